"""ctypes mirror of include/rt_abi.h (the C ABI of libbwrt.so).

The structs are byte-compatible with the reference's world types
(/root/reference/bwidman-raytracer/src/WorldTypes.cuh:4-53, Math.cuh:35-39);
tests/test_abi.py pins every size and offset.

Loading policy: the library is the product, so a missing or unloadable
libbwrt.so raises immediately.  Its scalar C++ CPU fallback (rt_create_cpu)
lives in the same library and runs only when asked for explicitly.  When PyTorch is
used in the same process (bench.py, multi-GPU), import torch BEFORE calling
load(): libbwrt.so then binds to the HIP runtime torch already loaded
(same soname libamdhip64.so.7), so device pointers and streams are shared.
"""
from __future__ import annotations

import ctypes as C
import os
import re

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "lib", "libbwrt.so")
HEADER_PATH = os.path.join(REPO_DIR, "include", "rt_abi.h")


class Vec3(C.Structure):
    """Math.cuh:35-39 vec3d / color (12 B)."""
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]

    def tolist(self):
        return [self.x, self.y, self.z]


class Material(C.Structure):
    """WorldTypes.cuh:15-20 (24 B)."""
    _fields_ = [("albedo", Vec3), ("emittance", C.c_float), ("roughness", C.c_float),
                ("refractive_index", C.c_float)]


class Sphere(C.Structure):
    """WorldTypes.cuh:22-26 (40 B)."""
    _fields_ = [("position", Vec3), ("radius", C.c_float), ("mat", Material)]


class Plane(C.Structure):
    """WorldTypes.cuh:28-32 (60 B)."""
    _fields_ = [("origin", Vec3), ("directions", Vec3 * 2), ("mat", Material)]


class Triangle(C.Structure):
    """WorldTypes.cuh:34-37 (60 B)."""
    _fields_ = [("vertices", Vec3 * 3), ("mat", Material)]


class Quad(C.Structure):
    """WorldTypes.cuh:39-42 (72 B)."""
    _fields_ = [("vertices", Vec3 * 4), ("mat", Material)]


class Camera(C.Structure):
    """WorldTypes.cuh:9-13 (24 B)."""
    _fields_ = [("position", Vec3), ("angle", C.c_float * 2), ("fov", C.c_float)]


class SceneStruct(C.Structure):
    """WorldTypes.cuh:44-53 (88 B); pointers are host pointers here."""
    _fields_ = [("camera", Camera),
                ("spheres", C.POINTER(Sphere)), ("sphere_count", C.c_int),
                ("planes", C.POINTER(Plane)), ("plane_count", C.c_int),
                ("triangles", C.POINTER(Triangle)), ("triangle_count", C.c_int),
                ("quads", C.POINTER(Quad)), ("quad_count", C.c_int)]


class RenderParams(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("samples", C.c_int),
                ("max_bounces", C.c_int), ("first_frame", C.c_uint),
                ("row_offset", C.c_int), ("row_stride", C.c_int)]


RT_OK = 0
RT_ERR_INVALID_ARGUMENT = -1
RT_ERR_NO_DEVICE = -2
RT_ERR_UNSUPPORTED = -6
RT_MAX_BOUNCES = 32
RT_DEFAULT_MAX_BOUNCES = 5

_lib = None


def _proto(lib):
    P = C.POINTER
    vp = C.c_void_p
    sigs = {
        "rt_version": (C.c_char_p, []),
        "rt_material_default": (Material, []),
        "rt_device_count": (C.c_int, []),
        "rt_create": (C.c_int, [C.c_int, P(vp)]),
        "rt_destroy": (None, [vp]),
        "rt_cpu_threads": (C.c_int, []),
        "rt_create_cpu": (C.c_int, [C.c_int, P(vp)]),
        "rt_context_threads": (C.c_int, [vp]),
        "rt_render_cpu": (C.c_int, [vp, P(RenderParams), C.c_int, vp, vp]),
        "rt_set_scene": (C.c_int, [vp, P(SceneStruct)]),
        "rt_set_camera": (C.c_int, [vp, P(Camera)]),
        "rt_reset_accumulation": (C.c_int, [vp]),
        "rt_frame_counter": (C.c_uint, [vp]),
        "rt_set_max_bounces": (C.c_int, [vp, C.c_int]),
        "rt_set_background": (C.c_int, [vp, C.c_float, C.c_float, C.c_float]),
        "rt_set_samples_per_pixel": (C.c_int, [vp, C.c_int]),
        "rt_get_camera": (C.c_int, [vp, P(Camera)]),
        "rt_apply_controls": (C.c_int, [P(Camera), C.c_uint, C.c_float]),
        "rt_controls": (C.c_int, [vp, C.c_uint, C.c_float]),
        "rt_init_rand": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.c_int]),
        "rt_render": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, vp]),
        "rt_render_ex": (C.c_int, [vp, P(RenderParams), vp, vp]),
        "rt_render_device": (C.c_int, [vp, P(RenderParams), vp, vp]),
        "rt_synchronize": (C.c_int, [vp]),
        "rt_get_stream": (vp, [vp]),
        "rt_render_multi": (C.c_int, [P(vp), C.c_int, C.c_int, C.c_int, C.c_int, vp]),
        "rt_last_kernel_ms": (C.c_float, [vp]),
        "rt_set_kernel_timing": (C.c_int, [vp, C.c_int]),
        "rt_shard_rows": (C.c_int, [C.c_int, C.c_int, C.c_int]),
        "rt_deinterleave_rows_device": (C.c_int, [vp, vp, vp, C.c_int, C.c_int, C.c_int,
                                                  C.c_int, vp]),
        "rt_get_state": (C.c_int, [vp, vp, vp]),
        "rt_set_state": (C.c_int, [vp, vp, vp, C.c_uint]),
        "rt_error_string": (C.c_char_p, [C.c_int]),
        "rt_last_error": (C.c_char_p, [vp]),
        "rt_last_kernel_name": (C.c_char_p, [vp]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def declared_functions(header: str = HEADER_PATH):
    """Names of every RT_API function declared in include/rt_abi.h."""
    with open(header) as f:
        text = f.read()
    return sorted(set(re.findall(r"RT_API[^;(]*?\b(rt_\w+)\s*\(", text)))


def load(path: str | None = None):
    """Load libbwrt.so (fails loudly if it is missing: no fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("BWRT_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise RuntimeError(
            f"libbwrt.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (the HIP library is the product; nothing runs without it)")
    lib = _proto(C.CDLL(p))
    if path is None:
        _lib = lib
    return lib


# Controls.cuh key bits (include/rt_abi.h RT_KEY_*)
KEYS = {"W": 1 << 0, "A": 1 << 1, "S": 1 << 2, "D": 1 << 3, "SPACE": 1 << 4, "LEFT_SHIFT": 1 << 5,
        "LEFT": 1 << 6, "RIGHT": 1 << 7, "UP": 1 << 8, "DOWN": 1 << 9, "ESCAPE": 1 << 10}
CONTROLS_MOVED = 1
CONTROLS_QUIT = 2


class RTError(RuntimeError):
    pass


def check(lib, status, ctx=None):
    if status != RT_OK:
        msg = lib.rt_error_string(status).decode()
        if ctx:
            last = lib.rt_last_error(ctx)
            if last:
                msg += ": " + last.decode()
        raise RTError(f"rt status {status}: {msg}")
    return status
