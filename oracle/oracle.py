"""ctypes wrapper of liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, as the checker / the CPU baseline.  The product (libbwrt.so,
bwrt package) never imports it.  See oracle.h for what the oracle restates
and how its parity is pinned.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or \
            os.path.getmtime(LIB_PATH) < max(os.path.getmtime(os.path.join(HERE, f))
                                             for f in ("oracle.c", "oracle.h")):
        subprocess.run(["make", "-B" if force else "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if LIB_PATH_IN_USE == LIB_PATH and not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH_IN_USE)
        L.orc_curand_init.argtypes = [C.c_ulonglong, C.POINTER(C.c_uint32)]
        L.orc_curand_init.restype = None
        L.orc_curand.argtypes = [C.POINTER(C.c_uint32)]
        L.orc_curand.restype = C.c_uint32
        for f in ("orc_atanf", "orc_sinf", "orc_cosf"):
            getattr(L, f).argtypes = [C.c_float]
            getattr(L, f).restype = C.c_float
        L.orc_render_rows.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_uint, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_int, C.c_int]
        L.orc_render_rows.restype = C.c_int
        L.orc_set_background.argtypes = [C.c_float, C.c_float, C.c_float]
        L.orc_set_background.restype = None
        L.orc_set_samples_per_pixel.argtypes = [C.c_int]
        L.orc_set_samples_per_pixel.restype = None
        L.orc_last_counters.argtypes = [C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]
        L.orc_last_counters.restype = None
        _lib = L
    return _lib


def use_library(path: str):
    """Switch to another build of the oracle (the pin-sensitivity mutants,
    tests/golden/make_pin_sensitivity.py); use_library(LIB_PATH) goes back."""
    global _lib, LIB_PATH_IN_USE
    _lib = None
    LIB_PATH_IN_USE = path
    return lib()


LIB_PATH_IN_USE = LIB_PATH


def curand_stream(seed: int, n: int) -> np.ndarray:
    st = (C.c_uint32 * 6)()
    lib().orc_curand_init(seed, st)
    return np.array([lib().orc_curand(st) for _ in range(n)], dtype=np.uint32)


def curand_init(seed: int) -> np.ndarray:
    st = (C.c_uint32 * 6)()
    lib().orc_curand_init(seed, st)
    return np.array(list(st), dtype=np.uint32)


class OracleState:
    """Progressive state of one shard: rng planes (6,rows,W), accum (rows,W,3)."""

    def __init__(self, width, height, row_offset=0, row_stride=1):
        self.width, self.height = width, height
        self.row_offset, self.row_stride = row_offset, row_stride
        self.rows = len(range(row_offset, height, row_stride))
        self.rng = np.zeros((6, self.rows, width), dtype=np.uint32)
        self.accum = np.zeros((self.rows, width, 3), dtype=np.float32)
        self.rgba = np.zeros((self.rows, width, 4), dtype=np.uint8)
        self.seeded = False
        self.frame = 1


def render(scene, state: OracleState, passes: int, max_bounces: int,
           first_frame: int | None = None, threads: int = 0, background=(0.0, 0.0, 0.0),
           samples_per_pixel: int = 1) -> np.ndarray:
    """Render `passes` progressive frames; returns the RGBA8 rows (row 0 = bottom).
    samples_per_pixel: the reference's in-frame loop (Main.cu:27, 296-299)."""
    ff = state.frame if first_frame is None else first_frame
    lib().orc_set_background(*[float(c) for c in background])
    lib().orc_set_samples_per_pixel(int(samples_per_pixel))
    rc = lib().orc_render_rows(C.cast(scene.ptr(), C.c_void_p), state.width, state.height,
                               state.row_offset, state.row_stride, state.rows, ff, passes,
                               max_bounces, state.rng.ctypes.data, state.accum.ctypes.data,
                               state.rgba.ctypes.data, 0 if state.seeded else 1, threads)
    if rc != 0:
        raise ValueError("orc_render_rows: bad arguments")
    state.seeded = True
    state.frame = ff + passes
    return state.rgba


def render_image(scene, width, height, passes, max_bounces, row_offset=0, row_stride=1,
                 threads=0):
    st = OracleState(width, height, row_offset, row_stride)
    render(scene, st, passes, max_bounces, first_frame=1, threads=threads)
    return st


def last_counters():
    q, p = C.c_ulonglong(), C.c_ulonglong()
    lib().orc_last_counters(C.byref(q), C.byref(p))
    return q.value, p.value
