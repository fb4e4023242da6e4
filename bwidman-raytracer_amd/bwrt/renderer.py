"""Python host mirror of the reference's render driver over the C ABI.

Mirrors /root/reference/bwidman-raytracer/src/Main.cu: allocateScene()
(:38-109) -> Renderer.set_scene(); the frame loop's render() +
accumulatedFrames++ (:467-480) -> Renderer.render(); controls()' reset
(Controls.cuh:15..69) -> Renderer.reset_accumulation() / set_camera().
Every call goes to libbwrt.so: Renderer(device) renders with the HIP
kernels; Renderer.cpu(threads) makes a context of the library's scalar C++
CPU fallback (rt_create_cpu, the same per-ray arithmetic, bit-identical
results).  A GPU renderer never falls back to the CPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


class Renderer:
    def __init__(self, device: int = 0, lib=None, _cpu_threads=None):
        self.lib = lib or abi.load()
        self.ctx = C.c_void_p()
        if _cpu_threads is None:
            abi.check(self.lib, self.lib.rt_create(device, C.byref(self.ctx)))
        else:
            abi.check(self.lib, self.lib.rt_create_cpu(_cpu_threads, C.byref(self.ctx)))
        self.device = device if _cpu_threads is None else -1
        self.scene = None

    @classmethod
    def cpu(cls, threads: int = 0, lib=None) -> "Renderer":
        """A context of the scalar C++ CPU fallback on `threads` host threads
        (0 = every CPU this process may run on)."""
        return cls(-1, lib=lib, _cpu_threads=threads)

    @property
    def is_cpu(self) -> bool:
        return self.device < 0

    @property
    def threads(self) -> int:
        """Host threads of a CPU renderer (0 for a GPU one)."""
        return self.lib.rt_context_threads(self.ctx)

    # -- context lifetime -------------------------------------------------
    def close(self):
        if self.ctx:
            self.lib.rt_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, status):
        return abi.check(self.lib, status, self.ctx)

    # -- scene / camera / accumulation -----------------------------------
    def set_scene(self, scene):
        self.scene = scene
        self._check(self.lib.rt_set_scene(self.ctx, C.byref(scene.struct)))

    def set_camera(self, camera):
        self._check(self.lib.rt_set_camera(self.ctx, C.byref(camera)))

    def reset_accumulation(self):
        self._check(self.lib.rt_reset_accumulation(self.ctx))

    @property
    def frame_counter(self) -> int:
        return self.lib.rt_frame_counter(self.ctx)

    def set_max_bounces(self, mb: int):
        self._check(self.lib.rt_set_max_bounces(self.ctx, mb))

    def set_background(self, r: float, g: float, b: float):
        """backgroundColor (Main.cu:27): radiance of misses and the depth cut-off."""
        self._check(self.lib.rt_set_background(self.ctx, r, g, b))

    def set_samples_per_pixel(self, n: int):
        """samplesPerPixel (Main.cu:27, 296-299): n paths per frame from one
        jittered camera ray, the last one kept and scaled by 1/n (default 1)."""
        self._check(self.lib.rt_set_samples_per_pixel(self.ctx, n))

    def get_camera(self):
        from .abi import Camera
        cam = Camera()
        self._check(self.lib.rt_get_camera(self.ctx, C.byref(cam)))
        return cam

    def controls(self, keys, delta_time: float) -> int:
        """controls() (Controls.cuh:5-75) for one frame: `keys` is an int mask
        or an iterable of key names ("W", "LEFT", ...).  Returns the
        RT_CONTROLS_* flags; movement restarts accumulation."""
        from .abi import KEYS
        if not isinstance(keys, int):
            keys = sum(KEYS[k] for k in keys)
        flags = self.lib.rt_controls(self.ctx, keys, delta_time)
        if flags < 0:
            self._check(flags)
        return flags

    def init_rand(self, width, height, row_offset=0, row_stride=1):
        self._check(self.lib.rt_init_rand(self.ctx, width, height, row_offset, row_stride))

    # -- rendering ----------------------------------------------------------
    @staticmethod
    def params(width, height, samples, max_bounces, first_frame=0, row_offset=0, row_stride=1):
        return abi.RenderParams(width, height, samples, max_bounces, first_frame, row_offset,
                                row_stride)

    def render_simple(self, width: int, height: int, samples: int) -> np.ndarray:
        """Drop-in render(width, height, samples): continue accumulation."""
        out = np.empty((height, width, 4), dtype=np.uint8)
        self._check(self.lib.rt_render(self.ctx, width, height, samples, out.ctypes.data))
        return out

    def render(self, width, height, samples, max_bounces=abi.RT_DEFAULT_MAX_BOUNCES, first_frame=0,
               row_offset=0, row_stride=1, want_accum=False):
        rows = self.lib.rt_shard_rows(height, row_offset, row_stride)
        out = np.empty((rows, width, 4), dtype=np.uint8)
        acc = np.empty((rows, width, 3), dtype=np.float32) if want_accum else None
        p = self.params(width, height, samples, max_bounces, first_frame, row_offset, row_stride)
        self._check(self.lib.rt_render_ex(self.ctx, C.byref(p), out.ctypes.data,
                                          acc.ctypes.data if acc is not None else None))
        return (out, acc) if want_accum else out

    def render_cpu(self, width, height, samples, max_bounces=abi.RT_DEFAULT_MAX_BOUNCES, first_frame=0,
                   row_offset=0, row_stride=1, threads=0, want_accum=False):
        """rt_render_cpu: render() on a CPU renderer with this call's thread count."""
        rows = self.lib.rt_shard_rows(height, row_offset, row_stride)
        out = np.empty((rows, width, 4), dtype=np.uint8)
        acc = np.empty((rows, width, 3), dtype=np.float32) if want_accum else None
        p = self.params(width, height, samples, max_bounces, first_frame, row_offset, row_stride)
        self._check(self.lib.rt_render_cpu(self.ctx, C.byref(p), threads, out.ctypes.data,
                                           acc.ctypes.data if acc is not None else None))
        return (out, acc) if want_accum else out

    def render_device(self, params: abi.RenderParams, rgba_ptr: int, stream_ptr: int | None = None):
        self._check(self.lib.rt_render_device(self.ctx, C.byref(params), rgba_ptr, stream_ptr))

    def synchronize(self):
        self._check(self.lib.rt_synchronize(self.ctx))

    def stream_handle(self) -> int:
        """The context's own hipStream_t (rt_get_stream): renders on it defer
        their end event (no marker packet between back-to-back renders)."""
        return self.lib.rt_get_stream(self.ctx) or 0

    def last_kernel_ms(self) -> float:
        return self.lib.rt_last_kernel_ms(self.ctx)

    def last_kernel_name(self) -> str:
        """The render kernel the last GPU render launched (rt_last_kernel_name)."""
        return self.lib.rt_last_kernel_name(self.ctx).decode()

    def set_kernel_timing(self, enable: bool):
        """Per-launch timing events for last_kernel_ms (rt_set_kernel_timing)."""
        self._check(self.lib.rt_set_kernel_timing(self.ctx, int(bool(enable))))

    def deinterleave_device(self, gathered_ptr, image_ptr, width, height, shards, rows_per_shard,
                            stream_ptr=None):
        self._check(self.lib.rt_deinterleave_rows_device(self.ctx, gathered_ptr, image_ptr, width,
                                                         height, shards, rows_per_shard,
                                                         stream_ptr))

    # -- checkpoint / resume -----------------------------------------------
    def get_state(self, rows, width):
        rng = np.empty((6, rows, width), dtype=np.uint32)
        acc = np.empty((rows, width, 3), dtype=np.float32)
        self._check(self.lib.rt_get_state(self.ctx, rng.ctypes.data, acc.ctypes.data))
        return rng, acc

    def set_state(self, rng, acc, frame_counter):
        rng = np.ascontiguousarray(rng, dtype=np.uint32)
        acc = np.ascontiguousarray(acc, dtype=np.float32)
        self._check(self.lib.rt_set_state(self.ctx, rng.ctypes.data, acc.ctypes.data,
                                          frame_counter))


def shard_rows(height: int, row_offset: int, row_stride: int) -> int:
    return len(range(row_offset, height, row_stride)) if row_stride > 0 else 0


def render_multi(renderers, width: int, height: int, samples: int) -> np.ndarray:
    """rt_render_multi: one image across several Renderers (one per GPU, same
    scene/camera set on each) in this process; returns (H, W, 4) uint8, row 0
    = bottom.  Renderer i renders rows y = i (mod len(renderers))."""
    lib = renderers[0].lib
    arr = (C.c_void_p * len(renderers))(*[r.ctx.value for r in renderers])
    out = np.empty((height, width, 4), np.uint8)
    rc = lib.rt_render_multi(arr, len(renderers), width, height, samples, out.ctypes.data)
    if rc != abi.RT_OK:
        renderers[0]._check(rc)
    return out
