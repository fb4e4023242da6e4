"""bwrt — MI355X-native path tracer (host side over libbwrt.so's C ABI).

The product is the HIP library bwidman-raytracer_amd/lib/libbwrt.so
(include/rt_abi.h); this package is the Python host mirror of the
reference's driver (scenes, render loop, multi-GPU sharding).
"""
from . import abi, scenes  # noqa: F401
from .renderer import Renderer, render_multi, shard_rows  # noqa: F401

__all__ = ["abi", "scenes", "Renderer", "render_multi", "shard_rows"]
