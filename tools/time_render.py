#!/usr/bin/env python3
"""Median kernel time of one render on GPU 0: tools/time_render.py SCENE W H SPP MB [REPS]
(launch knobs from the BWRT_* environment, read when the context is made and
only under BWRT_TUNING=1, which this script sets)."""
import os
os.environ["BWRT_TUNING"] = "1"
import statistics
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bwidman-raytracer_amd")]
import torch  # noqa: E402,F401  (one HIP runtime with libbwrt)

from bwrt import Renderer, scenes  # noqa: E402

scene, w, h, spp, mb = sys.argv[1], *map(int, sys.argv[2:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
with Renderer(0) as r:
    r.set_scene(scenes.SCENES[scene]())
    r.init_rand(w, h)
    ts = []
    for _ in range(reps + 1):
        r.render(w, h, spp, mb, first_frame=1)
        ts.append(r.last_kernel_ms())
print(f"{scene} {w}x{h} {spp}spp mb{mb} {os.environ.get('BWRT_BVH_PAIRS', '0')}: median {statistics.median(ts[1:]):.3f} ms")
