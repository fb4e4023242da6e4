"""Extreme-scale parity probe: the stress scene scaled by 1e10 / 1e6 through the BVH and the
brute-force loop against the oracle (pixels, RNG and accumulators that differ).  GPU box only."""
import os, sys
os.environ["BWRT_TUNING"] = "1"  # the library reads BWRT_* knobs only under it
sys.path[:0] = ["bwidman-raytracer_amd", "oracle", "tests"]
import numpy as np
import oracle as O
from bwrt import Renderer, scenes
from test_gpu_parity import _scaled
O.build()
r = Renderer(0)
for k in [1e10, 1e6]:
    for mode in ["bvh", "brute"]:
        if mode == "brute": os.environ["BWRT_BVH_MIN"] = "100000000"
        else: os.environ.pop("BWRT_BVH_MIN", None)
        for mb in [0, 1, 3]:
            s = _scaled(scenes.stress_scene(), k)
            r.set_scene(s); r.init_rand(96, 54)
            img = r.render(96, 54, 2, mb, first_frame=1)
            st = O.OracleState(96, 54); O.render(s, st, 2, mb, first_frame=1)
            bad = np.argwhere((img != st.rgba).any(-1))
            rng, acc = r.get_state(st.rows, st.width)
            print(f"k={k:g} {mode} mb={mb}: {len(bad)} px differ {bad[:3].tolist()} rng diff {int((rng != st.rng).sum())} "
                  f"acc diff {int((~((acc == st.accum) | (np.isnan(acc) & np.isnan(st.accum)))).sum())}", flush=True)
            if len(bad):
                y, x = bad[0]; print("   gpu", img[y, x], "oracle", st.rgba[y, x], "acc", acc.reshape(54, 96, 3)[y, x], st.accum.reshape(54, 96, 3)[y, x])
