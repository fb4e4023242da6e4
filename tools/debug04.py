import sys, os
sys.path[:0] = ['bwidman-raytracer_amd', 'oracle', 'tests']
import torch  # noqa
import numpy as np
import oracle as O
from bwrt import Renderer, scenes
O.build()
r = Renderer(0)
bad = 0
for name, w, h, spp, mb in [("01", 256, 256, 1, 1), ("07", 1920, 1080, 8, 4)] + [("04", 1280, 720, 4, 3), ("07", 1920, 1080, 8, 4)] * 10:
    s = scenes.SCENES[name]()
    r.set_scene(s); r.init_rand(w, h)
    img = r.render(w, h, spp, mb, first_frame=1)
    st = O.OracleState(w, h)
    O.render(s, st, spp, mb, first_frame=1)
    rng, acc = r.get_state(h, w)
    d = np.argwhere((img != st.rgba).any(-1))
    bad += len(d) + int((rng != st.rng).sum())
    print(name, w, h, spp, mb, "pix diff", len(d), d[:3].tolist(), "rng diff", int((rng != st.rng).sum()),
          "acc diff", int((~((acc == st.accum) | (np.isnan(acc) & np.isnan(st.accum)))).sum()))
    if len(d):
        y, x = d[0]
        print("  gpu", img[y, x], "orc", st.rgba[y, x], "acc gpu", acc.reshape(-1,3)[y*w+x] if acc.ndim==2 else None)
print("TOTAL BAD", bad)
sys.exit(1 if bad else 0)
