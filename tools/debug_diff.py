import sys, os
sys.path[:0] = ['bwidman-raytracer_amd', 'oracle']
import numpy as np, oracle as O
from bwrt import Renderer, scenes
w, h, spp, mb = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
s = scenes.SCENES[sys.argv[5] if len(sys.argv) > 5 else '07']()
r = Renderer(0); r.set_scene(s)
img, acc = r.render(w, h, spp, mb, first_frame=1, want_accum=True)
rng, _ = r.get_state(h, w)
st = O.render_image(s, w, h, spp, mb)
d = np.argwhere((img != st.rgba).any(-1))
da = np.argwhere(~((acc == st.accum) | (np.isnan(acc) & np.isnan(st.accum))).all(-1))
dr = np.argwhere((rng != st.rng).any(0))
print('rgba diffs', len(d), 'accum diffs', len(da), 'rng diffs', len(dr))
for (y, x) in da[:10]:
    print(y, x, 'gpu', img[y, x], acc[y, x], 'orc', st.rgba[y, x], st.accum[y, x], 'rng eq', (rng[:, y, x] == st.rng[:, y, x]).all())
