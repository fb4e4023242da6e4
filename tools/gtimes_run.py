#!/usr/bin/env python3
"""Per-group start/end times of one render (-DRT_GTIMES build via BWRT_LIB):
group-duration spread and the chip's active-group count over time.
usage: BWRT_LIB=.../gtimes/libbwrt.so tools/gtimes_run.py [config] [stride]"""
import os

os.environ.setdefault("BWRT_TUNING", "1")  # the library reads BWRT_* knobs only under it
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "bwidman-raytracer_amd")]
import torch  # noqa: E402

from bwrt import Renderer, abi, scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
g = int(sys.argv[2]) if len(sys.argv) > 2 else 1
key, W, H, SPP, MB, _ = scenes.CONFIGS[cfg]
r = Renderer(0, lib=abi.load())
r.set_scene(scenes.SCENES[key]())
img = torch.empty(-(-H // g) * W, dtype=torch.int32, device="cuda")
p = r.params(W, H, SPP, MB, first_frame=1, row_offset=0, row_stride=g)
r.init_rand(W, H, 0, g)
r.render_device(p, img.data_ptr(), None)
torch.cuda.synchronize()
path = os.path.join(REPO, "gpurun_out", f"gtimes_{cfg}_{g}.bin")
os.makedirs(os.path.dirname(path), exist_ok=True)
os.environ["BWRT_GTIMES"] = path
r.render_device(p, img.data_ptr(), None)
torch.cuda.synchronize()
t = np.fromfile(path, dtype=np.uint64).reshape(-1, 2)
n = int(np.nonzero(t[:, 1])[0].max()) + 1
t = t[:n].astype(np.int64)
t0 = t[:, 0].min()
s, e = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # us (100 MHz)
dur = e - s
print(f"{cfg} stride {g}: {n} groups, kernel span {e.max():.1f} us; duration us: mean {dur.mean():.1f} "
      f"p10 {np.percentile(dur, 10):.1f} p50 {np.median(dur):.1f} p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f}")
print(f"  last start {s.max():.1f} us; groups ending after 90% of span: {(e > 0.9 * e.max()).sum()}")
grid = np.linspace(0, e.max(), 41)
act = [int(((s <= x) & (e > x)).sum()) for x in grid]
print("  active groups over time:", " ".join(str(a) for a in act))
# cost by tile row band (blockIdx order = tile rows bottom-up)
nb = 16
band = np.array_split(np.arange(n), nb)
print("  mean duration by blockIdx band:", " ".join(f"{dur[b].mean():.0f}" for b in band))
os.unlink(path)
