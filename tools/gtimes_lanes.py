#!/usr/bin/env python3
"""Config 5's tail, lane by lane (-DRT_GTIMES build via BWRT_LIB): per-wave
spans of the BVH refill kernel and, inside each wave, when each lane's pixel
finished — how much of the slowest waves' time runs with few live lanes.
usage: BWRT_LIB=.../c5gt/libbwrt.so tools/gtimes_lanes.py [config] [stride]"""
import os

os.environ.setdefault("BWRT_TUNING", "1")  # the library reads BWRT_* knobs only under it
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "bwidman-raytracer_amd")]
import torch  # noqa: E402

from bwrt import Renderer, abi, scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
g = int(sys.argv[2]) if len(sys.argv) > 2 else 8
key, W, H, SPP, MB, _ = scenes.CONFIGS[cfg]
r = Renderer(0, lib=abi.load())
r.set_scene(scenes.SCENES[key]())
img = torch.empty(-(-H // g) * W, dtype=torch.int32, device="cuda")
p = r.params(W, H, SPP, MB, first_frame=1, row_offset=0, row_stride=g)
r.init_rand(W, H, 0, g)
r.render_device(p, img.data_ptr(), None)
torch.cuda.synchronize()
r.init_rand(W, H, 0, g)
path = os.path.join(REPO, "gpurun_out", f"gtimes_lanes_{cfg}_{g}.bin")
os.makedirs(os.path.dirname(path), exist_ok=True)
os.environ["BWRT_GTIMES"] = path
r.render_device(p, img.data_ptr(), None)
torch.cuda.synchronize()
raw = np.fromfile(path, dtype=np.uint64).astype(np.int64)
os.unlink(path)
NG = 65536
se = raw[:2 * NG].reshape(-1, 2)
n = int(np.nonzero(se[:, 1])[0].max()) + 1
se = se[:n]
lanes = raw[2 * NG:2 * NG + 64 * n].reshape(n, 64)
t0 = se[:, 0].min()
s, e = (se[:, 0] - t0) / 100.0, (se[:, 1] - t0) / 100.0  # us
dur = e - s
print(f"{cfg} stride {g}: {n} waves, kernel span {e.max():.0f} us; wave span us: mean {dur.mean():.0f} "
      f"p50 {np.median(dur):.0f} p90 {np.percentile(dur, 90):.0f} p99 {np.percentile(dur, 99):.0f} max {dur.max():.0f}")
valid = lanes > 0
fin = np.where(valid, (lanes - t0) / 100.0 - s[:, None], np.nan)  # lane finish, us after its wave's start
print(f"  lane finish / wave span (all waves): mean {np.nanmean(fin / dur[:, None]):.3f}")
order = np.argsort(-dur)
for q in (1, 10, 100, 1000):
    sel = order[:q]
    f = np.sort(fin[sel], axis=1)
    # live lanes over the wave's life (in tenths of its span), averaged over the q slowest waves
    tl = np.linspace(0, 1, 11)
    live = [np.mean([(np.nan_to_num(fin[i], nan=-1) > x * dur[i]).sum() for i in sel]) for x in tl]
    print(f"  slowest {q:4d}: span {dur[sel].mean():.0f} us, median lane done at {np.nanmedian(f[:, :] / dur[sel][:, None]):.2f} "
          f"of span; live lanes at 0,.1..1 of span: " + " ".join(f"{v:.0f}" for v in live))
# time the slowest waves spend with <= k live lanes
for k in (32, 16, 8, 4):
    sel = order[:100]
    frac = []
    for i in sel:
        ft = np.sort(np.nan_to_num(fin[i], nan=0.0))
        live_from = ft[-(k + 1)] if k + 1 <= 64 else 0.0  # from this time on at most k lanes are live
        frac.append((dur[i] - live_from) / dur[i])
    print(f"  slowest 100: share of span with <= {k} live lanes: {np.mean(frac):.3f}")
