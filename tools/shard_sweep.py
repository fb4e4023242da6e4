#!/usr/bin/env python3
"""Per-rank kernel time of a row shard on ONE GPU (the work one rank of an
N-GPU run does), for several workgroup sizes: rehearses the N = 2/4/8 bench
on a single MI355X.  usage: tools/shard_sweep.py [--config c3] [--strides 1,2,4,8]
                                                  [--blocks 0,64,128,256] [--reps 20]
"""
import argparse
import os

os.environ.setdefault("BWRT_TUNING", "1")  # the library reads BWRT_* knobs only under it
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "bwidman-raytracer_amd")]
import torch  # noqa: E402

from bwrt import Renderer, abi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--strides", default="1,2,4,8")
    ap.add_argument("--blocks", default="0,64,128,256")
    ap.add_argument("--tiles", default="-1", help="wave tile widths; -1 = the library's launch policy")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    key, W, H, SPP, MB, _ = scenes.CONFIGS[a.config]
    lib = abi.load()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    for tile in [int(t) for t in a.tiles.split(",")]:
        for blk in [int(b) for b in a.blocks.split(",")]:
            os.environ["BWRT_BLOCK"] = str(blk)
            if tile >= 0:
                os.environ["BWRT_TILE"] = str(tile)
            else:
                os.environ.pop("BWRT_TILE", None)
            r = Renderer(0, lib=lib)
            r.set_scene(scenes.SCENES[key]())
            for g in [int(s) for s in a.strides.split(",")]:
                rows = -(-H // g)
                img = torch.empty(rows * W, dtype=torch.int32, device=dev)
                p = r.params(W, H, SPP, MB, first_frame=1, row_offset=0, row_stride=g)
                r.init_rand(W, H, 0, g)
                for _ in range(3):
                    r.render_device(p, img.data_ptr(), stream.cuda_stream)
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(a.reps)]
                for e0, e1 in evs:
                    e0.record(stream)
                    r.render_device(p, img.data_ptr(), stream.cuda_stream)
                    e1.record(stream)
                torch.cuda.synchronize()
                ms = sorted(e0.elapsed_time(e1) for e0, e1 in evs)
                print(f"{a.config} tile {tile:2d} block {blk:3d} stride {g}: median {ms[len(ms)//2]:.4f} ms "
                      f"min {ms[0]:.4f}  (x{g} = {ms[len(ms)//2]*g:.4f})", flush=True)
            r.close()


if __name__ == "__main__":
    main()
