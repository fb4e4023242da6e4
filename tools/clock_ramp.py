#!/usr/bin/env python3
"""Render time and shader clock per launch from a cold start (tools only):
config-3 renders back to back on the context's stream, each followed by a
50-us clock probe (tools/micro/clock_probe.hip: s_memtime ticks per
s_memrealtime tick), so a trend in the per-launch time can be read against
the GPU's clock.  usage: tools/clock_ramp.py [N_LAUNCHES] [--config c3] [--reseed-at K] [--pause-at K]
"""
import argparse
import ctypes as C
import os
import sys

os.environ.setdefault("BWRT_TUNING", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "bwidman-raytracer_amd")]
import torch  # noqa: E402

from bwrt import Renderer, abi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", nargs="?", type=int, default=60)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reseed-at", type=int, default=-1,
                    help="re-seed the RNG (y*W+x) before this launch: a transient that comes back is the RNG's")
    ap.add_argument("--pause-at", type=int, default=-1, help="idle the GPU 200 ms before this launch")
    a = ap.parse_args()
    probe = C.CDLL(os.path.join(REPO, "build", "libclockprobe.so"))
    probe.clock_probe_launch.argtypes = [C.c_void_p, C.c_uint, C.c_void_p]
    key, W, H, SPP, MB, _ = scenes.CONFIGS[a.config]
    lib = abi.load()
    r = Renderer(0, lib=lib)
    r.set_kernel_timing(False)
    r.set_scene(scenes.SCENES[key]())
    r.init_rand(W, H)
    dev = torch.device("cuda", 0)
    img = torch.empty(H * W, dtype=torch.int32, device=dev)
    out = torch.zeros((a.n, 2), dtype=torch.int64, device=dev)
    stream = torch.cuda.ExternalStream(r.stream_handle(), device=dev)
    p = r.params(W, H, SPP, MB, first_frame=1)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.n)]
    torch.cuda.synchronize()
    import time
    for i in range(a.n):
        if i == a.reseed_at:
            r.init_rand(W, H)  # (on the context's stream, ordered after the renders)
        if i == a.pause_at:
            torch.cuda.synchronize()
            time.sleep(0.2)
        evs[i][0].record(stream)
        r.render_device(p, img.data_ptr(), stream.cuda_stream)
        evs[i][1].record(stream)
        probe.clock_probe_launch(out[i].data_ptr(), 50, stream.cuda_stream)
    torch.cuda.synchronize()
    o = out.cpu().tolist()
    for i in range(a.n):
        ms = evs[i][0].elapsed_time(evs[i][1])
        mhz = o[i][0] / (o[i][1] * 10e-3) if o[i][1] else 0.0
        print(f"launch {i:3d}: render {ms:.4f} ms  shader clock {mhz:7.1f} MHz", flush=True)
    r.close()


if __name__ == "__main__":
    main()
