"""Config-5 fixtures at the config's own frame count (TEST INFRASTRUCTURE).

The oracle (oracle/oracle.c, the reference's brute-force loop over all 10,256
primitives) needs minutes for these rows, too long for a GPU test, so its
results are committed as SHA-256 digests of the arrays:

  rows8   rows y = 3 mod 135 (8 full-width rows) of the stress scene,
          1920x1080, 32 spp (frames 1..32), maxBounces 8
  rows15  rows y = 5 mod 72 (15 rows: every 9th row of the 8-GPU run's
          shard y = 5 mod 8), same workload

per sample: RGBA8 rows (row 0 = bottom), frameSum (rows, W, 3) float32 and
the RNG planes (6, rows, W) uint32 after the last frame.  Used by
tests/test_cpu_fallback.py (the CPU fallback reproduces them) and
tests/test_gpu_parity.py (the refill kernel does).

  python tests/golden/make_c5_golden.py   (about 8 minutes on 8 cores)
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "bwidman-raytracer_amd"), os.path.join(REPO, "oracle")]

import oracle as O  # noqa: E402
from bwrt import scenes  # noqa: E402

SAMPLES = {"rows8": (3, 135), "rows15": (5, 72)}
W, H, SPP, MB = 1920, 1080, 32, 8


def digests(rgba, accum, rng):
    return {"rgba": hashlib.sha256(rgba.tobytes()).hexdigest(),
            "accum": hashlib.sha256(accum.tobytes()).hexdigest(),
            "rng": hashlib.sha256(rng.tobytes()).hexdigest()}


def main():
    out = {"workload": f"stress scene {W}x{H}, {SPP} spp, maxBounces {MB}", "width": W, "height": H,
           "spp": SPP, "max_bounces": MB, "samples": {}}
    s = scenes.stress_scene()
    for name, (off, stride) in SAMPLES.items():
        t0 = time.time()
        st = O.OracleState(W, H, off, stride)
        O.render(s, st, SPP, MB, first_frame=1)
        out["samples"][name] = {"row_offset": off, "row_stride": stride, "rows": st.rows,
                                **digests(st.rgba, st.accum, st.rng),
                                "rgba_first_row_mean": float(st.rgba[0, :, :3].mean())}
        print(f"{name}: {st.rows} rows in {time.time() - t0:.0f} s", flush=True)
    with open(os.path.join(HERE, "c5_rows_32spp.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
