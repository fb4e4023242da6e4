"""Turn a tools/pmc.sh run into profiles/traffic_<tag>.json for bench.py.

HBM bytes per launch of rt_render_kernel/rt_render_sorted_kernel, corrected
as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KiB) reads exactly half
the bytes of a coalesced streaming read on gfx950 -> x2 (calibrated for this
kernel's 4-byte-per-lane, 256-B-per-wave reads: the corrected value equals
the 24 B/pixel of RNG state the launch must read), WRITE_SIZE (KiB) exact.
VALU: SQ_INSTS_VALU (wave instructions) and SQ_THREAD_CYCLES_VALU (active
lanes summed over VALU instructions) per launch.

usage: python tools/make_traffic_json.py PMC_DIR WORKLOAD_KEY OUT.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def main():
    pmc_dir, key, out = sys.argv[1], sys.argv[2], sys.argv[3]
    avg, dur = load(pmc_dir, "rt_render")
    fetch = avg["FETCH_SIZE"] * 1024 * 2
    write = avg["WRITE_SIZE"] * 1024
    rec = {
        "workload": key,
        "source": os.path.relpath(pmc_dir),
        "hbm_bytes_per_launch": fetch + write,
        "fetch_bytes_corrected": fetch,
        "write_bytes": write,
        "FETCH_SIZE_KiB_raw": avg["FETCH_SIZE"],
        "WRITE_SIZE_KiB_raw": avg["WRITE_SIZE"],
        "profiled_kernel_s": dur,
    }
    if "SQ_INSTS_VALU" in avg:
        rec["valu"] = {
            "insts_valu_per_launch": avg["SQ_INSTS_VALU"],
            "lane_ops_per_launch": avg.get("SQ_THREAD_CYCLES_VALU"),
            "active_lanes_per_valu": avg.get("SQ_THREAD_CYCLES_VALU", 0) / avg["SQ_INSTS_VALU"],
            "waves": avg.get("SQ_WAVES"),
        }
    if "TCP_TOTAL_CACHE_ACCESSES_sum" in avg:
        # L1 (vector cache) line accesses: tag lookups and the lines it
        # requests from L2 (its misses), per launch — bench.py's
        # l1_line_roofline
        rec["l1"] = {
            "tag_accesses_per_launch": avg["TCP_TOTAL_CACHE_ACCESSES_sum"],
            "l2_requests_per_launch": avg.get("TCP_TCC_READ_REQ_sum"),
        }
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
