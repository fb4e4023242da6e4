"""Copy the judged artefacts of a tools/gpu_round.sh run into profiles/<tag>/.

usage: python tools/collect_profiles.py TAG   (reads gpurun_out/TAG)

profiles/<tag>/: bench.log, pytest_gpu.log, smoke.log, rocprof kernel/domain
stats (rocprofv3 --kernel-trace --stats of `bench.py --no-cpu-baseline`),
pmc_summary.json (tools/pmc.sh counters averaged per launch of the render
kernel) and traffic.json (HBM bytes per launch, MI355X_MICROARCH.md
corrections); profiles/traffic_latest.json is the copy bench.py reads.
"""
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    src = os.path.join(REPO, "gpurun_out", tag)
    dst = os.path.join(REPO, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for f in ("bench.log", "pytest_gpu.log", "smoke.log"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    for f, g in (("run_kernel_stats.csv", "rocprof_kernel_stats.csv"),
                 ("run_domain_stats.csv", "rocprof_domain_stats.csv")):
        p = os.path.join(src, "prof", f)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, g))
    avg, dur = load(os.path.join(src, "pmc"), "rt_render")
    summ = dict(sorted(avg.items()))
    summ["profiled_kernel_s"] = dur
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(summ, f, indent=1)
    fetch = avg["FETCH_SIZE"] * 1024 * 2
    write = avg["WRITE_SIZE"] * 1024
    rec = {
        "workload": "07-1920x1080-8spp-4b-rows1",
        "source": f"profiles/{tag}/pmc_summary.json (tools/pmc.sh on MI355X)",
        "hbm_bytes_per_launch": fetch + write,
        "fetch_bytes_corrected": fetch,
        "write_bytes": write,
        "FETCH_SIZE_KiB_raw": avg["FETCH_SIZE"],
        "WRITE_SIZE_KiB_raw": avg["WRITE_SIZE"],
        "profiled_kernel_s": dur,
        "valu": {
            "insts_valu_per_launch": avg["SQ_INSTS_VALU"],
            "lane_ops_per_launch": avg.get("SQ_THREAD_CYCLES_VALU"),
            "active_lanes_per_valu": avg.get("SQ_THREAD_CYCLES_VALU", 0) / avg["SQ_INSTS_VALU"],
            "waves": avg.get("SQ_WAVES"),
        },
    }
    for p in (os.path.join(dst, "traffic.json"), os.path.join(REPO, "profiles", "traffic_latest.json")):
        with open(p, "w") as f:
            json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
