"""Per-phase VALU breakdown from tools/phase_lanes.sh: each RT_PHASE_TWICE
variant runs one phase a second time, so (variant - base) of SQ_INSTS_VALU /
SQ_THREAD_CYCLES_VALU per render launch is that phase's wave-instructions /
lane-cycles; the rest (posting, take-back, loop control, pixel load/store) is
base minus the four phases.  usage: tools/phase_lanes.py OUTDIR"""
import collections
import csv
import glob
import json
import os
import sys

PHASES = {"ph1": "closest hit (I-phase)", "ph2": "RANDDIR task (genRandomDirection)",
          "ph3": "SPEC task (microfacet sample, Fresnel, G)", "ph4": "path-end fold"}


def per_launch(d):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "rt_render_sorted_kernel" in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main(out):
    base = per_launch(os.path.join(out, "base"))
    rows, rest_i, rest_l = [], base["SQ_INSTS_VALU"], base["SQ_THREAD_CYCLES_VALU"]
    for v, name in PHASES.items():
        c = per_launch(os.path.join(out, v))
        di = c["SQ_INSTS_VALU"] - base["SQ_INSTS_VALU"]
        dl = c["SQ_THREAD_CYCLES_VALU"] - base["SQ_THREAD_CYCLES_VALU"]
        rest_i -= di
        rest_l -= dl
        rows.append({"phase": name, "valu_wave_insts": round(di), "lane_cycles": round(dl),
                     "lanes_per_valu": round(dl / di, 2) if di else None,
                     "share_of_insts": round(di / base["SQ_INSTS_VALU"], 4),
                     "idle_lane_slots": round(64 * di - dl),
                     "share_of_idle": round((64 * di - dl) / (64 * base["SQ_INSTS_VALU"] - base["SQ_THREAD_CYCLES_VALU"]), 4)})
    rows.append({"phase": "rest (posting, take-back, shading set-up, loop, load/store)", "valu_wave_insts": round(rest_i),
                 "lane_cycles": round(rest_l), "lanes_per_valu": round(rest_l / rest_i, 2),
                 "share_of_insts": round(rest_i / base["SQ_INSTS_VALU"], 4), "idle_lane_slots": round(64 * rest_i - rest_l),
                 "share_of_idle": round((64 * rest_i - rest_l) / (64 * base["SQ_INSTS_VALU"] - base["SQ_THREAD_CYCLES_VALU"]), 4)})
    res = {"base": {k: round(v) for k, v in base.items()},
           "base_lanes_per_valu": round(base["SQ_THREAD_CYCLES_VALU"] / base["SQ_INSTS_VALU"], 2), "phases": rows}
    print(json.dumps(res, indent=1))
    with open(os.path.join(out, "phase_lanes.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
