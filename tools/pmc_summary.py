"""Summarise tools/pmc.sh output: per-kernel counter averages + derived metrics."""
import collections, csv, glob, json, os, sys

def load(outdir, kernel_sub="rt_render"):
    vals = collections.defaultdict(list)
    durs = []
    for f in sorted(glob.glob(os.path.join(outdir, "pass*", "run_counter_collection.csv")) + glob.glob(os.path.join(outdir, "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kernel_sub in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    return avg, (sum(durs) / len(durs) if durs else None)

if __name__ == "__main__":
    avg, dur = load(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "rt_render")
    d = dict(avg)
    if "SQ_INSTS_VALU" in d and "SQ_THREAD_CYCLES_VALU" in d:
        d["lanes_per_valu"] = d["SQ_THREAD_CYCLES_VALU"] / d["SQ_INSTS_VALU"]
    if "SQ_WAVES" in d and "SQ_INSTS_VALU" in d:
        d["valu_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
    if "SQ_WAVE_CYCLES" in d:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in d: d[k + "_frac"] = d[k] / d["SQ_WAVE_CYCLES"]
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in sorted(d.items())}, indent=1))
