"""Sum SQ / SQC counters of the sweep kernel per dispatch (median over
dispatches) from rocprofv3 --pmc passes, and normalise per workgroup per node
step.  usage: pmc_sq.py OUTDIR N T_LOCAL"""
import csv
import glob
import os
import sys


def main():
    out, n, TL = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    kname = sys.argv[4] if len(sys.argv) > 4 else "ame_sweep"
    vals = {}
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kname not in row["Kernel_Name"]:
                    continue
                key = (row["Counter_Name"], os.path.dirname(f), row["Dispatch_Id"])
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    per = {}
    for (c, _, _), v in vals.items():
        per.setdefault(c, []).append(v)
    steps = TL * (n + 1)
    for c in sorted(per):
        v = sorted(per[c])
        med = v[len(v) // 2]
        print(f"{c:28s} per-dispatch {med:14.4g}   per WG-step {med / steps:10.1f}")
    if "SQ_WAVE_CYCLES" in per:
        wc = sorted(per["SQ_WAVE_CYCLES"])[len(per["SQ_WAVE_CYCLES"]) // 2]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS"):
            if c in per:
                print(f"  {c} / SQ_WAVE_CYCLES = {sorted(per[c])[len(per[c]) // 2] / wc:.3f}")


if __name__ == "__main__":
    main()
