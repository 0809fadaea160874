"""Per-launch HBM bytes of the sweep kernel from two rocprofv3 PMC passes.

MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide streaming reads, so it is
doubled; WRITE_SIZE is taken as is.  usage: pmc_summary.py OUTDIR CONFIG_TAG
"""
import csv
import glob
import json
import os
import sys


def per_launch(outdir, counter):
    vals = {}
    for f in glob.glob(os.path.join(outdir, f"pmc_{counter}", "**", "*counter_collection.csv"),
                       recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                key = row["Dispatch_Id"]
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows under {outdir}")
    v = sorted(vals.values())
    return v[len(v) // 2], len(v)   # median over launches


def main():
    outdir, tag = sys.argv[1], sys.argv[2]
    fetch_kib, nf = per_launch(outdir, "FETCH_SIZE")
    write_kib, nw = per_launch(outdir, "WRITE_SIZE")
    read_b = 2.0 * fetch_kib * 1024.0     # gfx950 FETCH_SIZE correction
    write_b = write_kib * 1024.0
    out = {
        "config_tag": tag,
        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; FETCH_SIZE x2 (gfx950)",
        "kernels": {"sweep": {"kernel": "ame_sweep3_kernel", "launches": [nf, nw],
                              "read_bytes_per_launch": read_b, "write_bytes_per_launch": write_b,
                              "hbm_bytes_per_launch": read_b + write_b}},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
