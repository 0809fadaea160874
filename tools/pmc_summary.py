"""Per-launch HBM bytes of the sweep / pair / covariance-terms kernels from two
rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, runs of their own, no kernel
filter).

MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide streaming reads, so it is
doubled; WRITE_SIZE is taken as is.  usage: pmc_summary.py OUTDIR CONFIG_TAG N T R
"""
import csv
import glob
import json
import os
import re
import sys

KERNELS = {"sweep": r"ame_sweep\d?_kernel", "pairs": r"ame_pairs2?_kernel", "cov": r"ame_cov_kernel"}


def per_launch(outdir, counter):
    """{kernel class: (median per-launch value, launches)}"""
    vals = {}
    for f in glob.glob(os.path.join(outdir, f"pmc_{counter}", "**", "*counter_collection.csv"),
                       recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                for cls, pat in KERNELS.items():
                    if re.search(pat, row["Kernel_Name"]):
                        key = (cls, row["Dispatch_Id"])
                        vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    out = {}
    for cls in KERNELS:
        v = sorted(x for (c, _), x in vals.items() if c == cls)
        if v:
            out[cls] = (v[len(v) // 2], len(v))
    if not out:
        raise SystemExit(f"no {counter} rows under {outdir}")
    return out


def main():
    outdir, tag = sys.argv[1], sys.argv[2]
    n, T, r = (int(x) for x in sys.argv[3:6])
    d = 2 + 2 * r
    alg = {"sweep": 8.0 * n * (n - 1) * T + 8.0 * n * T * d + 8.0 * n * T * d * d,
           "pairs": 4.0 * n * (n - 1) * T + 4.0 * n * T * 2 * r,
           "cov": 4.0 * n * T * d * d}
    fetch = per_launch(outdir, "FETCH_SIZE")
    write = per_launch(outdir, "WRITE_SIZE")
    kernels = {}
    for cls in KERNELS:
        if cls not in fetch:
            continue
        rd = 2.0 * fetch[cls][0] * 1024.0     # gfx950 FETCH_SIZE correction
        wr = write.get(cls, (0.0, 0))[0] * 1024.0
        kernels[cls] = {"kernel": KERNELS[cls], "launches": [fetch[cls][1], write.get(cls, (0, 0))[1]],
                        "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                        "hbm_bytes_per_launch": rd + wr, "alg_bytes": alg[cls],
                        "traffic_over_alg": (rd + wr) / alg[cls]}
    pp = os.path.join(outdir, "pmc_pairs.json")   # MFMA pass (tools/pmc_pairs.py), if taken
    if "pairs" in kernels and os.path.exists(pp):
        z = json.load(open(pp))
        if z.get("mfma_busy_est") is not None:
            kernels["pairs"]["mfma_busy"] = z["mfma_busy_est"]
            kernels["pairs"]["mfma_counters"] = {k: z.get(k) for k in
                                                 ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE")}
            kernels["pairs"]["mfma_method"] = ("SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs "
                                               "x 256 CUs x 4 SIMDs), median dispatch")
    out = {"config_tag": tag,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; FETCH_SIZE x2 (gfx950)",
           "kernels": kernels}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
