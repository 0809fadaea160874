"""ELBO pair kernel (K3, the MFMA U V^T kernel): HBM bytes and MFMA activity per
launch from rocprofv3 PMC passes (tools/gpu_profile.sh).  Counters are summed
over the rows of one dispatch and the median over dispatches is reported.
MFMA-busy estimate = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x CUs x 4
SIMDs) (GRBM_GUI_ACTIVE sums the 8 XCDs, MI355X_MICROARCH.md).  usage:
pmc_pairs.py OUTDIR"""
import csv
import glob
import json
import os
import sys


def per_launch(outdir, sub, counter, kernel="ame_pairs"):
    vals = {}
    for f in glob.glob(os.path.join(outdir, sub, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter and kernel in row["Kernel_Name"]:
                    k = row["Dispatch_Id"]
                    vals[k] = vals.get(k, 0.0) + float(row["Counter_Value"])
    if not vals:
        return None
    v = sorted(vals.values())
    return v[len(v) // 2]


def main():
    out = sys.argv[1]
    fetch = per_launch(out, "pmc_FETCH_SIZE", "FETCH_SIZE")
    mfma = per_launch(out, "pmc_pairs_mfma", "SQ_VALU_MFMA_BUSY_CYCLES")
    gui = per_launch(out, "pmc_pairs_mfma", "GRBM_GUI_ACTIVE")
    cus = 256
    res = {"kernel": "ame_pairs2_kernel<16> (K3, n=1024, T=128, r=16)",
           "hbm_read_bytes_per_launch": None if fetch is None else 2.0 * fetch * 1024.0,
           "algorithmic_read_bytes": 4.0 * 1024 * 1023 * 128,
           "SQ_VALU_MFMA_BUSY_CYCLES": mfma, "GRBM_GUI_ACTIVE": gui}
    if mfma is not None and gui:
        res["mfma_busy_est"] = mfma / (gui / 8.0 * cus * 4)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
