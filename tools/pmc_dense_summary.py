#!/usr/bin/env python
"""Per-kernel summary of rocprofv3 PMC passes over tools/exp_dense_one.py (tools/gpu/pmc_nt.sh):
counters averaged per dispatch (GRBM_GUI_ACTIVE is collected in two passes: averaged, not
summed), MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
(the rocprofv3 derived-metric formula), wait fractions per wave-cycle, HBM bytes per the
gfx950 correction (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md §HBM)."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> v
    for f in glob.glob(os.path.join(a.dir, "p*", "*counter_collection.csv")):
        pas = os.path.basename(os.path.dirname(f))
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if "gemm" not in k:
                continue
            k = k.split("(int")[0].replace("void (anonymous namespace)::", "")
            vals[k][row["Counter_Name"]][(pas, row["Dispatch_Id"])] += float(row["Counter_Value"])
    times = {}
    for f in glob.glob(os.path.join(a.dir, "kt", "*kernel_stats.csv")):
        for row in csv.DictReader(open(f)):
            k = row["Name"].split("(int")[0].replace("void (anonymous namespace)::", "")
            times[k] = float(row["AverageNs"]) * 1e-6
    out = {}
    for k, cs in vals.items():
        c = {n: sum(d.values()) / len(d) for n, d in cs.items()}  # mean over dispatches (and passes)
        rec = {"avg_ms": times.get(k), "counters_per_dispatch": {n: round(v) for n, v in sorted(c.items())}}
        g = c.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            rec["mfma_util"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024), 3)
            rec["clock_GHz"] = round(g / 8 / (times[k] * 1e-3) / 1e9, 2) if times.get(k) else None
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if n in c:
                    rec[n.lower() + "_frac"] = round(c[n] / wc, 3)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rec["hbm_bytes"] = round(2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024)
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            rec["lds_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
        out[k] = rec
    js = json.dumps(out, indent=1)
    print(js)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(js + "\n")


if __name__ == "__main__":
    main()
