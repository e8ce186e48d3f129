#!/usr/bin/env python
"""Summarise rocprofv3 CSV output (kernel stats / PMC counters) for one kernel.

  python tools/pmc_summary.py --fetch DIR_F --write DIR_W [--hits DIR_H] --kernel spmm_rows_kernel \
      --workload twitter-world-powerlaw-k300-fast --bytes 51696800004 --out profiles/r01/pmc_<workload>.json

HBM bytes per launch follow MI355X_MICROARCH.md §HBM for gfx950:
  FETCH_SIZE (KiB) reports 1/2 of the bytes of a wide coalesced (16 B/lane) read -> x2;
  WRITE_SIZE (KiB) is exact for 16 B/lane stores. Both counters are collected in
  separate passes (TCC slot limits), averaged over every dispatch of the kernel.
FETCH_SIZE counts L2 -> fabric requests; Infinity-Cache hits are counted, not excluded.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphconvgeo_amd._build import source_hash  # noqa: E402


def read_counters(d: str, kernel: str):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel not in row["Kernel_Name"]:
                    continue
                vals[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {c: list(v.values()) for c, v in vals.items()}


def mean(xs):
    return sum(xs) / len(xs) if xs else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--hits", default=None)
    ap.add_argument("--kernel", default="spmm_rows_kernel")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--bytes", type=int, required=True, help="algorithmic bytes per launch")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    f = read_counters(a.fetch, a.kernel)
    w = read_counters(a.write, a.kernel)
    fetch_kib = mean(f.get("FETCH_SIZE", []))
    write_kib = mean(w.get("WRITE_SIZE", []))
    rec = {
        "workload": a.workload, "kernel": a.kernel,
        "dispatches": {"fetch": len(f.get("FETCH_SIZE", [])), "write": len(w.get("WRITE_SIZE", []))},
        "FETCH_SIZE_KiB_per_launch": fetch_kib, "WRITE_SIZE_KiB_per_launch": write_kib,
        "correction": "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950, MI355X_MICROARCH.md §HBM)",
        "algorithmic_bytes_per_launch": a.bytes,
        # the library these counters describe (bench.load_traffic refuses another build's):
        # the tree's source hash, which the loaded library must match (_native._check_fresh)
        "gcg_source_hash": source_hash(),
    }
    if fetch_kib is not None and write_kib is not None:
        hbm = 2 * fetch_kib * 1024 + write_kib * 1024
        rec["hbm_bytes_per_launch"] = int(hbm)
        rec["hbm_over_algorithmic"] = round(hbm / a.bytes, 4)
    if a.hits:
        h = read_counters(a.hits, a.kernel)
        hit, miss = mean(h.get("TCC_HIT_sum", [])), mean(h.get("TCC_MISS_sum", []))
        if hit is not None and miss is not None and hit + miss > 0:
            rec["l2_hit_rate"] = round(hit / (hit + miss), 4)
            rec["TCC_HIT_sum"] = hit
            rec["TCC_MISS_sum"] = miss
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
