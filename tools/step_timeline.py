#!/usr/bin/env python
"""Print one training step's kernel timeline from a rocprofv3 --kernel-trace CSV: every
dispatch of the last step (the window between the last two Adam updates' first kernels is
approximated by the last 1/STEPS of the dispatches), with start offset, duration and stream,
plus the busy time per stream and the wall span -- which kernels sit on the critical path."""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, required=True, help="steps traced (warm-up included)")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = len(rows)
    per = n // a.steps
    last = rows[n - per:]
    t0 = int(last[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in last)
    busy = {}
    for r in last:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get("Stream_Id") or r.get("Queue_Id")
        busy[q] = busy.get(q, 0) + (e - s)
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:70]
        print(f"{(s - t0) / 1e6:8.3f} +{(e - s) / 1e6:7.3f} ms  q{q:>3}  {name}")
    print(f"step span {(t1 - t0) / 1e6:.3f} ms; busy per stream (ms):",
          {k: round(v / 1e6, 3) for k, v in busy.items()})


if __name__ == "__main__":
    main()
