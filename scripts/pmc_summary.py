#!/usr/bin/env python
"""Aggregate rocprofv3 --pmc counter CSVs per kernel (sum over dispatches)
into a markdown table: ``python scripts/pmc_summary.py gpurun_out/pmc_lstm``."""

import collections
import csv
import glob
import os
import sys


def collect(root):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add((f, r.get("Dispatch_Id", "")))
    return agg, calls


def main(root, pattern=""):
    agg, calls = collect(root)
    names = sorted(k for k in agg if pattern in k and not k.startswith("void at::") and "rocclr" not in k)
    counters = sorted({c for k in names for c in agg[k]})
    print("| kernel | " + " | ".join(counters) + " |")
    print("|---|" + "---:|" * len(counters))
    for k in names:
        short = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        print(f"| `{short}` | " + " | ".join(f"{agg[k].get(c, 0):.4g}" for c in counters) + " |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
