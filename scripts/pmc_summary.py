#!/usr/bin/env python
"""Aggregate rocprofv3 --pmc counter CSVs per kernel into a markdown table:
``python scripts/pmc_summary.py gpurun_out/pmc_lstm [name filter] [--per-dispatch]``
(default: sums over every dispatch of every counter pass; ``--per-dispatch``: the mean
per dispatch, each counter averaged over the dispatches of the pass that collected it)."""

import collections
import csv
import glob
import os
import sys


def collect(root, per_dispatch=False):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    ncount = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add((f, r.get("Dispatch_Id", "")))
            ncount[k][r["Counter_Name"]].add((f, r.get("Dispatch_Id", "")))
    if per_dispatch:
        for k in agg:
            for c in agg[k]:
                agg[k][c] /= max(1, len(ncount[k][c]))
    return agg, calls


def main(root, pattern="", per_dispatch=False):
    agg, calls = collect(root, per_dispatch)
    names = sorted(k for k in agg if pattern in k and not k.startswith("void at::") and "rocclr" not in k)
    counters = sorted({c for k in names for c in agg[k]})
    print("| kernel | " + " | ".join(counters) + " |")
    print("|---|" + "---:|" * len(counters))
    for k in names:
        short = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        print(f"| `{short}` | " + " | ".join(f"{agg[k].get(c, 0):.4g}" for c in counters) + " |")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--per-dispatch"]
    main(args[0], args[1] if len(args) > 1 else "", "--per-dispatch" in sys.argv)
