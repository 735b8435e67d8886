#!/usr/bin/env python
"""Summarise a rocprofv3 ``--kernel-trace --stats`` run into a markdown table
(``python scripts/prof_summary.py gpurun_out/prof/run_kernel_stats.csv``)."""

import csv
import sys


def summarise(path: str, top: int = 20) -> str:
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = [f"total kernel time: {tot / 1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} launches", "",
           "| ms total | calls | avg us | % | kernel |", "|---:|---:|---:|---:|---|"]
    for r in rows[:top]:
        name = r["Name"].replace("|", "/")
        if len(name) > 100:
            name = name[:100] + "…"
        out.append(f"| {float(r['TotalDurationNs']) / 1e6:.2f} | {r['Calls']} | "
                   f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} | `{name}` |")
    return "\n".join(out)


if __name__ == "__main__":
    print(summarise(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20))
