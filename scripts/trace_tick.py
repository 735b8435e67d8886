#!/usr/bin/env python
"""Print one steady-state tick of a rocprofv3 kernel trace as a timeline
(``python scripts/trace_tick.py gpurun_out/proflstm/run_kernel_trace.csv lstm_ae_kernel``):
every kernel between the last two launches of the anchor kernel, with start /
end relative to the first anchor and the HIP stream it ran on."""

import csv
import sys


def timeline(path: str, anchor: str, before: int = 40):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    i0, i1 = idx[-2], idx[-1]
    t0 = int(rows[i0]["Start_Timestamp"])
    out = []
    for r in rows[max(0, i0 - before):i1 + 1]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        out.append(f"{s:9.1f} {e:9.1f} {e - s:7.1f}  s{r.get('Stream_Id', '')}  {r['Kernel_Name'][:80]}")
    return "\n".join(out)


if __name__ == "__main__":
    print(timeline(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "lstm_ae_kernel"))
