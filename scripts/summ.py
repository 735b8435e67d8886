"""Print one line per bench record under gpurun_out/<dir>/ (``python scripts/summ.py r5ad``):
value, ms per step, p50 detect latency, detection TP / FP."""
import glob
import json
import os
import sys

for path in sorted(glob.glob(os.path.join("gpurun_out", sys.argv[1], "*.log"))):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{") and '"metric"' in line:
            d = json.loads(line)
            det = d.get("detection") or {}
            print(f"{os.path.basename(path)[:-4]:14s} {d['value']:>14,.0f} {d['unit']:10s} ms/step {d['ms_per_step']:8.3f} "
                  f"p50 {d.get('p50_detect_latency_ms')} tp {det.get('tp')} fp {det.get('fp')}")
            break
