"""Decode of a node tick's pod bodies as the rollout engine runs it: F family bodies with
the same series order through ONE shared key index into a [slots, F] block (column = family),
vs the same with each family's column in its own cache line ([slots, 16 F]).  CPU only."""
import sys, time, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from foremast_amd.ingest import native
from foremast_amd.ingest.tickdecode import pod_matrix_body

S, F = int(os.environ.get("S", 112000)), 5
th = [int(x) for x in os.environ.get("TH", "1,8,16").split(",")]
pods = [f'"namespace":"ns{a % 200}","pod":"app{a // 5}-v2-{a % 5}-7d9f8b6c5d"' for a in range(S)]
# SHUF=1: the pods' block rows are a random permutation (slots reused as jobs come and go)
rows = np.random.default_rng(1).permutation(S) if os.environ.get("SHUF") else np.arange(S)
ix = native.KeyTable.from_hashes(native.series_keys(pod_matrix_body("m", pods, 0, np.zeros(S)), "namespace", "pod"),
                                 rows, "namespace", "pod")
rng = np.random.default_rng(0)
bodies = [pod_matrix_body(f"namespace_pod:metric{f}", pods,
                          600000, rng.random(S).astype(np.float32) * 90 + 5) for f in range(F)]
mb = sum(map(len, bodies)) / 1e6
for pad in (1, 16):
    if os.environ.get("PIN"):  # page-locked block (as the rollout engine's tick block on a GPU box)
        import torch
        out = torch.empty((S, F * pad), dtype=torch.float32).pin_memory().numpy()
    else:
        out = np.empty((S, F * pad), dtype=np.float32)
    for t in th:
        for fill in (False, True):
            ts = []
            for _ in range(9):
                t0 = time.perf_counter()
                native.decode_bodies(bodies, [ix] * F, [600000.0] * F, 60.0, [1] * F, [f * pad for f in range(F)], out,
                                     threads=t, fill_nan=fill)
                ts.append((time.perf_counter() - t0) * 1e3)
            b = min(ts[2:])
            print({"pin": bool(os.environ.get("PIN")), "shuf": bool(os.environ.get("SHUF")), "pad": pad, "threads": t, "fill_nan": fill, "mb": round(mb, 1), "best_ms": round(b, 2),
                   "median_ms": round(sorted(ts[2:])[3], 2), "gb_per_s": round(mb / b, 2)}, flush=True)
