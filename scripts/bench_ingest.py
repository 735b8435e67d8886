"""Host decode rate of a 100k-series canary tick's Prometheus bodies (CPU only).

Renders one tick's ``query_range`` bodies exactly as ``bench.py --ingest prom``
does (5 metric families x canary/baseline pod sets, one point per (app, pod)
series) and times :class:`~foremast_amd.ingest.tickdecode.TickDecoder`.

    python scripts/bench_ingest.py --series 100000 --threads 8 --reps 5
"""

import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--series", type=int, default=100000)
    p.add_argument("--pods", type=int, default=5)
    p.add_argument("--threads", type=int, default=8)
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    n, P, ring = a.series, a.pods, 10080
    g = torch.Generator().manual_seed(0)
    host_ticks = (torch.rand((1, n, 2 * P), generator=g) * 90 + 5).float()
    t0 = time.perf_counter()
    dec, bodies = bench.prom_bodies(host_ticks, 0, P, ring, a.threads, False)
    nbytes = sum(len(b) for b in bodies[0])
    print(f"rendered {len(bodies[0])} bodies, {nbytes / 1e6:.1f} MB in {time.perf_counter() - t0:.1f} s", flush=True)
    ts = bench.T_STEP * ring
    times = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        blk, stats = dec.submit(bodies[0], ts, bench.T_STEP).result()
        times.append((time.perf_counter() - t0) * 1e3)
    got = blk.numpy().reshape(n, 2 * P)
    ok = np.array_equal(got, host_ticks[0].numpy())
    unmatched = sum(s[2] for s in stats)
    print({"series": n, "threads": a.threads, "mb": round(nbytes / 1e6, 1), "ms": [round(t, 2) for t in times],
           "best_ms": round(min(times), 2), "gb_per_s": round(nbytes / min(times) / 1e6, 2),
           "exact": bool(ok), "unmatched": int(unmatched)})
    dec.close()


if __name__ == "__main__":
    main()
