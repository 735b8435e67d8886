#!/usr/bin/env python
"""Holt-Winters variant-5 fit on gapped inputs (the masked-season kernel, hw_dg_kernel):
kernel time per 100k x 10,080 x 64 fit for dense series, a 30-minute outage in a fraction
of the series, isolated scrape misses at a rate, and (FOREMAST_HW_DG_ALL=1 rows) every pair
through the gapped kernel.  At the short seasons of variant 6 (hw_seq.hip, e.g. --season 72:
the 1200 s step) the ``v3dense`` / ``v3miss1e-3`` cases run the time-parallel variant 3 on the
same data (FOREMAST_HW_SEQ=0); ``s6*`` cases run variant 6 at m = 288 (FOREMAST_HW_SEQ288=1), ``g2*`` cases m = 144 with two grid
points per thread (FOREMAST_HW_SEQ_GPT144=2).  One JSON line per case; interleaved rounds."""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from foremast_amd.brain.engine import synthetic_history  # noqa: E402
from foremast_amd.models import smoothing as sm  # noqa: E402
from foremast_amd.ops import kernels as K  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--series", type=int, default=100_000)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--cases", default="dense,dgall,gap20,miss1e-4,miss1e-3")
    p.add_argument("--season", type=int, default=1440, help="points per day: 1440 (60 s step) or 288 (300 s)")
    args = p.parse_args()
    dev = torch.device("cuda:0")
    N, m = args.series, args.season
    R, C = 7 * m, 50 if m >= 1440 else 10
    base = synthetic_history(N, R, m, dev, seed=3).to(torch.bfloat16)
    grid = sm.make_grid(sm.MODE_HW, (0.1, 0.3, 0.5, 0.8), (0.0, 0.01, 0.05, 0.1), (0.05, 0.1, 0.3, 0.5)).to(dev)
    cur = base[:, -C:].float().contiguous()
    hz = 10 if m in K.SEQ_M else min(10, m // 32)
    spec = K.DetectSpec(horizons=torch.arange(1, hz + 1, dtype=torch.int32, device=dev).repeat(C // hz + 1)[:C],
                        max_horizon=hz,
                        threshold=torch.full((N,), 3.0, device=dev), bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.zeros(N, device=dev), cur=cur)
    g = torch.Generator(device=dev).manual_seed(5)
    hists = {}
    for case in args.cases.split(","):
        h = base.clone()
        kind = case[2:] if case[:2] in ("v3", "s6", "g2") else case
        if kind.startswith("gap"):
            frac = int(kind[3:]) / 100
            rows = torch.randperm(N, device=dev, generator=g)[: int(frac * N)]
            starts = torch.randint(m, R - 30, (rows.numel(),), device=dev, generator=g)
            cols = starts[:, None] + torch.arange(30, device=dev)[None, :]
            h[rows[:, None].expand(-1, 30), cols] = float("nan")
        elif kind.startswith("miss"):
            rate = float(kind[4:])
            h[torch.rand(h.shape, device=dev, generator=g) < rate] = float("nan")
        hists[case] = h
    res = {c: [] for c in hists}
    variant = {}
    outs = {}
    for _ in range(args.rounds):
        for case, h in hists.items():
            os.environ["FOREMAST_HW_DG_ALL"] = "1" if case == "dgall" else "0"
            os.environ["FOREMAST_HW_SEQ"] = "0" if case.startswith("v3") else "1"
            os.environ["FOREMAST_HW_SEQ288"] = "1" if case.startswith("s6") else "0"
            os.environ["FOREMAST_HW_SEQ_GPT144"] = "2" if case.startswith("g2") else "1"
            out = outs.setdefault(case[:2], {})
            for _w in range(2):
                K.smoothing_fit(h, 0, R, sm.MODE_HW, m, grid, spec, variant=5, out=out)
            torch.cuda.synchronize()
            d0 = K.hw_deferred_total(dev)
            ts = []
            for _r in range(5):
                torch.cuda.synchronize()
                t = time.perf_counter()
                K.smoothing_fit(h, 0, R, sm.MODE_HW, m, grid, spec, variant=5, out=out)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t) * 1e3)
            res[case].append((sorted(ts)[2], (K.hw_deferred_total(dev) - d0) / 5))
            variant[case] = K.last_hw_variant
    os.environ["FOREMAST_HW_DG_ALL"] = "0"
    os.environ["FOREMAST_HW_SEQ"] = "1"
    dense = sorted(x[0] for x in res.get("dense", [(float("nan"), 0)]))
    for case, xs in res.items():
        ms = sorted(x[0] for x in xs)
        rec = {"case": case, "season": m, "variant": variant[case], "points": R, "ms_median": round(ms[len(ms) // 2], 3),
               "ns_per_point": round(ms[len(ms) // 2] * 1e6 / (N * R), 4), "ms_all": [round(x, 3) for x in ms],
               "gapped_pairs_per_fit": xs[-1][1], "pairs": (N + 1) // 2,
               "vs_dense": round(ms[len(ms) // 2] / dense[len(dense) // 2], 3) if "dense" in res else None}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
