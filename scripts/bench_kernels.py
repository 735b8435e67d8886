#!/usr/bin/env python
"""Kernel micro-benchmarks on the flagship shapes (one process, interleaved
A/B rounds — cdna_hip_programming.md §5.4 rule 24).

Prints one JSON line per kernel/variant with median / min milliseconds and
the derived series/s; writes the same to ``gpurun_out/kernels.json``.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from foremast_amd.brain.engine import synthetic_history  # noqa: E402
from foremast_amd.models import smoothing as sm  # noqa: E402
from foremast_amd.ops import kernels as K  # noqa: E402


def timed(fn, reps=5):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    return ts


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--series", type=int, default=100_000)
    p.add_argument("--ring", type=int, default=10080)
    p.add_argument("--season", type=int, default=1440)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--variants", default="3,4")
    p.add_argument("--only", default="")
    args = p.parse_args()
    dev = torch.device("cuda:0")
    N, R, m, C = args.series, args.ring, args.season, 50
    hist = synthetic_history(N, R, m, dev, seed=3).to(torch.bfloat16)
    grid = sm.make_grid(sm.MODE_HW, (0.1, 0.3, 0.5, 0.8), (0.0, 0.01, 0.05, 0.1), (0.05, 0.1, 0.3, 0.5)).to(dev)
    cur = hist[:, -C:].float().contiguous()
    # current window: 5 pods x 10 one-minute slots (horizons 1..10 per pod)
    spec = K.DetectSpec(horizons=torch.arange(1, 11, dtype=torch.int32, device=dev).repeat(C // 10),
                        max_horizon=10,
                        threshold=torch.full((N,), 3.0, device=dev),
                        bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.zeros(N, device=dev), cur=cur)
    results = {}
    variants = [int(v) for v in args.variants.split(",") if v.strip()]
    outs = {}

    def run_hw(v, mode=sm.MODE_HW):
        outs[(v, mode)] = K.smoothing_fit(hist, 0, R, mode, m, grid if mode == sm.MODE_HW else grid[:4],
                                          spec, out=outs.get((v, mode)), variant=v)

    jobs = {}
    if not args.only or "hw" in args.only:
        for v in variants:
            jobs[f"holt_winters_v{v}"] = (lambda v=v: run_hw(v))
    es_grid = sm.make_grid(sm.MODE_ES, (0.1, 0.3, 0.6, 0.9), (0.0,), (0.0,)).to(dev)
    des_grid = sm.make_grid(sm.MODE_DES, (0.1, 0.3, 0.6, 0.9), (0.0, 0.05, 0.1, 0.2), (0.0,)).to(dev)

    def run_es(v, mode):
        g = es_grid if mode == sm.MODE_ES else des_grid
        outs[(v, mode)] = K.smoothing_fit(hist, 0, R, mode, 1, g, spec, out=outs.get((v, mode)), variant=v)

    if not args.only or "es" in args.only:
        for v in (-1, 0, 5):  # 5 = sequential K2 (csrc/es_seq.hip); -1 / 0 = time-parallel scan
            jobs[f"exp_smoothing_v{v}"] = (lambda v=v: run_es(v, sm.MODE_ES))
            jobs[f"double_exp_smoothing_v{v}"] = (lambda v=v: run_es(v, sm.MODE_DES))
    base = cur[:, :50].contiguous()
    rk = {}
    jobs["rank_tests"] = lambda: rk.update(K.rank_tests(base, cur + 0.1, 1, 0.05, out=rk))
    ws = {}
    jobs["window_stats"] = lambda: ws.update(K.window_stats(hist, 0, R, spec, out=ws))
    dc = {}
    if not args.only or "decompose" in args.only:
        jobs["seasonal_decompose"] = lambda: dc.update(K.seasonal_decompose(hist, 0, R, m, out=dc))
        ds = {}
        jobs["decompose_score"] = lambda: ds.update(K.decompose_score(hist, 0, R, m, spec, out=ds))
    for name, fn in jobs.items():  # warm-up / compile
        fn()
    torch.cuda.synchronize()
    samples = {k: [] for k in jobs}
    for _ in range(args.rounds):
        for name, fn in jobs.items():
            samples[name] += timed(fn, reps=3)
    for name, ts in samples.items():
        med = float(np.median(ts))
        results[name] = {"median_ms": round(med, 3), "min_ms": round(float(np.min(ts)), 3),
                         "series_per_s": round(N / (med / 1e3), 1), "n_series": N, "T": R}
        print(json.dumps({"kernel": name, **results[name]}), flush=True)
    # agreement between variants
    ref_v = -1 if -1 in variants else (variants[0] if variants else None)
    ref = outs.get((ref_v, sm.MODE_HW))
    if ref is not None:
        for v in variants:
            o = outs.get((v, sm.MODE_HW))
            if o is None or v == ref_v:
                continue
            same = (o["best"] == ref["best"]).float().mean().item()
            dsig = ((o["sigma"] - ref["sigma"]).abs() / ref["sigma"].abs().clamp(min=1e-6)).max().item()
            vagree = (o["verdict"] == ref["verdict"]).float().mean().item()
            dfc = ((o["forecast"] - ref["forecast"]).abs() / ref["forecast"].abs().clamp(min=1e-3)).max().item()
            print(json.dumps({"agree_vs": ref_v, "variant": v, "best_same": same, "max_rel_sigma": dsig,
                              "max_rel_forecast": dfc, "verdict_agree": vagree}), flush=True)
            results[f"agree_v{v}"] = {"best_same": same, "max_rel_sigma": dsig, "verdict_agree": vagree}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "kernels.json"), "w") as f:
        json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
