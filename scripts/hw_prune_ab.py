"""A/B of the Holt-Winters fit (variant 5), read by the launcher on every launch:
exhaustive grid (FOREMAST_HW_PRUNE=0), exact grid branch and bound in grid order and
with the previous winners first (FOREMAST_HW_HINTS).

Each timed fit slides the 7-day window one sample forward (``--shift``, as a tick of
the canary bench does), so the hints come from the fit of the previous window, not of
the same data.  Kernel time by HIP events; the last fit of every
mode is compared bit for bit with the exhaustive one."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from foremast_amd.brain.engine import synthetic_history  # noqa: E402
from foremast_amd.models import smoothing as sm  # noqa: E402
from foremast_amd.ops import kernels as K  # noqa: E402

MODES = {  # PRUNE, HINTS
    "noprune": ("0", "1"),
    "prune_gridorder": ("1", "0"),
    "prune_hints": ("1", "1"),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--series", type=int, default=100_000)
    p.add_argument("--window", type=int, default=10080)
    p.add_argument("--season", type=int, default=1440)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--modes", default=",".join(MODES))
    p.add_argument("--shift", type=int, default=1, help="samples the window moves between fits")
    p.add_argument("--mix", action="store_true",
                   help="vary the winning grid point: noisy / level-shifted / spiky / growing series mixed in")
    args = p.parse_args()
    dev = torch.device("cuda:0")
    N, T, m, C = args.series, args.window, args.season, 50
    R = T + args.shift * (args.iters + 3)
    hist = synthetic_history(N, R, m, dev, seed=3)
    if args.mix:
        g = torch.Generator(device=dev).manual_seed(5)
        lvl = hist.mean(1, keepdim=True)
        hist[1::7] += torch.randn(hist[1::7].shape, generator=g, device=dev) * 0.2 * lvl[1::7]
        hist[2::7, R // 2:] += 0.5 * lvl[2::7]
        hist[3::7, 2000::97] += 3.0 * lvl[3::7]
        hist[5::7] *= torch.linspace(1.0, 3.0, R, device=dev)
    hist = hist.to(torch.bfloat16)
    grid = sm.make_grid(sm.MODE_HW, (0.1, 0.3, 0.5, 0.8), (0.0, 0.01, 0.05, 0.1), (0.05, 0.1, 0.3, 0.5)).to(dev)
    cur = hist[:, -C:].float().contiguous()
    spec = K.DetectSpec(horizons=torch.arange(1, 11, dtype=torch.int32, device=dev).repeat(C // 10), max_horizon=10,
                        threshold=torch.full((N,), 3.0, device=dev), bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.zeros(N, device=dev), cur=cur)
    modes = args.modes.split(",")
    res, outs = {}, {}
    for name in modes * 2:
        os.environ["FOREMAST_HW_PRUNE"], os.environ["FOREMAST_HW_HINTS"] = MODES[name]
        o = K.smoothing_fit(hist, 0, T, sm.MODE_HW, m, grid, spec, variant=5)
        o = K.smoothing_fit(hist, args.shift, T, sm.MODE_HW, m, grid, spec, out=o, variant=5)
        torch.cuda.synchronize()
        ts = []
        for it in range(args.iters):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            o = K.smoothing_fit(hist, args.shift * (it + 2), T, sm.MODE_HW, m, grid, spec, out=o, variant=5)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        res.setdefault(name, []).append(round(ts[len(ts) // 2], 3))
        outs[name] = {k: v.clone() for k, v in o.items() if torch.is_tensor(v)}
    ref = modes[0]
    same = {n: all(torch.equal(outs[ref][k], outs[n][k]) for k in outs[ref]) for n in modes}
    wins = torch.bincount(outs[ref]["best"].long(), minlength=grid.shape[0])
    best = {n: min(v) for n, v in res.items()}
    print(json.dumps({"series": N, "mix": args.mix, "shift": args.shift, "median_ms": res, "best_ms": best,
                      "speedup_vs_" + ref: {n: round(best[ref] / best[n], 4) for n in modes},
                      "identical_to_" + ref: same, "distinct_winners": int((wins > 0).sum())}), flush=True)


if __name__ == "__main__":
    main()
