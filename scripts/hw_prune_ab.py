"""A/B of the Holt-Winters fit (variant 5) with and without the exact grid branch and
bound (FOREMAST_HW_PRUNE=0|1, read by the launcher on every launch): kernel time by
HIP events, outputs compared bit for bit."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from foremast_amd.brain.engine import synthetic_history  # noqa: E402
from foremast_amd.models import smoothing as sm  # noqa: E402
from foremast_amd.ops import kernels as K  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--series", type=int, default=100_000)
    p.add_argument("--ring", type=int, default=10080)
    p.add_argument("--season", type=int, default=1440)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--noise", type=float, default=0.03)
    args = p.parse_args()
    dev = torch.device("cuda:0")
    N, R, m, C = args.series, args.ring, args.season, 50
    hist = synthetic_history(N, R, m, dev, seed=3).to(torch.bfloat16)
    grid = sm.make_grid(sm.MODE_HW, (0.1, 0.3, 0.5, 0.8), (0.0, 0.01, 0.05, 0.1), (0.05, 0.1, 0.3, 0.5)).to(dev)
    cur = hist[:, -C:].float().contiguous()
    spec = K.DetectSpec(horizons=torch.arange(1, 11, dtype=torch.int32, device=dev).repeat(C // 10), max_horizon=10,
                        threshold=torch.full((N,), 3.0, device=dev), bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.zeros(N, device=dev), cur=cur)
    res, outs = {}, {}
    for mode in ("0", "1", "0", "1"):
        os.environ["FOREMAST_HW_PRUNE"] = mode
        o = None
        o = K.smoothing_fit(hist, 0, R, sm.MODE_HW, m, grid, spec, variant=5)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.iters):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            o = K.smoothing_fit(hist, 0, R, sm.MODE_HW, m, grid, spec, out=o, variant=5)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        res.setdefault(mode, []).append(ts[len(ts) // 2])
        outs[mode] = {k: v.clone() for k, v in o.items() if torch.is_tensor(v)}
    same = {k: bool(torch.equal(outs["0"][k], outs["1"][k])) for k in outs["0"]}
    print(json.dumps({"series": N, "median_ms_noprune": res["0"], "median_ms_prune": res["1"],
                      "speedup": min(res["0"]) / min(res["1"]), "identical": same}), flush=True)


if __name__ == "__main__":
    main()
