"""Rank tests (K5) at the product geometry: the sort-and-search path vs the O(n^2)
sweep, on the same windows (100k rows x 5 + 5 pods x 11 minutes, partly filled
canary windows, tied values).  Prints the kernel time of each path (CUDA events,
median of several launches) and the largest difference of their outputs; the
windows are also checked against the PyTorch fp64 reference on a sample.

    python scripts/bench_rank.py [--rows 100000] [--nb 55] [--nc 55]
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from foremast_amd.models import pairwise as pw  # noqa: E402
from foremast_amd.ops import kernels as K  # noqa: E402


def windows(N, nb, nc, dev, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    base = torch.randn(N, nb, generator=g) * 0.1 + 1.0
    cur = torch.randn(N, nc, generator=g) * 0.1 + 1.0
    cur[: N // 3] += 0.08                                   # a third of the rows shifted
    base[N // 2:] = torch.round(base[N // 2:] * 20) / 20    # ties in half of the rows
    cur[N // 2:] = torch.round(cur[N // 2:] * 20) / 20
    fill = torch.randint(1, nc + 1, (N,), generator=g)       # canary windows partly filled
    cur[torch.arange(nc)[None, :] >= fill[:, None]] = float("nan")
    base[torch.rand(N, nb, generator=g) < 0.02] = float("nan")
    return base.to(dev).contiguous(), cur.to(dev).contiguous()


def run(base, cur, sweep, reps, want_pvals=True):
    if sweep:
        os.environ["FOREMAST_RANK_SWEEP"] = "1"
    else:
        os.environ.pop("FOREMAST_RANK_SWEEP", None)
    out = {}
    K.rank_tests(base, cur, 1, 0.05, want_pvals=want_pvals, out=out)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        K.rank_tests(base, cur, 1, 0.05, want_pvals=want_pvals, out=out)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return out, float(np.median(ts)), float(np.min(ts))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=100_000)
    p.add_argument("--nb", type=int, default=55)
    p.add_argument("--nc", type=int, default=55)
    p.add_argument("--reps", type=int, default=20)
    a = p.parse_args()
    dev = torch.device("cuda:0")
    base, cur = windows(a.rows, a.nb, a.nc, dev)
    small, t_small, m_small = run(base, cur, False, a.reps)
    sweep, t_sweep, m_sweep = run(base, cur, True, a.reps)
    # the product tick's form: decisions only (|z| > z_crit, no p-values)
    zsmall, tz_small, _ = run(base, cur, False, a.reps, want_pvals=False)
    zsweep, tz_sweep, _ = run(base, cur, True, a.reps, want_pvals=False)
    os.environ.pop("FOREMAST_RANK_SWEEP", None)
    rows_differ = int(((small["pvals"] - sweep["pvals"]).abs() > 1e-6).any(1).sum())
    diff = {k: float((small[k] - sweep[k]).abs().max()) for k in ("pvals", "counts")}
    same = float((small["differs"] == sweep["differs"]).float().mean())
    bm = float(torch.nan_to_num((small["base_mean"] - sweep["base_mean"]).abs()).max())
    # fp64 reference (scipy-pinned models/pairwise.py) on a sample of rows
    idx = torch.arange(0, a.rows, max(1, a.rows // 2000))
    ref = pw.rank_tests(base[idx].double().cpu(), cur[idx].double().cpu())
    got = small["pvals"][idx].double().cpu()
    want = torch.stack([ref.p_mw, ref.p_wilcoxon, ref.p_kruskal], 1)
    ok = torch.isfinite(want)
    ref_err = float((got[ok] - want[ok]).abs().max())
    got_sw = sweep["pvals"][idx].double().cpu()
    ref_err_sweep = float((got_sw[ok] - want[ok]).abs().max())
    # per test: sampled rows further than 1e-4 from the fp64 reference, each path
    far = {name: [int(((g[:, j] - want[:, j]).abs() > 1e-4).sum()) for g in (got, got_sw)]
           for j, name in enumerate(("mw", "wilcoxon", "kruskal"))}
    print(json.dumps({"rows": a.rows, "nb": a.nb, "nc": a.nc, "small_ms": round(t_small, 4),
                      "small_min_ms": round(m_small, 4), "sweep_ms": round(t_sweep, 4),
                      "sweep_min_ms": round(m_sweep, 4), "speedup": round(t_sweep / t_small, 2),
                      "decisions_only_small_ms": round(tz_small, 4), "decisions_only_sweep_ms": round(tz_sweep, 4),
                      "decisions_only_agree_with_pvals": float((zsmall["differs"] == small["differs"]).float().mean()),
                      "decisions_only_small_vs_sweep": float((zsmall["differs"] == zsweep["differs"]).float().mean()),
                      "rows_pvals_differ_gt_1e-6": rows_differ,
                      "differs_agree": same, "max_abs_diff": diff, "base_mean_diff": bm,
                      "max_abs_err_vs_fp64_ref": ref_err, "sweep_max_abs_err_vs_fp64_ref": ref_err_sweep,
                      "sampled_rows": int(idx.numel()), "rows_off_ref_gt_1e-4_small_sweep": far}), flush=True)


if __name__ == "__main__":
    main()
