"""Detection-quality diagnostics of the LSTM-AE benches (configs 3 / 5).

Runs ``bench.setup_lstm`` on a reduced series count, scores the timed ticks
and prints the reconstruction-error / z-score distributions of regressed vs
healthy apps, and how many errors are non-finite.

    python scripts/lstm_detect_diag.py --config multivariate --series 20000
"""

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    args = bench.parse()
    world, rank, dev = bench.init_dist(args)
    F, fp8 = (2, True) if args.config == "multivariate" else (1, False)
    tick, health_host, meta, _, _ = bench.setup_lstm(args, world, rank, dev, F, fp8)
    out = None
    for k in range(args.warmup + args.steps):
        out = tick(k)
    truth_apps, n_apps = meta["_truth"]
    ent_per_app = max(1, bench.METRICS_PER_APP // F)
    err = out["err"].float().cpu().numpy()
    z = out["zscore"].float().cpu().numpy()
    v = out["verdict"].cpu().numpy()
    sh = meta["_shard"]
    bad = np.zeros(err.shape[0], dtype=bool)
    bad[meta["_bad"].numpy()] = True
    zg = (err - sh.mu) / sh.sigma
    print(f"global mu={sh.mu:.4g} sigma={sh.sigma:.4g} rho={sh.rho:.4g}")
    q = [0.0, 0.01, 0.1, 0.5, 0.9, 0.99, 1.0]
    for name, m in (("injected", bad), ("healthy", ~bad)):
        e, zz = err[m], z[m]
        fin = np.isfinite(e)
        print(f"{name}: n={m.sum()} nonfinite={int((~fin).sum())} flagged={int(v[m].sum())}")
        if fin.any():
            print("  err q", np.round(np.quantile(e[fin], q), 4).tolist())
            print("  z   q", np.round(np.quantile(zz[fin], q), 3).tolist())
            print("  zg  q", np.round(np.quantile(zg[m][fin], q), 3).tolist())
            for thr in (4.0, 8.0):
                print(f"  >thr {thr}: per-series {int((zz[fin] > thr).sum())} global {int((zg[m][fin] > thr).sum())}"
                      f" both {int(((zz[fin] > thr) & (zg[m][fin] > thr)).sum())}")
    print(bench.detection_report(health_host, truth_apps, n_apps))


if __name__ == "__main__":
    main()
