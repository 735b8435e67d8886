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
    tk_last = meta["_ticks"][-1, :, 0].float()
    lvl = meta["_params"][0]["lvl"][:, 0].float().cpu()
    bb = meta["_bad"].long()
    print("bad series with last tick > 2 x level:", int((tk_last[bb] > 2 * lvl[bb]).sum()), "of", len(bb),
          "| all ticks of bad > 2x:", int((meta["_ticks"][:, bb, 0] > 2 * lvl[bb][None]).all(0).sum()))
    # the injected series the detector missed: their scored window vs the fp32 model
    miss = np.nonzero(bad & (v == 0))[0][:6]
    if len(miss):
        idx = torch.as_tensor(miss, device=sh.device)
        x = sh._gather(idx, torch.zeros_like(idx))
        with torch.no_grad():
            ref = sh.model.recon_error(x).cpu().numpy()
            y = sh.model(x)
        for j, i in enumerate(miss.tolist()):
            xi = x[j, :, 0].cpu().numpy()
            print(f"miss {i}: kernel err {err[i]:.4g} fp32 err {ref[j]:.4g} mean {float(sh.mean[i, 0]):.4g} "
                  f"std {float(sh.std[i, 0]):.4g} x[0] {xi[0]:.3g} x[-1] {xi[-1]:.3g} y[-1] {float(y[j, -1, 0]):.3g}")
            ring = sh.rings[0]
            last = ring.logical()[i, -3:].float().cpu().numpy()
            tk = meta["_ticks"][-3:, i, 0].numpy()
            print(f"   lvl {float(meta['_params'][0]['lvl'][i]):.4g} ring last {np.round(last, 2)} ticks last {np.round(tk, 2)}")


if __name__ == "__main__":
    main()
