"""A/B of the K4 decomposition kernel: the in-tree kernel against an older build of
decompose.hip loaded from another shared library (``--old-lib``), same inputs, full
outputs and scoring mode.  Wall time per call (median of 10 after warm-up)."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from foremast_amd.brain.engine import synthetic_history  # noqa: E402
from foremast_amd.ops import _native as nat  # noqa: E402
from foremast_amd.ops import kernels as K  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--old-lib", required=True)
    p.add_argument("--series", type=int, default=100_000)
    args = p.parse_args()
    dev = torch.device("cuda:0")
    N, R, m, Cw = args.series, 10080, 1440, 50
    hist = synthetic_history(N, R, m, dev, seed=3).to(torch.bfloat16)
    cur = hist[:, -Cw:].float().contiguous()
    spec = K.DetectSpec(horizons=torch.arange(1, 11, dtype=torch.int32, device=dev).repeat(Cw // 10),
                        max_horizon=10, threshold=torch.full((N,), 3.0, device=dev),
                        bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.zeros(N, device=dev), cur=cur)
    real = nat.require()
    old = C.CDLL(os.path.abspath(args.old_lib))
    old.fm_seasonal_decompose.argtypes = real.fm_seasonal_decompose.argtypes
    old.fm_seasonal_decompose.restype = real.fm_seasonal_decompose.restype
    old.fm_decompose_lds_bytes.argtypes = real.fm_decompose_lds_bytes.argtypes
    old.fm_decompose_lds_bytes.restype = real.fm_decompose_lds_bytes.restype

    class Mixed:
        def __getattr__(self, k):
            return getattr(old if k in ("fm_seasonal_decompose", "fm_decompose_lds_bytes") else real, k)

    res = {}
    outs = {}
    for which in ("new", "old"):
        nat.require = (lambda: real) if which == "new" else (lambda: Mixed())
        K.nat.require = nat.require
        for mode in ("full", "score"):
            out = {}
            fn = ((lambda: K.seasonal_decompose(hist, 0, R, m, out=out)) if mode == "full"
                  else (lambda: K.decompose_score(hist, 0, R, m, spec, out=out)))
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(10):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
            ts.sort()
            res[f"{which}_{mode}_ms"] = round(ts[len(ts) // 2], 3)
            outs[(which, mode)] = {k: v.clone() for k, v in out.items()}
    for mode in ("full", "score"):
        a, b = outs[("new", mode)], outs[("old", mode)]
        for k in a:
            if a[k].is_floating_point():
                d = (a[k] - b[k]).abs()
                ok = ~torch.isnan(d)
                res[f"maxdiff_{mode}_{k}"] = float(d[ok].max()) if ok.any() else 0.0
            else:
                res[f"equal_{mode}_{k}"] = bool(torch.equal(a[k], b[k]))
    res["n_series"], res["T"], res["m"] = N, R, m
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
