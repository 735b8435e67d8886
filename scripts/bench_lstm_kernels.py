#!/usr/bin/env python
"""Micro-benchmark of the fused LSTM kernels: training kernel per phase
(enc fwd / dec fwd / dec bwd / enc bwd), weight-grad GEMMs, scoring kernel
(bf16 / fp8).  Prints one JSON line per measurement."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from foremast_amd.models.lstm_ae import LSTMAutoencoder  # noqa: E402
from foremast_amd.ops import lstm as L  # noqa: E402
from foremast_amd.ops.lstm_train import FusedLstmGrad  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dev = torch.device("cuda:0")
    B, T, F = int(os.environ.get("B", 4096)), int(os.environ.get("T", 32)), int(os.environ.get("F", 1))
    m = LSTMAutoencoder(F, 64).to(dev)
    x = torch.randn(B, T, F, device=dev)
    for variant in (() if os.environ.get("SKIP_TRAIN") else (0, 1)):
        fg = FusedLstmGrad(B, T, F, dev, variant=variant)
        for ph, name in [(15, "all"), (1, "enc_fwd"), (2, "dec_fwd"), (3, "fwd"), (4, "dec_bwd"), (8, "enc_bwd")]:
            fg.phases = ph
            print(json.dumps({"kernel": "lstm_train", "variant": variant, "phases": name, "B": B, "T": T,
                              "ms": round(timeit(lambda: fg.launch(m, x)), 4)}))
        fg.phases = 0
        for bg in (False, True):
            fg.batched_gemm = bg
            print(json.dumps({"kernel": "lstm_train+gemms", "variant": variant, "batched_gemm": bg, "B": B, "T": T,
                              "ms": round(timeit(lambda: fg.grads(m, x)), 4)}))
    for N in [int(v) for v in os.environ.get("N", "100000").split(",")]:  # N=a,b,c: a scoring-size sweep
        xs = torch.randn(N, T, F, device=dev)
        for fp8 in (False, True):
            p = L.pack(m, fp8=fp8, device=dev)
            out = {}
            ms = timeit(lambda: L.lstm_score(p, xs, out=out))
            print(json.dumps({"kernel": "lstm_score", "fp8": fp8, "N": N, "T": T, "ms": round(ms, 4)}))


if __name__ == "__main__":
    main()
