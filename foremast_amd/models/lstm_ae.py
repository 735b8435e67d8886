"""LSTM autoencoder for multi-metric anomaly scoring (``docs/guides/design.md:84``:
"3+ metrics → Deep Learning (LSTM)"; BASELINE configs 3 and 5).

Architecture (reference semantics for the fused ``lstm_ae`` kernel):

* input: a window ``x [B, T, F]`` of F metrics (z-scored per series with the
  series' historical mean/std);
* encoder: LSTM(F → H), zero initial state, PyTorch gate order (i, f, g, o);
* decoder: LSTM with zero input, initial state = the encoder's final
  ``(h, c)`` — ``gates = h W_hh^T + b``;
* output: ``y_t = h_t W_out^T + b_out`` (same time order as the input);
* score: reconstruction MSE per window ``mean_{t,f} (y - x)^2``; anomalous
  when ``err > mu + threshold * sigma`` (``mu``/``sigma`` calibrated on
  history windows).

Training uses plain PyTorch ops (matmuls → hipBLASLt) under autograd, one
process per GPU with gradient all-reduce (:mod:`foremast_amd.parallel.dp`).
Inference over 100k series runs in the fused gfx950 kernel
(``ops/csrc/lstm.hip``): both recurrences on MFMA with the hidden state
kept in registers across time steps.
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn as nn


class LSTMAutoencoder(nn.Module):
    def __init__(self, n_features: int, hidden: int = 64) -> None:
        super().__init__()
        F, H = n_features, hidden
        self.F, self.H = F, H
        k = 1.0 / math.sqrt(H)
        self.enc_w_ih = nn.Parameter(torch.empty(4 * H, F).uniform_(-k, k))
        self.enc_w_hh = nn.Parameter(torch.empty(4 * H, H).uniform_(-k, k))
        self.enc_b = nn.Parameter(torch.empty(4 * H).uniform_(-k, k))
        self.dec_w_hh = nn.Parameter(torch.empty(4 * H, H).uniform_(-k, k))
        self.dec_b = nn.Parameter(torch.empty(4 * H).uniform_(-k, k))
        self.out_w = nn.Parameter(torch.empty(F, H).uniform_(-k, k))
        self.out_b = nn.Parameter(torch.zeros(F))

    @staticmethod
    def _cell(gates: torch.Tensor, c: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        i, f, g, o = gates.chunk(4, dim=-1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
        h = torch.sigmoid(o) * torch.tanh(c)
        return h, c

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, T, F = x.shape
        H = self.H
        h = x.new_zeros(B, H)
        c = x.new_zeros(B, H)
        xin = x @ self.enc_w_ih.t() + self.enc_b  # [B, T, 4H] (one GEMM for all steps)
        for t in range(T):
            h, c = self._cell(xin[:, t] + h @ self.enc_w_hh.t(), c)
        ys = []
        for t in range(T):
            h, c = self._cell(h @ self.dec_w_hh.t() + self.dec_b, c)
            ys.append(h)
        hs = torch.stack(ys, 1)  # [B, T, H]
        return hs @ self.out_w.t() + self.out_b

    def recon_error(self, x: torch.Tensor) -> torch.Tensor:
        y = self.forward(x)
        return ((y - x) ** 2).mean(dim=(1, 2))


@dataclass
class Calibration:
    mu: float
    sigma: float


def calibrate(errors: torch.Tensor) -> Calibration:
    e = errors.detach().double()
    return Calibration(mu=float(e.mean()), sigma=float(e.std(unbiased=False)) + 1e-12)


def make_windows(series: torch.Tensor, T: int, count: int, generator: Optional[torch.Generator] = None
                 ) -> torch.Tensor:
    """Sample ``count`` windows of length T from ``series [N, L, F]`` → ``[count, T, F]``."""
    N, L, F = series.shape
    dev = series.device
    ni = torch.randint(0, N, (count,), generator=generator, device=dev)
    ti = torch.randint(0, L - T + 1, (count,), generator=generator, device=dev)
    idx = ti[:, None] + torch.arange(T, device=dev)[None, :]
    return series[ni[:, None], idx]


def normalize(series: torch.Tensor, eps: float = 1e-6):
    """Per-series, per-feature z-score over the history axis (dim 1)."""
    mu = series.mean(1, keepdim=True)
    sd = series.std(1, keepdim=True, unbiased=False).clamp(min=eps)
    return (series - mu) / sd, mu, sd
