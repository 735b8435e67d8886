"""Joint (multi-metric) scoring of analysis jobs with the LSTM autoencoder,
plus the brain's LRU model cache and its on-disk checkpoint.

Reference: "3+ metrics → Deep Learning (LSTM)" (``docs/guides/design.md:84``)
and the brain's in-memory model cache bounded by ``MAX_CACHE_SIZE``
(``foremast-brain/README.md:30``).  Per job:

1. the job's F metric histories are aligned on their common (last-aligned)
   grid, gaps forward-filled, z-scored per metric;
2. a model keyed by ``(namespace, app, metric aliases)`` is taken from the
   cache, or trained (Adam on random history windows — the fused K7 kernel on
   the GPU) and calibrated (reconstruction-error mean/std over history
   windows), then cached;
3. for every current timestamp present in all metrics, the window ending
   there (history tail + current points, pods averaged) is scored — the fused
   MFMA kernel on the GPU — and flagged when ``z > threshold``.

The cache checkpoints to safetensors (weights + a JSON index of keys,
calibration and normalisation stats), so a restarted brain resumes with its
trained models.
"""

from __future__ import annotations

import json
import os
import time
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..models.lstm_ae import LSTMAutoencoder


@dataclass
class CachedModel:
    model: LSTMAutoencoder
    mu: float
    sigma: float
    mean: np.ndarray          # [F] normalisation
    std: np.ndarray           # [F]
    window: int
    trained_at: float
    uses: int = 0
    meta: Dict[str, str] = field(default_factory=dict)


class ModelCache:
    """LRU cache of fitted joint models (``MAX_CACHE_SIZE`` entries)."""

    def __init__(self, capacity: int = 1000) -> None:
        self.capacity = max(1, int(capacity))
        self._d: "OrderedDict[str, CachedModel]" = OrderedDict()
        self.hits = self.misses = self.evictions = 0

    @staticmethod
    def key(namespace: str, app: str, aliases: Sequence[str]) -> str:
        return f"{namespace}/{app}/" + ",".join(aliases)

    def get(self, key: str) -> Optional[CachedModel]:
        m = self._d.get(key)
        if m is None:
            self.misses += 1
            return None
        self._d.move_to_end(key)
        self.hits += 1
        m.uses += 1
        return m

    def put(self, key: str, m: CachedModel) -> None:
        self._d[key] = m
        self._d.move_to_end(key)
        while len(self._d) > self.capacity:
            self._d.popitem(last=False)
            self.evictions += 1

    def __len__(self) -> int:
        return len(self._d)

    def keys(self) -> List[str]:
        return list(self._d)

    # ------------------------------------------------------------------ checkpoint
    def save(self, path: str) -> None:
        from safetensors.torch import save_file
        tensors: Dict[str, torch.Tensor] = {}
        index = []
        for i, (k, m) in enumerate(self._d.items()):
            for name, p in m.model.state_dict().items():
                tensors[f"{i}.{name}"] = p.detach().float().cpu().contiguous()
            index.append({"key": k, "F": m.model.F, "H": m.model.H, "mu": m.mu, "sigma": m.sigma,
                          "mean": m.mean.tolist(), "std": m.std.tolist(), "window": m.window,
                          "trained_at": m.trained_at})
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        tmp = path + ".tmp"
        save_file(tensors, tmp, metadata={"index": json.dumps(index), "format": "foremast-lstm-cache-v1"})
        os.replace(tmp, path)  # atomic: a crash never leaves a torn checkpoint

    @classmethod
    def load(cls, path: str, capacity: int = 1000, device="cpu") -> "ModelCache":
        from safetensors import safe_open
        c = cls(capacity)
        with safe_open(path, framework="pt") as f:
            index = json.loads(f.metadata()["index"])
            for i, e in enumerate(index):
                m = LSTMAutoencoder(int(e["F"]), int(e["H"]))
                m.load_state_dict({n: f.get_tensor(f"{i}.{n}") for n, _ in m.state_dict().items()})
                c.put(e["key"], CachedModel(model=m.to(device), mu=e["mu"], sigma=e["sigma"],
                                            mean=np.array(e["mean"], np.float32), std=np.array(e["std"], np.float32),
                                            window=int(e["window"]), trained_at=float(e["trained_at"])))
        c.hits = c.misses = 0
        return c


def _ffill(a: np.ndarray) -> np.ndarray:
    """Forward-fill NaNs along axis 0 (leading NaNs → first valid / 0)."""
    out = a.copy()
    for f in range(a.shape[1]):
        col = out[:, f]
        ok = ~np.isnan(col)
        if not ok.any():
            col[:] = 0.0
            continue
        idx = np.where(ok, np.arange(len(col)), 0)
        np.maximum.accumulate(idx, out=idx)
        first = np.argmax(ok)
        col[:] = col[idx]
        col[:first] = col[first]
    return out


class LstmJobScorer:
    def __init__(self, device=None, cache: Optional[ModelCache] = None, hidden: int = 64,
                 train_steps: int = 80, train_batch: int = 256, lr: float = 1e-2, threshold: float = 4.0,
                 max_age_s: float = 24 * 3600.0, seed: int = 0, fp8: bool = False) -> None:
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.gpu = self.device.type == "cuda"
        self.cache = cache if cache is not None else ModelCache()
        self.hidden, self.train_steps, self.train_batch, self.lr = hidden, train_steps, train_batch, lr
        self.threshold, self.max_age_s, self.seed = threshold, max_age_s, seed
        self.fp8 = fp8  # score with fp8 e4m3 weights/activations on MFMA (GPU)
        self.trained = 0

    # ------------------------------------------------------------------ fit
    def _windows(self, z: torch.Tensor, W: int, n: int, g: torch.Generator) -> torch.Tensor:
        T = z.shape[0]
        st = torch.randint(0, T - W + 1, (n,), generator=g, device=z.device)
        return z[st[:, None] + torch.arange(W, device=z.device)[None, :]]  # [n, W, F]

    def _train(self, hist: np.ndarray, now: float) -> CachedModel:
        F = hist.shape[1]
        h = _ffill(hist)
        mean = h.mean(0).astype(np.float32)
        std = np.maximum(h.std(0), 1e-6).astype(np.float32)
        z = torch.from_numpy((h - mean) / std).float().to(self.device)
        W = int(min(32, max(4, z.shape[0] // 4)))
        torch.manual_seed(self.seed)
        model = LSTMAutoencoder(F, self.hidden).to(self.device)
        opt = torch.optim.Adam(model.parameters(), lr=self.lr)
        g = torch.Generator(device=self.device)
        g.manual_seed(self.seed + 1)
        fused = None
        B = self.train_batch
        if self.gpu and B % 32 == 0 and F <= 7 and self.hidden == 64:
            from ..ops.lstm_train import FusedLstmGrad
            fused = FusedLstmGrad(B, W, F, self.device)
        for _ in range(self.train_steps):
            x = self._windows(z, W, B, g).contiguous()
            opt.zero_grad(set_to_none=False)
            if fused is not None:
                fused.grads(model, x)
            else:
                model.recon_error(x).mean().backward()
            opt.step()
        with torch.no_grad():
            e = model.recon_error(self._windows(z, W, 512, g)).double()
        self.trained += 1
        return CachedModel(model=model, mu=float(e.mean()), sigma=float(e.std(unbiased=False)) + 1e-12,
                           mean=mean, std=std, window=W, trained_at=now)

    # ------------------------------------------------------------------ score
    def score_job(self, key: str, hist: np.ndarray, cur_ts: np.ndarray, cur: np.ndarray,
                  now: Optional[float] = None) -> Tuple[int, List[int], np.ndarray]:
        """``hist [T, F]`` (NaN gaps), ``cur [C, F]`` at ``cur_ts [C]`` (rows with a
        NaN are skipped).  Returns (verdict, anomalous row indices, z [C])."""
        now = time.time() if now is None else now
        if hist.shape[0] < 8 or not np.isfinite(hist).any():
            return -1, [], np.full(len(cur_ts), np.nan)
        m = self.cache.get(key)
        if m is None or m.model.F != hist.shape[1] or now - m.trained_at > self.max_age_s:
            m = self._train(hist, now)
            self.cache.put(key, m)
        W = m.window
        h = _ffill(hist)
        ok = np.all(np.isfinite(cur), axis=1)
        seq = np.concatenate([h, np.where(np.isfinite(cur), cur, np.nan)], 0)
        seq = _ffill(seq)
        zs = (seq - m.mean) / m.std
        T0 = h.shape[0]
        rows = [i for i in range(len(cur_ts)) if ok[i]]
        if not rows:
            return -1, [], np.full(len(cur_ts), np.nan)
        win = np.stack([zs[T0 + i + 1 - W: T0 + i + 1] for i in rows]).astype(np.float32)  # [R, W, F]
        x = torch.from_numpy(win).to(self.device)
        if self.gpu and m.model.H == 64:
            from ..ops import lstm as L
            p = L.pack(m.model, fp8=self.fp8, device=self.device)
            err = L.lstm_score(p, x.contiguous(), m.mu, m.sigma)["err"]
        else:
            with torch.no_grad():
                err = m.model.recon_error(x)
        z = ((err.double() - m.mu) / m.sigma).cpu().numpy()
        zfull = np.full(len(cur_ts), np.nan)
        zfull[rows] = z
        bad = [rows[j] for j in range(len(rows)) if z[j] > self.threshold]
        return (1 if bad else 0), bad, zfull


def align_job(tasks) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """MetricTasks of one job → (hist [T, F] last-aligned, cur_ts [C], cur [C, F])
    with current points averaged across pods per timestamp and restricted to
    timestamps present for every metric."""
    T = min(len(t.hist) for t in tasks)
    hist = np.stack([t.hist[-T:] for t in tasks], 1).astype(np.float32)
    per = []
    for t in tasks:
        acc: Dict[float, List[float]] = {}
        for ts, v in zip(t.cur_ts.tolist(), t.cur_vals.tolist()):
            if np.isfinite(v):
                acc.setdefault(float(ts), []).append(v)
        per.append({ts: float(np.mean(v)) for ts, v in acc.items()})
    common = sorted(set.intersection(*[set(p) for p in per])) if per else []
    cur = np.array([[p[ts] for p in per] for ts in common], dtype=np.float32).reshape(len(common), len(tasks))
    return hist, np.array(common, dtype=np.float64), cur
