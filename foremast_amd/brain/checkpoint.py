"""Checkpoint / resume of the streaming engines.

The reference keeps no engine state on disk: its durable state is the
DeploymentMonitor status (etcd) and the job documents (ES), and its brain
refits from Prometheus on restart.  Here a GPU shard holds a week of history
per series in HBM, so re-fetching 100k x 10,080 points after a restart costs
minutes of Prometheus load; a snapshot brings a rank back in seconds:

* :func:`save_streaming_shard` / :func:`load_streaming_shard` — the history
  ring (bf16, physical layout + head/length), the current and baseline pod
  windows, the per-series thresholds / bounds / app ids and the last fitted
  per-series parameters (level, trend, sigma, best grid point);
* :func:`save_lstm_shard` / :func:`load_lstm_shard` — the LSTM autoencoder
  weights AND its Adam state (moments, step counts), the calibration of the
  reconstruction error, per-series normalisation, the history rings and the
  window sampler's generator state, so training resumes exactly where it
  stopped.

Files are safetensors (tensors + a JSON metadata record, no pickle: loading
executes nothing from the file) written atomically (temp file + rename, so a
crash never leaves a torn checkpoint).  Resuming reproduces the uninterrupted
run bit for bit (``tests/test_checkpoint.py``).
"""

from __future__ import annotations

import json
import os
from typing import Any, Dict, Optional, Tuple

import torch

from ..ingest.ringbuffer import RingState

FORMAT = "foremast-amd/checkpoint/v1"
_DTYPES = {"bfloat16": torch.bfloat16, "float32": torch.float32, "float16": torch.float16}


def _dtype_name(dt: torch.dtype) -> str:
    for k, v in _DTYPES.items():
        if v == dt:
            return k
    raise ValueError(f"unsupported ring dtype {dt}")


def _atomic_save(tensors: Dict[str, torch.Tensor], meta: Dict[str, Any], path: str) -> None:
    from safetensors.torch import save_file
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    save_file({k: v.detach().contiguous().cpu() for k, v in tensors.items()}, tmp,
              metadata={"foremast": json.dumps(meta)})
    os.replace(tmp, path)


def _read(path: str, device) -> Tuple[Dict[str, Any], Dict[str, torch.Tensor]]:
    from safetensors import safe_open
    with safe_open(path, framework="pt", device="cpu") as f:
        md = f.metadata() or {}
        if "foremast" not in md:
            raise ValueError(f"{path}: not a foremast-amd checkpoint")
        meta = json.loads(md["foremast"])
        tensors = {k: f.get_tensor(k).to(device) for k in f.keys()}
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: unsupported checkpoint format {meta.get('format')!r}")
    return meta, tensors


# ---------------------------------------------------------------------- streaming shard
def save_streaming_shard(shard, path: str, extra: Optional[Dict[str, Any]] = None) -> None:
    """Snapshot a :class:`~foremast_amd.brain.engine.StreamingShard`."""
    sp = shard.spec
    tensors = {"hist": shard.hist._store, "cur": shard.cur.data, "base": shard.base,
               "threshold": shard.threshold, "bound": shard.bound, "min_lower": shard.min_lower,
               "app_id": shard.app_id}
    for k in ("level", "trend", "sigma", "best", "mean", "std"):
        if k in shard.out:
            tensors["fit." + k] = shard.out[k]
    meta = {"format": FORMAT, "kind": "streaming_shard",
            "spec": {"n_series": sp.n_series, "ring_len": sp.ring_len, "season": sp.season, "pods": sp.pods,
                     "window": sp.window, "algorithm": sp.algorithm, "pairwise": sp.pairwise,
                     "dtype": _dtype_name(sp.dtype), "n_apps": int(shard.app_stats.shape[0]),
                     "want_band": sp.want_band},
            "head": shard.hist.head, "length": shard.hist.length, "ticks": shard.cur.ticks,
            "extra": extra or {}}
    _atomic_save(tensors, meta, path)


def load_streaming_shard(path: str, cfg=None, device="cpu"):
    """Rebuild a StreamingShard from :func:`save_streaming_shard`; the fitted
    parameters of the last tick are in ``shard.fitted``."""
    from .engine import ShardSpec, StreamingShard
    meta, t = _read(path, device)
    if meta.get("kind") != "streaming_shard":
        raise ValueError(f"{path}: not a streaming-shard checkpoint")
    s = dict(meta["spec"])
    s["dtype"] = _DTYPES[s["dtype"]]
    shard = StreamingShard(ShardSpec(**s), cfg, device, app_id=t["app_id"].to(torch.int32),
                           threshold=t["threshold"], bound=t["bound"], min_lower=t["min_lower"])
    if tuple(t["hist"].shape) != tuple(shard.hist._store.shape):
        raise ValueError(f"{path}: ring geometry {tuple(t['hist'].shape)} does not match the spec")
    shard.hist._store.copy_(t["hist"])
    shard.hist.state = RingState(head=int(meta["head"]), length=int(meta["length"]))
    shard.cur.data.copy_(t["cur"])
    shard.cur.ticks = int(meta["ticks"])
    shard.base.copy_(t["base"])
    shard._refresh_horizons()
    shard.fitted = {k[4:]: v for k, v in t.items() if k.startswith("fit.")}
    shard.checkpoint_extra = meta.get("extra", {})
    return shard


# ---------------------------------------------------------------------- LSTM shard
def save_lstm_shard(shard, path: str, extra: Optional[Dict[str, Any]] = None) -> None:
    """Snapshot a :class:`~foremast_amd.brain.lstm_engine.LstmShard`: weights,
    Adam state, calibration, normalisation, rings, sampler state."""
    tensors: Dict[str, torch.Tensor] = {}
    for f, ring in enumerate(shard.rings):
        tensors[f"ring{f}"] = ring._store
    for k, v in shard.model.state_dict().items():
        tensors["model." + k] = v
    opt = shard.trainer.opt.state_dict()
    for idx, st in opt["state"].items():
        for k, v in st.items():
            tensors[f"adam.{idx}.{k}"] = v if torch.is_tensor(v) else torch.tensor(v)
    for k in ("mean", "std", "rstd", "app_id"):
        tensors[k] = getattr(shard, k)
    tensors["gen_state"] = shard.gen.get_state()
    if shard.cal is not None:
        tensors["cal"] = shard.cal
    if shard.lvl_sig is not None:
        tensors["lvl_sig"] = shard.lvl_sig
    hidden = int(shard.model.H)
    meta = {"format": FORMAT, "kind": "lstm_shard",
            "args": {"n_series": shard.n, "ring_len": shard.R, "n_features": shard.F, "window": shard.T,
                     "hidden": hidden, "fp8": bool(shard.fp8), "n_apps": int(shard.app_stats.shape[0]),
                     "threshold": float(shard.threshold), "train_batch": int(shard.train_batch),
                     "restat_every": int(shard.restat_every), "fused_train": bool(shard.fused_train),
                     "dtype": _dtype_name(shard.rings[0].data.dtype), "cal_windows": int(shard.cal_windows),
                     "cal_ewma": float(shard.cal_ewma), "season": int(shard.season),
                     "level_points": int(shard.level_points), "level_cal": int(shard.level_cal),
                     "level_threshold": shard.level_threshold},
            "param_groups": opt["param_groups"], "trainer_steps": int(shard.trainer.steps),
            "mu": float(shard.mu), "sigma": float(shard.sigma), "rho": float(shard.rho), "ticks": int(shard.ticks),
            "rings": [[r.head, r.length] for r in shard.rings], "extra": extra or {}}
    _atomic_save(tensors, meta, path)


def load_lstm_shard(path: str, device="cpu"):
    from .lstm_engine import LstmShard
    meta, t = _read(path, device)
    if meta.get("kind") != "lstm_shard":
        raise ValueError(f"{path}: not an LSTM-shard checkpoint")
    a = dict(meta["args"])
    hidden = a.pop("hidden") or 64
    dtype = _DTYPES[a.pop("dtype")]
    lr = float(meta["param_groups"][0]["lr"]) if meta["param_groups"] else 1e-3
    shard = LstmShard(a["n_series"], a["ring_len"], a["n_features"], window=a["window"], hidden=hidden,
                      fp8=a["fp8"], device=device, app_id=t["app_id"].to(torch.int32), n_apps=a["n_apps"],
                      threshold=a["threshold"], train_batch=a["train_batch"], lr=lr,
                      restat_every=a["restat_every"], dtype=dtype, fused_train=a["fused_train"],
                      cal_windows=int(a.get("cal_windows", 0)), cal_ewma=float(a.get("cal_ewma", 0.0)),
                      season=int(a.get("season", 1440)), level_points=int(a.get("level_points", 8)),
                      level_cal=int(a.get("level_cal", 64)), level_threshold=a.get("level_threshold", None))
    for f, ring in enumerate(shard.rings):
        ring._store.copy_(t[f"ring{f}"])
        ring.state = RingState(head=int(meta["rings"][f][0]), length=int(meta["rings"][f][1]))
    shard.model.load_state_dict({k[6:]: v for k, v in t.items() if k.startswith("model.")})
    state: Dict[int, Dict[str, torch.Tensor]] = {}
    for k, v in t.items():
        if k.startswith("adam."):
            _, idx, name = k.split(".", 2)
            state.setdefault(int(idx), {})[name] = v
    shard.trainer.opt.load_state_dict({"state": state, "param_groups": meta["param_groups"]})
    shard.trainer.steps = int(meta["trainer_steps"])
    for k in ("mean", "std", "rstd"):
        getattr(shard, k).copy_(t[k])
    shard.gen.set_state(t["gen_state"].cpu())
    shard.mu, shard.sigma = float(meta["mu"]), float(meta["sigma"])
    shard.rho = float(meta.get("rho", 1.0))
    shard.cal = t["cal"].float().contiguous() if "cal" in t else None
    shard.lvl_sig = t["lvl_sig"].float().contiguous() if "lvl_sig" in t else None
    shard.ticks = int(meta["ticks"])
    shard.packed = None  # repacked for the fused scorer on the next score
    shard.checkpoint_extra = meta.get("extra", {})
    return shard
