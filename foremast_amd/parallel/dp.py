"""Data-parallel training for the LSTM autoencoder (RC3 / RC4).

One process per GPU.  Parameters are broadcast from rank 0 at start (RC4);
gradients live in contiguous flat buckets (``p.grad`` are views into them,
so backward accumulates straight into the communication buffer — no copy)
and each bucket is all-reduced with ONE collective as soon as every
gradient in it is final (post-accumulate hooks), overlapping the reduction
of late buckets with the rest of backward (RC3).  The LSTM-AE has ~35-70 k
parameters (≈0.1-0.3 MB fp32): one bucket, i.e. a single latency-bound
RCCL all-reduce per step over xGMI.  With ``world_size == 1`` everything is
local.  The same code runs under ``gloo`` on CPU for tests.
"""

from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import comm


def _world(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


class GradBuckets:
    def __init__(self, params: List[torch.nn.Parameter], bucket_bytes: int = 4 << 20, group=None,
                 overlap: bool = True) -> None:
        self.group = group
        self.world = _world(group)
        self.active = comm.active(group)
        self.params = [p for p in params if p.requires_grad]
        self.buckets: List[Dict] = []
        cur: List[torch.nn.Parameter] = []
        size = 0
        # reverse registration order ≈ order gradients become ready in backward
        for p in reversed(self.params):
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= bucket_bytes:
                self._make(cur)
                cur, size = [], 0
        if cur:
            self._make(cur)
        self.overlap = overlap and self.active
        self._handles: List = []
        if self.overlap:
            for bi, b in enumerate(self.buckets):
                for p in b["params"]:
                    p.register_post_accumulate_grad_hook(self._hook(bi))

    def _make(self, params: List[torch.nn.Parameter]) -> None:
        dtype = params[0].dtype
        dev = params[0].device
        n = sum(p.numel() for p in params)
        flat = torch.zeros(n, dtype=dtype, device=dev)
        off = 0
        for p in params:
            k = p.numel()
            p.grad = flat[off:off + k].view_as(p)
            off += k
        self.buckets.append({"flat": flat, "params": params, "ready": 0})

    def _hook(self, bi: int):
        def fn(_p):
            b = self.buckets[bi]
            b["ready"] += 1
            if b["ready"] == len(b["params"]):
                self._handles.append(dist.all_reduce(b["flat"], group=self.group, async_op=True))
        return fn

    def zero(self) -> None:
        for b in self.buckets:
            b["flat"].zero_()
            b["ready"] = 0

    def finish(self, weight: Optional[float] = None, flags: Optional[torch.Tensor] = None,
               timeout_s: Optional[float] = None) -> Optional[torch.Tensor]:
        """Complete the reduction (average over ranks).  Buckets whose hooks
        did not fire (gradients written directly, e.g. by the fused LSTM
        training kernel) are all-reduced here.

        ``weight``: this rank's share of the step (e.g. 0 for a rank with no
        series: it still joins the collective, with a zero gradient); the
        average is then weighted, the weights travelling in the same
        all-reduce as an extra element.  ``flags``: small float tensor of
        per-rank values summed in that same collective (returned reduced) —
        e.g. "some rank admitted series and needs a calibration pass".
        ``timeout_s``: host-side deadline on the reduction
        (:func:`~foremast_amd.parallel.comm.wait_bounded`)."""
        extra = None
        if weight is not None and self.overlap and any(b["ready"] for b in self.buckets):
            raise ValueError("weighted steps need GradBuckets(overlap=False): hooks reduce before the weight applies")
        if weight is not None or flags is not None:
            # a device-side fill, not torch.tensor([...], device=...): a pageable host copy
            # would block the host until the GPU drained every step queued before it
            parts = [torch.full((1,), 1.0 if weight is None else float(weight), dtype=torch.float32,
                                device=self.buckets[-1]["flat"].device)]
            if flags is not None:
                parts.append(flags.to(parts[0].device, torch.float32).reshape(-1))
            extra = torch.cat(parts)
            if weight is not None and weight != 1.0:
                for b in self.buckets:
                    b["flat"].mul_(float(weight))
        active = comm.active(self.group)
        if active:
            world = dist.get_world_size(self.group)
            for b in self.buckets:
                if not self.overlap or b["ready"] < len(b["params"]):
                    if extra is not None and b is self.buckets[-1]:
                        # one collective: the last bucket carries the weights / flags
                        cat = torch.cat([b["flat"], extra.to(b["flat"].dtype)])
                        self._handles.append((dist.all_reduce(cat, group=self.group, async_op=True), cat, b))
                    else:
                        self._handles.append((dist.all_reduce(b["flat"], group=self.group, async_op=True), None, b))
            for h in self._handles:
                if isinstance(h, tuple):
                    work, cat, b = h
                    if timeout_s is not None:
                        comm.wait_bounded(work, timeout_s, "gradient all-reduce")
                    else:
                        work.wait()
                    if cat is not None:
                        n = b["flat"].numel()
                        b["flat"].copy_(cat[:n])
                        extra = cat[n:].to(torch.float32)
                else:
                    h.wait()
            self._handles.clear()
        else:
            world = 1
        if extra is not None:
            if active and self.overlap and all(b["ready"] == len(b["params"]) for b in self.buckets):
                # hooks reduced every bucket already: reduce the extras on their own
                if timeout_s is not None:
                    w = dist.all_reduce(extra, group=self.group, async_op=True)
                    comm.wait_bounded(w, timeout_s, "gradient weights")
                else:
                    dist.all_reduce(extra, group=self.group)
            total = float(extra[0])
            for b in self.buckets:
                b["flat"].div_(max(total, 1e-12))
            return extra[1:]
        if active:
            for b in self.buckets:
                b["flat"].div_(world)
        return None


def broadcast_params(module: torch.nn.Module, src: int = 0, group=None) -> None:
    if comm.active(group):
        for p in module.parameters():
            dist.broadcast(p.data, src=src, group=group)


class DPTrainer:
    """Adam on the reconstruction loss with bucketed gradient all-reduce."""

    def __init__(self, model: torch.nn.Module, lr: float = 1e-3, group=None, bucket_bytes: int = 4 << 20,
                 overlap: bool = True, grad_fn=None) -> None:
        """``grad_fn(model, windows) -> loss`` (optional) writes ``p.grad`` itself
        (fused kernel path) instead of autograd."""
        self.model = model
        self.grad_fn = grad_fn
        broadcast_params(model, 0, group)
        self.buckets = GradBuckets(list(model.parameters()), bucket_bytes, group, overlap)
        on_gpu = next(model.parameters()).is_cuda
        # fused multi-tensor Adam on the GPU: one launch for all parameters; capturable (its
        # step counters on the device) so a training step can be part of a HIP graph
        self.opt = torch.optim.Adam(model.parameters(), lr=lr, fused=on_gpu or None, capturable=on_gpu)
        self.steps = 0

    def step(self, windows, grad_fn=None, weight: Optional[float] = None, flags: Optional[torch.Tensor] = None,
             timeout_s: Optional[float] = None) -> torch.Tensor:
        """``grad_fn`` overrides the constructor's for this step (e.g. the
        second half of a split fused-kernel gradient).  ``windows`` None with
        ``weight`` 0: this rank has no data and joins the reduction with a zero
        gradient (every rank's Adam then applies the same averaged step, so the
        replicas stay identical).  ``flags`` / ``timeout_s``: see
        :meth:`GradBuckets.finish`; the reduced flags are kept in ``last_flags``."""
        self.buckets.zero()
        grad_fn = grad_fn or self.grad_fn
        if windows is None and grad_fn is None:
            loss = torch.zeros((), device=self.buckets.buckets[0]["flat"].device)
        elif grad_fn is not None:
            loss = grad_fn(self.model, windows)
        else:
            loss = self.model.recon_error(windows).mean()
            loss.backward()
        self.last_flags = self.buckets.finish(weight, flags, timeout_s)
        self.opt.step()
        self.steps += 1
        return loss.detach()
