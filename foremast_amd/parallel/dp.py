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

    def finish(self) -> None:
        """Complete the reduction (average over ranks).  Buckets whose hooks
        did not fire (gradients written directly, e.g. by the fused LSTM
        training kernel) are all-reduced here."""
        if self.active:
            for b in self.buckets:
                if not self.overlap or b["ready"] < len(b["params"]):
                    self._handles.append(dist.all_reduce(b["flat"], group=self.group, async_op=True))
            for h in self._handles:
                h.wait()
            self._handles.clear()
            for b in self.buckets:
                b["flat"].div_(self.world)


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
        # fused multi-tensor Adam on the GPU: one launch for all parameters
        self.opt = torch.optim.Adam(model.parameters(), lr=lr, fused=on_gpu or None)
        self.steps = 0

    def step(self, windows, grad_fn=None) -> torch.Tensor:
        """``grad_fn`` overrides the constructor's for this step (e.g. the
        second half of a split fused-kernel gradient)."""
        self.buckets.zero()
        grad_fn = grad_fn or self.grad_fn
        if grad_fn is not None:
            loss = grad_fn(self.model, windows)
        else:
            loss = self.model.recon_error(windows).mean()
            loss.backward()
        self.buckets.finish()
        self.opt.step()
        self.steps += 1
        return loss.detach()
