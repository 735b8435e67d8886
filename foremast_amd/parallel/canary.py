"""Cross-shard canary A/B exchange (RC5).

Multi-cluster canary analysis compares a canary's range-vectors with the
baseline's (``BASELINE.json`` config 4).  When the baseline cluster's
samples are ingested by a different rank than the one that owns the series
(shards follow ``hash(namespace, app)``, ingest follows the scrape source),
the baseline windows must travel to the owner before the rank tests run.

One exchange per tick, two ``all_to_all_single`` calls (counts, then
payload) — the expert-parallel dispatch pattern, point-to-point over xGMI
with RCCL, each pair of GPUs on its own link:

* rows are grouped by destination rank (stable sort by owner);
* a [world] counts all-to-all sizes the receive buffers;
* ids (int64) and windows (float32, NaN-padded to W) move in one payload
  all-to-all each.
"""

from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist

from . import comm


def _world(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def exchange_windows(ids: torch.Tensor, values: torch.Tensor, owner: torch.Tensor,
                     group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Send row ``i`` (``ids[i]``, ``values[i, :]``) to rank ``owner[i]``.
    Returns the rows this rank received (ids, values), grouped by source rank."""
    world = _world(group)
    if not comm.active(group):
        return ids, values
    dev = values.device
    W = values.shape[1]
    order = torch.argsort(owner, stable=True)
    ids_s = ids[order].contiguous()
    vals_s = values[order].contiguous()
    send_counts = torch.bincount(owner.long(), minlength=world).to(torch.int64)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    n_recv = int(sum(rc))
    ids_r = torch.empty(n_recv, dtype=ids_s.dtype, device=dev)
    vals_r = torch.empty((n_recv, W), dtype=vals_s.dtype, device=dev)
    dist.all_to_all_single(ids_r, ids_s, rc, sc, group=group)
    dist.all_to_all_single(vals_r.view(-1), vals_s.view(-1), [c * W for c in rc], [c * W for c in sc], group=group)
    return ids_r, vals_r


def scatter_rows(dst: torch.Tensor, local_index: torch.Tensor, rows: torch.Tensor) -> None:
    """``dst[local_index[i]] = rows[i]`` (received windows into the owner's buffer)."""
    if rows.numel():
        dst.index_copy_(0, local_index.long(), rows.to(dst.dtype))


def owner_of(series_ids: torch.Tensor, starts: torch.Tensor) -> torch.Tensor:
    """Rank owning each global series id given the shard start offsets
    (``starts[r]`` = first id of rank r, ascending)."""
    return (torch.searchsorted(starts, series_ids, right=True) - 1).to(torch.int64)


def shard_starts(n_total: int, world: int, align: int = 1, device=None) -> torch.Tensor:
    from .health import shard_range
    return torch.tensor([shard_range(n_total, world, r, align)[0] for r in range(world)], dtype=torch.int64,
                        device=device)


def remote_baseline_ids(n_total: int, world: int, rank: int, align: int = 1) -> torch.Tensor:
    """Series whose baseline samples this rank ingests in the multi-cluster
    layout: the shard of rank ``(rank + 1) % world`` (the baseline cluster is
    scraped by the neighbour)."""
    from .health import shard_range
    s, e, _ = shard_range(n_total, world, (rank + 1) % world, align)
    return torch.arange(s, e, dtype=torch.int64)



class WindowExchanger:
    """Fixed routing for the per-tick baseline exchange: the (ids, owner)
    layout does not change between ticks, so the counts all-to-all and the
    destination sort run once; each tick is ONE payload ``all_to_all_single``."""

    def __init__(self, ids: torch.Tensor, owner: torch.Tensor, width: int, group=None) -> None:
        self.group = group
        self.world = _world(group)
        self.active = comm.active(group)
        self.width = width
        self.order = torch.argsort(owner, stable=True)
        dev = ids.device
        if not self.active:
            self.recv_ids = ids
            return
        send_counts = torch.bincount(owner.long(), minlength=self.world).to(torch.int64)
        recv_counts = torch.empty_like(send_counts)
        dist.all_to_all_single(recv_counts, send_counts, group=group)
        self.sc, self.rc = send_counts.tolist(), recv_counts.tolist()
        ids_s = ids[self.order].contiguous()
        self.recv_ids = torch.empty(int(sum(self.rc)), dtype=ids.dtype, device=dev)
        dist.all_to_all_single(self.recv_ids, ids_s, self.rc, self.sc, group=group)
        self.recv = torch.empty((int(sum(self.rc)), width), dtype=torch.float32, device=dev)

    def __call__(self, values: torch.Tensor) -> torch.Tensor:
        if not self.active:
            return values
        send = values[self.order].contiguous()
        W = self.width
        dist.all_to_all_single(self.recv.view(-1), send.view(-1), [c * W for c in self.rc],
                               [c * W for c in self.sc], group=self.group)
        return self.recv
