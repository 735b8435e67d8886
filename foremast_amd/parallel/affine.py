"""Cluster-affine ingest (RC5 in the product): each rank scrapes only its own
clusters' Prometheus, and the windows a job needs from another cluster cross
ranks over the node's process group.

The reference serves many clusters from one brain: every cluster runs a
barrelman pointing at the same service (``docs/guides/design.md:21``;
"aggregate service health check across multiple K8s clusters",
``README.md:27``).  On a GPU node the scrape of a cluster's Prometheus is
bound to ONE rank (network locality: each rank holds the connections and the
decode work of its clusters), a job is owned by the rank of the cluster its
new pods run in (history and current windows are then local), and the
windows that live in another cluster — the baseline pods of a cross-cluster
canary — are fetched and decoded by that cluster's rank and delivered to the
owner in the node's lockstep tick:

1. one ``all_gather`` of per-rank request counts (an int per rank, every tick);
2. when any rank has requests: every rank publishes its requests
   ``(family, start, n_points, [(namespace, pod), ...])`` in the node's key-value
   store and reads its peers' with a deadline (no object collective: a dead peer
   raises :class:`~foremast_amd.parallel.comm.CollectiveTimeout` instead of
   wedging the rank), every rank fetches and decodes the requests of its own
   clusters, and ONE ``all_to_all_single`` (RCCL over xGMI on the GPU, waited for
   with the same deadline) returns the ``[pods, n_points]`` values to the
   requesters, in an order every rank derives from the gathered requests.

Affinity: ``FOREMAST_CLUSTER_AFFINITY="<endpoint>=<rank>,..."`` or a stable
hash of the endpoint over the ranks.
"""

from __future__ import annotations

import datetime
import json
import os
import time
import zlib
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import comm

Request = Tuple[Tuple[str, str], float, int, List[Tuple[str, str]]]  # (family, start, n, pods)
CHUNK = 4 << 20   # bytes per store value of a published request list


def affinity_from_env() -> Callable[[str, int], int]:
    spec = os.environ.get("FOREMAST_CLUSTER_AFFINITY", "")
    table: Dict[str, int] = {}
    for part in spec.split(","):
        if "=" in part:
            ep, r = part.rsplit("=", 1)
            table[ep.strip()] = int(r)

    def rank_of(endpoint: str, world: int) -> int:
        if endpoint in table:
            return table[endpoint] % max(world, 1)  # a mapped rank that left: the survivors share it
        return zlib.crc32(endpoint.encode()) % max(world, 1)
    return rank_of


class ClusterRouter:
    def __init__(self, rank_of: Callable[[str, int], int], device, group=None,
                 timeout_s: Optional[float] = None, kv=None, home: Optional[Sequence[str]] = None) -> None:
        self.rank_of = rank_of
        # home: the endpoints this rank scrapes itself (default: those rank_of maps to it).  A
        # 1-rank rehearsal of the N-rank layout names its own cluster here, so the windows of
        # the "other" clusters still travel through the collective exchange (served by itself)
        self.home = set(home) if home is not None else None
        self.device = torch.device(device)
        self.group = group
        self.timeout_s = comm.exchange_timeout_s() if timeout_s is None else float(timeout_s)
        self.kv = kv        # request store (None: the default process group's store)
        self.seq = 0        # exchanges with requests so far (lockstep: equal on every rank)
        self.exchanges = 0
        self.values_moved = 0
        self.request_bytes = 0      # request payloads this rank published (pod lists, at admission)
        self.last = {"ms": 0.0, "bytes": 0, "requests": 0}   # the last exchange (tick record)
        self._stale: Optional[List[str]] = None   # this rank's request keys of the last exchange
        self._mine_keys: List[str] = []

    def reset(self, kv=None) -> None:
        """After a re-formation: the new generation's store, sequence from zero."""
        self.kv, self.seq, self._stale = kv, 0, None

    def _store(self):
        if self.kv is None:
            self.kv = dist.PrefixStore("affine", dist.distributed_c10d._get_default_store())
        return self.kv

    def _gather_requests(self, mine: Sequence[Request], world: int, rank: int) -> List[List[Request]]:
        """Publish this rank's requests and read every peer's: one set, one wait on all the
        peers' keys, one multi-get (two store round trips at any world size)."""
        kv, seq = self._store(), self.seq
        payload = json.dumps([[list(q[0]), q[1], q[2], [list(p) for p in q[3]]] for q in mine]).encode()
        # the store caps one value at 8 MiB: a burst of admissions is published in chunks, the
        # chunk count last (a reader that sees it sees every chunk)
        chunks = [payload[i:i + CHUNK] for i in range(0, len(payload), CHUNK)] or [b""]
        for i, c in enumerate(chunks):
            kv.set(f"req/{seq}/{rank}/{i}", c)
        kv.set(f"req/{seq}/{rank}", str(len(chunks)))
        self._mine_keys = [f"req/{seq}/{rank}"] + [f"req/{seq}/{rank}/{i}" for i in range(len(chunks))]
        self.request_bytes += len(payload)
        peers = [r for r in range(world) if r != rank]
        keys = [f"req/{seq}/{r}" for r in peers]

        def dec(v) -> str:
            return v.decode() if isinstance(v, (bytes, bytearray)) else bytes(v).decode()
        try:
            raws = []
            if keys:
                kv.wait(keys, datetime.timedelta(seconds=self.timeout_s))
                mget = kv.multi_get if hasattr(kv, "multi_get") else (lambda ks: [kv.get(k) for k in ks])
                counts = [int(dec(v)) for v in mget(keys)]
                ckeys = [f"req/{seq}/{r}/{i}" for r, n in zip(peers, counts) for i in range(n)]
                parts = mget(ckeys)
                pos = 0
                for n in counts:
                    raws.append(b"".join(bytes(v) for v in parts[pos:pos + n]))
                    pos += n
        except Exception as e:  # noqa: BLE001 - store timeout: a peer is gone
            raise comm.CollectiveTimeout(f"affine requests of ranks {peers} (exchange {seq}) not published: {e}") from e
        out: List[List[Request]] = [list(mine) if r == rank else [] for r in range(world)]
        for r, raw in zip(peers, raws):
            out[r] = [(tuple(q[0]), float(q[1]), int(q[2]), [tuple(p) for p in q[3]]) for q in json.loads(raw.decode())]
        return out

    @property
    def rank(self) -> int:
        return dist.get_rank(self.group) if comm.active(self.group) else 0

    @property
    def world(self) -> int:
        return dist.get_world_size(self.group) if comm.active(self.group) else 1

    def local(self, endpoint: str) -> bool:
        if self.home is not None:
            return endpoint in self.home
        return self.rank_of(endpoint, self.world) == self.rank

    async def exchange(self, mine: Sequence[Request], serve) -> List[torch.Tensor]:
        """Lockstep (every rank calls it once per tick).  ``mine``: this rank's
        requests for windows of other ranks' clusters; ``serve(requests) ->
        [values [pods, n]]`` fetches and decodes requests of this rank's own
        clusters (awaitable).  Returns the values of ``mine``, in order, as views of ONE
        device buffer (the all-to-all's output: the caller scatters them on the device;
        nothing is copied back to the host).

        Requests are route changes, not per-tick traffic: a job's remote window is
        requested once, at admission, and a tick without admissions costs one gather of
        request counts.  ``FOREMAST_FORCE_COLLECTIVES=1`` runs the collective path at one
        rank too (the 1-GPU rehearsal of the N-rank exchange)."""
        world, rank = self.world, self.rank
        t_start = time.perf_counter()
        if world <= 1 and not (comm.force_collectives() and comm.active(self.group)):
            if not mine:
                return []
            vals = list(await serve(list(mine)))
            self.last = {"ms": round((time.perf_counter() - t_start) * 1e3, 3), "bytes": 0, "requests": len(mine)}
            return [torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32)).to(self.device) for v in vals]
        cnt = torch.tensor([len(mine)], dtype=torch.int64, device=self.device)
        counts = torch.empty(world, dtype=torch.int64, device=self.device)
        work = dist.all_gather_into_tensor(counts, cnt, group=self.group, async_op=True)
        comm.wait_bounded(work, self.timeout_s, "affine request counts")
        if self._stale is not None:
            # every rank has entered this tick's count gather, so every rank is done reading the
            # last exchange's requests (a peer that exchanged no bytes with this rank in the
            # all-to-all may not have synchronised with it there: deleting the key right after
            # it could pull it from under that peer's read)
            try:
                for k in self._stale:
                    self._store().delete_key(k)
            except Exception:  # noqa: BLE001 - best-effort cleanup
                pass
            self._stale = None
        if int(counts.sum()) == 0:
            self.last = {"ms": round((time.perf_counter() - t_start) * 1e3, 3), "bytes": 0, "requests": 0}
            return []
        gathered = self._gather_requests(mine, world, rank)
        self.exchanges += 1
        # every rank derives the same order: requester q's requests by index, routed to the
        # rank whose cluster serves the family
        served_by = [[self.rank_of(req[0][0], world) for req in (gathered[q] or [])] for q in range(world)]
        to_serve = [(q, i, req) for q in range(world) for i, req in enumerate(gathered[q] or [])
                    if served_by[q][i] == rank]
        values = await serve([req for _, _, req in to_serve]) if to_serve else []
        send_parts: List[List[np.ndarray]] = [[] for _ in range(world)]
        for (q, _i, req), v in zip(to_serve, values):
            send_parts[q].append(np.asarray(v, dtype=np.float32).reshape(len(req[3]), req[2]))
        send_sizes = [sum(p.size for p in parts) for parts in send_parts]
        recv_sizes = [sum(len(req[3]) * req[2] for i, req in enumerate(mine) if served_by[rank][i] == a)
                      for a in range(world)]
        send = np.concatenate([p.reshape(-1) for parts in send_parts for p in parts]) if sum(send_sizes) else \
            np.zeros(0, dtype=np.float32)
        send_t = torch.from_numpy(send)
        if self.device.type == "cuda":  # one pinned staging copy, one H2D
            send_t = send_t.pin_memory().to(self.device, non_blocking=True)
        recv_t = torch.empty(sum(recv_sizes), dtype=torch.float32, device=self.device)
        work = dist.all_to_all_single(recv_t, send_t, output_split_sizes=recv_sizes, input_split_sizes=send_sizes,
                                      group=self.group, async_op=True)
        comm.wait_bounded(work, self.timeout_s, "affine window all-to-all")
        self._stale = list(self._mine_keys)   # deleted after the next tick's count gather
        self.seq += 1
        self.values_moved += int(recv_t.numel())
        offs = np.concatenate([[0], np.cumsum(recv_sizes)])
        out: List[Optional[torch.Tensor]] = [None] * len(mine)
        pos = {a: int(offs[a]) for a in range(world)}
        for i, req in enumerate(mine):  # rank a's part holds my requests to a, in index order
            a = served_by[rank][i]
            sz = len(req[3]) * req[2]
            out[i] = recv_t[pos[a]:pos[a] + sz].view(len(req[3]), req[2])
            pos[a] += sz
        self.last = {"ms": round((time.perf_counter() - t_start) * 1e3, 3),
                     "bytes": int(recv_t.numel() + send_t.numel()) * 4,
                     "requests": int(sum(len(g or []) for g in gathered))}
        return out  # type: ignore[return-value]
