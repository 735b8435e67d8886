"""Node health table of the production brain: RC1 + RC2 as ONE all-gather per tick.

Every brain rank (one process per GPU) owns a disjoint set of apps
(``brain/node.py`` shards apps by a stable hash of (namespace, app)), so the
per-app counters need no reduction: rank r contributes the fixed-size int32
record

    [roster_version, n_apps, cap_request, n_series | anomalous_0, scored_0, ...]

and ONE ``all_gather_into_tensor`` (RCCL over xGMI on the GPU, gloo on CPU)
gives every rank the whole node's table.  The records carry counters only;
the app NAMES behind each rank's rows travel in a control-plane
``all_gather_object`` that runs only when some rank's roster version changed
(jobs started or finished) — every rank sees the same gathered headers, so
all take that branch together and the collective sequence stays matched.
When a rank needs more rows than the record holds it asks for a larger
``cap`` in its header; every rank adopts the maximum on the next tick.

Failure handling: the all-gather is issued ``async_op=True`` and waited for
on the host with a deadline (:func:`~foremast_amd.parallel.comm.wait_bounded`),
so a dead or SIGSTOPped peer raises :class:`~foremast_amd.parallel.comm.CollectiveTimeout`
instead of wedging the rank in a D2H copy until the RCCL watchdog kills it;
with a key-value store (``kv``: the generation's prefix store of the elastic
world) the app rosters travel through the store, read with the same deadline,
instead of an object collective.

At 100k series over 8 ranks (~2.5k apps per rank) the record is ~20 KB, so the
exchange is latency bound (one collective, tens of microseconds on xGMI).
"""

from __future__ import annotations

import datetime
import json
import time
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import comm

HDR = 4


def _world(group=None) -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


class ClusterHealth:
    def __init__(self, device, cap: int = 256, group=None, kv=None, timeout_s: Optional[float] = None) -> None:
        self.device = torch.device(device)
        self.cap = max(1, int(cap))
        self.group = group
        self.kv = kv                       # roster store (None: all_gather_object)
        self.timeout_s = comm.exchange_timeout_s() if timeout_s is None else float(timeout_s)
        self._versions: Optional[List[int]] = None
        self._rosters: List[Dict[str, Any]] = []
        self._published: Optional[int] = None
        self._mine: Optional[Dict[str, Any]] = None   # roster record of _mine_version
        self._mine_version: Optional[int] = None
        self.roster_exchanges = 0
        self.last_ms = 0.0

    def reset(self, kv=None) -> None:
        """Forget the peers' rosters (after the process group was re-formed);
        ``kv``: the new generation's roster store."""
        self._versions = None
        self._rosters = []
        self._published = None
        if kv is not None:
            self.kv = kv

    def _read_roster(self, r: int, version: int) -> Dict[str, Any]:
        key = f"roster/{r}/{version}"
        try:
            self.kv.wait([key], datetime.timedelta(seconds=self.timeout_s))
            return json.loads(self.kv.get(key))
        except Exception as e:  # noqa: BLE001 - store timeout: the peer is gone
            raise comm.CollectiveTimeout(f"roster of rank {r} (version {version}) not published: {e}") from e

    def exchange(self, names: Sequence[Tuple[str, str]], counts: torch.Tensor, roster_version: int,
                 n_series: int, info: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        """One tick: gather every rank's per-app counters; returns the node table
        ``{"ranks", "members", "apps": {"ns/app": {anomalous, scored, rank}}, ...}``."""
        world, rank = _world(self.group)
        t0 = time.perf_counter()
        cap_req = 1
        while cap_req < len(names):
            cap_req *= 2
        chunk = HDR + 2 * self.cap
        send = torch.zeros(chunk, dtype=torch.int32, device=self.device)
        k = min(len(names), self.cap)
        hdr = torch.tensor([roster_version, len(names), cap_req, n_series], dtype=torch.int32)
        send[:HDR].copy_(hdr.to(self.device, non_blocking=True))
        if k:
            send[HDR:HDR + 2 * k].copy_(counts[:k].reshape(-1))
        # this rank's roster record, built only when the roster changed (O(apps) per change,
        # not per tick: a node holds tens of thousands of apps)
        if self._mine is None or self._mine_version != roster_version:
            # (namespace, app) tuples as given (JSON writes them as lists; a C-level copy,
            # not a Python loop: the roster of a node with arrivals changes every tick)
            self._mine = {"names": list(names), "version": roster_version}
            self._mine_version = roster_version
        mine = dict(info or {}, **self._mine)
        if self.kv is not None and comm.active(self.group) and self._published != roster_version:
            # publish before the gather that announces the version: a peer that sees it can read it
            self.kv.set(f"roster/{rank}/{roster_version}", json.dumps(mine))
            if self._published is not None:
                try:
                    self.kv.delete_key(f"roster/{rank}/{self._published}")
                except Exception:  # noqa: BLE001 - best effort cleanup
                    pass
            self._published = roster_version
        if comm.active(self.group):
            recv = torch.empty(world * chunk, dtype=torch.int32, device=self.device)
            work = dist.all_gather_into_tensor(recv, send, group=self.group, async_op=True)
            comm.fault_point("exchange")
            comm.wait_bounded(work, self.timeout_s, "health all-gather")
        else:
            recv = send
        host = recv.cpu().view(world, chunk)
        versions = host[:, 0].tolist()
        if versions != self._versions or len(self._rosters) != world:
            if not comm.active(self.group):
                rosters: List[Any] = [mine]
            elif self.kv is not None:
                rosters = [mine if r == rank else self._read_roster(r, int(versions[r])) for r in range(world)]
            else:
                rosters = [None] * world
                dist.all_gather_object(rosters, mine, group=self.group)
            self._rosters, self._versions = rosters, versions
            self.roster_exchanges += 1
        self.cap = max(self.cap, int(host[:, 2].max()))  # every rank adopts the same cap next tick
        self.last_ms = (time.perf_counter() - t0) * 1e3
        members, anomalous = [], []
        for r in range(world):
            ro = self._rosters[r]
            n = min(int(host[r, 1]), (chunk - HDR) // 2, len(ro["names"]))
            bad = torch.nonzero(host[r, HDR:HDR + 2 * n:2] > 0).flatten().tolist()
            anomalous += [f"{ro['names'][i][0]}/{ro['names'][i][1]}" for i in bad if ro["names"][i]]
            members.append({k: v for k, v in ro.items() if k not in ("names", "version")}
                           | {"rank": r, "apps": int(host[r, 1]), "series": int(host[r, 3])})
        return NodeTable({"ranks": world, "members": members, "anomalous_apps": sorted(anomalous),
                          "collective_ms": round(self.last_ms, 3), "updated": time.time()},
                         host, self._rosters, chunk)


class NodeTable(dict):
    """The node health table of one tick.  ``table["apps"]`` — one entry per app
    of the node (``{"ns/app": {anomalous, scored, rank}}``) — is built from the
    gathered counters on first access only: at 20k apps building it costs tens
    of milliseconds of Python, and the tick itself needs just the anomalous
    apps (computed vectorised)."""

    def __init__(self, base: Dict[str, Any], host: torch.Tensor, rosters: List[Dict[str, Any]], chunk: int) -> None:
        super().__init__(base)
        self._host, self._rosters, self._chunk = host, rosters, chunk

    def __missing__(self, key):
        if key != "apps":
            raise KeyError(key)
        apps: Dict[str, Dict[str, int]] = {}
        for r, ro in enumerate(self._rosters):
            n = min(int(self._host[r, 1]), (self._chunk - HDR) // 2, len(ro["names"]))
            cnt = self._host[r, HDR:HDR + 2 * n].view(n, 2).tolist()
            for name, (an, sc) in zip(ro["names"][:n], cnt):
                if name:  # None: a free index of the rank's stable app table
                    apps[f"{name[0]}/{name[1]}"] = {"anomalous": an, "scored": sc, "rank": r}
        self["apps"] = apps
        return apps

    def full(self) -> Dict[str, Any]:
        """Plain dict with every key (for publishing / JSON)."""
        return dict(self, apps=self["apps"])
