"""Node health table of the production brain: RC1 + RC2 as ONE all-gather per tick.

Every brain rank (one process per GPU) owns a disjoint set of apps
(``brain/node.py`` shards apps by a stable hash of (namespace, app)), so the
per-app counters need no reduction: rank r contributes the fixed-size int32
record

    [roster_seq, n_apps, cap_request, n_series, full_seq | anomalous_0, scored_0, ...]

and ONE ``all_gather_into_tensor`` (RCCL over xGMI on the GPU, gloo on CPU)
gives every rank the whole node's table.  The records carry counters only;
the app NAMES behind each rank's rows travel through the node's key-value
store as DELTAS: when a rank's roster changes it publishes the ``(index,
name)`` changes since its last publication under ``roster/<rank>/d/<seq>``
(a full roster ``roster/<rank>/f/<seq>`` the first time, after a reset, when
the changes exceed half the roster, or every ``FULL_EVERY`` publications),
then announces ``seq`` and the seq of its last full roster in its header.  A
peer one publication behind reads one delta; one that lost track reads the
full roster and the deltas after it.  Under a steady deployment stream (the
roster changes every tick) the host work and the bytes per tick are
O(apps that changed), not O(apps).  Keys older than the previous full roster
are deleted.  When a rank needs more rows than the record holds it asks for a
larger ``cap`` in its header; every rank adopts the maximum on the next tick.

Failure handling: the all-gather is issued ``async_op=True`` and waited for
on the host with a deadline (:func:`~foremast_amd.parallel.comm.wait_bounded`),
so a dead or SIGSTOPped peer raises :class:`~foremast_amd.parallel.comm.CollectiveTimeout`
instead of wedging the rank in a D2H copy until the RCCL watchdog kills it;
roster reads wait on the store with the same deadline.  ``kv`` is the
generation's prefix store of the elastic world (``parallel/elastic.py``), or
the default process group's store; only without any store do full rosters
travel as objects.

At 100k series over 8 ranks (~2.5k apps per rank) the record is ~20 KB, so the
exchange is latency bound (one collective, tens of microseconds on xGMI).
"""

from __future__ import annotations

import datetime
import json
import time
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import comm

HDR = 5          # [roster seq, n_apps, cap_req, n_series, seq of the last full roster]
FULL_EVERY = 256  # a full roster at least every this many publications (bounds a reader's catch-up)


def _world(group=None) -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def _label(name) -> str:
    """``"namespace/app"`` of a roster entry: a (namespace, app) tuple (this rank's
    engines) or the label itself (a peer's roster, as published); "" for a free index."""
    if not name:
        return ""
    return name if isinstance(name, str) else f"{name[0]}/{name[1]}"


def _diff(old: Sequence, new: Sequence) -> List[Tuple[int, Any]]:
    """Index changes turning roster ``old`` into ``new`` (the fallback when the
    caller keeps no change log)."""
    out = [(i, n) for i, (o, n) in enumerate(zip(old, new)) if o != n]
    out += [(i, new[i]) for i in range(len(old), len(new))]
    out += [(i, None) for i in range(len(new), len(old)) if old[i] is not None]
    return out


class _Peer:
    __slots__ = ("seq", "names", "info")

    def __init__(self) -> None:
        self.seq = -1
        self.names: List[Any] = []
        self.info: Dict[str, Any] = {}


class ClusterHealth:
    def __init__(self, device, cap: int = 256, group=None, kv=None, timeout_s: Optional[float] = None) -> None:
        self.device = torch.device(device)
        self.cap = max(1, int(cap))
        self.group = group
        self.kv = kv                       # roster store (None: the default group's store)
        self.timeout_s = comm.exchange_timeout_s() if timeout_s is None else float(timeout_s)
        self.roster_exchanges = 0          # ticks on which some peer's roster had to be read
        self.roster_full_reads = 0
        self.last_ms = 0.0
        self.last_roster_bytes = 0         # roster bytes written + read by the last exchange
        self.last_phases_ms: Dict[str, float] = {}
        self._reset_state()

    def _reset_state(self) -> None:
        self._peers: Dict[int, _Peer] = {}
        self._seq = 0                      # roster publications of this rank
        self._fseq = -1                    # seq of its last full roster (-1: none yet)
        self._delta_n = 0                  # delta entries published since that full roster
        self._mine_version: Optional[int] = None
        self._pub_names: Optional[List[Any]] = None   # roster as last published (diff fallback only)
        self._keys: List[Tuple[int, str]] = []        # (seq, key) this rank published, oldest first
        self._info: Dict[str, Any] = {}

    def reset(self, kv=None) -> None:
        """Forget the peers' rosters (after the process group was re-formed);
        ``kv``: the new generation's roster store.  The next exchange publishes a
        full roster."""
        self._reset_state()
        if kv is not None:
            self.kv = kv

    def _store(self):
        if self.kv is None:
            try:
                self.kv = dist.PrefixStore("health", dist.distributed_c10d._get_default_store())
            except Exception:  # noqa: BLE001 - no default store: rosters travel as objects
                return None
        return self.kv

    def _publish(self, kv, rank: int, names: Sequence, version: int, info: Dict[str, Any],
                 changes: Optional[Tuple[bool, List[Tuple[int, Any]]]]) -> None:
        """Roster publication of this tick (only when the roster changed): the
        changes since the last publication, or a full roster when a reader could
        not catch up cheaply (first publication, a reset of the caller's table,
        more changes than half the roster, or every FULL_EVERY publications)."""
        if changes is None:
            items = _diff(self._pub_names or [], names)
            reset = self._pub_names is None
            self._pub_names = list(names)
        else:
            reset, items = changes
        self._seq += 1
        seq = self._seq
        full = (reset or self._fseq < 0 or seq - self._fseq >= FULL_EVERY
                or self._delta_n + len(items) > max(64, len(names) // 2))
        if full:
            key, rec = f"roster/{rank}/f/{seq}", {"n": [_label(n) for n in names], "info": info}
        else:
            key, rec = f"roster/{rank}/d/{seq}", {"i": [i for i, _ in items], "n": [_label(n) for _, n in items],
                                                  "info": info}
        raw = json.dumps(rec)
        kv.set(key, raw)   # published before the gather that announces it: a peer that sees it can read it
        self.last_roster_bytes += len(raw)
        self._keys.append((seq, key))
        if full:
            # readers still finishing the last tick need keys from the previous full roster on
            old_f, self._fseq, self._delta_n = self._fseq, seq, 0
            while self._keys and self._keys[0][0] < old_f:
                try:
                    kv.delete_key(self._keys.pop(0)[1])
                except Exception:  # noqa: BLE001 - best-effort cleanup
                    pass
        else:
            self._delta_n += len(items)

    def _read_many(self, keys: List[str]) -> List[Dict[str, Any]]:
        """Records under ``keys`` in two store round trips (one wait for all, one
        multi-get), however many peers they come from."""
        try:
            self.kv.wait(keys, datetime.timedelta(seconds=self.timeout_s))
            raws = self.kv.multi_get(keys) if hasattr(self.kv, "multi_get") else [self.kv.get(k) for k in keys]
        except Exception as e:  # noqa: BLE001 - store timeout: a peer is gone
            raise comm.CollectiveTimeout(f"peer rosters {keys[:4]}... not published: {e}") from e
        self.last_roster_bytes += sum(len(x) for x in raws)
        return [json.loads(x) for x in raws]

    def _catch_up(self, want: Dict[int, Tuple[int, int]]) -> None:
        """Bring each peer ``r`` of ``want`` (r -> (seq, full seq)) to publication
        ``seq``: its deltas, or its last full roster plus the deltas after it — all
        peers' records in one batched read."""
        plan: List[Tuple[int, int, str]] = []   # (peer, seq, kind) in apply order
        for r, (seq, fseq) in want.items():
            p = self._peers.setdefault(r, _Peer())
            q0 = p.seq
            if q0 < fseq:
                plan.append((r, fseq, "f"))
                q0 = fseq
            plan += [(r, q, "d") for q in range(q0 + 1, seq + 1)]
        recs = self._read_many([f"roster/{r}/{k}/{q}" for r, q, k in plan]) if plan else []
        for (r, q, kind), rec in zip(plan, recs):
            p = self._peers[r]
            if kind == "f":
                p.names, p.info = [n or None for n in rec["n"]], rec.get("info", {})
                self.roster_full_reads += 1
            else:
                names = p.names
                idx = rec["i"]
                if idx and max(idx) >= len(names):
                    names.extend([None] * (max(idx) + 1 - len(names)))
                for i, n in zip(idx, rec["n"]):
                    names[i] = n or None
                p.info = rec.get("info", p.info)
            p.seq = q
        for r, (seq, _f) in want.items():
            self._peers[r].seq = seq

    def exchange(self, names: Sequence[Tuple[str, str]], counts: torch.Tensor, roster_version: int,
                 n_series: int, info: Optional[Dict[str, Any]] = None,
                 changes: Optional[Tuple[bool, List[Tuple[int, Any]]]] = None) -> Dict[str, Any]:
        """One tick: gather every rank's per-app counters; returns the node table
        ``{"ranks", "members", "apps": {"ns/app": {anomalous, scored, rank}}, ...}``.
        ``names``: this rank's roster (index -> (namespace, app), None for a free
        index); ``changes``: its ``(reset, [(index, name)])`` since the last call
        (:class:`~foremast_amd.parallel.roster.ChangeLog`; None: diffed here)."""
        world, rank = _world(self.group)
        t0 = time.perf_counter()
        self.last_roster_bytes = 0
        active = comm.active(self.group)
        cap_req = 1
        while cap_req < len(names):
            cap_req *= 2
        info = dict(info or {})
        kv = self._store() if active else None
        if roster_version != self._mine_version or info != self._info:
            if active and kv is not None:
                self._publish(kv, rank, names, roster_version, info, changes)
            elif changes is None:
                self._pub_names = None
            self._mine_version, self._info = roster_version, info
        chunk = HDR + 2 * self.cap
        send = torch.zeros(chunk, dtype=torch.int32, device=self.device)
        k = min(len(names), self.cap)
        hdr = torch.tensor([self._seq, len(names), cap_req, n_series, self._fseq], dtype=torch.int32)
        send[:HDR].copy_(hdr.to(self.device, non_blocking=True))
        if k:
            send[HDR:HDR + 2 * k].copy_(counts[:k].reshape(-1))
        t1 = time.perf_counter()
        if active:
            recv = torch.empty(world * chunk, dtype=torch.int32, device=self.device)
            work = dist.all_gather_into_tensor(recv, send, group=self.group, async_op=True)
            comm.fault_point("exchange")
            comm.wait_bounded(work, self.timeout_s, "health all-gather")
        else:
            recv = send
        host = recv.cpu().view(world, chunk)
        t2 = time.perf_counter()
        rosters: List[Tuple[Sequence, Dict[str, Any]]] = []
        read = False
        if active and kv is None:  # no store at all: full rosters as objects, every tick
            objs: List[Any] = [None] * world
            dist.all_gather_object(objs, {"names": list(names), "info": info}, group=self.group)
            rosters = [(o["names"], o["info"]) for o in objs]
            read = True
        else:
            seqs, fseqs = host[:, 0].tolist(), host[:, 4].tolist()
            want = {r: (int(seqs[r]), int(fseqs[r])) for r in range(world) if r != rank
                    and (r not in self._peers or self._peers[r].seq != seqs[r])}
            if want:
                self._catch_up(want)
                read = True
            for r in range(world):
                p = self._peers.get(r)
                rosters.append((names, info) if r == rank else (p.names, p.info))
        t3 = time.perf_counter()
        if read:
            self.roster_exchanges += 1
        self.cap = max(self.cap, int(host[:, 2].max()))  # every rank adopts the same cap next tick
        self.last_ms = (time.perf_counter() - t0) * 1e3
        # anomalous apps of every rank in one pass over the gathered counters
        hn = host.numpy()
        lim = np.minimum(np.minimum(hn[:, 1], (chunk - HDR) // 2), [len(ro) for ro, _ in rosters])
        bad = hn[:, HDR::2] > 0
        bad &= np.arange(bad.shape[1])[None, :] < lim[:, None]
        anomalous = [_label(rosters[r][0][i]) for r, i in zip(*np.nonzero(bad)) if rosters[r][0][i]]
        members = [dict(rosters[r][1]) | {"rank": r, "apps": int(hn[r, 1]), "series": int(hn[r, 3])}
                   for r in range(world)]
        t4 = time.perf_counter()
        # where the exchange's time went: roster publication, the counter all-gather (includes
        # waiting for the slowest rank to reach it), peer roster reads, the table
        self.last_phases_ms = {"publish": round((t1 - t0) * 1e3, 3), "gather": round((t2 - t1) * 1e3, 3),
                               "rosters": round((t3 - t2) * 1e3, 3), "table": round((t4 - t3) * 1e3, 3)}
        return NodeTable({"ranks": world, "members": members, "anomalous_apps": sorted(anomalous),
                          "collective_ms": round(self.last_ms, 3), "roster_bytes": self.last_roster_bytes,
                          "exchange_phases_ms": self.last_phases_ms, "updated": time.time()},
                         host, [ro for ro, _ in rosters], chunk)


class NodeTable(dict):
    """The node health table of one tick.  ``table["apps"]`` — one entry per app
    of the node (``{"ns/app": {anomalous, scored, rank}}``) — is built from the
    gathered counters on first access only: at 20k apps building it costs tens
    of milliseconds of Python, and the tick itself needs just the anomalous
    apps (computed vectorised)."""

    def __init__(self, base: Dict[str, Any], host: torch.Tensor, rosters: List[Sequence], chunk: int) -> None:
        super().__init__(base)
        self._host, self._rosters, self._chunk = host, rosters, chunk

    def __missing__(self, key):
        if key != "apps":
            raise KeyError(key)
        apps: Dict[str, Dict[str, int]] = {}
        for r, ro in enumerate(self._rosters):
            n = min(int(self._host[r, 1]), (self._chunk - HDR) // 2, len(ro))
            cnt = self._host[r, HDR:HDR + 2 * n].view(n, 2).tolist()
            for name, (an, sc) in zip(ro[:n], cnt):
                if name:  # None: a free index of the rank's stable app table
                    apps[_label(name)] = {"anomalous": an, "scored": sc, "rank": r}
        self["apps"] = apps
        return apps

    def full(self) -> Dict[str, Any]:
        """Plain dict with every key (for publishing / JSON)."""
        return dict(self, apps=self["apps"])
