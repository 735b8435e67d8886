"""The node's resident 7-day history, keyed by series.

A one-shot canary / rollingUpdate job asks for the 7-day history of every
metric it watches (``namespace_app_per_pod:<m>{namespace, app}`` over
``[start - 7d, start]``, ``metricsquery.go:73-79``).  The reference brain
re-fetches that week of points per job and cycle.  Here the week of every
series a job has used stays in HBM (100k series x 10,080 points x 2 B = 2 GB
bf16 of the 288 GB) and is kept current with ONE short range query per metric
family per tick, so a job on an app seen before (re-deploys, canaries of a
continuously watched app) starts scoring without any history fetch:

* rows: one per (endpoint, metric, namespace, app); a row is referenced by
  the jobs that use it (:meth:`want` / :meth:`unwant`) and retained for
  ``retain_s`` after its last job (``FOREMAST_HISTORY_RETAIN_S``), then
  freed in place; the table grows by doubling;
* columns: one shared time axis at the query step, newest point at
  ``t_last`` (a full ring: unknown points are NaN, the kernels skip them);
* loads: a new series' week arrives in (time chunk x app group) queries that
  stay below Prometheus' ``--query.max-samples``, decoded by the native keyed
  parser into one pinned block and copied H2D once; a key whose load had a
  failed query stays pending and is retried next sync;
* advance: the tick's newest points of every resident row (one query per
  family, split into time chunks after an outage); if any of them fails the
  ring does not move, so the next sync fetches the same minutes again
  instead of leaving NaN holes; behind by more than the ring, every row is
  reloaded.
"""

from __future__ import annotations

import asyncio
import collections
import itertools
import logging
import operator
import os
import re
import time
from collections import _count_elements  # the C helper of Counter.update
from typing import Dict, Iterable, List, Optional, Sequence, Set, Tuple
from urllib.parse import quote

import numpy as np
import torch

from ..ingest import native
from ..ingest.ringbuffer import HistoryRing

log = logging.getLogger("foremast.resident")

Key = Tuple[str, str, str, str]  # (endpoint, metric, namespace, app)

_RE2_SPECIAL = re.compile(r"([\\.^$|?*+()\[\]{}])")


_RE2_SPECIAL_NOBAR = re.compile(r"[\\.^$?*+()\[\]{}]")


def re_alt(values: Iterable[str]) -> str:
    """RE2 alternation of literal label values, escaped for a PromQL string (values
    without RE2 metacharacters -- every k8s pod / app name without a dot -- are
    joined as they are: one scan of the joined string instead of one per value)."""
    vals = sorted(values)
    joined = "|".join(vals)
    if "|" not in "".join(vals) and _RE2_SPECIAL_NOBAR.search(joined) is None:
        return joined
    return "|".join(_RE2_SPECIAL.sub(r"\\\\\1", v) for v in vals)


# urllib.parse.quote(s, safe="") for ASCII selectors as one str.replace per special
# character present (quote builds a list of per-character strings, and str.translate does
# a dict lookup per character: both take milliseconds on the 30 KB pod alternations of a
# window query; a selector holds a handful of distinct special characters)
_SPECIAL = [c for c in map(chr, range(32, 127)) if not (c.isalnum() or c in "_.-~%")]


def _quote(s: str) -> str:
    if not (s.isascii() and s.isprintable()):
        return quote(s, safe="")
    if "%" in s:  # first: the escapes below introduce '%'
        s = s.replace("%", "%25")
    for c in _SPECIAL:
        if c in s:
            s = s.replace(c, f"%{ord(c):02X}")
    return s


def quote_selector(selector: str) -> str:
    return _quote(selector)


def range_url_quoted(endpoint: str, quoted: str, start: float, n: int, step: float) -> str:
    """:func:`range_url` of an already URL-quoted selector."""
    return f"{endpoint}query_range?query={quoted}&start={int(start)}&end={int(start + (n - 1) * step)}&step={int(step)}"


def range_url(endpoint: str, selector: str, start: float, n: int, step: float) -> str:
    return range_url_quoted(endpoint, _quote(selector), start, n, step)


async def fetch_decode(prom, reqs: Sequence[Tuple[str, float, int, int]], tables: Sequence[native.KeyTable],
                       out: np.ndarray, step: float, threads: int,
                       timings: Optional[Dict[str, float]] = None, fill_nan: bool = False) -> List[bool]:
    """Fetch ``reqs`` = (url, start, n_points, col0) and scatter every body through
    its key table into ``out`` (one native call on a thread pool, off the event
    loop).  Returns per request whether it was fetched and decoded; ``timings``
    receives ``fetch_ms`` / ``native_ms`` / ``resume_ms`` (executor hand-back).
    ``fill_nan``: the native threads first set the bodies' column span of every
    row of ``out`` to NaN (the caller did not pre-fill it)."""
    t0 = time.perf_counter()
    bodies = await prom.fetch_raw_many([u for u, *_ in reqs])
    t1 = time.perf_counter()
    ok = [not isinstance(b, Exception) for b in bodies]
    for (url, *_), b in zip(reqs, bodies):
        if isinstance(b, Exception):
            log.warning("fetch %s failed: %s", url.split("?")[0], b)
    good = [j for j in range(len(reqs)) if ok[j]]
    if not good:
        return ok
    args = ([bodies[j] for j in good], [tables[j] for j in good], [reqs[j][1] for j in good],
            [reqs[j][2] for j in good], [reqs[j][3] for j in good])
    span = [0.0, 0.0]

    def run():
        span[0] = time.perf_counter()
        r = native.decode_bodies(args[0], args[1], args[2], step, args[3], args[4], out, threads=threads,
                                 fill_nan=fill_nan)
        span[1] = time.perf_counter()
        return r
    stats = await asyncio.get_running_loop().run_in_executor(None, run)
    if timings is not None:
        t2 = time.perf_counter()
        timings["fetch_ms"] = (t1 - t0) * 1e3
        timings["native_ms"] = (span[1] - span[0]) * 1e3
        timings["resume_ms"] = ((span[0] - t1) + (t2 - span[1])) * 1e3
        timings["body_mb"] = sum(len(b) for b in args[0]) / 1e6
    for j, (series, _dropped, _unmatched) in zip(good, stats):
        if series < 0:
            log.warning("malformed response for %s", reqs[j][0].split("?")[0])
            ok[j] = False
    return ok


def history_key_hash(k: Key) -> int:
    """64-bit key of a history series: series_key of "endpoint\x1fmetric" and
    "namespace\x1fapp" (the key ``ingest/csrc/job_plan.cpp`` emits per series)."""
    return native.key_hash(k[0] + "\x1f" + k[1], k[2] + "\x1f" + k[3])


class ResidentHistory:
    """Rows are indexed by the 64-bit history key (:func:`history_key_hash`), so a
    batch of admitted jobs finds its rows with integer dict lookups; the key tuple
    of a row is kept for its queries.  The tuple API (:meth:`want`, :meth:`ready`,
    :meth:`row_of`) hashes once per distinct key."""

    def __init__(self, prom, device, ring_len: int = 10080, step: float = 60.0, clock=time.time,
                 chunk_points: int = 1440, apps_per_query: int = 256, decode_threads: Optional[int] = None,
                 min_capacity: int = 64, retain_s: float = 86400.0, dtype: Optional[torch.dtype] = None) -> None:
        self.prom = prom
        self.device = torch.device(device)
        self.R, self.step, self.clock = int(ring_len), float(step), clock
        self.chunk_pts = max(1, int(chunk_points))
        self.apps_per_query = max(1, int(apps_per_query))
        self.decode_threads = max(1, int(decode_threads or native.default_threads()))
        self.min_capacity = max(1, int(min_capacity))
        self.retain_s = float(retain_s)
        self.dtype = dtype or (torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        self.ring: Optional[HistoryRing] = None
        self.t_last = 0.0
        self.rows: Dict[int, int] = {}                 # history key -> row
        self.keys: List[Optional[Key]] = []            # row -> key tuple (None: free)
        self.refs: Dict[int, int] = {}
        self.last_used: Dict[int, float] = {}
        self.pending: Set[int] = set()
        self._tuples: Dict[int, Key] = {}              # key tuples of wanted keys without a row yet
        self._hash: Dict[Key, int] = {}                # tuple -> key (tuple API)
        self._idle: "collections.deque[Tuple[float, int]]" = collections.deque()  # (last use, key) of unreferenced rows
        self._stage: Dict[Tuple[int, int], List[torch.Tensor]] = {}
        self._stage_i = 0
        self._tables: Optional[Dict[Tuple[str, str], native.KeyTable]] = None
        self._fam_ids: Dict[Tuple[str, str], int] = {}
        self._row_fam = np.zeros(0, dtype=np.int64)   # row -> family id (-1: free)
        self._row_app = np.zeros(0, dtype=np.uint64)  # row -> (namespace, app) decode key
        self._free_rows: List[int] = []
        self.history_queries = 0
        self.tick_queries = 0
        self.failed_queries = 0
        self.reloads = 0
        # cold loads: at most load_budget_s of week loads per call (in batches of load_batch
        # keys), the rest stays pending for the next tick, so a node filling up with
        # thousands of new apps keeps scoring the jobs it already holds every tick
        self.load_batch = max(1, int(os.environ.get("FOREMAST_HISTORY_LOAD_BATCH", "4096")))
        env_budget = os.environ.get("FOREMAST_HISTORY_LOAD_BUDGET_S", "")
        self.load_budget_s: Optional[float] = float(env_budget) if env_budget else None
        self.load_stats = {"keys": 0, "body_bytes": 0, "fetch_s": 0.0, "decode_s": 0.0, "h2d_s": 0.0, "h2d_bytes": 0,
                           "batches": 0}

    # ------------------------------------------------------------------ references
    def key_hash(self, k: Key) -> int:
        h = self._hash.get(k)
        if h is None:
            if len(self._hash) > 1 << 20:
                self._hash.clear()
            h = self._hash[k] = history_key_hash(k)
        return h

    def want(self, keys: Iterable[Key], now: float) -> None:
        keys = list(keys)
        self.want_h([self.key_hash(k) for k in keys], now, keys.__getitem__)

    def want_h(self, hashes: Sequence[int], now: float, key_of) -> None:
        """Reference history keys; ``key_of(i)`` gives the tuple of ``hashes[i]``
        (asked only for keys without a row).  Bulk dict operations in C: a deploy
        burst references thousands of keys per tick, nearly all with rows."""
        hashes = list(hashes)
        _count_elements(self.refs, hashes)
        self.last_used.update(dict.fromkeys(hashes, now))
        rows = self.rows
        if all(map(rows.__contains__, hashes)):
            return
        for i, h in enumerate(hashes):
            if h not in rows:
                self.pending.add(h)
                if h not in self._tuples:
                    self._tuples[h] = key_of(i)

    def unwant(self, keys: Iterable[Key], now: float) -> None:
        self.unwant_h([self.key_hash(k) for k in keys], now)

    def unwant_h(self, hashes: Iterable[int], now: float) -> None:
        """Release references (bulk: counts, lookups and updates in C; Python touches
        only the keys whose last reference goes)."""
        dec: Dict[int, int] = {}
        _count_elements(dec, hashes)
        if not dec:
            return
        refs = self.refs
        keys = list(dec)
        left = (np.fromiter(map(refs.get, keys, itertools.repeat(0)), dtype=np.int64, count=len(keys))
                - np.fromiter(dec.values(), dtype=np.int64, count=len(keys)))
        keep = left > 0
        if keep.any():
            refs.update(zip(itertools.compress(keys, keep), left[keep].tolist()))
        gone = list(itertools.compress(keys, ~keep))
        collections.deque(map(refs.pop, gone, itertools.repeat(None)), maxlen=0)  # pops in C
        self._idle.extend(zip(itertools.repeat(now), gone))  # expiry candidates (checked in time order)
        self.last_used.update(dict.fromkeys(keys, now))

    def ready(self, key: Key) -> bool:
        return self.ready_h(self.key_hash(key))

    def ready_h(self, h: int) -> bool:
        return h in self.rows and h not in self.pending

    def ready_mask(self, hashes: np.ndarray) -> np.ndarray:
        """:meth:`ready_h` of every key (uint64 array) at once."""
        hs = hashes.tolist()
        # membership through map(dict.__contains__) in C (a set difference against the
        # keys view would first copy every resident key into a set)
        ok = np.fromiter(map(self.rows.__contains__, hs), dtype=bool, count=len(hs))
        if self.pending:
            ok &= ~np.fromiter(map(self.pending.__contains__, hs), dtype=bool, count=len(hs))
        return ok

    def rows_of_h(self, hashes: Sequence[int]) -> np.ndarray:
        """Rows of keys that have one (KeyError otherwise), one C-level lookup."""
        hashes = list(hashes)
        if not hashes:
            return np.zeros(0, dtype=np.int64)
        if len(hashes) == 1:
            return np.array([self.rows[hashes[0]]], dtype=np.int64)
        return np.array(operator.itemgetter(*hashes)(self.rows), dtype=np.int64)

    def row_of(self, key: Key) -> int:
        return self.rows[self.key_hash(key)]

    @property
    def n_rows(self) -> int:
        return len(self.rows)

    # ------------------------------------------------------------------ storage
    def _grow(self, capacity: int) -> None:
        new = HistoryRing(capacity, self.R, self.dtype, self.device)
        new.state.head, new.state.length = 0, self.R
        if self.ring is not None:
            n = self.ring.n
            new._store[:n].copy_(self.ring._store)
            new.state.head = self.ring.head
        old = len(self.keys)
        self.keys.extend([None] * (capacity - old))
        self._row_fam = np.concatenate([self._row_fam, np.full(capacity - old, -1, dtype=np.int64)])
        self._row_app = np.concatenate([self._row_app, np.zeros(capacity - old, dtype=np.uint64)])
        self._free_rows += list(range(capacity - 1, old - 1, -1))
        self.ring = new

    def _assign(self, now: float) -> List[Tuple[Key, int]]:
        """Free expired rows, give pending keys rows; returns the (key, row)
        pairs whose history must be (re)loaded."""
        expired = []
        while self._idle and now - self._idle[0][0] > self.retain_s:
            t, h = self._idle.popleft()
            # still unreferenced and not used again since it went idle
            if h in self.rows and h not in self.refs and self.last_used.get(h, 0.0) <= t:
                expired.append(h)
        freed = [self.rows.pop(h) for h in expired]
        for h in expired:
            self.last_used.pop(h, None)
            self.pending.discard(h)
        for row in freed:
            self.keys[row] = None
            self._free_rows.append(row)
        if freed:
            self._row_fam[freed] = -1
        if not self.pending and not expired:
            return []
        self.pending = {h for h in self.pending if h in self.refs or h in self.rows}
        new = sorted((h for h in self.pending if h not in self.rows), key=lambda h: self._tuples[h])
        need = len(self.rows) + len(new)
        if self.ring is None or need > self.ring.n:
            cap = max(self.min_capacity, self.ring.n if self.ring is not None else 1)
            while cap < need:
                cap *= 2
            self._grow(cap)
        if freed:
            idx = torch.tensor(freed, dtype=torch.long, device=self.device)
            self.ring._store.index_fill_(0, idx, float("nan"))
        if new:
            self._free_rows.sort(reverse=True)  # lowest rows first (pop from the end)
            keys = [self._tuples.pop(h) for h in new]
            rows = [self._free_rows.pop() for _ in new]
            for h, k, row in zip(new, keys, rows):
                self.keys[row] = k
                self.rows[h] = row
            fam = [self._fam_ids.setdefault((k[0], k[1]), len(self._fam_ids)) for k in keys]
            self._row_fam[rows] = fam
            self._row_app[rows] = native.key_hashes([k[2] for k in keys], [k[3] for k in keys])
        for h in [h for h in self._tuples if h not in self.refs]:
            self._tuples.pop(h)  # wanted and released before they got a row
        if expired or new:
            self._tables = None
        return sorted(((self.keys[self.rows[h]], self.rows[h]) for h in self.pending), key=lambda kr: kr[1])

    def _key_tables(self) -> Dict[Tuple[str, str], native.KeyTable]:
        """Per metric family (endpoint, metric): (namespace, app) -> row."""
        if self._tables is None:
            tabs = {}
            for fam, fid in self._fam_ids.items():
                rows = np.nonzero(self._row_fam == fid)[0]
                if len(rows):
                    tabs[fam] = native.KeyTable.indexed(self._row_app[rows], rows.astype(np.int64), "namespace", "app")
            self._tables = tabs
        return self._tables

    def _staging(self, rows: int, cols: int, reuse: bool = False) -> Tuple[torch.Tensor, np.ndarray]:
        """NaN-filled host block (pinned for the GPU).  ``reuse``: one of two
        per-shape buffers kept across ticks (a tick's H2D has completed before
        the buffer comes round again: every tick ends with a D2H sync)."""
        if reuse:
            bufs = self._stage.get((rows, cols))
            if bufs is None:
                bufs = [torch.empty((rows, cols), dtype=torch.float32) for _ in range(2)]
                if self.device.type == "cuda":
                    bufs = [b.pin_memory() for b in bufs]
                self._stage = {(rows, cols): bufs}  # one live shape: the ring's capacity
            self._stage_i ^= 1
            t = bufs[self._stage_i]
            a = t.numpy()
            a.fill(np.nan)
            return t, a
        t = torch.full((rows, cols), float("nan"), dtype=torch.float32)
        if self.device.type == "cuda":
            t = t.pin_memory()
        return t, t.numpy()

    # ------------------------------------------------------------------ sync
    async def sync(self, now: Optional[float] = None, load: bool = True) -> None:
        """Advance the ring to ``now``; with ``load``, free expired rows and load
        pending keys too (:meth:`load_pending`)."""
        now = self.clock() if now is None else now
        t_new = float(np.floor(now / self.step) * self.step)
        if self.t_last == 0.0:
            self.t_last = t_new
        elif self.rows:
            await self._advance(t_new)
        else:
            self.t_last = max(self.t_last, t_new)
        if load:
            await self.load_pending(now)

    async def load_pending(self, now: Optional[float] = None, budget_s: Optional[float] = None) -> None:
        """Free expired rows, give pending keys rows and load their week: batches of
        ``load_batch`` keys while the time budget (``budget_s`` / ``load_budget_s``,
        None: no limit) lasts; keys left over stay pending for the next call."""
        now = self.clock() if now is None else now
        if self.t_last == 0.0:
            self.t_last = float(np.floor(now / self.step) * self.step)
        todo = self._assign(now)
        budget = self.load_budget_s if budget_s is None else budget_s
        t0 = time.perf_counter()
        for i in range(0, len(todo), self.load_batch):
            await self._load(todo[i:i + self.load_batch])
            if budget is not None and time.perf_counter() - t0 >= budget:
                break

    async def _advance(self, t_new: float) -> None:
        n_new = int(round((t_new - self.t_last) / self.step))
        if n_new <= 0:
            return
        if n_new >= self.R:  # down for longer than the ring: reload every row
            self.t_last = t_new
            self.ring.state.head = 0
            self.ring._store.fill_(float("nan"))
            self.pending |= set(self.rows)
            self.reloads += 1
            return
        tables = self._key_tables()
        block_t, block = self._staging(self.ring.n, n_new, reuse=True)
        reqs, tabs = [], []
        s = self.t_last + self.step
        for fam, table in tables.items():
            for c0 in range(0, n_new, self.chunk_pts):  # catch-up after an outage: time chunks
                n = min(self.chunk_pts, n_new - c0)
                reqs.append((range_url(fam[0], fam[1], s + c0 * self.step, n, self.step), s + c0 * self.step, n, c0))
                tabs.append(table)
        self.tick_queries += len(reqs)
        ok = await fetch_decode(self.prom, reqs, tabs, block, self.step, self.decode_threads)
        if not all(ok):
            self.failed_queries += ok.count(False)
            return  # all or nothing: the next sync fetches these minutes again
        self._append(block_t, n_new)
        self.t_last = t_new

    def _append(self, block_t: torch.Tensor, n: int) -> None:
        ring = self.ring
        col = ring.head  # full ring: the oldest column is overwritten
        if self.device.type == "cuda":
            from ..ops import kernels as K
            K.ring_append(ring.data, col, block_t.to(self.device, non_blocking=True))
            ring.state.head = (ring.head + n) % self.R
        else:
            ring.append_(block_t)

    async def _load(self, todo: List[Tuple[Key, int]]) -> None:
        """The R points ending at ``t_last`` of the given rows, in (time chunk x
        app group) queries, into one pinned block; one H2D and row scatter."""
        R = self.R
        first = self.t_last - (R - 1) * self.step
        by_fam: Dict[Tuple[str, str], List[Tuple[Key, int]]] = {}
        for i, (key, _row) in enumerate(todo):
            by_fam.setdefault((key[0], key[1]), []).append((key, i))
        block_t, block = self._staging(len(todo), R)
        reqs, tabs, groups = [], [], []
        for fam, items in by_fam.items():
            for g in range(0, len(items), self.apps_per_query):
                grp = items[g:g + self.apps_per_query]
                table = native.KeyTable([((k[2], k[3]), i) for k, i in grp])
                sel = (f'{fam[1]}{{namespace=~"{re_alt({k[2] for k, _ in grp})}",'
                       f'app=~"{re_alt({k[3] for k, _ in grp})}"}}')
                for c0 in range(0, R, self.chunk_pts):
                    n = min(self.chunk_pts, R - c0)
                    reqs.append((range_url(fam[0], sel, first + c0 * self.step, n, self.step),
                                 first + c0 * self.step, n, c0))
                    tabs.append(table)
                    groups.append([k for k, _ in grp])
        self.history_queries += len(reqs)
        tm: Dict[str, float] = {}
        ok = await fetch_decode(self.prom, reqs, tabs, block, self.step, self.decode_threads, timings=tm)
        failed: Set[Key] = set()
        for good, keys in zip(ok, groups):
            if not good:
                failed.update(keys)
        self.failed_queries += ok.count(False)
        rows = torch.tensor([row for _, row in todo], dtype=torch.long)
        t0 = time.perf_counter()
        self._write_rows(rows, block_t)
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        st = self.load_stats
        st["h2d_s"] += time.perf_counter() - t0
        st["h2d_bytes"] += int(block_t.numel()) * 4
        st["keys"] += len(todo) - len(failed)
        st["body_bytes"] += int(tm.get("body_mb", 0.0) * 1e6)
        st["fetch_s"] += tm.get("fetch_ms", 0.0) / 1e3
        st["decode_s"] += tm.get("native_ms", 0.0) / 1e3
        st["batches"] += 1
        # this batch's keys are loaded, except those of a failed query (retried next call)
        self.pending -= {self.key_hash(k) for k, _row in todo if k not in failed}

    def _write_rows(self, rows: torch.Tensor, values: torch.Tensor) -> None:
        """``values [k, R]`` oldest first into the rotated ring (two column slices)."""
        ring = self.ring
        dev = self.device
        rows = rows.to(dev)
        v = values.to(dev, non_blocking=True).to(ring.data.dtype)
        head, R = ring.head, self.R
        n1 = R - head
        ring.data[:, head:].index_copy_(0, rows, v[:, :n1])
        if head:
            ring.data[:, :head].index_copy_(0, rows, v[:, n1:])

    def load_rows(self, keys: Sequence[Key], values: torch.Tensor) -> None:
        """Adopt known histories (``values [k, R]`` oldest first, ending at
        ``t_last``) for keys that already have rows — e.g. a warm node restored
        from a snapshot, or a benchmark's synthetic week — without a fetch."""
        hs = [self.key_hash(k) for k in keys]
        rows = torch.tensor([self.rows[h] for h in hs], dtype=torch.long)
        self._write_rows(rows, values)
        self.pending -= set(hs)

    async def assign_only(self, now: Optional[float] = None) -> None:
        """Give pending keys rows without loading them (then :meth:`load_rows`)."""
        now = self.clock() if now is None else now
        if self.t_last == 0.0:
            self.t_last = float(np.floor(now / self.step) * self.step)
        self._assign(now)

    # ------------------------------------------------------------------ reads
    def gather(self, rows: Sequence[int], drop_newest: int = 0) -> Tuple[torch.Tensor, int, int]:
        """Rows' histories for a batched fit: ``(hist [k, R] view of a 16-byte
        aligned block, head, length)`` where the logical window is the ring's
        minus its ``drop_newest`` newest points (a job's history ends at its
        start time, ``metricsquery.go:73-79``)."""
        ring = self.ring
        idx = torch.as_tensor(list(rows), dtype=torch.long, device=self.device)
        buf = torch.index_select(ring._store, 0, idx)
        length = max(1, self.R - max(0, int(drop_newest)))
        return buf[:, :self.R], ring.head, length

    def column_time(self) -> float:
        """Time of the newest column."""
        return self.t_last
