"""App rosters of the node health exchange, kept incrementally.

Each resident engine of a rank (streaming, rollout, LSTM monitors) holds its
apps at stable indices of an app table whose ``[A, 2]`` device counters it
fills every tick.  The node health table needs the rank's apps merged into ONE
table (an app can have series in two engines) and every peer's roster.  Under
a steady deployment stream the roster changes every tick, so both are kept as
change logs, never rebuilt:

* :class:`ChangeLog` — an engine records ``(index, name or None)`` whenever a
  slot of its app table is set or freed; a consumer drains it once per tick.
  An engine that renumbers its table (or a log that grew past its bound without
  a consumer) marks a reset: the consumer then re-reads the whole table once.
* :class:`NodeRoster` — the rank's merged table.  While at most one engine
  holds apps (a rollout-only or continuous-only node, the common case) it IS
  that engine's table: same indices, the engine's changes forwarded as they
  are, its counters used as they are — no per-change work at all.  When a
  second engine holds apps it switches to a merged table: node index per app
  with a reference count over the engines, an index map per engine (engine
  index → node index) mirrored on the device, so the merged counters are one
  ``index_add_`` per engine.  Either way its change log feeds the exchange's
  roster deltas (:class:`~foremast_amd.parallel.cluster.ClusterHealth`), so the
  host work per tick is O(apps that changed), not O(apps).

The reference brain has no such table; it is what "aggregate service health
check across multiple K8s clusters" (``/root/reference/README.md:27``) needs
on a node whose ranks own disjoint apps (``docs/guides/design.md:37-41``).
"""

from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

Name = Tuple[str, str]


class ChangeLog:
    """``(index, name-or-None)`` changes of an app table since the last drain."""

    LIMIT = 1 << 16

    def __init__(self) -> None:
        self.items: List[Tuple[int, Optional[Name]]] = []
        self.reset = True       # a fresh table: the consumer reads it whole once

    def note(self, i: int, name: Optional[Name]) -> None:
        if self.reset:
            return
        self.items.append((int(i), name))
        if len(self.items) > self.LIMIT:   # nobody drains: stop logging, resync on the next drain
            self.mark_reset()

    def note_many(self, items: Iterable[Tuple[int, Optional[Name]]]) -> None:
        if not self.reset:
            self.items.extend(items)
            if len(self.items) > self.LIMIT:
                self.mark_reset()

    def mark_reset(self) -> None:
        self.items = []
        self.reset = True

    def drain(self) -> Tuple[bool, List[Tuple[int, Optional[Name]]]]:
        out = (self.reset, self.items)
        self.items, self.reset = [], False
        return out


class NodeRoster:
    """The rank's merged app table over its engines (stable node indices)."""

    def __init__(self, n_engines: int, device) -> None:
        self.device = torch.device(device)
        self.names: List[Optional[Name]] = []
        self.index: Dict[Name, int] = {}
        self.refs: Dict[Name, int] = {}
        self.free: List[int] = []
        self.maps = [np.zeros(0, dtype=np.int64) for _ in range(n_engines)]
        self._dev_maps: List[Optional[torch.Tensor]] = [None] * n_engines
        self.log = ChangeLog()
        self.version = 0
        self.n_apps = 0
        self._changes = 0
        self.mode: Optional[Tuple[str, int]] = None   # ("pass", engine) or ("merged", -1)

    # ------------------------------------------------------------------ node index refcounts
    def _ref(self, name: Name) -> int:
        i = self.index.get(name)
        if i is None:
            i = self.free.pop() if self.free else len(self.names)
            if i == len(self.names):
                self.names.append(name)
            else:
                self.names[i] = name
            self.index[name] = i
            self.refs[name] = 0
            self.log.note(i, name)
            self.n_apps += 1
            self._changes += 1
        self.refs[name] += 1
        return i

    def _unref(self, i: int) -> None:
        name = self.names[i]
        if name is None:
            return
        n = self.refs[name] - 1
        if n > 0:
            self.refs[name] = n
            return
        del self.refs[name], self.index[name]
        self.names[i] = None
        self.free.append(i)
        self.log.note(i, None)
        self.n_apps -= 1
        self._changes += 1

    def _set(self, k: int, i: int, name: Optional[Name]) -> None:
        m = self.maps[k]
        if i >= len(m):
            grow = max(i + 1, 2 * len(m), 64) - len(m)
            m = self.maps[k] = np.concatenate([m, np.full(grow, -1, dtype=np.int64)])
        old = int(m[i])
        if old >= 0:
            if name is not None and self.names[old] == name:
                return
            self._unref(old)
        m[i] = self._ref(name) if name is not None else -1

    # ------------------------------------------------------------------ per tick
    def _clear(self) -> None:
        self.names = []
        self.index, self.refs, self.free = {}, {}, []
        self.maps = [np.zeros(0, dtype=np.int64) for _ in self.maps]
        self._dev_maps = [None] * len(self.maps)
        self.n_apps = 0

    def update(self, engines: Sequence[Tuple[bool, List[Tuple[int, Optional[Name]]], object, Optional[int]]]) -> bool:
        """Apply each engine's drained change log ``(reset, items, names, n_apps)``
        (``names``: a callable returning the engine's current table, called only
        when needed; ``n_apps``: its app count, None if unknown); returns whether
        the node roster changed."""
        active = [k for k, e in enumerate(engines) if e[3] is None or e[3] > 0]
        if len(active) <= 1:  # one engine holds every app: its table is the node's
            k = active[0] if active else 0
            reset, items, names_fn, n = engines[k]
            changed = False
            if self.mode != ("pass", k):
                self._clear()
                self.mode = ("pass", k)
                self.log.mark_reset()
                changed = True
                reset = True
            self.n_apps = int(n or 0)
            # the node's names are this rank's OWN list, as of this exchange: the engine
            # frees and reuses indices in place later in the tick (intake), so aliasing its
            # list would pair this tick's counters with the next tick's names
            if reset:
                self.names = list(names_fn())
                self.log.mark_reset()
                changed = True
            elif items:
                names = self.names
                for i, nm in items:
                    if i >= len(names):
                        names.extend([None] * (i + 1 - len(names)))
                    names[i] = nm
                self.log.note_many(items)
                changed = True
            if changed:
                self.version += 1
            return changed
        c0 = self._changes
        if self.mode != ("merged", -1):  # rebuild from every engine's whole table
            self._clear()
            self.mode = ("merged", -1)
            self.log.mark_reset()
            self._changes += 1
            engines = [(True, [], names_fn, n) for _r, _i, names_fn, n in engines]
        for k, (reset, items, names_fn, _n) in enumerate(engines):
            if reset:
                m = self.maps[k]
                for i in np.flatnonzero(m >= 0).tolist():
                    self._unref(int(m[i]))
                names = names_fn()
                self.maps[k] = np.full(max(64, len(names)), -1, dtype=np.int64)
                for i, nm in enumerate(names):
                    if nm is not None:
                        self.maps[k][i] = self._ref(nm)
                self._dev_maps[k] = None
            elif items:
                for i, nm in items:
                    self._set(k, i, nm)
                self._dev_maps[k] = None
        changed = self._changes != c0
        if changed:
            self.version += 1
        return changed

    def counts(self, tables: Sequence[torch.Tensor]) -> torch.Tensor:
        """``[A, 2]`` int32 node counters from each engine's ``[A_k, 2]`` counters."""
        A = len(self.names)
        if self.mode is not None and self.mode[0] == "pass":
            c = tables[self.mode[1]]
            return c[:A]
        out = torch.zeros((max(A, 1), 2), dtype=torch.int32, device=self.device)
        for k, c in enumerate(tables):
            m = self.maps[k]
            n = min(len(m), c.shape[0])
            if not n or not (m[:n] >= 0).any():
                continue
            dm = self._dev_maps[k]
            if dm is None or dm[0] != n:
                sel = np.flatnonzero(m[:n] >= 0)
                dm = self._dev_maps[k] = (n, torch.from_numpy(sel).to(self.device),
                                          torch.from_numpy(m[sel]).to(self.device))
            _, src, dst = dm
            out.index_add_(0, dst, c[:n].index_select(0, src).to(device=self.device, dtype=torch.int32))
        return out[:A] if A else out[:0]
