"""Failure detection and elastic recovery for the per-GPU scorer ranks.

The reference scales brains as shared-nothing replicas coordinated only by
job-table leases (``docs/guides/design.md:37-41``).  The MI355X engine shards
series over one process per GPU joined by RCCL, so a dead rank must not take
the node's scoring down (SURVEY §5.3 "New build"):

* every member (stable id, independent of its current rank) heartbeats into a
  key-value store (the torchrun rendezvous TCPStore, or any ``c10d.Store``);
* before each tick — and whenever a collective fails or times out — members
  check heartbeat freshness;
* on a membership change the survivors agree on ONE new member list: the
  first ``compare_set`` on the generation's key wins, everyone adopts it;
* the process group's communicators are ABORTED (``ncclCommAbort`` through
  ``_abort_process_group``: a wedged RCCL communicator cannot hang the
  teardown), destroyed and re-created over the survivors under a
  generation-prefixed store, and the caller re-shards its series with the new
  (rank, world);
* under RCCL the watchdog is told to abort communicators without killing the
  process (``TORCH_NCCL_ASYNC_ERROR_HANDLING=2``, CleanUpOnly) and the per-tick
  exchange waits on the host with a deadline (``comm.wait_bounded``), so a peer
  that dies or stops mid-collective surfaces as an exception in the survivors.

Works with ``gloo`` (CPU tests) and ``nccl`` (= RCCL on ROCm).
"""

from __future__ import annotations

import datetime
import json
import os
import threading
import time
from typing import Callable, List, Optional, Sequence

import torch.distributed as dist


class ElasticWorld:
    def __init__(self, store, member_id: str, members: Sequence[str], backend: str = "gloo",
                 heartbeat_timeout_s: float = 5.0, collective_timeout_s: float = 30.0,
                 device_id=None, heartbeat_store=None) -> None:
        self.store = store
        # A TCPStore client is one socket: a heartbeat thread sharing it would
        # queue behind the main thread's blocking rendezvous reads and look
        # dead.  Heartbeats get their own connection.
        if heartbeat_store is None and hasattr(store, "host") and hasattr(store, "port"):
            heartbeat_store = dist.TCPStore(store.host, store.port, is_master=False,
                                            timeout=datetime.timedelta(seconds=30))
        self.hb_store = heartbeat_store if heartbeat_store is not None else store
        self.id = member_id
        self.members: List[str] = sorted(members)
        self.backend = backend
        self.hb_timeout = heartbeat_timeout_s
        self.coll_timeout = datetime.timedelta(seconds=collective_timeout_s)
        self.device_id = device_id
        self.generation = 0
        self.pstore = None
        self.rank = -1
        self.world = 0
        self.reforms = 0

    # ------------------------------------------------------------------ heartbeats
    def beat(self, store=None) -> None:
        (store or self.store).set(f"hb/{self.id}", repr(time.time()))

    def start_heartbeat(self, period_s: Optional[float] = None) -> threading.Thread:
        """Background heartbeat (keeps beating while the rank is inside a
        long kernel or a blocked collective)."""
        period = period_s if period_s is not None else self.hb_timeout / 4
        self._hb_stop = threading.Event()
        self._hb_dead = threading.Event()
        # a transient store error must not silence a healthy rank: retry on the next
        # period; only after errors spanning a whole heartbeat timeout does the thread
        # give up, and then it says so (changed() beats on the main thread instead)
        give_up_after = max(3, int(self.hb_timeout / max(period, 1e-3)) + 1)

        def loop():
            fails = 0
            while not self._hb_stop.wait(period):
                try:
                    self.beat(self.hb_store)
                    fails = 0
                except Exception:  # noqa: BLE001 - store hiccup: retry next period
                    fails += 1
                    if fails >= give_up_after:
                        self._hb_dead.set()
                        return

        self.beat()
        th = threading.Thread(target=loop, daemon=True, name=f"heartbeat-{self.id}")
        th.start()
        return th

    def stop_heartbeat(self) -> None:
        ev = getattr(self, "_hb_stop", None)
        if ev is not None:
            ev.set()

    def last_beat(self, member: str) -> float:
        key = f"hb/{member}"
        try:
            if not self.store.check([key]):
                return 0.0
            return float(self.store.get(key).decode())
        except Exception:  # noqa: BLE001 - store hiccup counts as stale
            return 0.0

    def _beats(self, members: Sequence[str]) -> List[float]:
        """Last beat of each member in two store round trips (an existence check of
        every key, then one multi-get) instead of two per member: the check runs
        before every tick."""
        keys = [f"hb/{m}" for m in members]
        try:
            if keys and hasattr(self.store, "multi_get") and self.store.check(keys):
                return [float(v.decode() if isinstance(v, (bytes, bytearray)) else bytes(v).decode())
                        for v in self.store.multi_get(keys)]
        except Exception:  # noqa: BLE001 - fall back to one member at a time
            pass
        return [self.last_beat(m) for m in members]

    def live(self, now: Optional[float] = None) -> List[str]:
        now = time.time() if now is None else now
        others = [m for m in self.members if m != self.id]
        beats = dict(zip(others, self._beats(others)))
        return [m for m in self.members if m == self.id or now - beats[m] <= self.hb_timeout]

    # ------------------------------------------------------------------ group management
    def _agree(self, proposal: List[str]) -> List[str]:
        key = f"gen/{self.generation}/members"
        want = json.dumps(sorted(proposal)).encode()
        got = self.store.compare_set(key, b"", want)  # first proposer wins
        if got in (b"", None):
            got = self.store.get(key)
        return json.loads(got.decode() if isinstance(got, (bytes, bytearray)) else got)

    def form(self) -> None:
        """(Re)create the process group over the agreed members of this
        generation.  Generation 0 is the configured member list (start-up waits
        for everyone, like a rendezvous); later generations use liveness."""
        members = self._agree(self.members if self.generation == 0 else self.live())
        if self.id not in members:
            raise RuntimeError(f"{self.id} was voted out of generation {self.generation}")
        self.members = members
        self.rank = members.index(self.id)
        self.world = len(members)
        pstore = dist.PrefixStore(f"pg/{self.generation}", self.store)
        self.pstore = dist.PrefixStore(f"kv/{self.generation}", self.store)  # per-generation records (rosters)
        kw = {}
        if self.device_id is not None:
            kw["device_id"] = self.device_id
        if self.backend == "nccl":
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")  # abort comms, keep the process
        # beat before the group's rendezvous: once any member is past it, every member has a
        # fresh beat (a peer still between form() and start_heartbeat() must not look dead)
        self.beat()
        dist.init_process_group(self.backend, store=pstore, rank=self.rank, world_size=self.world,
                                timeout=self.coll_timeout, **kw)

    def changed(self) -> bool:
        if (getattr(self, "_hb_stop", None) is None or self._hb_stop.is_set()
                or self._hb_dead.is_set()):
            self.beat()  # no (live) heartbeat thread: this call is the beat
        return len(self.live()) != len(self.members)

    def reform(self, settle_s: float = 0.0) -> None:
        """Tear the group down and re-form it over the live members."""
        if dist.is_initialized():
            try:  # abort first: destroying a communicator with a collective in flight can block
                from torch.distributed.distributed_c10d import _abort_process_group
                _abort_process_group()
            except Exception:  # noqa: BLE001 - backends without abort (gloo) fall through to destroy
                pass
            if dist.is_initialized():
                try:
                    dist.destroy_process_group()
                except Exception:  # noqa: BLE001 - a broken communicator may fail to close cleanly
                    pass
        if settle_s:
            time.sleep(settle_s)
        self.beat()
        self.generation += 1
        self.reforms += 1
        self.form()

    def run_tick(self, fn: Callable[[], object], max_attempts: int = 3):
        """Run one tick's collective work; on failure or membership change,
        re-form and retry (the caller's ``fn`` must re-read rank/world)."""
        last: Optional[BaseException] = None
        for _attempt in range(max_attempts):
            if self.changed():
                self.reform()
            try:
                return fn()
            except (RuntimeError, dist.DistBackendError) as e:  # peer died mid-collective
                last = e
                # wait until the dead peer's heartbeat is stale, then re-form
                t_end = time.time() + self.hb_timeout * 2
                while time.time() < t_end and not self.changed():
                    time.sleep(self.hb_timeout / 10)
                self.reform()
        raise RuntimeError(f"tick failed after {max_attempts} re-formations: {last}")
