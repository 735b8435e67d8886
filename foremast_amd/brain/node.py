"""The node brain: one scorer process per GPU, sharded by app, joined by RCCL.

The reference scales its brain as shared-nothing replicas that only meet in
the ES job table (``docs/guides/design.md:37-41``) and promises "aggregate
service health check across multiple K8s clusters" (``README.md:27``).  Here
the brains of one node form a process group (``nccl`` = RCCL over xGMI on the
GPU, ``gloo`` on CPU):

* ownership: continuous jobs are sharded by a stable hash of (namespace, app)
  over the current members, so every app's series live on one rank and the
  per-app counters need no reduction (:func:`owner_of`);
* each tick every rank scores its own :class:`StreamingMonitor` shard, then the
  ranks exchange their per-app counters in ONE all-gather
  (:class:`~foremast_amd.parallel.cluster.ClusterHealth`); rank 0 publishes
  the node health table into the job store (``put_meta("cluster_health")``),
  which ``GET /v1/healthcheck/cluster`` serves;
* failure detection / elastic recovery: members heartbeat into
  the node's key-value store; when one goes silent (or a collective fails)
  the survivors agree on a new member list, re-form the process group
  (:class:`~foremast_amd.parallel.elastic.ElasticWorld`), hand back the
  leases of apps that moved to another rank, and take over the dead rank's
  jobs at once (``steal_from``) instead of after the 90 s stuck-job timeout.

:func:`launch_node` is the launcher (``python -m foremast_amd.brain
--streaming --nproc N``): it hosts the key-value store itself, so the store
outlives any rank, starts N rank processes and never touches the GPU.
"""

from __future__ import annotations

import asyncio
import datetime
import gc
import logging
import os
import signal
import socket
import subprocess
import sys
import time
import zlib
from typing import Dict, List, Optional, Set

import torch
import torch.distributed as dist

from ..parallel.cluster import ClusterHealth
from ..parallel.roster import NodeRoster
from ..parallel import comm
from ..parallel.elastic import ElasticWorld
from .streaming import StreamingMonitor, app_of

log = logging.getLogger("foremast.node")

META_KEY = "cluster_health"


def owner_of(namespace: str, app: str, world: int) -> int:
    """Rank index that owns an app (stable across processes and restarts)."""
    return zlib.crc32(f"{namespace}/{app}".encode()) % max(world, 1)


def worker_id_of(member: str) -> str:
    return f"node-{member}"


class NodeBrain:
    """``mon``: the continuous-job monitor; ``extra``: further resident engines
    on the same rank (the rollout monitor for canary / rollingUpdate jobs),
    all sharded by app with the same ownership function and merged into one
    per-app record for the exchange."""

    def __init__(self, mon: StreamingMonitor, world: Optional[ElasticWorld], store, device,
                 publish: bool = True, extra=()) -> None:
        self.mon = mon
        self.monitors = [mon] + [m for m in extra if m is not None]
        self.world = world
        self.store = store
        self.device = torch.device(device)
        self.health = ClusterHealth(self.device)
        self.roster = NodeRoster(len(self.monitors), self.device)
        self._mver: Dict[int, int] = {}
        self.publish = publish
        self.dead: Set[str] = set()
        self.table: Dict = {}
        self.ticks = 0
        # the full per-app table goes to the store at most every publish_every_s (and at once
        # when the anomalous set changes): GET /v1/healthcheck/cluster is polled like barrelman's 10 s
        self.publish_every_s = float(os.environ.get("FOREMAST_PUBLISH_EVERY_S", "10"))
        self._published = -1e18
        self._last_anomalous = None
        self.gc_freeze_min = int(os.environ.get("FOREMAST_GC_FREEZE_MIN", "256"))
        self.gc_full_every_s = float(os.environ.get("FOREMAST_GC_FULL_EVERY_S", "600"))
        self._full_gc_at = time.monotonic()
        self._admitted_since = 0
        # young-generation threshold: a tick allocates ~10^5 short-lived objects (decoded
        # rows, query strings); the default 700 runs ~150 young collections per tick
        t0 = int(os.environ.get("FOREMAST_GC_THRESHOLD0", "50000"))
        if t0 > 0:
            th = gc.get_threshold()
            gc.set_threshold(max(th[0], t0), th[1], th[2])
        self.timings: Dict[str, float] = {}
        self._frozen_at = 0
        for m in self.monitors:
            m.owns = self._owns_for(m)

    @property
    def rank(self) -> int:
        return self.world.rank if self.world is not None else 0

    @property
    def size(self) -> int:
        return self.world.world if self.world is not None else 1

    def owns(self, doc) -> bool:
        ns, app = app_of(doc)
        return owner_of(ns, app, self.size) == self.rank

    def _owns_for(self, m):
        """Ownership a monitor claims by: by app, or — a rollout monitor in
        cluster-affine mode — by the cluster of the job's new pods."""
        return m.owns_affine if getattr(m, "router", None) is not None else self.owns

    def _suffixes(self) -> Set[str]:
        """Worker-id suffixes of this rank's monitors (``node-<member>`` + "", "-rollout",
        "-lstm"): a dead member's leases are held under each of them."""
        base = worker_id_of(self.world.id) if self.world is not None else ""
        out = {""}
        for m in self.monitors:
            wid = getattr(m, "worker_id", "")
            if base and wid.startswith(base):
                out.add(wid[len(base):])
        return out

    def _after_reform(self, before: List[str]) -> None:
        """The node re-formed: dead members' leases become stealable, jobs whose owner
        moved are released, per-generation stores are reset, and the monitors' re-formation
        collectives (the LSTM replicas adopt rank 0's weights, RC4) run under the world's
        deadline-and-re-form guard — a member lost during them re-forms the node again,
        and this repeats over the newer membership."""
        gen = None
        while gen != self.world.generation:
            gen = self.world.generation
            members = list(self.world.members)
            gone = set(before) - set(members)
            self.dead |= {worker_id_of(m) + sfx for m in gone for sfx in self._suffixes()}
            moved = sum(m.release(lambda d, o=self._owns_for(m): not o(d)) for m in self.monitors)
            for m in self.monitors:
                if getattr(m, "router", None) is not None:
                    m.router.reset(kv=dist.PrefixStore("affine", self.world.pstore))
            self.health.reset(kv=self.world.pstore)
            log.warning("node re-formed: generation %d, members %s (lost %s); released %d moved jobs",
                        self.world.generation, members, sorted(gone), moved)
            self.world.run_tick(self._reform_collectives)
            before = members

    def _reform_collectives(self) -> None:
        for m in self.monitors:
            if hasattr(m, "after_reform"):
                m.after_reform()

    def app_table(self):
        """(node app roster, ``[A, 2]`` device counters, roster version, live series)
        of every monitor of this rank, merged per app.  The merged roster is kept
        from the monitors' change logs (:class:`~foremast_amd.parallel.roster.NodeRoster`):
        O(apps that changed) per tick, one ``index_add_`` per monitor on the device."""
        engines, tables = [], []
        for k, m in enumerate(self.monitors):
            log = getattr(m, "roster_log", None)
            if log is not None:
                reset, items = log.drain()
            else:  # a monitor without a change log: re-read its table when its version moves
                v = getattr(m, "roster_version", 0)
                reset, items = v != self._mver.get(k), []
                self._mver[k] = v
            apps = getattr(m, "apps", None)
            n_apps = len(apps) if isinstance(apps, dict) else None
            if hasattr(m, "app_counts"):
                tables.append(m.app_counts())
                engines.append((reset, items, m.roster_names, n_apps))
            else:
                names, c = m.app_table()
                tables.append(c)
                engines.append((reset, items, lambda names=names: names, n_apps))
        self.roster.update(engines)
        counts = self.roster.counts(tables)
        return self.roster.names, counts, self.roster.version, sum(m.n_live for m in self.monitors)

    def _exchange(self) -> Dict:
        names, counts, version, n_live = self.app_table()
        info = {"member": self.world.id if self.world else "m0", "pid": os.getpid()}
        for m in self.monitors:
            if hasattr(m, "model_digest"):
                info["lstm_model"] = m.model_digest()
        return self.health.exchange(names, counts, version, n_live, info, changes=self.roster.log.drain())

    def _freeze_admitted(self) -> None:
        """Admission builds long-lived per-job state (plans, slot maps, documents):
        after an intake of ``gc_freeze_min`` jobs, ``gc.freeze()`` moves everything
        alive into the permanent generation (O(1)), so the generational collections
        of the following ticks no longer walk the admitted jobs' objects (a 100+ ms
        gen-2 pause in a ~9 ms tick at 10k jobs otherwise).  Frozen objects are
        still freed by reference counting when their jobs finish; what only the
        cycle collector could reclaim is reclaimed by a full collection every
        ``gc_full_every_s`` (default 10 min), off the steady ticks' path."""
        self._admitted_since += sum(getattr(m, "timings", {}).get("admitted", 0) or 0 for m in self.monitors
                                    if hasattr(m, "intake"))
        n = sum(len(getattr(m, "jobs", ())) for m in self.monitors)
        now = time.monotonic()
        if now - self._full_gc_at >= self.gc_full_every_s:
            gc.unfreeze()
            gc.collect()
            gc.freeze()
            self._full_gc_at = now
            self._frozen_at, self._admitted_since = n, 0
        elif n - self._frozen_at >= self.gc_freeze_min or self._admitted_since >= self.gc_freeze_min:
            gc.freeze()
            self._frozen_at, self._admitted_since = n, 0
        elif n < self._frozen_at:
            self._frozen_at = n  # jobs finished: the next intake of the same size freezes again

    async def tick(self) -> Dict:
        """One node tick: every monitor scores its running jobs, the ranks exchange
        the node health table — the verdicts are out (``timings["detect_ms"]``) —
        then the monitors that split their tick (:meth:`RolloutMonitor.intake`)
        claim and admit new jobs (``timings["intake_ms"]``): a deploy burst never
        delays the verdicts of the jobs already running."""
        t0 = time.perf_counter()
        split = []
        for m in self.monitors:
            try:
                if hasattr(m, "intake"):
                    split.append(m)
                    await m.score_tick()
                else:
                    await m.tick()
            except Exception as e:  # noqa: BLE001 - a scoring failure must not desynchronise the collectives
                log.exception("%s tick failed: %s", type(m).__name__, e)
        if self.world is None:
            table = self._exchange()
        else:
            before, gen = list(self.world.members), self.world.generation
            table = self.world.run_tick(self._exchange)
            if self.world.generation != gen:
                self._after_reform(before)
        t1 = time.perf_counter()
        # claims are intake: a monitor's new jobs are leased after the verdicts are out (a
        # claim scans the store's open documents, e.g. a burst of another monitor's jobs)
        # and admitted by its next tick
        for m in self.monitors:
            if m not in split:
                try:
                    m.sync(steal_from=self.dead or None)
                except Exception as e:  # noqa: BLE001 - the store may be briefly unavailable
                    log.exception("%s claim failed: %s", type(m).__name__, e)
        for m in split:
            try:
                m.sync(steal_from=self.dead or None)
            except Exception as e:  # noqa: BLE001 - the store may be briefly unavailable
                log.exception("%s claim failed: %s", type(m).__name__, e)
            try:
                await m.intake()  # every rank, every tick: it may run the lockstep window exchange
            except Exception as e:  # noqa: BLE001 - e.g. the job store is briefly unavailable
                log.exception("%s intake failed: %s", type(m).__name__, e)
        self._freeze_admitted()
        self.timings = {"detect_ms": (t1 - t0) * 1e3, "intake_ms": (time.perf_counter() - t1) * 1e3}
        table["generation"] = self.world.generation if self.world else 0
        table["backend"] = dist.get_backend() if dist.is_available() and dist.is_initialized() else "none"
        table["collectives"] = comm.active()
        self.table = table
        self.ticks += 1
        now = time.monotonic()
        shape = (table["ranks"], table["generation"], table["anomalous_apps"])
        if self.publish and self.rank == 0 and (now - self._published >= self.publish_every_s
                                                 or shape != self._last_anomalous):
            try:
                self.store.put_meta(META_KEY, table.full() if hasattr(table, "full") else table)
                self._published, self._last_anomalous = now, shape
            except Exception as e:  # noqa: BLE001 - the store may be briefly unavailable
                log.warning("publishing the node health table failed: %s", e)
        return table

    def start(self) -> None:
        """Join the node: form the elastic world's process group (a no-op if it is
        formed), point the health exchange and the affine router at the
        generation's key-value store, start heartbeating.  Every rank of a
        multi-GPU node runs this once before its first tick (``run_forever``, and
        the node benches under ``torch.distributed.run``)."""
        if self.world is None:
            return
        if not dist.is_initialized():
            self.world.form()
        self.health.reset(kv=self.world.pstore)
        for m in self.monitors:
            if getattr(m, "router", None) is not None:
                m.router.reset(kv=dist.PrefixStore("affine", self.world.pstore))
        self.world.start_heartbeat()

    def stop(self) -> None:
        if self.world is not None:
            self.world.stop_heartbeat()

    async def run_forever(self, stop: asyncio.Event, period: float) -> None:
        self.start()
        try:
            while not stop.is_set():
                t0 = time.monotonic()
                await self.tick()
                try:
                    await asyncio.wait_for(stop.wait(), timeout=max(0.0, period - (time.monotonic() - t0)))
                except asyncio.TimeoutError:
                    pass
        finally:
            self.stop()


def elastic_world_from_env(device: torch.device, force: bool = False) -> Optional[ElasticWorld]:
    """The rank's ElasticWorld: under :func:`launch_node` (``FOREMAST_NODE_STORE``)
    or under torchrun (``WORLD_SIZE`` > 1: the agent's store at MASTER_ADDR:PORT);
    None for a single brain process — unless ``force`` (``FOREMAST_FORCE_COLLECTIVES=1``
    runs: a 1-member world on a store this process hosts, so one GPU exercises
    the deployed RCCL exchange, its deadlines and its re-formation)."""
    hb = float(os.environ.get("FOREMAST_HEARTBEAT_S", "5"))
    backend = os.environ.get("FOREMAST_DIST_BACKEND", "nccl" if device.type == "cuda" else "gloo")
    # RCCL aborts a wedged communicator at once (ncclCommAbort); gloo's teardown waits for
    # in-flight work until the group timeout, so a gloo node bounds it near the heartbeat
    coll = float(os.environ.get("FOREMAST_COLLECTIVE_TIMEOUT_S", "60" if backend == "nccl" else str(2 * hb)))
    if os.environ.get("FOREMAST_NODE_STORE"):
        host, port = os.environ["FOREMAST_NODE_STORE"].rsplit(":", 1)
        n = int(os.environ["FOREMAST_NODE_MEMBERS"])
        me = int(os.environ["FOREMAST_NODE_MEMBER"])
    elif int(os.environ.get("WORLD_SIZE", "1")) > 1:
        host, port = os.environ.get("MASTER_ADDR", "127.0.0.1"), os.environ["MASTER_PORT"]
        n, me = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    elif force:
        kv = dist.TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False,
                           timeout=datetime.timedelta(seconds=60))
        return ElasticWorld(kv, "m0", ["m0"], backend=backend, heartbeat_timeout_s=hb, collective_timeout_s=coll,
                            device_id=device if backend == "nccl" else None)
    else:
        return None
    kv = dist.TCPStore(host, int(port), is_master=False, timeout=datetime.timedelta(seconds=60))
    return ElasticWorld(kv, f"m{me}", [f"m{i}" for i in range(n)], backend=backend, heartbeat_timeout_s=hb,
                        collective_timeout_s=coll, device_id=device if backend == "nccl" else None)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_node(nproc: int, argv: List[str]) -> int:
    """Start ``nproc`` brain ranks (``python -m foremast_amd.brain <argv>``) around a
    key-value store this process hosts.  A rank that dies is not restarted: the
    survivors re-shard its apps.  Returns when every rank has exited (SIGTERM /
    SIGINT are forwarded); the exit code is 0 if any rank exited cleanly."""
    port = _free_port()
    kv = dist.TCPStore("127.0.0.1", port, is_master=True, wait_for_workers=False,
                       timeout=datetime.timedelta(seconds=60))
    procs = []
    for i in range(nproc):
        env = dict(os.environ, FOREMAST_NODE_STORE=f"127.0.0.1:{port}", FOREMAST_NODE_MEMBERS=str(nproc),
                   FOREMAST_NODE_MEMBER=str(i), LOCAL_RANK=str(i), HSA_ENABLE_IPC_MODE_LEGACY="0")
        env.pop("WORLD_SIZE", None)
        procs.append(subprocess.Popen([sys.executable, "-m", "foremast_amd.brain"] + argv, env=env))
    kv.set("launcher/pids", ",".join(str(p.pid) for p in procs))

    def forward(sig, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)
    old = {s: signal.signal(s, forward) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        codes = [p.wait() for p in procs]
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    del kv
    return 0 if any(c == 0 for c in codes) else (codes[0] or 1)
