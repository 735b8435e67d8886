"""Barrelman: Deployment watcher, job launcher and status poller.

Behaviour follows ``foremast-barrelman/pkg/controller/Barrelman.go``; Go
goroutines become asyncio tasks and client-go informers become
``KubeAPI.watch`` streams.  Reference quirks fixed here:

* Q9  — no loop-variable capture: every task gets its own copy;
* Q10 — deleting a Deployment (with ``aca=true``) deletes its
        DeploymentMonitor, not the DeploymentMetadata;
* Q15 — the poller lists monitors cluster-wide instead of per namespace;
* Q17 — the canary path passes the ``canary`` strategy (the reference passes
        ``rollingUpdate``, so canaries never got a baseline query);
* Q18 — a monitor whose ``waitUntil`` passed is persisted as Healthy+expired
        even when the analyst still says in-progress (the reference only
        persisted status changes);
* updates use ``resourceVersion`` with one re-read on conflict (no lost
  updates between the poller and the MonitorController).
"""

from __future__ import annotations

import asyncio
import copy
import logging
import os
import time
from typing import Any, Awaitable, Callable, Dict, List, Optional, Tuple

from ..api import crd
from ..api import rest as r
from ..api import status as st
from ..k8s.api import ApiError, Conflict, KubeAPI, NotFound, Obj, revision_of
from ..utils.timeutil import format_rfc3339, parse_rfc3339
from .analyst import AnalystClient, AnalystError

log = logging.getLogger("foremast.barrelman")

WATCH_TIME_MIN = 10       # Barrelman.go:52
WAIT_UNTIL_MAX_MIN = 30   # Barrelman.go:54
POLL_SECONDS = 10.0       # Barrelman.go:467
CONTINUOUS_COOLDOWN = 60  # Barrelman.go:579
NAMESPACE_BLACKLIST = ("kube-public", "kube-system", "opa", "monitoring")  # Barrelman.go:93-98


class TTLCache:
    def __init__(self, ttl: float, clock: Callable[[], float]) -> None:
        self.ttl = ttl
        self.clock = clock
        self._d: Dict[str, Tuple[float, Any]] = {}

    def get(self, key: str):
        v = self._d.get(key)
        if v is None:
            return None, False
        if self.clock() - v[0] > self.ttl:
            self._d.pop(key, None)
            return None, False
        return v[1], True

    def set(self, key: str, value: Any) -> None:
        self._d[key] = (self.clock(), value)

    def clear(self) -> None:
        self._d.clear()


def _containers(depl: Obj) -> List[Obj]:
    return ((depl.get("spec") or {}).get("template") or {}).get("spec", {}).get("containers", []) or []


def _env_equal(a: List[Obj], b: List[Obj]) -> bool:
    if len(a or []) != len(b or []):
        return False
    return all(x.get("name") == y.get("name") and x.get("value") == y.get("value") for x, y in zip(a or [], b or []))


class Barrelman:
    def __init__(self, kube: KubeAPI, namespace: Optional[str] = None,
                 clock: Callable[[], float] = time.time,
                 sleep: Callable[[float], Awaitable[None]] = asyncio.sleep,
                 analyst_factory: Optional[Callable[[str], AnalystClient]] = None,
                 poll_seconds: float = POLL_SECONDS, pod_retry_sleep: float = 5.0,
                 watch_time_min: int = WATCH_TIME_MIN, wait_until_min: int = WAIT_UNTIL_MAX_MIN) -> None:
        self.kube = kube
        self.namespace = namespace if namespace is not None else os.environ.get("NAMESPACE", "")
        self.clock = clock
        self.sleep = sleep
        self.analyst_factory = analyst_factory or (lambda ep: AnalystClient(ep))
        self.poll_seconds = poll_seconds
        self.pod_retry_sleep = pod_retry_sleep
        self.watch_time = watch_time_min
        self.wait_until = wait_until_min
        self.ns_cache = TTLCache(300, clock)
        self.md_cache = TTLCache(60, clock)
        self.tasks: set = set()
        self.events: List[Dict[str, str]] = []

    # ------------------------------------------------------------------ helpers
    def spawn(self, coro) -> asyncio.Task:
        t = asyncio.ensure_future(coro)
        self.tasks.add(t)
        t.add_done_callback(self.tasks.discard)
        return t

    async def drain(self) -> None:
        while self.tasks:
            await asyncio.gather(*list(self.tasks), return_exceptions=True)

    async def record_event(self, obj: Obj, reason: str, message: str, etype: str = "Normal") -> None:
        md = obj.get("metadata", {})
        ev = {"metadata": {"generateName": md.get("name", "x") + ".", "namespace": md.get("namespace", "default")},
              "involvedObject": {"kind": obj.get("kind", ""), "name": md.get("name", ""),
                                 "namespace": md.get("namespace", ""), "uid": md.get("uid", "")},
              "reason": reason, "message": message, "type": etype, "source": {"component": "barrelman"},
              "lastTimestamp": format_rfc3339(self.clock())}
        self.events.append({"reason": reason, "message": message, "name": md.get("name", "")})
        try:
            await self.kube.create("events", ev)
        except ApiError:
            pass

    async def is_monitoring(self, namespace: str) -> bool:
        """``isMonitoring`` (Barrelman.go:477-494)."""
        if namespace in NAMESPACE_BLACKLIST:
            return False
        cached, found = self.ns_cache.get(namespace)
        if found:
            return bool(cached)
        try:
            ns = await self.kube.get("namespaces", "", namespace)
        except ApiError:
            return False
        result = ((ns.get("metadata") or {}).get("annotations") or {}).get(crd.ANNOTATION_MONITORING) != "false"
        self.ns_cache.set(namespace, result)
        return result

    async def get_metadata(self, namespace: str, app: str, depl: Obj) -> Optional[crd.DeploymentMetadata]:
        """app name → appType label → ``$NAMESPACE`` (Barrelman.go:139-174)."""
        key = namespace + ":" + app
        cached, found = self.md_cache.get(key)
        if found:
            return cached
        result = None
        for ns, name in ((namespace, app),):
            try:
                result = crd.DeploymentMetadata.from_dict(await self.kube.get("deploymentmetadatas", ns, name))
            except ApiError:
                result = None
        if result is None:
            app_type = ((depl.get("metadata") or {}).get("labels") or {}).get("appType")
            if app_type:
                for ns in (namespace, self.namespace):
                    if not ns:
                        continue
                    try:
                        result = crd.DeploymentMetadata.from_dict(
                            await self.kube.get("deploymentmetadatas", ns, app_type))
                        break
                    except ApiError:
                        result = None
        self.md_cache.set(key, result)
        return result

    async def _get_monitor(self, namespace: str, name: str) -> Optional[crd.DeploymentMonitor]:
        try:
            return crd.DeploymentMonitor.from_dict(await self.kube.get("deploymentmonitors", namespace, name))
        except NotFound:
            return None

    async def save_monitor(self, mon: crd.DeploymentMonitor, create: bool,
                           mutate: Optional[Callable[[crd.DeploymentMonitor], None]] = None) -> Optional[Obj]:
        """Create or update; on a resourceVersion conflict re-read, re-apply
        ``mutate`` and retry once."""
        try:
            if create:
                try:
                    return await self.kube.create("deploymentmonitors", mon.to_dict())
                except ApiError as e:
                    if e.reason != "AlreadyExists":
                        raise
                    cur = await self._get_monitor(mon.namespace, mon.name)
                    if cur is None:
                        raise
                    mon.metadata["resourceVersion"] = cur.resource_version
            return await self.kube.update("deploymentmonitors", mon.to_dict())
        except Conflict:
            cur = await self._get_monitor(mon.namespace, mon.name)
            if cur is None or mutate is None:
                return None
            mutate(cur)
            try:
                return await self.kube.update("deploymentmonitors", cur.to_dict())
            except ApiError as e:
                log.info("monitor update failed twice: %s", e)
                return None

    # ------------------------------------------------------------------ deployment events
    async def on_deployment_added(self, depl: Obj) -> None:
        md = depl.get("metadata", {})
        name, ns = md.get("name", ""), md.get("namespace", "")
        app = (md.get("labels") or {}).get("app")
        if not app or not await self.is_monitoring(ns):
            return
        meta = await self.get_metadata(ns, app, depl)
        if meta is None:
            return
        strategy = r.STRATEGY_CANARY if name.endswith(crd.CANARY_SUFFIX) else r.STRATEGY_ROLLING_UPDATE
        now = self.clock()
        old = await self._get_monitor(ns, name)
        create = old is None
        if create:
            old = crd.DeploymentMonitor(metadata={"name": name, "namespace": ns,
                                                  "annotations": {crd.ANNOTATION_DEPLOYMENT_NAME: name}})
            remediation = crd.RemediationAction(option=crd.REMEDIATION_NONE)
            continuous = False
        else:
            remediation = old.spec.remediation
            continuous = old.spec.continuous
        mon = copy.deepcopy(old)

        def apply(m: crd.DeploymentMonitor) -> None:
            m.spec = crd.DeploymentMonitorSpec(
                selector=(depl.get("spec") or {}).get("selector"), analyst=copy.deepcopy(meta.spec.analyst),
                start_time=format_rfc3339(now), wait_until=format_rfc3339(now + self.wait_until * 60),
                metrics=copy.deepcopy(meta.spec.metrics), logs=copy.deepcopy(meta.spec.logs),
                remediation=copy.deepcopy(remediation), continuous=continuous, rollback_revision=0)
            m.status = crd.DeploymentMonitorStatus(job_id="", phase=crd.PHASE_HEALTHY)

        apply(mon)
        await self.save_monitor(mon, create, apply)
        if strategy == r.STRATEGY_CANARY:
            base_name = name[: -len(crd.CANARY_SUFFIX)]
            try:
                base = await self.kube.get("deployments", ns, base_name)
            except ApiError:
                return
            await self.monitor_deployment(app, base, depl, strategy=r.STRATEGY_CANARY)

    async def on_deployment_updated(self, old: Obj, new: Obj) -> None:
        ns = new.get("metadata", {}).get("namespace", "")
        if not await self.is_monitoring(ns):
            return
        new_app = (new.get("metadata", {}).get("labels") or {}).get("app")
        old_app = (old.get("metadata", {}).get("labels") or {}).get("app")
        if not new_app or not old_app or new_app != old_app:
            return
        await self.monitor_deployment(new_app, old, new)

    async def on_deployment_deleted(self, depl: Obj) -> None:
        md = depl.get("metadata", {})
        if not await self.is_monitoring(md.get("namespace", "")):
            return
        if (md.get("annotations") or {}).get("aca") != "true":
            return
        try:
            await self.kube.delete("deploymentmonitors", md.get("namespace", ""), md.get("name", ""))
        except ApiError:
            pass

    async def monitor_deployment(self, app: str, old: Obj, new: Obj,
                                 strategy: str = r.STRATEGY_ROLLING_UPDATE) -> Optional[asyncio.Task]:
        """``monitorDeployment`` (Barrelman.go:205-263)."""
        ns = new.get("metadata", {}).get("namespace", "")
        meta = await self.get_metadata(ns, app, new)
        if meta is None:
            return None
        oc, nc = _containers(old), _containers(new)
        if len(oc) != len(nc):
            return None
        changed = any(a.get("image") != b.get("image") or not _env_equal(a.get("env"), b.get("env"))
                      for a, b in zip(oc, nc))
        if not changed and strategy != r.STRATEGY_CANARY:
            return None
        rb_new = (new.get("metadata", {}).get("annotations") or {}).get(crd.ANNOTATION_ROLLBACK_ID)
        rb_old = (old.get("metadata", {}).get("annotations") or {}).get(crd.ANNOTATION_ROLLBACK_ID)
        if rb_new and rb_new != rb_old:
            return None  # the rollout our own rollback triggered (revision numbers move on, so
            #              the reference's `revision == rollbackRevision` test cannot see it)
        name = new.get("metadata", {}).get("name", "")
        mon = await self._get_monitor(ns, name)
        not_found = mon is None
        if mon is not None:
            rev = revision_of(new)
            if rev > 0 and rev == mon.spec.rollback_revision:
                return None  # this rollout IS our rollback
            if (old.get("metadata", {}).get("annotations") or {}).get("deprecated.deployment.rollback.to"):
                return None
        return self.spawn(self.monitor_new_deployment(app, copy.deepcopy(old), copy.deepcopy(new), meta,
                                                      mon, not_found, strategy))

    async def monitor_continuously(self, monitor: crd.DeploymentMonitor) -> None:
        """``monitorContinuously`` (Barrelman.go:176-203)."""
        name = monitor.annotations.get(crd.ANNOTATION_DEPLOYMENT_NAME) or monitor.name
        try:
            depl = await self.kube.get("deployments", monitor.namespace, name)
        except ApiError:
            return
        app = (depl.get("metadata", {}).get("labels") or {}).get("app")
        if not app:
            return
        meta = await self.get_metadata(depl["metadata"].get("namespace", ""), app, depl)
        if meta is None:
            return
        await self.monitor_new_deployment(app, depl, depl, meta, monitor, False, r.STRATEGY_CONTINUOUS)

    # ------------------------------------------------------------------ pods
    async def _owned_replicasets(self, ns: str, uids: Tuple[str, ...]) -> List[Obj]:
        out = []
        for rs in await self.kube.list("replicasets", ns):
            owners = rs.get("metadata", {}).get("ownerReferences") or []
            if not owners or owners[0].get("uid") not in uids:
                continue
            spec_r = int((rs.get("spec") or {}).get("replicas") or 0)
            stat_r = int((rs.get("status") or {}).get("replicas") or 0)
            if spec_r > 0 or stat_r > 0:
                out.append(rs)
        return out

    async def get_pod_names(self, old: Obj, new: Obj) -> List[List[str]]:
        """``getPodNames`` (Barrelman.go:650-780): ``[current(new), baseline(old)]``.

        New/old ReplicaSets are told apart by owner (canary: two Deployments)
        or by revision (rolling update: one Deployment), instead of the
        reference's condition-message heuristic."""
        ns = new.get("metadata", {}).get("namespace", "")
        old_uid = old.get("metadata", {}).get("uid", "")
        new_uid = new.get("metadata", {}).get("uid", "")
        for attempt in range(4):
            rss = await self._owned_replicasets(ns, (old_uid, new_uid))
            if old_uid != new_uid:
                new_rs = sorted([x for x in rss if x["metadata"]["ownerReferences"][0]["uid"] == new_uid],
                                key=revision_of)
                old_rs = sorted([x for x in rss if x["metadata"]["ownerReferences"][0]["uid"] == old_uid],
                                key=revision_of)
                new_rs = new_rs[-1:] if new_rs else []
                old_rs = old_rs[-1:] if old_rs else []
            else:
                rss = sorted(rss, key=revision_of)
                new_rs = rss[-1:]
                old_rs = rss[-2:-1]
            if not new_rs:
                if attempt < 3:
                    await self.sleep(self.pod_retry_sleep)
                    continue
                raise NotFound("no ReplicaSet for " + new.get("metadata", {}).get("name", ""))
            hashes = [x["metadata"]["labels"].get("pod-template-hash", "") for x in new_rs + old_rs]
            sel = "pod-template-hash in (" + ",".join(h for h in hashes if h) + ")"
            pods = await self.kube.list("pods", ns, sel)
            new_uids = {x["metadata"]["uid"] for x in new_rs}
            cur, base = [], []
            for p in pods:
                owners = p.get("metadata", {}).get("ownerReferences") or []
                pname = p["metadata"]["name"]
                if owners and owners[0].get("uid") in new_uids:
                    if pname not in cur:
                        cur.append(pname)
                elif pname not in base:
                    base.append(pname)
            if not cur and attempt < 3:
                await self.sleep(self.pod_retry_sleep)
                continue
            return [cur, base] if base else [cur]
        return [[]]

    # ------------------------------------------------------------------ job launch
    async def monitor_new_deployment(self, app: str, old: Obj, new: Obj, meta: crd.DeploymentMetadata,
                                     old_monitor: Optional[crd.DeploymentMonitor], not_found: bool,
                                     strategy: str) -> None:
        """``monitorNewDeployment`` (Barrelman.go:783-899)."""
        ns = new["metadata"].get("namespace", "")
        name = new["metadata"]["name"]
        pods: List[List[str]] = []
        if strategy != r.STRATEGY_CONTINUOUS:
            try:
                pods = await self.get_pod_names(old, new)
            except ApiError as e:
                log.info("pod resolution failed for %s/%s: %s", ns, name, e)
                return
            if not pods or not pods[0]:
                return
        fresh = await self._get_monitor(ns, name)
        if fresh is not None:
            old_monitor = fresh
            not_found = False
        job_id, phase = "", crd.PHASE_RUNNING
        if strategy == r.STRATEGY_CONTINUOUS or old_monitor is None or not old_monitor.spec.continuous:
            client = self.analyst_factory(meta.spec.analyst.endpoint)
            for attempt in range(2):
                try:
                    job_id = await client.start_analyzing(ns, app, pods, meta.spec.metrics, self.watch_time,
                                                          strategy, now=self.clock())
                    break
                except (AnalystError, ApiError, Exception) as e:  # noqa: BLE001 - network errors
                    log.info("start analyzing failed (attempt %d): %s", attempt + 1, e)
            if not job_id:
                return
        else:
            job_id, phase = old_monitor.status.job_id, old_monitor.status.phase
        now = self.clock()
        mon = old_monitor if old_monitor is not None else crd.DeploymentMonitor(
            metadata={"name": name, "namespace": ns})
        old_rev = mon.spec.rollback_revision
        if strategy == r.STRATEGY_ROLLING_UPDATE:
            old_rev = revision_of(old)
        option = mon.spec.remediation.option or crd.REMEDIATION_NONE
        continuous = mon.spec.continuous

        def apply(m: crd.DeploymentMonitor) -> None:
            m.metadata["name"], m.metadata["namespace"] = name, ns
            m.annotations[crd.ANNOTATION_DEPLOYMENT_NAME] = name
            m.spec = crd.DeploymentMonitorSpec(
                selector=(new.get("spec") or {}).get("selector"), analyst=copy.deepcopy(meta.spec.analyst),
                start_time=format_rfc3339(now), wait_until=format_rfc3339(now + self.wait_until * 60),
                metrics=copy.deepcopy(meta.spec.metrics), logs=copy.deepcopy(meta.spec.logs),
                remediation=crd.RemediationAction(option=option), continuous=continuous,
                rollback_revision=old_rev)
            m.status = crd.DeploymentMonitorStatus(job_id=job_id, phase=phase, timestamp=format_rfc3339(now))

        apply(mon)
        await self.save_monitor(mon, not_found, apply)
        await self.record_event(new, "MonitoringStarted", f"job {job_id} strategy {strategy}")

    # ------------------------------------------------------------------ poller
    async def check_running_status(self) -> None:
        """``checkRunningStatus`` (Barrelman.go:496-591), cluster-wide list (Q15)."""
        try:
            items = await self.kube.list("deploymentmonitors")
        except ApiError as e:
            log.info("listing monitors failed: %s", e)
            return
        for raw in items:
            item = crd.DeploymentMonitor.from_dict(raw)
            if item.status.phase == crd.PHASE_RUNNING:
                await self._poll_one(item)
            elif item.spec.continuous:
                if item.status.phase == crd.PHASE_UNHEALTHY:
                    try:
                        ts = parse_rfc3339(item.status.timestamp).timestamp()
                    except ValueError:
                        continue
                    if self.clock() - ts > CONTINUOUS_COOLDOWN:
                        self.spawn(self.monitor_continuously(copy.deepcopy(item)))
                else:
                    self.spawn(self.monitor_continuously(copy.deepcopy(item)))

    async def _poll_one(self, item: crd.DeploymentMonitor) -> None:
        changed = False
        now = self.clock()
        new_phase, anomaly = item.status.phase, None
        if not item.status.expired:
            if not item.status.job_id:
                new_phase = crd.PHASE_HEALTHY
                changed = True
            else:
                try:
                    resp, new_phase = await self.analyst_factory(item.spec.analyst.endpoint).get_status(
                        item.status.job_id)
                except (AnalystError, Exception) as e:  # noqa: BLE001
                    log.info("status poll failed for %s/%s: %s", item.namespace, item.name, e)
                    return
                if resp.anomaly:
                    anomaly = crd.anomaly_from_flat({k: {"tags": v.tags, "values": v.values or []}
                                                     for k, v in resp.anomaly.items()})
                    changed = True
                if new_phase != item.status.phase:
                    changed = True
        expire = False
        if new_phase == crd.PHASE_RUNNING and item.spec.wait_until:
            try:
                if parse_rfc3339(item.spec.wait_until).timestamp() < now:
                    expire = True
                    changed = True
            except ValueError:
                pass
        if not changed:
            return
        no_job = not item.status.job_id and not item.status.expired

        def apply(m: crd.DeploymentMonitor) -> None:
            if m.status.phase != crd.PHASE_RUNNING:
                return  # someone else moved it on
            m.status.phase = new_phase
            if anomaly is not None:
                m.status.anomaly = anomaly
            if expire or no_job:
                m.status.phase = crd.PHASE_HEALTHY
                m.status.expired = True
            m.status.timestamp = format_rfc3339(now)
            m.status.remediation_taken = False

        apply(item)
        await self.save_monitor(item, False, apply)

    # ------------------------------------------------------------------ run loops
    async def watch_deployments(self) -> None:
        async for ev in self.kube.watch("deployments"):
            try:
                if ev["type"] == "ADDED":
                    await self.on_deployment_added(ev["object"])
                elif ev["type"] == "MODIFIED" and ev.get("old") is not None:
                    await self.on_deployment_updated(ev["old"], ev["object"])
                elif ev["type"] == "DELETED":
                    await self.on_deployment_deleted(ev["object"])
            except ApiError as e:
                log.info("deployment event failed: %s", e)

    async def poll_forever(self) -> None:
        while True:
            await self.check_running_status()
            await self.sleep(self.poll_seconds)
