"""MonitorController: reacts to DeploymentMonitor phase changes, remediates.

``foremast-barrelman/pkg/controller/MonitorController.go``:

* phase becomes ``Unhealthy`` and ``remediationTaken`` is false → set it,
  persist, then run the configured action: ``AutoRollback`` → roll back to
  ``spec.rollbackRevision``; ``AutoPause`` → ``spec.paused = true``;
  ``Auto`` (a TODO in the reference) → rollback when a revision is known,
  otherwise pause (design decision);
* a continuous monitor that is not running is re-launched (60 s cooldown
  after Unhealthy); toggling ``spec.continuous`` on starts it.

Fixes: Q8 (the reference compared against a hard-coded ``oldPhase = ""``),
Q16 (rollback re-applies the ReplicaSet template — what ``kubectl rollout
undo`` does — instead of the removed extensions/v1beta1 DeploymentRollback).
"""

from __future__ import annotations

import copy
import logging
from typing import Optional

from ..api import crd
from ..k8s.api import ApiError, KubeAPI, Obj, revision_of
from ..utils.timeutil import parse_rfc3339
from .barrelman import CONTINUOUS_COOLDOWN, Barrelman

log = logging.getLogger("foremast.monitor")


class MonitorController:
    def __init__(self, kube: KubeAPI, barrelman: Barrelman) -> None:
        self.kube = kube
        self.barrelman = barrelman
        self.clock = barrelman.clock
        self.actions = {crd.REMEDIATION_AUTO_ROLLBACK: self.rollback, crd.REMEDIATION_AUTO_PAUSE: self.pause,
                        crd.REMEDIATION_AUTO: self.auto}

    def deployment_name(self, m: crd.DeploymentMonitor) -> str:
        return m.annotations.get(crd.ANNOTATION_DEPLOYMENT_NAME) or m.name

    async def on_monitor_updated(self, old_raw: Obj, new_raw: Obj) -> None:
        old = crd.DeploymentMonitor.from_dict(old_raw)
        new = crd.DeploymentMonitor.from_dict(new_raw)
        new_phase, old_phase = new.status.phase, old.status.phase
        continuous_change = old.spec.continuous != new.spec.continuous
        if new_phase == old_phase:
            if continuous_change and new.spec.continuous and new_phase != crd.PHASE_RUNNING:
                self.barrelman.spawn(self.barrelman.monitor_continuously(new))
            return
        if new_phase == crd.PHASE_UNHEALTHY and not new.status.remediation_taken:
            action = self.actions.get(new.spec.remediation.option)
            if action is not None:
                def mark(m: crd.DeploymentMonitor) -> None:
                    m.status.remediation_taken = True
                mark(new)
                saved = await self.barrelman.save_monitor(new, False, mark)
                if saved is not None:
                    self.barrelman.spawn(action(copy.deepcopy(new)))
                return
        if new.spec.continuous and new_phase != crd.PHASE_RUNNING:
            if new_phase == crd.PHASE_UNHEALTHY:
                try:
                    ts = parse_rfc3339(new.status.timestamp).timestamp()
                except ValueError:
                    return
                if self.clock() - ts > CONTINUOUS_COOLDOWN:
                    self.barrelman.spawn(self.barrelman.monitor_continuously(new))
            else:
                self.barrelman.spawn(self.barrelman.monitor_continuously(new))

    async def _get_deployment(self, m: crd.DeploymentMonitor) -> Optional[Obj]:
        try:
            return await self.kube.get("deployments", m.namespace, self.deployment_name(m))
        except ApiError:
            return None

    async def rollback(self, m: crd.DeploymentMonitor) -> bool:
        rev = m.spec.rollback_revision
        if rev == 0:
            return False
        depl = await self._get_deployment(m)
        if depl is None:
            return False
        if revision_of(depl) == rev:
            log.info("already at revision %d", rev)
            return False
        if (depl.get("spec") or {}).get("paused"):
            await self.barrelman.record_event(depl, "RollbackSkipped", "deployment is paused", "Warning")
            return False
        msg = f"Foremast detected unhealthy, so roll it back automatically to revision:{rev}"
        try:
            await self.kube.rollback(m.namespace, self.deployment_name(m), rev, msg)
        except ApiError as e:
            log.info("rollback failed: %s", e)
            return False
        await self.barrelman.record_event(depl, "RollbackProgressing", msg, "Warning")
        return True

    async def pause(self, m: crd.DeploymentMonitor) -> bool:
        depl = await self._get_deployment(m)
        if depl is None:
            return False
        try:
            await self.kube.patch("deployments", m.namespace, self.deployment_name(m), {"spec": {"paused": True}})
        except ApiError as e:
            log.info("pause failed: %s", e)
            return False
        if hasattr(self.kube, "actions"):
            self.kube.actions.append({"action": "pause", "namespace": m.namespace, "name": self.deployment_name(m)})
        await self.barrelman.record_event(depl, "ForemastPaused",
                                          "Foremast detected unhealthy, so paused this deployment", "Warning")
        return True

    async def auto(self, m: crd.DeploymentMonitor) -> bool:
        if m.spec.rollback_revision:
            return await self.rollback(m)
        return await self.pause(m)

    async def watch_monitors(self) -> None:
        async for ev in self.kube.watch("deploymentmonitors"):
            if ev["type"] == "MODIFIED" and ev.get("old") is not None:
                try:
                    await self.on_monitor_updated(ev["old"], ev["object"])
                except ApiError as e:
                    log.info("monitor event failed: %s", e)
