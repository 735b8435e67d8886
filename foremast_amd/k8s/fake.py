"""In-memory Kubernetes cluster for tests and local runs.

Features the controller relies on:

* object store keyed by (plural, namespace, name) with ``uid``,
  ``resourceVersion`` (optimistic concurrency on ``update``),
  ``creationTimestamp``;
* watch streams (ADDED / MODIFIED / DELETED with the previous object);
* label selectors (equality / set-based);
* a simulated deployment controller: creating a Deployment or changing its
  pod template creates a ReplicaSet (owner = Deployment UID, label
  ``pod-template-hash``, revision annotation) and its pods.  The old
  ReplicaSet keeps its pods until :meth:`finish_rollout` (so canary /
  rolling-update baselines exist), mirroring a rollout in progress;
* ``rollback`` re-applies the template of the ReplicaSet at a revision, like
  ``kubectl rollout undo --to-revision`` (Q16: the reference used the
  removed ``extensions/v1beta1`` DeploymentRollback);
* an ``actions`` log so tests can assert on remediation.
"""

from __future__ import annotations

import asyncio
import copy
import hashlib
import itertools
import json
import time
import uuid
from typing import Any, AsyncIterator, Dict, List, Optional, Tuple

from .api import (API_VERSION_OF, CLUSTER_SCOPED, KIND_OF, AlreadyExists, Conflict, NotFound, Obj,
                  field_matches, matches, parse_field_selector, revision_of)

REV = "deployment.kubernetes.io/revision"


def _now_rfc3339() -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())


def template_hash(template: Obj) -> str:
    t = copy.deepcopy(template)
    (t.get("metadata") or {}).get("labels", {}).pop("pod-template-hash", None)
    raw = json.dumps(t, sort_keys=True).encode()
    return hashlib.sha256(raw).hexdigest()[:10]


class FakeCluster:
    def __init__(self, simulate_controllers: bool = True) -> None:
        self._objs: Dict[Tuple[str, str, str], Obj] = {}
        self._rv = itertools.count(1)
        self._watchers: List[Tuple[str, Optional[str], asyncio.Queue]] = []
        self.simulate = simulate_controllers
        self.actions: List[Dict[str, Any]] = []

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _key(kind: str, namespace: Optional[str], name: str):
        return (kind, "" if kind in CLUSTER_SCOPED else (namespace or ""), name)

    def _emit(self, kind: str, etype: str, obj: Obj, old: Optional[Obj] = None) -> None:
        ns = (obj.get("metadata") or {}).get("namespace")
        for wk, wns, q in list(self._watchers):
            if wk == kind and (wns is None or wns == ns):
                q.put_nowait({"type": etype, "object": copy.deepcopy(obj),
                              "old": copy.deepcopy(old) if old is not None else None})

    def _stamp(self, kind: str, obj: Obj) -> Obj:
        md = obj.setdefault("metadata", {})
        md["resourceVersion"] = str(next(self._rv))
        obj.setdefault("apiVersion", API_VERSION_OF.get(kind, "v1"))
        obj.setdefault("kind", KIND_OF.get(kind, kind))
        return obj

    # ------------------------------------------------------------------ sync core
    def get_sync(self, kind: str, namespace: str, name: str) -> Obj:
        o = self._objs.get(self._key(kind, namespace, name))
        if o is None:
            raise NotFound(f"{kind} {namespace}/{name}")
        return copy.deepcopy(o)

    def list_sync(self, kind: str, namespace: Optional[str] = None,
                  label_selector: Optional[str] = None, field_selector: Optional[str] = None) -> List[Obj]:
        fields = parse_field_selector(kind, field_selector)
        out = []
        for (k, ns, _), o in sorted(self._objs.items()):
            if k != kind:
                continue
            if namespace and kind not in CLUSTER_SCOPED and ns != namespace:
                continue
            if label_selector and not matches((o.get("metadata") or {}).get("labels"), label_selector):
                continue
            if fields and not field_matches(o, fields):
                continue
            out.append(copy.deepcopy(o))
        return out

    def create_sync(self, kind: str, obj: Obj) -> Obj:
        obj = copy.deepcopy(obj)
        md = obj.setdefault("metadata", {})
        if not md.get("name") and md.get("generateName"):
            md["name"] = md["generateName"] + uuid.uuid4().hex[:5]
        key = self._key(kind, md.get("namespace"), md["name"])
        if key in self._objs:
            raise AlreadyExists(f"{kind} {key[1]}/{key[2]}")
        md["uid"] = str(uuid.uuid4())
        md.setdefault("creationTimestamp", _now_rfc3339())
        md.setdefault("generation", 1)
        self._stamp(kind, obj)
        self._objs[key] = obj
        self._emit(kind, "ADDED", obj)
        if self.simulate and kind == "deployments":
            self._reconcile_deployment(obj, None)
        return copy.deepcopy(obj)

    def update_sync(self, kind: str, obj: Obj) -> Obj:
        obj = copy.deepcopy(obj)
        md = obj.setdefault("metadata", {})
        key = self._key(kind, md.get("namespace"), md.get("name", ""))
        old = self._objs.get(key)
        if old is None:
            raise NotFound(f"{kind} {key[1]}/{key[2]}")
        rv = md.get("resourceVersion")
        if rv and rv != old["metadata"].get("resourceVersion"):
            raise Conflict(f"{kind} {key[1]}/{key[2]}: resourceVersion {rv} is stale")
        md["uid"] = old["metadata"]["uid"]
        md["creationTimestamp"] = old["metadata"].get("creationTimestamp")
        if kind == "deployments" and old.get("spec", {}).get("template") != obj.get("spec", {}).get("template"):
            md["generation"] = int(old["metadata"].get("generation", 1)) + 1
        self._stamp(kind, obj)
        self._objs[key] = obj
        self._emit(kind, "MODIFIED", obj, old)
        if self.simulate and kind == "deployments":
            self._reconcile_deployment(obj, old)
        return copy.deepcopy(obj)

    def patch_sync(self, kind: str, namespace: str, name: str, patch: Obj) -> Obj:
        cur = self.get_sync(kind, namespace, name)
        merged = _merge_patch(cur, patch)
        merged["metadata"].pop("resourceVersion", None)
        return self.update_sync(kind, merged)

    def delete_sync(self, kind: str, namespace: str, name: str) -> None:
        key = self._key(kind, namespace, name)
        o = self._objs.pop(key, None)
        if o is None:
            raise NotFound(f"{kind} {namespace}/{name}")
        self._emit(kind, "DELETED", o)

    # ------------------------------------------------------------------ async API
    async def get(self, kind, namespace, name):
        return self.get_sync(kind, namespace, name)

    async def list(self, kind, namespace=None, label_selector=None, field_selector=None):
        return self.list_sync(kind, namespace, label_selector, field_selector)

    async def create(self, kind, obj):
        return self.create_sync(kind, obj)

    async def update(self, kind, obj):
        return self.update_sync(kind, obj)

    async def patch(self, kind, namespace, name, patch):
        return self.patch_sync(kind, namespace, name, patch)

    async def delete(self, kind, namespace, name):
        self.delete_sync(kind, namespace, name)

    async def watch(self, kind: str, namespace: Optional[str] = None) -> AsyncIterator[Dict[str, Any]]:
        q: asyncio.Queue = asyncio.Queue()
        entry = (kind, namespace, q)
        self._watchers.append(entry)
        try:
            # initial ADDED events for existing objects (informer list+watch)
            for o in self.list_sync(kind, namespace):
                yield {"type": "ADDED", "object": o, "old": None, "initial": True}
            while True:
                ev = await q.get()
                yield ev
        finally:
            if entry in self._watchers:
                self._watchers.remove(entry)

    async def rollback(self, namespace: str, name: str, revision: int, message: str = "") -> Obj:
        return self.rollback_sync(namespace, name, revision, message)

    # ------------------------------------------------------------------ simulated controllers
    def _owned_rs(self, depl: Obj) -> List[Obj]:
        uid = depl["metadata"]["uid"]
        ns = depl["metadata"].get("namespace")
        return [rs for rs in self.list_sync("replicasets", ns)
                if any(o.get("uid") == uid for o in rs["metadata"].get("ownerReferences", []))]

    def _reconcile_deployment(self, depl: Obj, old: Optional[Obj]) -> None:
        tpl = depl.get("spec", {}).get("template") or {}
        h = template_hash(tpl)
        ns = depl["metadata"].get("namespace")
        owned = self._owned_rs(depl)
        existing = next((rs for rs in owned if rs["metadata"]["labels"].get("pod-template-hash") == h), None)
        max_rev = max([revision_of(rs) for rs in owned] + [0])
        replicas = int(depl.get("spec", {}).get("replicas", 1))
        if existing is not None:
            if revision_of(existing) != max_rev or revision_of(depl) != revision_of(existing):
                # template reverted to an older RS (rollback): it becomes the newest revision
                new_rev = max_rev + 1 if revision_of(existing) != max_rev else max_rev
                existing["metadata"].setdefault("annotations", {})[REV] = str(new_rev)
                existing["metadata"].pop("resourceVersion", None)
                existing["spec"]["replicas"] = replicas
                self.update_sync("replicasets", existing)
                self._set_depl_revision(depl, new_rev)
                self._ensure_pods(self.get_sync("replicasets", ns, existing["metadata"]["name"]), replicas)
            return
        rev = max_rev + 1
        labels = dict((tpl.get("metadata") or {}).get("labels") or {})
        labels["pod-template-hash"] = h
        rs = {
            "metadata": {
                "name": f"{depl['metadata']['name']}-{h}", "namespace": ns, "labels": labels,
                "annotations": {REV: str(rev)},
                "ownerReferences": [{"apiVersion": "apps/v1", "kind": "Deployment",
                                     "name": depl["metadata"]["name"], "uid": depl["metadata"]["uid"],
                                     "controller": True}],
            },
            "spec": {"replicas": replicas, "template": copy.deepcopy(tpl),
                     "selector": depl.get("spec", {}).get("selector")},
            "status": {"replicas": replicas},
        }
        rs = self.create_sync("replicasets", rs)
        self._ensure_pods(rs, replicas)
        self._set_depl_revision(depl, rev)

    def _set_depl_revision(self, depl: Obj, rev: int) -> None:
        key = self._key("deployments", depl["metadata"].get("namespace"), depl["metadata"]["name"])
        cur = self._objs.get(key)
        if cur is None:
            return
        if revision_of(cur) == rev:
            return
        old = copy.deepcopy(cur)
        cur["metadata"].setdefault("annotations", {})[REV] = str(rev)
        conds = cur.setdefault("status", {}).setdefault("conditions", [])
        conds[:] = [c for c in conds if c.get("type") != "Progressing"]
        rs_name = f"{cur['metadata']['name']}-{template_hash(cur['spec'].get('template') or {})}"
        conds.append({"type": "Progressing", "status": "True", "reason": "NewReplicaSetAvailable",
                      "message": f'ReplicaSet "{rs_name}" has successfully progressed.'})
        self._stamp("deployments", cur)
        self._emit("deployments", "MODIFIED", cur, old)

    def _ensure_pods(self, rs: Obj, replicas: int) -> None:
        ns = rs["metadata"].get("namespace")
        h = rs["metadata"]["labels"].get("pod-template-hash")
        have = [p for p in self.list_sync("pods", ns, f"pod-template-hash={h}")]
        for i in range(len(have), replicas):
            labels = dict(rs["metadata"]["labels"])
            self.create_sync("pods", {
                "metadata": {"name": f"{rs['metadata']['name']}-{uuid.uuid4().hex[:5]}", "namespace": ns,
                             "labels": labels,
                             "ownerReferences": [{"apiVersion": "apps/v1", "kind": "ReplicaSet",
                                                  "name": rs["metadata"]["name"], "uid": rs["metadata"]["uid"],
                                                  "controller": True}]},
                "spec": copy.deepcopy((rs["spec"].get("template") or {}).get("spec") or {}),
                "status": {"phase": "Running"},
            })

    def finish_rollout(self, namespace: str, name: str) -> None:
        """Scale every non-current ReplicaSet of the deployment to 0 and delete its pods."""
        depl = self.get_sync("deployments", namespace, name)
        h = template_hash(depl["spec"].get("template") or {})
        for rs in self._owned_rs(depl):
            if rs["metadata"]["labels"].get("pod-template-hash") == h:
                continue
            for p in self.list_sync("pods", namespace,
                                    f"pod-template-hash={rs['metadata']['labels'].get('pod-template-hash')}"):
                self.delete_sync("pods", namespace, p["metadata"]["name"])
            rs["spec"]["replicas"] = 0
            rs["status"]["replicas"] = 0
            rs["metadata"].pop("resourceVersion", None)
            self.update_sync("replicasets", rs)

    def rollback_sync(self, namespace: str, name: str, revision: int, message: str = "") -> Obj:
        depl = self.get_sync("deployments", namespace, name)
        if depl.get("spec", {}).get("paused"):
            raise Conflict("you cannot rollback a paused deployment")
        target = next((rs for rs in self._owned_rs(depl) if revision_of(rs) == revision), None)
        if target is None:
            raise NotFound(f"revision {revision} of {namespace}/{name}")
        tpl = copy.deepcopy(target["spec"]["template"])
        tpl.get("metadata", {}).get("labels", {}).pop("pod-template-hash", None)
        depl["spec"]["template"] = tpl
        ann = depl["metadata"].setdefault("annotations", {})
        ann["deployment.foremast.ai/rollback-id"] = f"{revision}-{time.time_ns()}"
        if message:
            ann["deployment.foremast.ai/rollbackMessage"] = message
        depl["metadata"].pop("resourceVersion", None)
        self.actions.append({"action": "rollback", "namespace": namespace, "name": name,
                             "revision": revision, "message": message})
        return self.update_sync("deployments", depl)

    # ------------------------------------------------------------------ conveniences
    def add_namespace(self, name: str, annotations: Optional[Dict[str, str]] = None) -> Obj:
        return self.create_sync("namespaces", {"metadata": {"name": name, "annotations": annotations or {}}})

    def apply_deployment(self, namespace: str, name: str, app: str, image: str, env=None, replicas: int = 1,
                         labels: Optional[Dict[str, str]] = None) -> Obj:
        lbl = {"app": app}
        lbl.update(labels or {})
        tpl = {"metadata": {"labels": {"app": app}},
               "spec": {"containers": [{"name": app, "image": image, "env": env or []}]}}
        try:
            cur = self.get_sync("deployments", namespace, name)
        except NotFound:
            return self.create_sync("deployments", {
                "metadata": {"name": name, "namespace": namespace, "labels": lbl},
                "spec": {"replicas": replicas, "selector": {"matchLabels": {"app": app}}, "template": tpl},
                "status": {}})
        cur["spec"]["template"] = tpl
        cur["spec"]["replicas"] = replicas
        cur["metadata"]["labels"] = lbl
        cur["metadata"].pop("resourceVersion", None)
        return self.update_sync("deployments", cur)


def _merge_patch(target: Any, patch: Any) -> Any:
    """RFC 7386 JSON merge patch."""
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    out = copy.deepcopy(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = _merge_patch(out.get(k), v)
    return out
