"""The Kubernetes surface the controller needs, as an async protocol.

Kinds are addressed by their REST plural: ``deployments``, ``replicasets``,
``pods``, ``namespaces``, ``events``, ``deploymentmonitors``,
``deploymentmetadatas``.  Objects are plain JSON dicts (the API server's
wire form).  Implementations: :class:`~foremast_amd.k8s.fake.FakeCluster`
(in-memory, with a simulated deployment controller — the analogue of the
generated fake clientset the reference ships but never uses,
``pkg/client/clientset/versioned/fake``) and
:class:`~foremast_amd.k8s.http.HttpKube` (a real API server over HTTPS).
"""

from __future__ import annotations

from typing import Any, AsyncIterator, Dict, List, Optional, Protocol

Obj = Dict[str, Any]

CLUSTER_SCOPED = {"namespaces"}

KIND_OF = {
    "deployments": "Deployment", "replicasets": "ReplicaSet", "pods": "Pod", "namespaces": "Namespace",
    "events": "Event", "deploymentmonitors": "DeploymentMonitor", "deploymentmetadatas": "DeploymentMetadata",
}
API_VERSION_OF = {
    "deployments": "apps/v1", "replicasets": "apps/v1", "pods": "v1", "namespaces": "v1", "events": "v1",
    "deploymentmonitors": "deployment.foremast.ai/v1alpha1",
    "deploymentmetadatas": "deployment.foremast.ai/v1alpha1",
}


class ApiError(Exception):
    def __init__(self, code: int, reason: str, message: str = "") -> None:
        super().__init__(f"{code} {reason}: {message}")
        self.code = code
        self.reason = reason


class NotFound(ApiError):
    def __init__(self, message: str = "") -> None:
        super().__init__(404, "NotFound", message)


class Conflict(ApiError):
    def __init__(self, message: str = "") -> None:
        super().__init__(409, "Conflict", message)


class AlreadyExists(ApiError):
    def __init__(self, message: str = "") -> None:
        super().__init__(409, "AlreadyExists", message)


class KubeAPI(Protocol):
    async def get(self, kind: str, namespace: str, name: str) -> Obj: ...

    async def list(self, kind: str, namespace: Optional[str] = None,
                   label_selector: Optional[str] = None) -> List[Obj]: ...

    async def create(self, kind: str, obj: Obj) -> Obj: ...

    async def update(self, kind: str, obj: Obj) -> Obj: ...

    async def patch(self, kind: str, namespace: str, name: str, patch: Obj) -> Obj: ...

    async def delete(self, kind: str, namespace: str, name: str) -> None: ...

    def watch(self, kind: str, namespace: Optional[str] = None) -> AsyncIterator[Dict[str, Any]]: ...

    async def rollback(self, namespace: str, name: str, revision: int, message: str = "") -> Obj: ...


# ---------------------------------------------------------------------------------
# label selectors (the subset barrelman uses: equality and set-based "in")
# ---------------------------------------------------------------------------------

def parse_selector(sel: Optional[str]):
    reqs = []
    if not sel:
        return reqs
    s = sel.strip()
    i = 0
    parts = []
    depth = 0
    cur = ""
    for ch in s:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur:
        parts.append(cur)
    del i
    for p in parts:
        p = p.strip()
        if " in " in p or " in(" in p:
            k, rest = p.split(" in", 1)
            vals = rest.strip().lstrip("(").rstrip(")")
            reqs.append((k.strip(), "in", {v.strip() for v in vals.split(",") if v.strip()}))
        elif " notin " in p:
            k, rest = p.split(" notin", 1)
            vals = rest.strip().lstrip("(").rstrip(")")
            reqs.append((k.strip(), "notin", {v.strip() for v in vals.split(",") if v.strip()}))
        elif "!=" in p:
            k, v = p.split("!=", 1)
            reqs.append((k.strip(), "!=", v.strip()))
        elif "==" in p:
            k, v = p.split("==", 1)
            reqs.append((k.strip(), "=", v.strip()))
        elif "=" in p:
            k, v = p.split("=", 1)
            reqs.append((k.strip(), "=", v.strip()))
        else:
            reqs.append((p, "exists", None))
    return reqs


def matches(labels: Optional[Dict[str, str]], sel: Optional[str]) -> bool:
    labels = labels or {}
    for k, op, v in parse_selector(sel):
        have = labels.get(k)
        if op == "=" and have != v:
            return False
        if op == "!=" and have == v:
            return False
        if op == "in" and have not in v:
            return False
        if op == "notin" and have in v:
            return False
        if op == "exists" and k not in labels:
            return False
    return True


def revision_of(obj: Obj) -> int:
    """``deploymentutil.Revision``: the revision annotation as int (0 if absent)."""
    ann = (obj.get("metadata") or {}).get("annotations") or {}
    try:
        return int(ann.get("deployment.kubernetes.io/revision", "0"))
    except ValueError:
        return 0
