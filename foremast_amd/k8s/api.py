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

from typing import Any, AsyncIterator, Dict, List, Optional, Protocol, Tuple

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
                   label_selector: Optional[str] = None, field_selector: Optional[str] = None) -> List[Obj]: ...

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


# ---------------------------------------------------------------------------------
# field selectors: metadata.name / metadata.namespace for every kind, plus the
# DeploymentMonitor status fields the reference registers as field labels
# (v1alpha1/register.go:38-53: status.jobId, status.phase); the generated CRD declares
# them as selectableFields so a real API server filters on them too (deploy/schema.py)
# ---------------------------------------------------------------------------------

FIELD_LABELS: Dict[str, Tuple[str, ...]] = {
    "deploymentmonitors": ("metadata.name", "metadata.namespace", "status.jobId", "status.phase"),
}
DEFAULT_FIELD_LABELS = ("metadata.name", "metadata.namespace")


class BadRequest(ApiError):
    def __init__(self, message: str = "") -> None:
        super().__init__(400, "BadRequest", message)


def parse_field_selector(kind: str, sel: Optional[str]) -> List[Tuple[str, str, str]]:
    """``a=b`` / ``a==b`` / ``a!=b`` terms joined by commas (ANDed); an unsupported
    field label is a 400, like the API server's."""
    out = []
    allowed = FIELD_LABELS.get(kind, DEFAULT_FIELD_LABELS)
    for term in (sel or "").split(","):
        term = term.strip()
        if not term:
            continue
        if "!=" in term:
            k, v = term.split("!=", 1)
            op = "!="
        elif "==" in term:
            k, v = term.split("==", 1)
            op = "="
        elif "=" in term:
            k, v = term.split("=", 1)
            op = "="
        else:
            raise BadRequest(f"invalid field selector term {term!r}")
        k = k.strip()
        if k not in allowed:
            raise BadRequest(f'field label not supported: "{k}"')
        out.append((k, op, v.strip()))
    return out


def field_value(obj: Obj, path: str) -> str:
    cur: Any = obj
    for part in path.split("."):
        cur = cur.get(part) if isinstance(cur, dict) else None
    return "" if cur is None else str(cur)


def field_matches(obj: Obj, terms: List[Tuple[str, str, str]]) -> bool:
    for k, op, v in terms:
        have = field_value(obj, k)
        if (op == "=" and have != v) or (op == "!=" and have == v):
            return False
    return True


def revision_of(obj: Obj) -> int:
    """``deploymentutil.Revision``: the revision annotation as int (0 if absent)."""
    ann = (obj.get("metadata") or {}).get("annotations") or {}
    try:
        return int(ann.get("deployment.kubernetes.io/revision", "0"))
    except ValueError:
        return 0
