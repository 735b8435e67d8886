"""Kubernetes API server client (REST over HTTPS) implementing :class:`KubeAPI`.

The reference builds generated typed clientsets, informers and listers for
``apps/v1`` Deployments and the Foremast CRDs
(``foremast-barrelman/pkg/client/clientset/versioned/clientset.go:43-92``,
``.../informers/externalversions/factory.go:79-180``).  Here one small async
client covers every kind the controller touches, addressed by REST plural:

* CRUD: ``GET/POST/PUT/DELETE`` and JSON merge-patch, with API ``Status``
  bodies mapped to :class:`NotFound` / :class:`Conflict` / :class:`AlreadyExists`
  (optimistic concurrency through ``metadata.resourceVersion`` — the
  reference's unconditional ``Update`` calls lose updates);
* :meth:`HttpKube.watch` is an *informer*: list → ``ADDED`` (``initial``) for
  the current state, then a streaming ``?watch=true`` from the list's
  resourceVersion; it keeps the last-seen object per key so ``MODIFIED``
  events carry ``old`` (what ``UpdateFunc(old, new)`` gets in client-go),
  relists and diffs after ``410 Gone`` / dropped streams, and re-delivers the
  cache every ``resync`` seconds (the reference's 30 s / 10 s informer resync,
  ``foremast-barrelman/cmd/manager/main.go:74,76``);
* :meth:`HttpKube.rollback` does what ``kubectl rollout undo --to-revision``
  does (copy the target ReplicaSet's pod template into the Deployment), since
  the ``extensions/v1beta1`` rollback subresource the reference calls
  (``MonitorController.go:150-175``) no longer exists in current clusters.

Configuration: in-cluster service account, a kubeconfig (server + token or
client certificate), or an explicit base URL / transport (tests).
"""

from __future__ import annotations

import asyncio
import base64
import copy
import json
import os
import tempfile
import time
from dataclasses import dataclass
from typing import Any, AsyncIterator, Dict, List, Optional, Tuple

import httpx

from .api import (API_VERSION_OF, CLUSTER_SCOPED, AlreadyExists, ApiError, Conflict, NotFound, Obj,
                  revision_of)

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


@dataclass
class KubeConfig:
    server: str
    token: Optional[str] = None
    ca_file: Optional[str] = None
    cert_file: Optional[str] = None
    key_file: Optional[str] = None
    verify: bool = True

    @classmethod
    def in_cluster(cls) -> "KubeConfig":
        host, port = os.environ["KUBERNETES_SERVICE_HOST"], os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        with open(os.path.join(SA_DIR, "token")) as f:
            token = f.read().strip()
        return cls(server=f"https://{host}:{port}", token=token, ca_file=os.path.join(SA_DIR, "ca.crt"))

    @classmethod
    def from_kubeconfig(cls, path: Optional[str] = None, context: Optional[str] = None) -> "KubeConfig":
        import yaml
        path = path or os.environ.get("KUBECONFIG") or os.path.expanduser("~/.kube/config")
        with open(path) as f:
            cfg = yaml.safe_load(f)
        ctx_name = context or cfg.get("current-context")
        ctx = next(c["context"] for c in cfg.get("contexts", []) if c["name"] == ctx_name)
        cluster = next(c["cluster"] for c in cfg.get("clusters", []) if c["name"] == ctx["cluster"])
        user = next((u["user"] for u in cfg.get("users", []) if u["name"] == ctx.get("user")), {}) or {}

        def materialise(data_key: str, file_key: str, src: Dict[str, Any]) -> Optional[str]:
            if src.get(file_key):
                return src[file_key]
            if src.get(data_key):
                fd, p = tempfile.mkstemp(prefix="foremast-kube-")
                with os.fdopen(fd, "wb") as out:
                    out.write(base64.b64decode(src[data_key]))
                return p
            return None

        return cls(server=cluster["server"], token=user.get("token"),
                   ca_file=materialise("certificate-authority-data", "certificate-authority", cluster),
                   cert_file=materialise("client-certificate-data", "client-certificate", user),
                   key_file=materialise("client-key-data", "client-key", user),
                   verify=not cluster.get("insecure-skip-tls-verify", False))

    @classmethod
    def auto(cls) -> "KubeConfig":
        if os.environ.get("KUBERNETES_SERVICE_HOST") and os.path.exists(os.path.join(SA_DIR, "token")):
            return cls.in_cluster()
        return cls.from_kubeconfig()


def resource_path(kind: str, namespace: Optional[str] = None, name: Optional[str] = None) -> str:
    api = API_VERSION_OF[kind]
    prefix = "/api/v1" if api == "v1" else f"/apis/{api}"
    if kind in CLUSTER_SCOPED or not namespace:
        p = f"{prefix}/{kind}"
    else:
        p = f"{prefix}/namespaces/{namespace}/{kind}"
    return f"{p}/{name}" if name else p


def _raise_for(resp: httpx.Response) -> None:
    if resp.status_code < 400:
        return
    try:
        body = resp.json()
    except ValueError:
        body = {}
    reason, msg = body.get("reason", ""), body.get("message", resp.text[:200])
    if resp.status_code == 404:
        raise NotFound(msg)
    if resp.status_code == 409:
        raise AlreadyExists(msg) if reason == "AlreadyExists" else Conflict(msg)
    raise ApiError(resp.status_code, reason or resp.reason_phrase, msg)


def _key(o: Obj) -> Tuple[str, str]:
    md = o.get("metadata") or {}
    return md.get("namespace", ""), md.get("name", "")


class HttpKube:
    def __init__(self, config: Optional[KubeConfig] = None, base_url: Optional[str] = None,
                 transport: Optional[httpx.AsyncBaseTransport] = None, timeout: float = 30.0,
                 resync: Optional[float] = None) -> None:
        headers = {"Accept": "application/json"}
        kw: Dict[str, Any] = {"timeout": httpx.Timeout(timeout, read=None)}
        if config is not None:
            base_url = base_url or config.server
            if config.token:
                headers["Authorization"] = f"Bearer {config.token}"
            kw["verify"] = (config.ca_file or True) if config.verify else False
            if config.cert_file and config.key_file:
                kw["cert"] = (config.cert_file, config.key_file)
        if transport is not None:
            kw["transport"] = transport
        self.http = httpx.AsyncClient(base_url=base_url or "http://127.0.0.1:8001", headers=headers, **kw)
        self.resync = resync

    async def aclose(self) -> None:
        await self.http.aclose()

    # ------------------------------------------------------------------ CRUD
    async def get(self, kind: str, namespace: str, name: str) -> Obj:
        resp = await self.http.get(resource_path(kind, namespace, name))
        _raise_for(resp)
        return resp.json()

    async def _list_raw(self, kind: str, namespace: Optional[str], label_selector: Optional[str] = None,
                        field_selector: Optional[str] = None):
        params = {k: v for k, v in (("labelSelector", label_selector), ("fieldSelector", field_selector)) if v}
        resp = await self.http.get(resource_path(kind, namespace), params=params or None)
        _raise_for(resp)
        return resp.json()

    async def list(self, kind: str, namespace: Optional[str] = None,
                   label_selector: Optional[str] = None, field_selector: Optional[str] = None) -> List[Obj]:
        return list((await self._list_raw(kind, namespace, label_selector, field_selector)).get("items") or [])

    async def create(self, kind: str, obj: Obj) -> Obj:
        ns = (obj.get("metadata") or {}).get("namespace")
        body = dict(obj)
        body.setdefault("apiVersion", API_VERSION_OF[kind])
        resp = await self.http.post(resource_path(kind, ns), json=body)
        _raise_for(resp)
        return resp.json()

    async def update(self, kind: str, obj: Obj) -> Obj:
        ns, name = _key(obj)
        resp = await self.http.put(resource_path(kind, ns, name), json=obj)
        _raise_for(resp)
        return resp.json()

    async def patch(self, kind: str, namespace: str, name: str, patch: Obj) -> Obj:
        resp = await self.http.patch(resource_path(kind, namespace, name), content=json.dumps(patch),
                                     headers={"Content-Type": "application/merge-patch+json"})
        _raise_for(resp)
        return resp.json()

    async def delete(self, kind: str, namespace: str, name: str) -> None:
        resp = await self.http.delete(resource_path(kind, namespace, name))
        _raise_for(resp)

    # ------------------------------------------------------------------ informer-style watch
    async def _stream(self, kind: str, namespace: Optional[str], rv: str) -> AsyncIterator[Dict[str, Any]]:
        params = {"watch": "true", "resourceVersion": rv, "allowWatchBookmarks": "true"}
        async with self.http.stream("GET", resource_path(kind, namespace), params=params) as resp:
            if resp.status_code == 410:
                raise _Gone()
            _raise_for(resp)
            async for line in resp.aiter_lines():
                if line.strip():
                    yield json.loads(line)

    async def watch(self, kind: str, namespace: Optional[str] = None,
                    resync: Optional[float] = None) -> AsyncIterator[Dict[str, Any]]:
        resync = self.resync if resync is None else resync
        cache: Dict[Tuple[str, str], Obj] = {}
        first = True
        while True:
            lst = await self._list_raw(kind, namespace)
            rv = (lst.get("metadata") or {}).get("resourceVersion", "0")
            seen = set()
            for o in lst.get("items") or []:
                k = _key(o)
                seen.add(k)
                old = cache.get(k)
                cache[k] = o
                if old is None:
                    yield {"type": "ADDED", "object": copy.deepcopy(o), "old": None, "initial": first}
                elif (old.get("metadata") or {}).get("resourceVersion") != (o.get("metadata") or {}).get(
                        "resourceVersion"):
                    yield {"type": "MODIFIED", "object": copy.deepcopy(o), "old": old}
            for k in [k for k in cache if k not in seen]:  # deleted while we were not watching
                yield {"type": "DELETED", "object": cache.pop(k), "old": None}
            first = False
            next_resync = time.monotonic() + resync if resync else None
            try:
                async for ev in self._stream(kind, namespace, rv):
                    et, o = ev.get("type"), ev.get("object") or {}
                    if et == "BOOKMARK":
                        continue
                    if et == "ERROR":
                        if (o.get("code") == 410):
                            raise _Gone()
                        raise ApiError(int(o.get("code", 500)), o.get("reason", "Error"), o.get("message", ""))
                    k = _key(o)
                    if et == "DELETED":
                        cache.pop(k, None)
                        yield {"type": "DELETED", "object": o, "old": None}
                    else:
                        old = cache.get(k)
                        cache[k] = o
                        yield {"type": "ADDED" if old is None else "MODIFIED", "object": copy.deepcopy(o),
                               "old": old}
                    if next_resync is not None and time.monotonic() >= next_resync:
                        for c in list(cache.values()):
                            yield {"type": "MODIFIED", "object": copy.deepcopy(c), "old": c, "resync": True}
                        next_resync = time.monotonic() + resync
            except _Gone:
                pass  # resourceVersion too old: relist and diff
            except (httpx.ReadError, httpx.RemoteProtocolError, httpx.ReadTimeout):
                await asyncio.sleep(1.0)

    # ------------------------------------------------------------------ rollback
    async def rollback(self, namespace: str, name: str, revision: int, message: str = "") -> Obj:
        depl = await self.get("deployments", namespace, name)
        if (depl.get("spec") or {}).get("paused"):
            raise Conflict("you cannot rollback a paused deployment")
        uid = depl["metadata"]["uid"]
        owned = [rs for rs in await self.list("replicasets", namespace)
                 if any(o.get("uid") == uid for o in rs["metadata"].get("ownerReferences", []))]
        if revision == 0:  # previous revision
            cur = revision_of(depl)
            older = sorted((revision_of(rs) for rs in owned if revision_of(rs) < cur), reverse=True)
            if not older:
                raise NotFound(f"no previous revision of {namespace}/{name}")
            revision = older[0]
        target = next((rs for rs in owned if revision_of(rs) == revision), None)
        if target is None:
            raise NotFound(f"revision {revision} of {namespace}/{name}")
        tpl = copy.deepcopy(target["spec"]["template"])
        (tpl.get("metadata") or {}).get("labels", {}).pop("pod-template-hash", None)
        ann = {"deployment.foremast.ai/rollback-id": f"{revision}-{time.time_ns()}"}
        if message:
            ann["deployment.foremast.ai/rollbackMessage"] = message
        patch: Obj = {"spec": {"template": tpl}, "metadata": {"annotations": ann}}
        return await self.patch("deployments", namespace, name, patch)


class _Gone(Exception):
    pass
