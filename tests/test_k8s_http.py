"""HttpKube (REST client + informer-style watch) against the fake API server
over a real socket (uvicorn on 127.0.0.1)."""

import asyncio
import socket
import threading
import time

import pytest

from foremast_amd.k8s.api import AlreadyExists, Conflict, NotFound, revision_of
from foremast_amd.k8s.fake import FakeCluster
from foremast_amd.k8s.fake_apiserver import create_apiserver
from foremast_amd.k8s.http import HttpKube, KubeConfig, resource_path


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture()
def apiserver():
    import uvicorn
    cluster = FakeCluster()
    app = create_apiserver(cluster)
    port = _free_port()
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="error"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    t0 = time.time()
    while not server.started and time.time() - t0 < 20:
        time.sleep(0.05)
    assert server.started
    yield f"http://127.0.0.1:{port}", app
    server.should_exit = True
    th.join(timeout=10)


def _depl(ns, name, image):
    tpl = {"metadata": {"labels": {"app": name}}, "spec": {"containers": [{"name": name, "image": image}]}}
    return {"metadata": {"name": name, "namespace": ns, "labels": {"app": name}},
            "spec": {"replicas": 1, "selector": {"matchLabels": {"app": name}}, "template": tpl}, "status": {}}


def test_resource_paths():
    assert resource_path("pods", "ns") == "/api/v1/namespaces/ns/pods"
    assert resource_path("namespaces", None, "ns") == "/api/v1/namespaces/ns"
    assert resource_path("deployments", "ns", "d") == "/apis/apps/v1/namespaces/ns/deployments/d"
    assert resource_path("deploymentmonitors", "ns") == \
        "/apis/deployment.foremast.ai/v1alpha1/namespaces/ns/deploymentmonitors"


def test_kubeconfig_parsing(tmp_path):
    import base64
    cfg = tmp_path / "config"
    cfg.write_text(f"""
apiVersion: v1
current-context: c1
contexts: [{{name: c1, context: {{cluster: k1, user: u1}}}}]
clusters: [{{name: k1, cluster: {{server: "https://10.0.0.1:6443",
  certificate-authority-data: "{base64.b64encode(b'CA').decode()}"}}}}]
users: [{{name: u1, user: {{token: abc}}}}]
""")
    kc = KubeConfig.from_kubeconfig(str(cfg))
    assert kc.server == "https://10.0.0.1:6443" and kc.token == "abc"
    assert open(kc.ca_file, "rb").read() == b"CA"


def test_http_crud_watch_rollback(apiserver):
    base, app = apiserver

    async def run():
        kube = HttpKube(base_url=base, resync=None)
        try:
            await kube.create("namespaces", {"metadata": {"name": "demo"}})
            assert [n["metadata"]["name"] for n in await kube.list("namespaces")] == ["demo"]
            events = []

            async def watcher():
                async for ev in kube.watch("deployments", "demo"):
                    events.append(ev)

            wt = asyncio.create_task(watcher())
            await asyncio.sleep(0.3)
            d = await kube.create("deployments", _depl("demo", "web", "web:1"))
            with pytest.raises(AlreadyExists):
                await kube.create("deployments", _depl("demo", "web", "web:1"))
            with pytest.raises(NotFound):
                await kube.get("deployments", "demo", "nope")
            stale = dict(d)
            d2 = await kube.patch("deployments", "demo", "web",
                                  {"spec": {"template": {"spec": {"containers": [{"name": "web", "image": "web:2"}]}}}})
            with pytest.raises(Conflict):
                await kube.update("deployments", stale)
            assert revision_of(d2) == 2 or revision_of(await kube.get("deployments", "demo", "web")) == 2
            rs = await kube.list("replicasets", "demo", "app=web")
            assert sorted(revision_of(r) for r in rs) == [1, 2]
            back = await kube.rollback("demo", "web", 0, "foremast: unhealthy")
            assert back["spec"]["template"]["spec"]["containers"][0]["image"] == "web:1"
            assert back["metadata"]["annotations"]["deployment.foremast.ai/rollbackMessage"] == "foremast: unhealthy"
            mon = await kube.create("deploymentmonitors", {"metadata": {"name": "web", "namespace": "demo"},
                                                           "spec": {"continuous": False}, "status": {}})
            assert mon["apiVersion"] == "deployment.foremast.ai/v1alpha1"
            await kube.delete("deployments", "demo", "web")
            for _ in range(100):
                if any(e["type"] == "DELETED" for e in events):
                    break
                await asyncio.sleep(0.05)
            wt.cancel()
            types = [e["type"] for e in events]
            assert types[0] == "ADDED" and "MODIFIED" in types and types[-1] == "DELETED"
            mod = next(e for e in events if e["type"] == "MODIFIED")
            assert mod["old"] is not None and mod["old"]["metadata"]["name"] == "web"
        finally:
            await kube.aclose()

    asyncio.run(run())


def test_watch_relists_after_gone(apiserver):
    base, app = apiserver

    async def run():
        kube = HttpKube(base_url=base)
        try:
            await kube.create("namespaces", {"metadata": {"name": "ns"}})
            await kube.create("deployments", _depl("ns", "a", "a:1"))
            app.state.watch_state["min_rv"] = 10 ** 9  # every watch answers 410 Gone → relist loop
            seen = []
            agen = kube.watch("deployments", "ns")
            ev = await asyncio.wait_for(agen.__anext__(), 10)
            seen.append(ev)
            app.state.watch_state["min_rv"] = 0
            await kube.create("deployments", _depl("ns", "b", "b:1"))
            ev = await asyncio.wait_for(agen.__anext__(), 10)
            seen.append(ev)
            await agen.aclose()
            assert seen[0]["initial"] and seen[0]["object"]["metadata"]["name"] == "a"
            assert seen[1]["type"] == "ADDED" and seen[1]["object"]["metadata"]["name"] == "b"
        finally:
            await kube.aclose()

    asyncio.run(run())


def test_field_selectors_status_job_id_and_phase():
    """The reference's DeploymentMonitor field labels (v1alpha1/register.go:38-53):
    status.jobId / status.phase filter lists on the fake cluster and through the
    REST client + fake API server; other fields are a 400; the generated CRD
    declares them as selectableFields."""
    import asyncio
    import httpx
    from foremast_amd.deploy import schema
    from foremast_amd.k8s.api import ApiError
    from foremast_amd.k8s.fake import FakeCluster
    from foremast_amd.k8s.fake_apiserver import create_apiserver as apiserver
    from foremast_amd.k8s.http import HttpKube
    kube = FakeCluster()
    kube.add_namespace("a")
    for i, phase in enumerate(("Running", "Healthy", "Running")):
        kube.create_sync("deploymentmonitors", {"metadata": {"name": f"m{i}", "namespace": "a"},
                                                "status": {"jobId": f"j{i}", "phase": phase}})
    names = lambda objs: [o["metadata"]["name"] for o in objs]  # noqa: E731
    assert names(kube.list_sync("deploymentmonitors", field_selector="status.phase=Running")) == ["m0", "m2"]
    assert names(kube.list_sync("deploymentmonitors", field_selector="status.phase!=Running")) == ["m1"]
    assert names(kube.list_sync("deploymentmonitors", field_selector="status.jobId==j2,status.phase=Running")) == ["m2"]
    with pytest.raises(ApiError) as e:
        kube.list_sync("deploymentmonitors", field_selector="spec.continuous=true")
    assert e.value.code == 400

    async def go():
        client = HttpKube(base_url="http://k8s", transport=httpx.ASGITransport(app=apiserver(kube)))
        got = await client.list("deploymentmonitors", "a", field_selector="status.jobId=j1")
        assert names(got) == ["m1"]
        with pytest.raises(ApiError):
            await client.list("deploymentmonitors", "a", field_selector="status.bogus=1")
    asyncio.run(go())
    assert all("selectableFields" not in c["spec"]["versions"][0] for c in schema.crds())  # any k8s version
    dm = [c for c in schema.crds(selectable=True) if c["spec"]["names"]["kind"] == "DeploymentMonitor"][0]
    assert dm["spec"]["versions"][0]["selectableFields"] == [{"jsonPath": ".status.jobId"},
                                                             {"jsonPath": ".status.phase"}]
