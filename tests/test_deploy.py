"""Deployment bundle: generated CRD schemas accept what the controller
writes, recording rules cover every series the query builder reads, the
rendered YAML in deploy/ is current, and the process entrypoints start."""

import asyncio
import os
import subprocess
import sys

import yaml

from foremast_amd.api import crd
from foremast_amd.controller import queries
from foremast_amd.deploy import manifests, rules, schema

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _crd_schema(kind):
    c = next(c for c in schema.crds() if c["spec"]["names"]["kind"] == kind)
    return c["spec"]["versions"][0]["schema"]["openAPIV3Schema"]


def test_crd_schema_required_fields_match_go_tags():
    st = _crd_schema("DeploymentMonitor")["properties"]["status"]
    assert set(st["required"]) == {"phase", "remediationTaken", "timestamp", "expired"}
    spec = _crd_schema("DeploymentMetadata")["properties"]["spec"]
    assert set(spec["required"]) == {"analyst", "metrics"}
    val = st["properties"]["anomaly"]["properties"]["anomalousMetrics"]["items"]["properties"]["values"]
    assert val["items"]["properties"]["time"]["type"] == "integer"


def test_controller_objects_validate_against_crds():
    m = crd.DeploymentMonitor(metadata={"name": "demo", "namespace": "ns"})
    m.status.phase = crd.PHASE_UNHEALTHY
    m.status.timestamp = "2020-01-01T00:00:00Z"
    m.status.anomaly = crd.anomaly_from_flat({"error5xx": {"tags": "", "values": [1577836920, 40.5]}})
    m.spec.remediation.option = crd.REMEDIATION_AUTO_ROLLBACK
    m.spec.rollback_revision = 3
    d = m.to_dict()
    assert schema.validate(d, _crd_schema("DeploymentMonitor")) == []
    bad = dict(d, status={"phase": "Running"})
    assert any("required" in e for e in schema.validate(bad, _crd_schema("DeploymentMonitor")))
    md = manifests.default_metadata()
    assert schema.validate(md, _crd_schema("DeploymentMetadata")) == []


def test_recording_rules_cover_queries():
    names = set(rules.recorded_names())
    md = crd.DeploymentMetadata.from_dict(manifests.default_metadata())
    for mon in md.spec.metrics.monitoring:
        for prefix in ("namespace_pod:", "namespace_app_per_pod:", "namespace_app:"):
            assert prefix + mon.metric_name in names
    q = queries.create_map("ns", "app", ["p1", "p2"], md.spec.metrics, 1000, 1600, "rollingupdate")
    assert q  # the builder produces queries over the recorded families
    for fam in list(rules.HTTP_FAMILIES) + list(rules.RESOURCE_FAMILIES):
        assert f"namespace_app_per_pod:{fam}" in names


def test_rendered_bundle_is_current():
    for rel, docs in manifests.bundle().items():
        path = os.path.join(ROOT, "deploy", "foremast", rel)
        with open(path) as f:
            on_disk = [d for d in yaml.safe_load_all(f) if d is not None]
        assert on_disk == docs, f"{rel} is stale: run `make deploy`"
    brain = manifests.brain()[0]
    c = brain["spec"]["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 8
    env = {e["name"]: e.get("value") for e in c["env"]}
    assert env["ML_ALGORITHM"] == "moving_average_all" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_kubectl_helpers_are_executable():
    for n in ("kubectl-watch", "kubectl-unwatch"):
        p = os.path.join(ROOT, "bin", n)
        assert os.access(p, os.X_OK)
        assert "continuous" in open(p).read()


def test_brain_entrypoint_runs(tmp_path):
    env = dict(os.environ, FOREMAST_JOB_STORE=f"sqlite:///{tmp_path}/jobs.db", PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "-m", "foremast_amd.brain", "--metrics-port", "0", "--run-seconds", "1"],
                         capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]


def test_controller_entrypoint_fake_cluster():
    from foremast_amd.controller import __main__ as cli
    args = cli.parse(["--fake", "--run-seconds", "0.3", "--poll-seconds", "0.05"])
    bm = asyncio.run(cli.run(args))
    assert bm.namespace == "foremast"
