"""The deployment bundle as data (rendered to YAML by ``python -m foremast_amd.deploy``).

Mirrors the reference's ``deploy/foremast`` layout — namespace, CRDs,
barrelman (+RBAC, default DeploymentMetadata, recording rules), job store,
service, brain — with the MI355X brain: one pod per 8-GPU node running one
scorer process per GPU (``torchrun --nproc-per-node 8``), ``amd.com/gpu``
resources, the reference's brain environment block verbatim
(:func:`~foremast_amd.utils.config.reference_default_env`) and the
``:8000`` metrics port scraped by a ServiceMonitor.
"""

from __future__ import annotations

from typing import Any, Dict, List

from ..api import crd
from ..utils.config import reference_default_env
from . import rules, schema

NS = "foremast"
IMAGE = "foremast-amd:latest"
SERVICE_URL = f"http://foremast-service.{NS}.svc.cluster.local:8099"
ES_URL = f"http://elasticsearch-discovery.{NS}.svc.cluster.local:9200"
PROM_URL = "http://prometheus-k8s.monitoring.svc.cluster.local:9090/"


def _labels(app: str) -> Dict[str, str]:
    return {"app": app, "app.kubernetes.io/part-of": "foremast"}


def namespace() -> Dict[str, Any]:
    return {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": NS}}


def barrelman_rbac() -> List[Dict[str, Any]]:
    group = crd.API_VERSION.split("/")[0]
    return [
        {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "foremast-barrelman", "namespace": NS}},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
         "metadata": {"name": "foremast-barrelman"},
         "rules": [
             {"apiGroups": ["apps"], "resources": ["deployments"],
              "verbs": ["get", "list", "watch", "update", "patch"]},
             {"apiGroups": ["apps"], "resources": ["replicasets"], "verbs": ["get", "list", "watch"]},
             {"apiGroups": [""], "resources": ["pods", "namespaces"], "verbs": ["get", "list", "watch"]},
             {"apiGroups": [""], "resources": ["events"], "verbs": ["create", "patch"]},
             {"apiGroups": [group], "resources": ["deploymentmonitors", "deploymentmetadatas",
                                                  "deploymentmonitors/status"],
              "verbs": ["get", "list", "watch", "create", "update", "patch", "delete"]},
         ]},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
         "metadata": {"name": "foremast-barrelman"},
         "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "foremast-barrelman"},
         "subjects": [{"kind": "ServiceAccount", "name": "foremast-barrelman", "namespace": NS}]},
    ]


def _deployment(name: str, containers: List[Dict[str, Any]], replicas: int = 1, sa: str = None,
                extra_spec: Dict[str, Any] = None) -> Dict[str, Any]:
    pod_spec: Dict[str, Any] = {"containers": containers}
    if sa:
        pod_spec["serviceAccountName"] = sa
    pod_spec.update(extra_spec or {})
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": name, "namespace": NS, "labels": _labels(name)},
            "spec": {"replicas": replicas, "selector": {"matchLabels": {"app": name}},
                     "template": {"metadata": {"labels": _labels(name)}, "spec": pod_spec}}}


def _service(name: str, port: int, target: int = None, port_name: str = "http") -> Dict[str, Any]:
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name, "namespace": NS, "labels": _labels(name)},
            "spec": {"selector": {"app": name}, "ports": [{"name": port_name, "port": port,
                                                           "targetPort": target or port}]}}


def _probe(path: str, port: int) -> Dict[str, Any]:
    return {"httpGet": {"path": path, "port": port}, "initialDelaySeconds": 10, "periodSeconds": 10}


def barrelman() -> List[Dict[str, Any]]:
    c = {"name": "barrelman", "image": IMAGE, "command": ["python", "-m", "foremast_amd.controller"],
         "env": [{"name": "NAMESPACE", "valueFrom": {"fieldRef": {"fieldPath": "metadata.namespace"}}}],
         "resources": {"requests": {"cpu": "100m", "memory": "128Mi"}, "limits": {"memory": "512Mi"}}}
    return barrelman_rbac() + [_deployment("foremast-barrelman", [c], sa="foremast-barrelman")]


def default_metadata() -> Dict[str, Any]:
    """``spring-boot`` appType defaults (reference C29): the 5xx error rate."""
    m = crd.DeploymentMetadata(metadata={"name": "spring-boot", "namespace": NS})
    m.spec.analyst.endpoint = SERVICE_URL + "/v1/healthcheck/"
    m.spec.metrics.data_source_type = "prometheus"
    m.spec.metrics.endpoint = PROM_URL + "api/v1/"
    m.spec.metrics.monitoring = [crd.Monitoring(metric_name="http_server_requests_error_5xx",
                                                metric_type="counter", metric_alias="error5xx")]
    d = m.to_dict()
    d.pop("status", None)
    return d


def elasticsearch() -> List[Dict[str, Any]]:
    c = {"name": "elasticsearch", "image": "docker.elastic.co/elasticsearch/elasticsearch-oss:6.8.23",
         "env": [{"name": "discovery.type", "value": "single-node"},
                 {"name": "ES_JAVA_OPTS", "value": "-Xms512m -Xmx512m"}],
         "ports": [{"containerPort": 9200}],
         "resources": {"requests": {"memory": "1Gi"}, "limits": {"memory": "2Gi"}}}
    return [_deployment("elasticsearch", [c]),
            {**_service("elasticsearch", 9200), "metadata": {"name": "elasticsearch-discovery", "namespace": NS}}]


def service() -> List[Dict[str, Any]]:
    c = {"name": "foremast-service", "image": IMAGE, "command": ["python", "-m", "foremast_amd.service"],
         "env": [{"name": "ELASTIC_URL", "value": ES_URL}, {"name": "QUERY_SERVICE_ENDPOINT", "value": PROM_URL}],
         "ports": [{"containerPort": 8099}],
         "readinessProbe": _probe("/healthz", 8099), "livenessProbe": _probe("/healthz", 8099)}
    return [_deployment("foremast-service", [c], replicas=2), _service("foremast-service", 8099)]


def brain(gpus: int = 8) -> List[Dict[str, Any]]:
    env = [{"name": k, "value": v} for k, v in reference_default_env().items()]
    env += [{"name": "ES_ENDPOINT", "value": ES_URL}, {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"},
            {"name": "FOREMAST_DTYPE", "value": "bf16"},
            # resident engines: continuous (streaming) + canary / rollingUpdate (rollout) jobs on the GPUs
            {"name": "FOREMAST_STREAMING", "value": "1"}, {"name": "FOREMAST_ROLLOUT", "value": "1"},
            # "reference": the reference brain's per-point thresholds (no window correction, one point
            # outside the lowered band fires, one-step sigma); "engine" (default): docs/SCORING.md
            {"name": "FOREMAST_DETECTION_PRESET", "value": "engine"}]
    c = {"name": "foremast-brain", "image": IMAGE,
         "command": ["python", "-m", "torch.distributed.run", "--standalone", f"--nproc-per-node={gpus}",
                     "-m", "foremast_amd.brain"],
         "env": env, "ports": [{"containerPort": 8000 + r, "name": f"metrics-{r}"} for r in range(gpus)],
         "resources": {"limits": {"amd.com/gpu": gpus, "memory": "256Gi"}, "requests": {"cpu": "16"}}}
    # one exposition port per scorer rank (8000 + LOCAL_RANK)
    svc = _service("foremast-brain", 8000, port_name="metrics-0")
    svc["spec"]["ports"] = [{"name": f"metrics-{r}", "port": 8000 + r, "targetPort": 8000 + r} for r in range(gpus)]
    monitor = {"apiVersion": "monitoring.coreos.com/v1", "kind": "ServiceMonitor",
               "metadata": {"name": "foremast-brain", "namespace": NS, "labels": _labels("foremast-brain")},
               "spec": {"selector": {"matchLabels": {"app": "foremast-brain"}},
                        "endpoints": [{"port": f"metrics-{r}", "interval": "15s"} for r in range(gpus)]}}
    return [_deployment("foremast-brain", [c], extra_spec={"tolerations": [
        {"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}]}), svc, monitor]


def bundle() -> Dict[str, List[Dict[str, Any]]]:
    """file name → documents (numbered like the reference's apply order)."""
    return {
        "00_namespace.yaml": [namespace()],
        "1_crds/crds.yaml": schema.crds(),
        "2_barrelman/barrelman.yaml": barrelman(),
        "2_barrelman/deployment-metadata-default.yaml": [default_metadata()],
        "2_barrelman/metrics-rules.yaml": [rules.prometheus_rule()],
        "3_brain/elasticsearch.yaml": elasticsearch(),
        "3_brain/foremast-service.yaml": service(),
        "3_brain/foremast-brain.yaml": brain(),
        # opt-in, Kubernetes >= 1.31: field selectors on status.jobId / status.phase
        "../optional/crds-selectable.yaml": schema.crds(selectable=True),
    }
