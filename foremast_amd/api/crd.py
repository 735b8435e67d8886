"""CRD types: ``DeploymentMetadata`` and ``DeploymentMonitor``.

Group/version ``deployment.foremast.ai/v1alpha1`` — field names, omitempty
behaviour and the phase / remediation constants mirror
``foremast-barrelman/pkg/apis/deployment/v1alpha1/types.go:14-305`` so that
objects written by this framework are readable by the reference barrelman
and vice versa.  ``ObjectMeta`` / ``LabelSelector`` are kept as plain dicts
(they are Kubernetes-owned types).
"""

from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

from .gojson import from_go, gofield, to_go

GROUP = "deployment.foremast.ai"
VERSION = "v1alpha1"
API_VERSION = f"{GROUP}/{VERSION}"
PLURAL_MONITOR = "deploymentmonitors"
PLURAL_METADATA = "deploymentmetadatas"
KIND_MONITOR = "DeploymentMonitor"
KIND_METADATA = "DeploymentMetadata"

# Phases (types.go:241-255)
PHASE_HEALTHY = "Healthy"
PHASE_RUNNING = "Running"
PHASE_FAILED = "Failed"
PHASE_UNHEALTHY = "Unhealthy"
PHASE_WARNING = "Warning"
PHASE_EXPIRED = "Expired"
PHASE_ABORT = "Abort"
PHASES = (PHASE_HEALTHY, PHASE_RUNNING, PHASE_FAILED, PHASE_UNHEALTHY,
          PHASE_WARNING, PHASE_EXPIRED, PHASE_ABORT)

# Remediation options (types.go:258-269)
REMEDIATION_NONE = "None"
REMEDIATION_AUTO_ROLLBACK = "AutoRollback"
REMEDIATION_AUTO_PAUSE = "AutoPause"
REMEDIATION_AUTO = "Auto"
REMEDIATIONS = (REMEDIATION_NONE, REMEDIATION_AUTO_ROLLBACK, REMEDIATION_AUTO_PAUSE,
                REMEDIATION_AUTO)

# Annotations / naming (Barrelman.go:56-62, MonitorController.go:168)
ANNOTATION_DEPLOYMENT_NAME = "deployment.kubernetes.io/name"
# set by our rollback on the Deployment (a fresh value per rollback): the
# rollout it triggers is the remediation itself and must not start a new job
ANNOTATION_ROLLBACK_ID = "deployment.foremast.ai/rollback-id"
ANNOTATION_STRATEGY = "deployment.foremast.ai/strategy"
ANNOTATION_MONITORING = "foremast.ai/monitoring"
ANNOTATION_ROLLBACK_MESSAGE = "deployment.foremast.ai/rollbackMessage"
ANNOTATION_REVISION = "deployment.kubernetes.io/revision"
CANARY_SUFFIX = "-foremast-canary"


@dataclass
class Analyst:
    endpoint: str = gofield("endpoint", default="")
    version: str = gofield("version", omitempty=True, default="")


@dataclass
class ImageSpec:
    src: str = gofield("src", default="")
    size: str = gofield("size", omitempty=True, default="")
    type: str = gofield("type", omitempty=True, default="")


@dataclass
class ContactData:
    name: str = gofield("name", omitempty=True, default="")
    url: str = gofield("url", omitempty=True, default="")
    email: str = gofield("email", omitempty=True, default="")


@dataclass
class Link:
    description: str = gofield("description", omitempty=True, default="")
    url: str = gofield("url", omitempty=True, default="")


@dataclass
class Descriptor:
    type: str = gofield("type", omitempty=True, default="")
    version: str = gofield("version", omitempty=True, default="")
    description: str = gofield("description", omitempty=True, default="")
    icons: List[ImageSpec] = gofield("icons", omitempty=True, default_factory=list)
    maintainers: List[ContactData] = gofield("maintainers", omitempty=True, default_factory=list)
    owners: List[ContactData] = gofield("owners", omitempty=True, default_factory=list)
    keywords: List[str] = gofield("keywords", omitempty=True, default_factory=list)
    links: List[Link] = gofield("links", omitempty=True, default_factory=list)
    notes: str = gofield("notes", omitempty=True, default="")


@dataclass
class Monitoring:
    metric_name: str = gofield("metricName", default="")
    metric_type: str = gofield("metricType", omitempty=True, default="")
    metric_alias: str = gofield("metricAlias", default="")


@dataclass
class Metrics:
    data_source_type: str = gofield("dataSourceType", default="")
    endpoint: str = gofield("endpoint", default="")
    monitoring: List[Monitoring] = gofield("monitoring", omitempty=True, default_factory=list)


@dataclass
class Logs:
    log_name: str = gofield("logName", default="")
    log_type: str = gofield("logType", default="")
    file_pattern: str = gofield("filePattern", omitempty=True, default="")


@dataclass
class DeploymentMetadataSpec:
    analyst: Analyst = gofield("analyst", default_factory=Analyst)
    description: str = gofield("description", omitempty=True, default="")
    metrics: Metrics = gofield("metrics", default_factory=Metrics)
    logs: List[Logs] = gofield("logs", omitempty=True, default_factory=list)
    descriptor: Descriptor = gofield("descriptor", omitempty=True, default_factory=Descriptor)


@dataclass
class DeploymentMetadataStatus:
    observed_generation: int = gofield("observedGeneration", omitempty=True, default=0)


@dataclass
class RemediationAction:
    option: str = gofield("option", default="")
    parameters: Dict[str, str] = gofield("parameters", omitempty=True, default_factory=dict)


@dataclass
class AnomalousMetricValue:
    time: int = gofield("time", default=0)
    value: float = gofield("value", default=0.0)


@dataclass
class AnomalousMetric:
    name: str = gofield("name", default="")
    tags: str = gofield("tags", omitempty=True, default="")
    values: List[AnomalousMetricValue] = gofield("values", default_factory=list)


@dataclass
class Anomaly:
    anomalous_metrics: List[AnomalousMetric] = gofield("anomalousMetrics", omitempty=True,
                                                       default_factory=list)


@dataclass
class DeploymentMonitorSpec:
    selector: Optional[Dict[str, Any]] = gofield("selector", omitempty=True, default=None)
    analyst: Analyst = gofield("analyst", omitempty=True, default_factory=Analyst)
    start_time: str = gofield("startTime", omitempty=True, default="")
    wait_until: str = gofield("waitUntil", omitempty=True, default="")
    metrics: Metrics = gofield("metrics", omitempty=True, default_factory=Metrics)
    logs: List[Logs] = gofield("logs", omitempty=True, default_factory=list)
    continuous: bool = gofield("continuous", omitempty=True, default=False)
    remediation: RemediationAction = gofield("remediation", omitempty=True,
                                             default_factory=RemediationAction)
    rollback_revision: int = gofield("rollbackRevision", omitempty=True, default=0)


@dataclass
class DeploymentMonitorStatus:
    observed_generation: int = gofield("observedGeneration", omitempty=True, default=0)
    job_id: str = gofield("jobId", omitempty=True, default="")
    phase: str = gofield("phase", default="")
    remediation_taken: bool = gofield("remediationTaken", default=False)
    anomaly: Anomaly = gofield("anomaly", omitempty=True, default_factory=Anomaly)
    timestamp: str = gofield("timestamp", default="")
    expired: bool = gofield("expired", default=False)


def _meta_default() -> Dict[str, Any]:
    return {}


@dataclass
class _Object:
    """Common envelope: TypeMeta (inline) + ObjectMeta as a plain dict."""

    metadata: Dict[str, Any] = field(default_factory=_meta_default)

    # --- ObjectMeta convenience --------------------------------------------------
    @property
    def name(self) -> str:
        return self.metadata.get("name", "")

    @property
    def namespace(self) -> str:
        return self.metadata.get("namespace", "")

    @property
    def annotations(self) -> Dict[str, str]:
        return self.metadata.setdefault("annotations", {})

    @property
    def labels(self) -> Dict[str, str]:
        return self.metadata.setdefault("labels", {})

    @property
    def resource_version(self) -> str:
        return self.metadata.get("resourceVersion", "")

    def deepcopy(self):
        return copy.deepcopy(self)


@dataclass
class DeploymentMetadata(_Object):
    spec: DeploymentMetadataSpec = field(default_factory=DeploymentMetadataSpec)
    status: DeploymentMetadataStatus = field(default_factory=DeploymentMetadataStatus)

    def to_dict(self) -> Dict[str, Any]:
        d = {"apiVersion": API_VERSION, "kind": KIND_METADATA,
             "metadata": copy.deepcopy(self.metadata), "spec": to_go(self.spec)}
        st = to_go(self.status)
        d["status"] = st
        return d

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "DeploymentMetadata":
        return cls(metadata=copy.deepcopy(d.get("metadata") or {}),
                   spec=from_go(DeploymentMetadataSpec, d.get("spec")),
                   status=from_go(DeploymentMetadataStatus, d.get("status")))


@dataclass
class DeploymentMonitor(_Object):
    spec: DeploymentMonitorSpec = field(default_factory=DeploymentMonitorSpec)
    status: DeploymentMonitorStatus = field(default_factory=DeploymentMonitorStatus)

    def to_dict(self) -> Dict[str, Any]:
        return {"apiVersion": API_VERSION, "kind": KIND_MONITOR,
                "metadata": copy.deepcopy(self.metadata), "spec": to_go(self.spec),
                "status": to_go(self.status)}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "DeploymentMonitor":
        return cls(metadata=copy.deepcopy(d.get("metadata") or {}),
                   spec=from_go(DeploymentMonitorSpec, d.get("spec")),
                   status=from_go(DeploymentMonitorStatus, d.get("status")))


def anomaly_from_flat(anomaly_info: Dict[str, Dict[str, Any]]) -> Anomaly:
    """Convert the analyst's ``{alias: {tags, values: [t0, v0, t1, v1, ...]}}``
    into the CRD ``Anomaly`` (``Barrelman.go:593-620`` ``convertToAnomaly``).

    Aliases are visited in sorted order (Go iterates maps randomly; sorting
    makes the CRD status deterministic).  A trailing unpaired time is dropped,
    as in the reference.
    """
    out = Anomaly(anomalous_metrics=[])
    for key in sorted(anomaly_info):
        value = anomaly_info[key] or {}
        m = AnomalousMetric(name=key, tags=value.get("tags", "") or "", values=[])
        vals = value.get("values") or []
        t = None
        for i, v in enumerate(vals):
            if i % 2 == 1:
                m.values.append(AnomalousMetricValue(time=int(t), value=float(v)))
            else:
                t = v
        out.anomalous_metrics.append(m)
    return out
