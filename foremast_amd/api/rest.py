"""foremast-service REST wire format.

Mirrors ``foremast-service/pkg/models/models.go:6-146`` and the barrelman
side ``foremast-barrelman/pkg/client/analyst/analystclient.go:27-61``.

Compatibility decisions:

* Q2 — ``GET /id/:id`` returns the ``anomaly`` map (the reference service
  drops it, ``converter.go:48-61``).
* Q3 — anomaly ``values`` are emitted as JSON numbers that are floats when
  the value is fractional (barrelman decodes ``[]float64``; the service
  declared ``[]int64``).
* Q11 — fields whose Go tag was malformed (``json:"x",omitempty``) are always
  emitted, exactly as Go does.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List, Optional

from .gojson import from_go, gofield, to_go

CATEGORY_CURRENT = "current"
CATEGORY_BASELINE = "baseline"
CATEGORY_HISTORICAL = "historical"
CATEGORIES = (CATEGORY_CURRENT, CATEGORY_BASELINE, CATEGORY_HISTORICAL)

STRATEGY_ROLLING_UPDATE = "rollingUpdate"
STRATEGY_CANARY = "canary"
STRATEGY_CONTINUOUS = "continuous"
STRATEGIES = (STRATEGY_ROLLING_UPDATE, STRATEGY_CANARY, STRATEGY_CONTINUOUS)

DATASOURCE_PROMETHEUS = "prometheus"
DATASOURCE_WAVEFRONT = "wavefront"


@dataclass
class MetricQuery:
    data_source_type: str = gofield("dataSourceType", default="")
    parameters: Dict[str, Any] = gofield("parameters", omitempty=True, default_factory=dict)


@dataclass
class MetricsInfo:
    current: Dict[str, MetricQuery] = gofield("current", default=None)
    baseline: Dict[str, MetricQuery] = gofield("baseline", omitempty=True, default=None)
    historical: Dict[str, MetricQuery] = gofield("historical", omitempty=True, default=None)


@dataclass
class ApplicationHealthAnalyzeRequest:
    app_name: str = gofield("appName", default="")
    start_time: str = gofield("startTime", default="")
    end_time: str = gofield("endTime", default="")
    metrics: MetricsInfo = gofield("metrics", default_factory=MetricsInfo)
    strategy: str = gofield("strategy", default="")

    def to_dict(self) -> Dict[str, Any]:
        return to_go(self)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "ApplicationHealthAnalyzeRequest":
        return from_go(cls, d)


@dataclass
class AnomalyInfo:
    tags: str = gofield("tags", default="")
    values: List[float] = gofield("values", default=None)


@dataclass
class ApplicationHealthAnalyzeResponse:
    """Status response (``models.go:66-72``; field order as in Go)."""

    job_id: str = gofield("jobId", default="")
    status_code: int = gofield("statusCode", default=0)
    status: str = gofield("status", default="")
    reason: str = gofield("reason", omitempty=True, default="")
    anomaly: Optional[Dict[str, AnomalyInfo]] = gofield("anomaly", default=None)

    def to_dict(self) -> Dict[str, Any]:
        d = to_go(self)
        if d.get("anomaly"):
            for info in d["anomaly"].values():
                info["values"] = [_num(v) for v in (info.get("values") or [])]
        return d

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "ApplicationHealthAnalyzeResponse":
        return from_go(cls, d)


@dataclass
class ApplicationHealthAnalyzeResponseNew:
    """Create response (``models.go:75-80``)."""

    job_id: str = gofield("jobId", default="")
    status_code: int = gofield("statusCode", default=0)
    status: str = gofield("status", default="")
    reason: str = gofield("reason", omitempty=True, default="")

    def to_dict(self) -> Dict[str, Any]:
        return to_go(self)


def _num(v: Any) -> Any:
    """Emit integral floats as ints (timestamps) and keep fractional values."""
    if isinstance(v, float) and v.is_integer() and abs(v) < 2 ** 53:
        return int(v)
    return v


# ----------------------------------------------------------------------------------
# Job document (Elasticsearch index "documents", type "document").
# ----------------------------------------------------------------------------------

ES_INDEX = "documents"
ES_TYPE = "document"

# Internal job statuses (converter.go:12-29 + the brain state diagram).
ST_INITIAL = "initial"
ST_PREPROCESS_INPROGRESS = "preprocess_inprogress"
ST_PREPROCESS_COMPLETED = "preprocess_completed"
ST_POSTPROCESS_INPROGRESS = "postprocess_inprogress"
ST_REPROGRESS = "reprogress"
ST_COMPLETED_HEALTH = "completed_health"
ST_COMPLETED_UNHEALTH = "completed_unhealth"
ST_COMPLETED_UNKNOWN = "completed_unknown"
ST_PREPROCESS_FAILED = "preprocess_failed"
ST_ABORT = "abort"

OPEN_STATUSES = (ST_INITIAL, ST_REPROGRESS)
INPROGRESS_STATUSES = (ST_PREPROCESS_INPROGRESS, ST_POSTPROCESS_INPROGRESS,
                       ST_PREPROCESS_COMPLETED)
TERMINAL_STATUSES = (ST_COMPLETED_HEALTH, ST_COMPLETED_UNHEALTH, ST_COMPLETED_UNKNOWN,
                     ST_PREPROCESS_FAILED, ST_ABORT)

DOCUMENT_FIELDS = (
    "id", "appName", "created_at", "startTime", "endTime", "modified_at",
    "currentConfig", "baselineConfig", "historicalConfig",
    "currentMetricStore", "baselineMetricStore", "historicalMetricStore",
    "status", "statusCode", "strategy", "reason", "processingContent", "anomalyInfo",
)


@dataclass
class DocumentRequest:
    """``models.go:104-116``; field order defines the job-id hash input."""

    app_name: str = ""
    start_time: str = ""
    end_time: str = ""
    current_config: str = ""
    baseline_config: str = ""
    historical_config: str = ""
    current_metric_store: str = ""
    baseline_metric_store: str = ""
    historical_metric_store: str = ""
    status_code: str = "200"
    strategy: str = ""

    def hash_input(self) -> str:
        """``elasticsearchstore.go:152-166`` ConvertDocumentRequestToString
        (statusCode is deliberately not part of it)."""
        return (self.app_name + self.start_time + self.end_time + self.current_config
                + self.baseline_config + self.historical_config + self.current_metric_store
                + self.baseline_metric_store + self.historical_metric_store + self.strategy)
