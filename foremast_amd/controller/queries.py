"""PromQL query builder — ``MetricsInfo{current, baseline, historical}``.

Re-implements ``foremast-barrelman/pkg/client/metrics/metricsquery.go:21-127``
with identical PromQL strings and time windows:

* step 60 s; ``nowUnix = floor(now/60)*60``;
* current  = ``[nowUnix+60, floor((now+(W+1)min)/60)*60]`` over the new pods
  (``namespace_pod:<m>{namespace=..,pod=~"a|b"}``) or, for the continuous
  strategy, ``namespace_app_per_pod:<m>{namespace=..,app=..}``;
* baseline = ``[floor((now-W min)/60)*60, nowUnix]`` over the old pods
  (only when there are old pods and the strategy is not rollingUpdate);
* historical = 7 days of ``namespace_app_per_pod:<m>``.

Extension — downstream impact (reference ``README.md:24``): a monitoring entry
with ``metricType: downstream`` reads the per-caller recordings instead
(``namespace_pod_caller:<m>`` / ``namespace_app_caller_per_pod:<m>``, one series
per calling service, ``deploy/rules.py``); the brain scores every caller of the
deployed app separately and names the impacted one in the verdict.
``metricType: api`` does the same per request path (``uri``): anomalies
aggregated at API level (reference ``README.md:26``).
"""

from __future__ import annotations

import time
from typing import Dict, List, Optional, Sequence

from ..api import crd
from ..api import rest as r

STEP = 60
HISTORICAL_DAYS = 7
METRIC_TYPE_DOWNSTREAM = "downstream"
METRIC_TYPE_API = "api"
# metricType -> (per-pod prefix, per-app-per-pod prefix) of the split recordings (deploy/rules.py)
_SPLIT = {METRIC_TYPE_DOWNSTREAM: ("namespace_pod_caller:", "namespace_app_caller_per_pod:"),
          METRIC_TYPE_API: ("namespace_pod_uri:", "namespace_app_uri_per_pod:")}


class QueryError(ValueError):
    pass


def _pod_selector(namespace: str, metric: str, pods: Sequence[str], prefix: str = "namespace_pod:") -> str:
    if len(pods) > 1:
        return (prefix + metric + '{namespace="' + namespace + '",pod=~"'
                + "|".join(pods) + '"}')
    return prefix + metric + '{namespace="' + namespace + '",pod="' + pods[0] + '"}'


def _app_selector(namespace: str, metric: str, app: str, prefix: str = "namespace_app_per_pod:") -> str:
    return prefix + metric + '{namespace="' + namespace + '",app="' + app + '"}'


def create_map(namespace: str, app_name: str, pod_names: Sequence[str], metrics: crd.Metrics,
               category: str, time_window_min: int, strategy: str,
               now: Optional[float] = None) -> Dict[str, r.MetricQuery]:
    now = time.time() if now is None else now
    out: Dict[str, r.MetricQuery] = {}
    for mon in metrics.monitoring:
        pod_pfx, app_pfx = _SPLIT.get((mon.metric_type or "").lower(), ("namespace_pod:", "namespace_app_per_pod:"))
        now_unix = (int(now) // STEP) * STEP
        before = (int(now - time_window_min * 60) // STEP) * STEP
        p: Dict[str, object] = {"endpoint": metrics.endpoint, "step": STEP}
        if category == r.CATEGORY_CURRENT:
            p["start"] = now_unix + STEP
            p["end"] = (int(now + (time_window_min + 1) * 60) // STEP) * STEP
            if strategy == r.STRATEGY_CONTINUOUS:
                p["query"] = _app_selector(namespace, mon.metric_name, app_name, app_pfx)
            else:
                if not pod_names:
                    raise QueryError("No valid pod names")
                p["query"] = _pod_selector(namespace, mon.metric_name, pod_names, pod_pfx)
        elif category == r.CATEGORY_BASELINE:
            if not pod_names:
                raise QueryError("No valid pod names")
            p["start"] = before
            p["end"] = now_unix
            p["query"] = _pod_selector(namespace, mon.metric_name, pod_names, pod_pfx)
        elif category == r.CATEGORY_HISTORICAL:
            t = now - HISTORICAL_DAYS * 24 * 3600
            p["start"] = (int(t) // STEP) * STEP
            p["end"] = now_unix
            p["query"] = _app_selector(namespace, mon.metric_name, app_name, app_pfx)
        out[mon.metric_alias] = r.MetricQuery(data_source_type=metrics.data_source_type,
                                              parameters=p)
    return out


def create_metrics_info(namespace: str, app_name: str, pod_names: List[List[str]],
                        metrics: crd.Metrics, time_window_min: int, strategy: str,
                        now: Optional[float] = None) -> r.MetricsInfo:
    """``CreateMetricsInfo`` (``metricsquery.go:91-127``)."""
    if strategy != r.STRATEGY_CONTINUOUS and len(pod_names) == 0:
        raise QueryError("No valid pod names")
    if metrics.data_source_type != r.DATASOURCE_PROMETHEUS:
        raise QueryError("Unsupported DataSourceType:" + metrics.data_source_type)
    pods: List[str] = [] if strategy == r.STRATEGY_CONTINUOUS else list(pod_names[0])
    info = r.MetricsInfo(current=create_map(namespace, app_name, pods, metrics,
                                            r.CATEGORY_CURRENT, time_window_min, strategy, now))
    if strategy != r.STRATEGY_ROLLING_UPDATE and len(pod_names) > 1 and pod_names[1]:
        info.baseline = create_map(namespace, app_name, pod_names[1], metrics,
                                   r.CATEGORY_BASELINE, time_window_min, strategy, now)
    info.historical = create_map(namespace, app_name, pods, metrics, r.CATEGORY_HISTORICAL,
                                 time_window_min, strategy, now)
    return info
