"""Prometheus recording rules the query builder depends on.

Every Foremast query reads a *recorded* series at one of three levels
(``foremast_amd/controller/queries.py``; reference ``metricsquery.go``):
``namespace_pod:<m>`` (current/baseline pods), ``namespace_app_per_pod:<m>``
(continuous + 7-day history) and ``namespace_app:<m>``.  The reference
ships these as a hand-written PrometheusRule
(``deploy/foremast/2_barrelman/metrics-rules-default.yaml``); here they are
generated from one table of metric families so every family exists at all
three levels and the per-pod level is always ``app / pod_count``.
"""

from __future__ import annotations

from typing import Dict, List, Tuple

HTTP = "http_server_requests_seconds"

# family -> (instant selector body over the app's request metrics, kind)
# "rate" families sum per-second rates; "ratio" divides two rates (latency).
HTTP_FAMILIES: Dict[str, Tuple[str, str]] = {
    "http_server_requests_error_4xx": (f'{HTTP}_count{{status=~"4[0-9]+"}}', "rate"),
    "http_server_requests_error_5xx": (f'{HTTP}_count{{status=~"5[0-9]+"}}', "rate"),
    "http_server_requests_errors": (f'{HTTP}_count{{status=~"[4-5][0-9]+"}}', "rate"),
    "http_server_requests_2xx": (f'{HTTP}_count{{status=~"2[0-9]+"}}', "rate"),
    "http_server_requests_count": (f"{HTTP}_count", "rate"),
    "http_server_requests_latency": (f'{HTTP}_sum{{status="200"}}|{HTTP}_count{{status="200"}}', "ratio"),
}

# container resource families (cAdvisor, kubelet job; k8s >= 1.16 label names)
RESOURCE_FAMILIES: Dict[str, str] = {
    "cpu_usage_seconds_total":
        'rate(container_cpu_usage_seconds_total{job="kubelet", image!="", container!=""}[1m])',
    "memory_usage_bytes": 'container_memory_usage_bytes{job="kubelet", image!="", container!=""}',
}

# Downstream impact (reference README.md:24, CallerWebMvcTagsProvider.java:22-25): the
# metrics starter tags every request with the calling service (``caller``, from the
# X-CALLER header), so each HTTP family is also recorded per caller — the query builder
# reads these for ``metricType: downstream`` and the brain scores each caller of the
# deployed app (controller/queries.py, brain/worker.py).
CALLER_PREFIX = {"pod": "namespace_pod_caller:", "app": "namespace_app_caller:",
                 "app_per_pod": "namespace_app_caller_per_pod:"}
# API level (reference README.md:26, "metrics anomaly aggregated at service or API
# level"): the same families recorded per request path (Micrometer's ``uri`` tag),
# read for ``metricType: api``
URI_PREFIX = {"pod": "namespace_pod_uri:", "app": "namespace_app_uri:",
              "app_per_pod": "namespace_app_uri_per_pod:"}
# split label -> recorded prefixes
SPLIT_PREFIXES = {"caller": CALLER_PREFIX, "uri": URI_PREFIX}

POD_COUNT = "namespace_app:pod_count"
APP_LABEL = 'label_replace({inner}, "app", "$1", "label_app", "(.*)")'


def _http_expr(sel: str, kind: str, by: str) -> str:
    if kind == "rate":
        return f"sum(rate({sel}[1m])) by ({by})"
    num, den = sel.split("|")
    return f"sum(rate({num}[1m])) by ({by}) / sum(rate({den}[1m])) by ({by})"


def _pod_app_join(expr_by_pod: str) -> str:
    """Attach the pod's ``app`` label (from kube-state-metrics pod labels)."""
    pod_app = APP_LABEL.format(inner='kube_pod_labels{job="kube-state-metrics"}')
    return f"sum by (namespace, app) ({expr_by_pod} * on (namespace, pod) group_left(app) max by (namespace, pod, app) ({pod_app}))"


def rules() -> List[Dict[str, str]]:
    out: List[Dict[str, str]] = [{
        "record": POD_COUNT,
        "expr": "count by (namespace, app) (" + APP_LABEL.format(
            inner='kube_pod_labels{job="kube-state-metrics"}') + ")",
    }]
    for fam, (sel, kind) in HTTP_FAMILIES.items():
        out.append({"record": f"namespace_pod:{fam}", "expr": _http_expr(sel, kind, "namespace, pod")})
        # apps expose the `app` tag themselves (metrics starter, C27)
        out.append({"record": f"namespace_app:{fam}", "expr": _http_expr(sel, kind, "namespace, app")})
        out.append({"record": f"namespace_app_per_pod:{fam}", "expr": f"namespace_app:{fam} / on (namespace, app) {POD_COUNT}"})
    for label, cp in SPLIT_PREFIXES.items():
        for fam, (sel, kind) in HTTP_FAMILIES.items():
            out.append({"record": cp["pod"] + fam, "expr": _http_expr(sel, kind, f"namespace, pod, {label}")})
            out.append({"record": cp["app"] + fam, "expr": _http_expr(sel, kind, f"namespace, app, {label}")})
            out.append({"record": cp["app_per_pod"] + fam,
                        "expr": f"{cp['app']}{fam} / on (namespace, app) group_left {POD_COUNT}"})
    for fam, inner in RESOURCE_FAMILIES.items():
        by_pod = f"sum by (namespace, pod) ({inner})"
        out.append({"record": f"namespace_pod:{fam}", "expr": by_pod})
        out.append({"record": f"namespace_app:{fam}", "expr": _pod_app_join(by_pod)})
        out.append({"record": f"namespace_app_per_pod:{fam}", "expr": f"namespace_app:{fam} / on (namespace, app) {POD_COUNT}"})
    return out


def prometheus_rule(namespace: str = "monitoring") -> Dict:
    return {
        "apiVersion": "monitoring.coreos.com/v1",
        "kind": "PrometheusRule",
        "metadata": {"name": "foremast-metrics-rules", "namespace": namespace,
                     "labels": {"prometheus": "k8s", "role": "alert-rules"}},
        "spec": {"groups": [{"name": "foremast.rules", "interval": "30s", "rules": rules()}]},
    }


def recorded_names() -> List[str]:
    return [r["record"] for r in rules()]
