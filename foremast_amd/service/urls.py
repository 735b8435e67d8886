"""Datasource URL builders and the job-document config-string format.

* Prometheus: ``<endpoint>query_range?query=<esc>&start=<int>&end=<int>&step=<int>``
  (``foremast-service/pkg/prometheus/prometheushelper.go:12-27``).
* Wavefront: ``<esc query>&&<start>&&<m|s|h|d>&&<end>``
  (``foremast-service/pkg/wavefront/wavefronthelper.go:12-34``; the
  reference file wrongly declares ``package prometheus`` — Q6).
* Config strings: ``alias== <url>`` entries joined by `` ||``
  (``foremast-service/cmd/manager/main.go:28-31,49-74``).  Go iterates the
  metric map in random order; we emit aliases in sorted order so the
  content-addressed job id is deterministic.
"""

from __future__ import annotations

from typing import Dict, List, Tuple
from urllib.parse import parse_qs, quote_plus, urlsplit

from ..api import rest as r

CONFIG_SEPARATOR = " ||"
KV_SEPARATOR = "== "


class ConfigError(ValueError):
    pass


def go_query_escape(s: str) -> str:
    """Go ``url.QueryEscape``: unreserved = ALPHA / DIGIT / ``-_.~``; space → ``+``."""
    return quote_plus(s, safe="-_.~")


def go_format_int(v) -> str:
    """``strconv.FormatFloat(v, 'f', 0, 64)`` (round-half-even, like Python)."""
    return f"{float(v):.0f}"


def _param(p: Dict, key: str):
    if key not in p:
        raise ConfigError(f"missing parameter {key!r}")
    return p[key]


def build_prometheus_url(q: r.MetricQuery) -> str:
    p = q.parameters
    return (str(_param(p, "endpoint")) + "query_range?query=" + go_query_escape(str(_param(p, "query")))
            + "&start=" + go_format_int(_param(p, "start"))
            + "&end=" + go_format_int(_param(p, "end"))
            + "&step=" + go_format_int(_param(p, "step")))


_WF_UNITS = {60: "m", 1: "s", 3600: "h", 86400: "d"}


def build_wavefront_url(q: r.MetricQuery) -> str:
    p = q.parameters
    step = float(_param(p, "step"))
    unit = _WF_UNITS.get(int(step), "") if step.is_integer() else ""
    return (go_query_escape(str(_param(p, "query"))) + "&&" + go_format_int(_param(p, "start"))
            + "&&" + unit + "&&" + go_format_int(_param(p, "end")))


def construct_url(q: r.MetricQuery) -> Tuple[int, str, str]:
    """``main.go:33-47`` constructURL → (errCode, dataSource, url)."""
    if not q.parameters:
        return 404, "", ""
    try:
        if q.data_source_type == r.DATASOURCE_PROMETHEUS:
            return 0, r.DATASOURCE_PROMETHEUS, build_prometheus_url(q)
        if q.data_source_type == r.DATASOURCE_WAVEFRONT:
            return 0, r.DATASOURCE_WAVEFRONT, build_wavefront_url(q)
    except (ConfigError, TypeError, ValueError):
        return 404, q.data_source_type, ""
    return 404, q.data_source_type, ""


def flatten_queries(metric: Dict[str, r.MetricQuery]) -> Tuple[int, str, str]:
    """``convertMetricQuerys`` → (errCode, config string, metric-store string)."""
    if not metric:
        return 404, "", ""
    out: List[str] = []
    stores: List[str] = []
    for key in sorted(metric):
        code, source, url = construct_url(metric[key])
        if code != 0:
            return 404, url, source
        out.append(key + KV_SEPARATOR + url)
        stores.append(key + KV_SEPARATOR + source)
    return 0, CONFIG_SEPARATOR.join(out), CONFIG_SEPARATOR.join(stores)


def flatten_metrics_info(m: r.MetricsInfo) -> Tuple[int, str, List[str], List[str]]:
    """``convertMetricInfoString`` (``main.go:76-127``)."""
    configs = ["", "", ""]
    sources = ["", "", ""]
    if not m.current:
        return 404, "MetricInfo current is empty ", configs, sources
    error_code = 0
    reason: List[str] = []
    code, ret, src = flatten_queries(m.current)
    if code != 0:
        reason.append("current query encount error " + ret + "\n")
        error_code = 404
    configs[0], sources[0] = ret, src
    if m.baseline is not None:
        bcode, ret, src = flatten_queries(m.baseline)
        if bcode != 0:
            reason.append(" baseline query encount error " + ret)
        configs[1], sources[1] = ret, src
    if m.historical is not None:
        hcode, ret, src = flatten_queries(m.historical)
        if hcode != 0:
            reason.append(" historical query encount error " + ret)
        if code != 0 and hcode != 0:
            error_code = 404
        configs[2], sources[2] = ret, src
    elif code != 0:
        error_code = 404
    return error_code, "".join(reason), configs, sources


def parse_config(config: str) -> Dict[str, str]:
    """Inverse of :func:`flatten_queries`: ``{alias: url}`` (brain side)."""
    out: Dict[str, str] = {}
    if not config:
        return out
    for entry in config.split(CONFIG_SEPARATOR):
        entry = entry.strip()
        if not entry:
            continue
        if KV_SEPARATOR not in entry:
            raise ConfigError(f"malformed config entry {entry!r}")
        alias, url = entry.split(KV_SEPARATOR, 1)
        out[alias.strip()] = url.strip()
    return out


def parse_prometheus_url(url: str) -> Dict[str, object]:
    """Split a Prometheus ``query_range`` URL into endpoint/query/start/end/step."""
    parts = urlsplit(url)
    qs = parse_qs(parts.query, keep_blank_values=True)
    base = url.split("query_range?", 1)[0]

    def one(k, conv):
        v = qs.get(k)
        if not v:
            raise ConfigError(f"url missing {k}: {url}")
        return conv(v[0])

    return {"endpoint": base, "query": one("query", str), "start": one("start", float),
            "end": one("end", float), "step": one("step", float)}


def parse_wavefront_url(s: str) -> Dict[str, object]:
    from urllib.parse import unquote_plus
    parts = s.split("&&")
    if len(parts) != 4:
        raise ConfigError(f"malformed wavefront query {s!r}")
    inv = {v: k for k, v in _WF_UNITS.items()}
    return {"query": unquote_plus(parts[0]), "start": float(parts[1]),
            "step": float(inv.get(parts[2], 60)), "end": float(parts[3])}
