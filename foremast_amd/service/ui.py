"""Health dashboard served by the service at ``/ui/{namespace}/{app}``.

Equivalent of foremast-browser (reference C26, ``foremast-browser/src/App.js``):
every 15 s it fetches the last 15 minutes at a 15 s step, through this
service's query proxy, for four metric families and draws for each the
observed series (``namespace_app_per_pod:<m>``), the brain's band
(``foremastbrain:namespace_app_per_pod:<m>_{upper,lower}``, an area) and
anomaly points (``..._anomaly``), plus the error-rate vs latency scatter
(one point per step, coloured by time: the reference's 3-D time x 5xx x
latency chart as a projection).  Unlike the reference (highcharts + React
build, namespace/app hard-coded to foremast-examples/demo), this is one
self-contained page with inline SVG — no external assets, so it works in
air-gapped clusters — and namespace/app come from the URL.
"""

from __future__ import annotations

import html
import json
from typing import Dict, List

# family → (title, scale applied to values, unit)
PANELS: Dict[str, List] = {
    "http_server_requests_error_5xx": ["5XX errors", 1, "req/s"],
    "http_server_requests_latency": ["Latency", 1000, "ms"],
    "cpu_usage_seconds_total": ["CPU", 1, "cores"],
    "memory_usage_bytes": ["Memory", 1.0 / (1 << 20), "MiB"],
}

# the reference's scatter: time x 5xx x latency (ScatterChart.js:144-173)
SCATTER = ("http_server_requests_error_5xx", "http_server_requests_latency")

REFRESH_S = 15
WINDOW_S = 15 * 60
STEP_S = 15


def queries(namespace: str, app: str) -> Dict[str, Dict[str, str]]:
    """PromQL per panel and role (base/upper/lower/anomaly).  Brain gauges are
    scraped from the brain pod, so their ``namespace`` label arrives as
    ``exported_namespace``."""
    out = {}
    for fam in PANELS:
        name = "namespace_app_per_pod:" + fam
        brain = "foremastbrain:" + name
        own = f'{{namespace="{namespace}",app="{app}"}}'
        exp = f'{{exported_namespace="{namespace}",app="{app}"}}'
        out[fam] = {"base": name + own, "upper": brain + "_upper" + exp, "lower": brain + "_lower" + exp,
                    "anomaly": brain + "_anomaly" + exp}
    return out


_PAGE = r"""<!doctype html>
<html><head><meta charset="utf-8"><title>Foremast · __TITLE__</title>
<style>
body{font-family:system-ui,sans-serif;margin:0;background:#0f1419;color:#d6dde6}
header{padding:12px 20px;background:#18212b;display:flex;gap:16px;align-items:baseline}
header h1{font-size:18px;margin:0} header span{color:#8a97a6;font-size:13px}
main{display:grid;grid-template-columns:repeat(auto-fit,minmax(520px,1fr));gap:16px;padding:16px}
.panel{background:#18212b;border-radius:8px;padding:12px}
.panel h2{font-size:14px;margin:0 0 8px 0;font-weight:600}
svg{width:100%;height:220px} .err{color:#e57373;font-size:12px}
.legend{font-size:12px;color:#8a97a6} .legend b{display:inline-block;width:10px;height:10px;margin:0 4px 0 10px}
</style></head><body>
<header><h1>__TITLE__</h1><span id="status">loading…</span></header>
<main id="panels"></main>
<script>
const CFG = __CFG__;
const fmt = t => new Date(t * 1000).toLocaleTimeString();
function parseProxy(body) {            // the proxy double-encodes (reference wire format)
  let v = body; for (let i = 0; i < 2 && typeof v === "string"; i++) v = JSON.parse(v); return v;
}
async function fetchSeries(q, start, end) {
  const url = "/api/v1/query_range?query=" + encodeURIComponent(q) + "&start=" + start + "&end=" + end + "&step=" + CFG.step;
  const r = await fetch(url); const d = parseProxy(await r.json());
  const res = (d && d.data && d.data.result) || [];
  const pts = {};
  for (const s of res) for (const [t, v] of s.values) { const x = parseFloat(v); if (!isNaN(x)) pts[t] = (pts[t] || 0) + x; }
  return Object.keys(pts).map(Number).sort((a, b) => a - b).map(t => [t, pts[t]]);
}
function draw(el, data, scale, unit) {
  const W = 600, H = 220, P = 36;
  const all = [...data.base, ...data.upper, ...data.lower].map(p => p[1] * scale);
  const ts = [...data.base, ...data.upper].map(p => p[0]);
  if (!all.length) { el.innerHTML = '<div class="err">no data</div>'; return; }
  let lo = Math.min(...all), hi = Math.max(...all); if (hi === lo) { hi += 1; lo -= 1; }
  const t0 = Math.min(...ts), t1 = Math.max(...ts) || t0 + 1;
  const X = t => P + (W - 2 * P) * (t - t0) / Math.max(t1 - t0, 1), Y = v => H - P + (2 * P - H) * (v * scale - lo) / (hi - lo);
  const path = pts => pts.map((p, i) => (i ? "L" : "M") + X(p[0]).toFixed(1) + "," + Y(p[1]).toFixed(1)).join("");
  let band = "";
  if (data.upper.length && data.lower.length) {
    const up = data.upper, dn = [...data.lower].reverse();
    band = '<path d="' + path(up) + dn.map(p => "L" + X(p[0]).toFixed(1) + "," + Y(p[1]).toFixed(1)).join("") + 'Z" fill="#4fc3f733" stroke="none"/>';
  }
  const anom = data.anomaly.filter(p => p[1] !== 0).map(p => {
    const b = data.base.find(q => q[0] === p[0]); const v = b ? b[1] : p[1];
    return '<circle cx="' + X(p[0]).toFixed(1) + '" cy="' + Y(v).toFixed(1) + '" r="4" fill="#e57373"/>'; }).join("");
  const ticks = [0, 0.5, 1].map(f => { const v = lo + f * (hi - lo); const y = H - P + (2 * P - H) * f;
    return '<text x="2" y="' + (y + 4) + '" font-size="10" fill="#8a97a6">' + v.toPrecision(3) + '</text>'; }).join("");
  el.innerHTML = '<svg viewBox="0 0 ' + W + ' ' + H + '">' + band + '<path d="' + path(data.base) + '" fill="none" stroke="#ffd54f" stroke-width="1.5"/>' +
    anom + ticks + '<text x="' + P + '" y="' + (H - 6) + '" font-size="10" fill="#8a97a6">' + fmt(t0) + '</text>' +
    '<text x="' + (W - P - 50) + '" y="' + (H - 6) + '" font-size="10" fill="#8a97a6">' + fmt(t1) + '</text></svg>' +
    '<div class="legend"><b style="background:#ffd54f"></b>observed (' + unit + ')<b style="background:#4fc3f7"></b>expected band<b style="background:#e57373"></b>anomaly</div>';
}
// error rate vs latency, one point per timestamp, colour = time (old → new): the
// reference's 3-D time x 5xx x latency scatter (ScatterChart.js) as a projection
function drawScatter(el, err, lat, latScale) {
  const W = 600, H = 220, P = 40;
  const lm = new Map(lat.map(p => [p[0], p[1] * latScale]));
  const pts = err.filter(p => lm.has(p[0])).map(p => [p[0], lm.get(p[0]), p[1]]);
  if (!pts.length) { el.innerHTML = '<div class="err">no data</div>'; return; }
  const xs = pts.map(p => p[1]), ys = pts.map(p => p[2]), ts = pts.map(p => p[0]);
  let x0 = Math.min(...xs), x1 = Math.max(...xs), y0 = Math.min(...ys), y1 = Math.max(...ys);
  if (x1 === x0) { x1 += 1; x0 -= 1; } if (y1 === y0) { y1 += 1; y0 -= 1; }
  const t0 = Math.min(...ts), t1 = Math.max(...ts);
  const X = v => P + (W - 2 * P) * (v - x0) / (x1 - x0), Y = v => H - P + (2 * P - H) * (v - y0) / (y1 - y0);
  const dots = pts.map(p => { const f = t1 > t0 ? (p[0] - t0) / (t1 - t0) : 1;
    return '<circle cx="' + X(p[1]).toFixed(1) + '" cy="' + Y(p[2]).toFixed(1) + '" r="3.5" fill="hsl(' + (200 - 200 * f).toFixed(0) + ',80%,60%)"><title>' + fmt(p[0]) + '</title></circle>'; }).join("");
  el.innerHTML = '<svg viewBox="0 0 ' + W + ' ' + H + '">' + dots +
    '<text x="' + P + '" y="' + (H - 6) + '" font-size="10" fill="#8a97a6">latency ' + x0.toPrecision(3) + '…' + x1.toPrecision(3) + ' ms</text>' +
    '<text x="2" y="14" font-size="10" fill="#8a97a6">5xx ' + y1.toPrecision(3) + '</text>' +
    '<text x="2" y="' + (H - P) + '" font-size="10" fill="#8a97a6">' + y0.toPrecision(3) + '</text></svg>' +
    '<div class="legend">one point per ' + CFG.step + ' s step; colour: ' + fmt(t0) + ' (blue) → ' + fmt(t1) + ' (red)</div>';
}
async function refresh() {
  const end = Math.floor(Date.now() / 1000), start = end - CFG.window;
  const panels = document.getElementById("panels");
  for (const [fam, [title, scale, unit]] of Object.entries(CFG.panels)) {
    let el = document.getElementById(fam);
    if (!el) { const d = document.createElement("div"); d.className = "panel"; d.innerHTML = "<h2>" + title + "</h2><div id='" + fam + "'></div>"; panels.appendChild(d); el = document.getElementById(fam); }
    try {
      const q = CFG.queries[fam], data = {};
      for (const role of ["base", "upper", "lower", "anomaly"]) data[role] = await fetchSeries(q[role], start, end);
      draw(el, data, scale, unit);
    } catch (e) { el.innerHTML = '<div class="err">' + e + '</div>'; }
  }
  let sc = document.getElementById("scatter");
  if (!sc) { const d = document.createElement("div"); d.className = "panel"; d.innerHTML = "<h2>5XX errors vs latency</h2><div id='scatter'></div>"; panels.appendChild(d); sc = document.getElementById("scatter"); }
  try {
    const err = await fetchSeries(CFG.queries[CFG.scatter[0]].base, start, end);
    const lat = await fetchSeries(CFG.queries[CFG.scatter[1]].base, start, end);
    drawScatter(sc, err, lat, CFG.panels[CFG.scatter[1]][1]);
  } catch (e) { sc.innerHTML = '<div class="err">' + e + '</div>'; }
  document.getElementById("status").textContent = "updated " + new Date().toLocaleTimeString() + " · every " + CFG.refresh + " s";
}
refresh(); setInterval(refresh, CFG.refresh * 1000);
</script></body></html>
"""


def page(namespace: str, app: str) -> str:
    cfg = {"panels": PANELS, "queries": queries(namespace, app), "refresh": REFRESH_S, "window": WINDOW_S,
           "step": STEP_S, "scatter": list(SCATTER)}
    # </script> can't appear inside JSON from these inputs after escaping '<'
    blob = json.dumps(cfg).replace("<", "\\u003c")
    return _PAGE.replace("__CFG__", blob).replace("__TITLE__", html.escape(f"{namespace} : {app}"))
