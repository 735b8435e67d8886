"""Rollout job plans: what the resident engine needs of a canary / rollingUpdate job.

A job document carries the reference service's flattened query strings
(``foremast-service/cmd/manager/main.go:28-31,49-127``) around the selectors
barrelman writes (``foremast-barrelman/pkg/client/metrics/metricsquery.go:21-89``).
The plan of a job is, per metric alias: the 7-day history series (endpoint,
metric, namespace, app), the pod metric family and pods of the current window,
the baseline pods and window (canary), and the window geometry.

Two decoders produce the same plans:

* :func:`plan_many` — documents in batches through the native decoder
  (``ingest/csrc/job_plan.cpp``: one pass per document, ~2 us instead of the
  ~250 us of the general Python parser), into a columnar :class:`PlanCols`
  (numeric columns, 64-bit keys of every pod / family / history series) that
  the engine admits with array operations;
* :func:`_plan` — the general Python parser, for the documents the native one
  declines (any shape outside the common one: general URL forms, escapes,
  regex pods, offsets in endTime, ...).

``tests/test_job_plan.py`` checks the two agree on every document the native
decoder accepts.
"""

from __future__ import annotations

import ctypes
import itertools
import os
import re
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple
from urllib.parse import unquote

import numpy as np

from ..api import rest as r
from ..ingest import native
from ..promql.selector import SelectorError, parse_selector
from ..service import urls
from ..utils.timeutil import TimeFormatError, parse_rfc3339

STRATEGIES = ("canary", "rollingupdate")
UNIVARIATE = ("holt_winters", "exponential_smoothing", "double_exponential_smoothing", "moving_average",
              "moving_average_all", "seasonal_decompose")
# multi-metric algorithms (docs/guides/design.md:53-89): every metric keeps a univariate
# row (moving_average_all, as brain/batch.py scores it), and the job gets a joint model
JOINT_ALGORITHMS = ("bivariate_normal", "lstm", "auto")
ALGORITHMS = UNIVARIATE + JOINT_ALGORITHMS
JOINT_SERVED = ("biv", "lstm")   # joint models the resident engine serves


def joint_kind(algorithm: str, n_metrics: int) -> Optional[str]:
    """The joint model of a job with ``n_metrics`` aliases: ``"biv"`` (bivariate
    normal over its first two aliases), ``"lstm"`` (LSTM autoencoder over all) or
    None — the dispatch of ``brain/worker.py`` ``_multivariate``: ``auto`` sends 2
    metrics to the bivariate normal and 3+ to the LSTM (``design.md:76-84``)."""
    if algorithm == "auto":
        return "biv" if n_metrics == 2 else ("lstm" if n_metrics >= 3 else None)
    if algorithm == "bivariate_normal":
        return "biv" if n_metrics >= 2 else None
    if algorithm == "lstm":
        return "lstm" if n_metrics >= 2 else None
    return None
_SPLIT = ("namespace_pod_caller:", "namespace_app_caller:", "namespace_app_caller_per_pod:",
          "namespace_pod_uri:", "namespace_app_uri:", "namespace_app_uri_per_pod:")
_REGEX_META = re.compile(r"[*+?()\[\]{}^$\\]")
DOC_FIELDS = ("strategy", "endTime", "currentConfig", "baselineConfig", "historicalConfig",
              "currentMetricStore", "baselineMetricStore", "historicalMetricStore")

Key = Tuple[str, str, str, str]  # (endpoint, metric, namespace, app)


@dataclass
class RolloutSeries:
    """One (job, metric alias): a row of the rollout table."""
    alias: str
    hkey: Key                       # 7-day history series (endpoint, metric, namespace, app)
    fam: Tuple[str, str]            # (endpoint, pod metric) of the current window
    namespace: str
    cur_pods: Tuple[str, ...]
    base_pods: Tuple[str, ...]
    cur_start: float
    cur_n: int
    base_start: float
    base_n: int
    hist_end: float
    base_fam: Tuple[str, str] = ("", "")  # (endpoint, pod metric) of the baseline window (may be another cluster)


class Interned:
    """A per-row column of a few distinct values, stored as row -> index into them
    (a decoded batch of 10k rows has a handful of aliases and families)."""

    __slots__ = ("vals", "idx")

    def __init__(self, vals: List, idx: np.ndarray) -> None:
        self.vals, self.idx = vals, idx

    def __getitem__(self, s):
        return self.vals[self.idx[s]]

    def __len__(self) -> int:
        return len(self.idx)

    def __iter__(self):
        return (self.vals[i] for i in self.idx.tolist())


class PlanCols:
    """Columnar plans of a batch of jobs: series rows ``[S]`` and pods ``[Q]``.

    ``f64 [S, 3]`` cur_start, base_start, hist_end; ``i32 [S, 7]`` cur_n, base_n,
    cur pod0, cur npod, base pod0, base npod, has_base; ``u64 [S, 6]`` history key,
    family key, baseline family key, history family key, (namespace, app) key,
    (alias, history metric) key;
    ``pod_u64 [Q]`` (namespace, pod) keys.  The few distinct strings (alias,
    families) are interned per row at construction; a row's history key tuple,
    namespace and pod names are decoded on demand from ``text`` (``span``)."""

    __slots__ = ("text", "f64", "i32", "u64", "span", "pod_span", "pod_u64", "alias", "fam", "base_fam", "hfam",
                 "_hkey", "_ns", "_pods")

    def __init__(self, text: bytes, f64, i32, u64, span, pod_span, pod_u64, alias, fam, base_fam, hfam,
                 hkey=None, ns=None) -> None:
        self.text, self.f64, self.i32, self.u64, self.span = text, f64, i32, u64, span
        self.pod_span, self.pod_u64 = pod_span, pod_u64
        self.alias, self.fam, self.base_fam, self.hfam = alias, fam, base_fam, hfam
        S = len(alias)
        self._hkey: List[Optional[Key]] = hkey if hkey is not None else [None] * S
        self._ns: List[Optional[str]] = ns if ns is not None else [None] * S
        self._pods: Dict[Tuple[int, int], Tuple[str, ...]] = {}

    def _str(self, k: int, s: int) -> str:
        a = self.span[s]
        return self.text[a[2 * k]:a[2 * k] + a[2 * k + 1]].decode()

    def ns_at(self, s: int) -> str:
        v = self._ns[s]
        if v is None:
            v = self._ns[s] = self._str(3, s)
        return v

    def hkey_at(self, s: int) -> Key:
        v = self._hkey[s]
        if v is None:
            hf = self.hfam[s]
            v = self._hkey[s] = (hf[0], hf[1], self.ns_at(s), self._str(4, s))
        return v

    @property
    def hkey(self) -> List[Key]:
        return [self.hkey_at(s) for s in range(len(self.alias))]

    def pods(self, p0: int, n: int) -> Tuple[str, ...]:
        got = self._pods.get((p0, n))
        if got is None:
            t, sp = self.text, self.pod_span
            got = tuple(t[sp[q, 0]:sp[q, 0] + sp[q, 1]].decode() for q in range(p0, p0 + n))
            self._pods[(p0, n)] = got
        return got

    def pods_alt(self, s: int, base: bool) -> bytes:
        """The row's current (or baseline) pods as the RE2 alternation ``a|b|c``
        (sorted, distinct; empty for rows of the Python parser: use :meth:`pods`)."""
        if self.span is None:
            return b""
        a = self.span[s]
        k = 18 if base else 16
        return bytes(self.text[a[k]:a[k] + a[k + 1]])

    def cur_pods(self, s: int) -> Tuple[str, ...]:
        return self.pods(int(self.i32[s, 2]), int(self.i32[s, 3]))

    def base_pods(self, s: int) -> Tuple[str, ...]:
        return self.pods(int(self.i32[s, 4]), int(self.i32[s, 5]))

    def series(self, s: int) -> RolloutSeries:
        f, i = self.f64[s], self.i32[s]
        return RolloutSeries(alias=self.alias[s], hkey=self.hkey_at(s), fam=self.fam[s], namespace=self.ns_at(s),
                             cur_pods=self.cur_pods(s), base_pods=self.base_pods(s), cur_start=float(f[0]),
                             cur_n=int(i[0]), base_start=float(f[1]), base_n=int(i[1]), hist_end=float(f[2]),
                             base_fam=self.base_fam[s])

    @classmethod
    def from_series(cls, series: Sequence[RolloutSeries]) -> "PlanCols":
        """Columns of plans the Python parser made (the rare path)."""
        S = len(series)
        f64 = np.array([[s.cur_start, s.base_start, s.hist_end] for s in series], dtype=np.float64).reshape(S, 3)
        pods: List[Tuple[str, str]] = []
        i32 = np.zeros((S, 7), dtype=np.int32)
        u64 = np.zeros((S, 6), dtype=np.uint64)
        for k, s in enumerate(series):
            i32[k, 0], i32[k, 1] = s.cur_n, s.base_n
            i32[k, 2], i32[k, 3] = len(pods), len(s.cur_pods)
            pods += [(s.namespace, p) for p in s.cur_pods]
            i32[k, 4], i32[k, 5] = len(pods), len(s.base_pods)
            pods += [(s.namespace, p) for p in s.base_pods]
            i32[k, 6] = 1 if s.base_fam[0] or s.base_fam[1] else 0
            u64[k, 0] = hkey_hash(s.hkey)
            u64[k, 1] = native.key_hash(*s.fam)
            u64[k, 2] = native.key_hash(*s.base_fam) if i32[k, 6] else 0
            u64[k, 3] = native.key_hash(s.hkey[0], s.hkey[1])
            u64[k, 4] = native.key_hash(s.hkey[2], s.hkey[3])
            u64[k, 5] = native.key_hash(s.alias, s.hkey[1])
        text = "".join(p for _, p in pods).encode()
        lens = np.array([len(p.encode()) for _, p in pods], dtype=np.int64)
        span = np.zeros((len(pods), 2), dtype=np.int64)
        if len(pods):
            span[1:, 0] = np.cumsum(lens)[:-1]
            span[:, 1] = lens
        pod_u64 = native.key_hashes([a for a, _ in pods], [b for _, b in pods]) if pods else np.zeros(0, np.uint64)
        out = cls(text, f64, i32, u64, None, span, pod_u64, [s.alias for s in series], [s.fam for s in series],
                  [s.base_fam for s in series], [(s.hkey[0], s.hkey[1]) for s in series],
                  hkey=[s.hkey for s in series], ns=[s.namespace for s in series])
        for k, s in enumerate(series):  # the pod tuples as parsed (no re-decode)
            out._pods[(int(i32[k, 2]), len(s.cur_pods))] = tuple(s.cur_pods)
            out._pods[(int(i32[k, 4]), len(s.base_pods))] = tuple(s.base_pods)
        return out


def hkey_hash(k: Key) -> int:
    """The history-series key of the native decoder (series_key of "endpoint\\x1fmetric"
    and "namespace\\x1fapp")."""
    return native.key_hash(k[0] + "\x1f" + k[1], k[2] + "\x1f" + k[3])


_NO_ROWS = np.zeros(0, dtype=np.int64)
_NO_KEYS = np.zeros(0, dtype=np.uint64)
_NO_ROWS.flags.writeable = False   # shared by every unadmitted plan: replaced, never written
_NO_KEYS.flags.writeable = False


class RolloutPlan:
    """A job's plan: its series are rows ``[s0, s0 + n)`` of ``cols``."""

    __slots__ = ("doc_id", "app", "end_ts", "doc", "rows", "cols", "s0", "n", "pod_keys", "_series", "jslot")

    def __init__(self, doc_id: str, app: Tuple[str, str], end_ts: float, cols: PlanCols, s0: int, n: int,
                 doc: Optional[Dict] = None) -> None:
        self.doc_id, self.app, self.end_ts = doc_id, app, end_ts
        self.cols, self.s0, self.n = cols, s0, n
        self.doc: Dict = doc if doc is not None else {}
        self.rows = _NO_ROWS        # table rows of the admitted job's series
        self.pod_keys = _NO_KEYS    # pod slots the admitted job holds
        self.jslot = -1                                # the admitted job's slot in the engine's job table
        self._series: Optional[List[RolloutSeries]] = None

    @property
    def series(self) -> List[RolloutSeries]:
        if self._series is None:
            self._series = [self.cols.series(s) for s in range(self.s0, self.s0 + self.n)]
        return self._series

    @property
    def hkeys(self) -> List[Key]:
        return [self.cols.hkey_at(s) for s in range(self.s0, self.s0 + self.n)]

    @property
    def first_fam(self) -> Tuple[str, str]:
        return self.cols.fam[self.s0]


# ---------------------------------------------------------------------- Python parser
def _pods_of(sel) -> Optional[Tuple[str, Tuple[str, ...]]]:
    """(namespace, pods) of ``<m>{namespace="ns", pod="a"}`` / ``pod=~"a|b"``."""
    ns, pods = None, None
    for label, op, val in sel.matchers:
        if label == "namespace" and op == "=":
            ns = val
        elif label == "pod" and op == "=":
            pods = (val,)
        elif label == "pod" and op == "=~":
            if _REGEX_META.search(val):
                return None
            pods = tuple(p for p in val.split("|") if p)
        else:
            return None
    if ns is None or not pods:
        return None
    return ns, tuple(sorted(set(pods)))


_SIMPLE_SEL = re.compile(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)\{((?:[a-zA-Z_][a-zA-Z0-9_]*(?:=~|=)"[^"\\]*",?)*)\}$')


class _Sel:
    __slots__ = ("name", "matchers")

    def __init__(self, name, matchers):
        self.name, self.matchers = name, matchers


def _selector(q: str):
    """The plain selectors barrelman writes (``name{l="v",l=~"a|b"}``, no
    escapes) split without the general PromQL matcher regex; anything else
    goes through :func:`parse_selector`."""
    m = _SIMPLE_SEL.match(q)
    if m is None:
        return parse_selector(q)
    out = []
    for part in m.group(2).split('",'):
        if not part:
            continue
        label, _, rest = part.partition("=")
        op = "=~" if rest.startswith("~") else "="
        out.append((label, op, rest[2 if op == "=~" else 1:].rstrip('"')))
    return _Sel(m.group(1), tuple(out))


def _grid(url: str) -> Tuple[str, object, float, float, float]:
    """(endpoint, selector, start, end, step) of a flattened Prometheus
    ``query_range`` URL (``prometheushelper.go:12-27`` shape: four parameters,
    only the query percent-encoded); other shapes take the general parser."""
    ep, sep, qs = url.partition("query_range?")
    fields = dict(kv.partition("=")[::2] for kv in qs.split("&")) if sep else {}
    if set(fields) != {"query", "start", "end", "step"}:
        p = urls.parse_prometheus_url(url)
        return ep, parse_selector(str(p["query"])), float(p["start"]), float(p["end"]), float(p["step"])
    return (ep, _selector(_unquote(fields["query"])), float(fields["start"]), float(fields["end"]),
            float(fields["step"]))


_ESC = (("%3A", ":"), ("%7B", "{"), ("%7D", "}"), ("%3D", "="), ("%22", '"'), ("%2C", ","), ("%7C", "|"),
        ("%7E", "~"), ("%2F", "/"))


def _unquote(q: str) -> str:
    """Percent-decoding of a selector: the escapes a PromQL selector of k8s
    names produces are replaced directly (C string ops); any other escape
    takes ``urllib.parse.unquote``."""
    if "%" not in q:
        return q
    for a, b in _ESC:
        q = q.replace(a, b)
    return unquote(q) if "%" in q else q


def _plan_series(doc, step, window_cols) -> Optional[Tuple[Tuple[str, str], float, List[RolloutSeries]]]:
    if (doc.get("strategy") or "").lower() not in STRATEGIES:
        return None
    try:
        cur = urls.parse_config(doc.get("currentConfig", ""))
        base = urls.parse_config(doc.get("baselineConfig", ""))
        hist = urls.parse_config(doc.get("historicalConfig", ""))
        stores = [v for k in ("currentMetricStore", "baselineMetricStore", "historicalMetricStore")
                  for v in urls.parse_config(doc.get(k, "")).values()]
    except urls.ConfigError:
        return None
    if not cur or any(s and s != r.DATASOURCE_PROMETHEUS for s in stores):
        return None
    try:
        end_ts = parse_rfc3339(doc.get("endTime", "")).timestamp()
    except TimeFormatError:
        return None
    out, app = [], None
    for alias in sorted(cur):
        if alias not in hist:
            return None
        try:
            ep_h, sel_h, _hs, h_end, h_step = _grid(hist[alias])
            ep_c, sel_c, c_start, c_end, c_step = _grid(cur[alias])
        except (urls.ConfigError, SelectorError, KeyError, ValueError):
            return None
        lab = {k: v for k, op, v in sel_h.matchers if op == "="}
        if (len(sel_h.matchers) != 2 or set(lab) != {"namespace", "app"} or not sel_h.name or not sel_c.name
                or sel_h.name.startswith(_SPLIT) or sel_c.name.startswith(_SPLIT)
                or h_step != step or c_step != step or ep_c != ep_h):
            return None
        pc = _pods_of(sel_c)
        if pc is None or pc[0] != lab["namespace"]:
            return None
        b_pods, b_start, b_n = (), 0.0, 0
        if alias in base:
            try:
                ep_b, sel_b, b_start, b_end, b_step = _grid(base[alias])
            except (urls.ConfigError, SelectorError, KeyError, ValueError):
                return None
            pb = _pods_of(sel_b)
            # the baseline may live in another cluster (its own Prometheus): multi-cluster canary
            if pb is None or sel_b.name != sel_c.name or b_step != step or pb[0] != pc[0]:
                return None
            b_pods, b_n = pb[1], min(window_cols, int(round((b_end - b_start) / step)) + 1)
            if b_n > 0 and int(round((b_end - b_start) / step)) + 1 > window_cols:
                b_start = b_end - (window_cols - 1) * step  # the newest window_cols points
        app = app or (lab["namespace"], lab["app"])
        out.append(RolloutSeries(
            alias=alias, hkey=(ep_h, sel_h.name, lab["namespace"], lab["app"]), fam=(ep_c, sel_c.name),
            namespace=pc[0], cur_pods=pc[1], base_pods=b_pods, cur_start=c_start,
            cur_n=max(0, min(window_cols, int(round((c_end - c_start) / step)) + 1)),
            base_start=b_start, base_n=b_n, hist_end=h_end,
            base_fam=(ep_b, sel_b.name) if alias in base else ("", "")))
    return app, end_ts, out


def _plan(doc, step, window_cols) -> Optional[RolloutPlan]:
    got = _plan_series(doc, step, window_cols)
    if got is None:
        return None
    app, end_ts, series = got
    p = RolloutPlan(doc["id"], app, end_ts, PlanCols.from_series(series), 0, len(series), doc=doc)
    p._series = series
    return p


# ---------------------------------------------------------------------- native batches
# interned strings of the few distinct aliases / families (keyed by bytes or 64-bit key)
_INTERN_A: Dict[int, str] = {}
_INTERN_H: Dict[int, Tuple[str, str]] = {}
_INTERN_F: Dict[int, Tuple[str, str]] = {}


def _native_call(lib, blob, off, N, step, window_cols, ser_cap, pod_cap, text_cap):
    job_i32 = np.zeros((N, 3), dtype=np.int32)
    job_f64 = np.zeros(N, dtype=np.float64)
    job_span = np.zeros((N, 4), dtype=np.int64)
    f64 = np.empty((ser_cap, 3), dtype=np.float64)
    i32 = np.empty((ser_cap, 7), dtype=np.int32)
    span = np.empty((ser_cap, 20), dtype=np.int64)
    u64 = np.empty((ser_cap, 6), dtype=np.uint64)
    pod_span = np.empty((pod_cap, 2), dtype=np.int64)
    pod_u64 = np.empty(pod_cap, dtype=np.uint64)
    text = bytearray(text_cap)  # kept as the PlanCols text (no copy of the decoded strings)
    text_ptr = ctypes.addressof((ctypes.c_char * text_cap).from_buffer(text))
    S = lib.fm_plan_rollout(blob, off.ctypes.data, N, float(step), int(window_cols), job_i32.ctypes.data,
                            job_f64.ctypes.data, job_span.ctypes.data, f64.ctypes.data, i32.ctypes.data,
                            span.ctypes.data, u64.ctypes.data, ser_cap, pod_span.ctypes.data, pod_u64.ctypes.data,
                            pod_cap, text_ptr, text_cap)
    if S < 0:
        return None
    return S, job_i32, job_f64, job_span, f64, i32, span, u64, pod_span, pod_u64, text


def _native_batch(docs: Sequence[Dict], step: float, window_cols: int) -> Optional[Tuple[np.ndarray, List]]:
    """Native decode of ``docs``: (accepted mask, plans) — None when the library is absent."""
    lib = native._load()
    if lib is None or not docs:
        return None
    # document-major [d0.f0, d0.f1, ..., d1.f0, ...] with C-level loops (one map per field)
    n_d = len(docs)
    fields = list(itertools.chain.from_iterable(zip(*[map(dict.get, docs, itertools.repeat(k, n_d),
                                                          itertools.repeat("", n_d)) for k in DOC_FIELDS])))
    if set(map(type, fields)) != {str}:
        fields = [f if isinstance(f, str) else "" for f in fields]
    joined = "".join(fields)
    if joined.isascii():  # one encode; byte offsets = character offsets
        lens = np.fromiter(map(len, fields), dtype=np.int64, count=len(fields))
        blob = joined.encode("ascii") or b"\0"
    else:
        parts = [f.encode() for f in fields]
        lens = np.fromiter(map(len, parts), dtype=np.int64, count=len(parts))
        blob = b"".join(parts) or b"\0"
    off = np.zeros(len(fields) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    N = len(docs)
    nchunk = max(1, min(_THREADS, N // 256))
    bounds = [N * c // nchunk for c in range(nchunk + 1)]

    def run(c):
        d0, d1 = bounds[c], bounds[c + 1]
        o = off[8 * d0:8 * d1 + 1]
        # capacities (grown and retried if short), scaled from the chunk's first document
        # (a batch is one shape of job; counting the whole chunk's text cost more than the
        # decode): series <= entries of the configs, pods <= escaped pod separators + one
        # per series and kind
        first = joined[off[8 * d0]:off[8 * d0 + 8]]
        scale = 1.25 * (int(o[-1] - o[0]) + 1) / (len(first) + 1)  # chunk text / first document's
        ser_cap = max(16, int(first.count("== ") * scale) + 16)
        pod_cap = max(64, int((first.count("%7C") + first.count("|")) * scale) + 2 * ser_cap)
        text_cap = int(o[-1] - o[0]) + 1024
        for _ in range(4):
            got = _native_call(lib, blob, o, d1 - d0, step, window_cols, ser_cap, pod_cap, text_cap)
            if got is not None:
                return got
            ser_cap, pod_cap, text_cap = 2 * ser_cap, 2 * pod_cap, 2 * text_cap
        return None
    # the decoder releases the GIL: a deploy burst is decoded on several cores
    outs = list(_pool().map(run, range(nchunk))) if nchunk > 1 else [run(0)]
    if any(o is None for o in outs):
        return None
    oks, plans = [], []
    for c, got in enumerate(outs):
        ok, pl_ = _columns(got, docs[bounds[c]:bounds[c + 1]])
        oks.append(ok)
        plans += pl_
    return np.concatenate(oks), plans


_THREADS = max(1, min(8, (os.cpu_count() or 1)))
_POOL = None


def _pool():
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _POOL = ThreadPoolExecutor(_THREADS, thread_name_prefix="plan")
    return _POOL


def _columns(got, docs: Sequence[Dict]) -> Tuple[np.ndarray, List]:
    """PlanCols and plans of one decoded chunk."""
    S, job_i32, job_f64, job_span, f64, i32, span, u64, pod_span, pod_u64, text = got
    tb = text
    sp = span[:S]

    def interned(col: int, table: Dict, make, mask=None) -> Interned:
        """Per row, the interned value of its key column (one decode per distinct key);
        rows outside ``mask`` get ("", "")."""
        u, first, inv = np.unique(u64[:S, col], return_index=True, return_inverse=True)
        vals = []
        for k, r0 in zip(u.tolist(), first.tolist()):
            v = table.get(k)
            if v is None:
                v = table[k] = make(sp[r0].tolist())
            vals.append(v)
        inv = inv.reshape(-1).astype(np.int32)
        if mask is not None and not mask.all():
            vals.append(("", ""))
            inv = np.where(mask, inv, len(vals) - 1).astype(np.int32)
        return Interned(vals, inv)

    def st(a, k):
        return tb[a[2 * k]:a[2 * k] + a[2 * k + 1]].decode()
    alias = interned(5, _INTERN_A, lambda a: st(a, 0))
    hfam = interned(3, _INTERN_H, lambda a: (st(a, 1), st(a, 2)))
    fam = interned(1, _INTERN_F, lambda a: (st(a, 1), st(a, 5)))
    has_b = i32[:S, 6] > 0
    bfam = interned(2, _INTERN_F, lambda a: (st(a, 6), st(a, 7)) if a[13] or a[15] else ("", ""), has_b)
    for d in (_INTERN_A, _INTERN_H, _INTERN_F):
        if len(d) > 1 << 16:
            d.clear()
    Q = int(i32[S - 1, 4] + i32[S - 1, 5]) if S else 0
    cols = PlanCols(tb, f64[:S].copy(), i32[:S].copy(), u64[:S].copy(), span[:S].copy(), pod_span[:Q].copy(),
                    pod_u64[:Q].copy(), alias, fam, bfam, hfam)
    plans: List[Optional[RolloutPlan]] = [None] * len(docs)
    ok = job_i32[:, 0] == 1
    ji, jf, js = job_i32.tolist(), job_f64.tolist(), job_span.tolist()
    for d in np.nonzero(ok)[0].tolist():
        a = js[d]
        plans[d] = RolloutPlan(docs[d]["id"], (tb[a[0]:a[0] + a[1]].decode(), tb[a[2]:a[2] + a[3]].decode()),
                               jf[d], cols, ji[d][1], ji[d][2], doc=docs[d])
    return ok, plans


_PLANS: "OrderedDict[Tuple[str, float, int], Optional[RolloutPlan]]" = OrderedDict()


def _remember(ck, plan) -> None:
    _PLANS[ck] = plan
    if len(_PLANS) > 1 << 17:
        _PLANS.popitem(last=False)


def plan_many(docs: Sequence[Dict], algorithm: str, step: float = 60.0,
              window_cols: int = 11) -> List[Optional[RolloutPlan]]:
    """Plans of ``docs`` (None: not keyable by the resident engine), memoised per
    job id (content-addressed: a job's request, hence its plan, never changes).
    Unseen documents are decoded natively in one batch; the ones the native
    decoder declines take the Python parser."""
    if algorithm not in ALGORITHMS:
        return [None] * len(docs)
    out: List[Optional[RolloutPlan]] = [None] * len(docs)
    todo = []
    for i, d in enumerate(docs):
        ck = (d.get("id", ""), step, window_cols)
        if ck in _PLANS:
            out[i] = _PLANS[ck]
        else:
            todo.append(i)
    if todo:
        got = _native_batch([docs[i] for i in todo], step, window_cols)
        for k, i in enumerate(todo):
            d = docs[i]
            p = got[1][k] if got is not None and got[0][k] else _plan(d, step, window_cols)
            out[i] = p
            _remember((d.get("id", ""), step, window_cols), p)
    if algorithm in JOINT_ALGORITHMS:  # jobs whose joint model the engine does not serve stay with BrainWorker
        for i, p in enumerate(out):
            if p is not None:
                k = joint_kind(algorithm, p.n)
                if k is not None and k not in JOINT_SERVED:
                    out[i] = None
    return out


def plan_rollout(doc: Dict, algorithm: str, step: float = 60.0, window_cols: int = 11) -> Optional[RolloutPlan]:
    return plan_many([doc], algorithm, step, window_cols)[0]
