"""Python binding of the native Prometheus matrix decoder (``csrc/prom_parse.cpp``).

``parse_matrix(body)`` → list of ``(labels, ts, values)``;
``parse_dense(body, start, step, T, out, row0)`` scatters straight into a
dense float32 matrix (e.g. a pinned host staging buffer for the GPU ring);
``parse_dense_keyed(body, start, step, T, out, table)`` puts each series in
the row of its (namespace, app) key.
Falls back to ``json`` when the native library cannot be built (no g++).
"""

from __future__ import annotations

import ctypes as C
import json
import os
import shutil
import subprocess
import threading
from typing import Dict, List, Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "prom_parse.cpp")
SRCS = [SRC, os.path.join(HERE, "csrc", "job_plan.cpp")]
LIBDIR = os.path.join(HERE, "_lib")
LIB = os.path.join(LIBDIR, "libforemast_ingest.so")

_lock = threading.Lock()
_lib: Optional[C.CDLL] = None


class ParseError(ValueError):
    pass


def build(verbose: bool = False) -> str:
    os.makedirs(LIBDIR, exist_ok=True)
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(x) for x in SRCS):
        return LIB
    cxx = os.environ.get("CXX") or shutil.which("g++") or shutil.which("clang++")
    if not cxx:
        raise RuntimeError("no C++ compiler for the ingest parser")
    cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-o", LIB + ".tmp", *SRCS]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"ingest parser build failed:\n{r.stderr}")
    os.replace(LIB + ".tmp", LIB)
    return LIB


def _load() -> Optional[C.CDLL]:
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        try:
            build()
            lib = C.CDLL(LIB)
        except (RuntimeError, OSError):
            return None
        LL, P = C.c_longlong, C.c_void_p
        lib.fm_prom_scan.argtypes = [C.c_char_p, LL, LL, P, P, P, P]
        lib.fm_prom_scan.restype = LL
        lib.fm_prom_fill.argtypes = [C.c_char_p, LL, P, P, LL]
        lib.fm_prom_fill.restype = LL
        lib.fm_prom_dense.argtypes = [C.c_char_p, LL, C.c_double, C.c_double, LL, P, LL, LL, LL, P]
        lib.fm_prom_dense.restype = LL
        lib.fm_prom_dense_keyed.argtypes = [C.c_char_p, LL, C.c_double, C.c_double, LL, P, LL, LL, C.c_char_p,
                                            C.c_char_p, P, P, LL, P, P]
        lib.fm_prom_dense_keyed.restype = LL
        lib.fm_prom_keys.argtypes = [C.c_char_p, LL, LL, C.c_char_p, C.c_char_p, P]
        lib.fm_prom_keys.restype = LL
        lib.fm_prom_render.argtypes = [C.c_char_p, P, LL, P, LL, C.c_double, C.c_double, P, LL]
        lib.fm_prom_render.restype = LL
        lib.fm_plan_rollout.argtypes = [C.c_char_p, P, LL, C.c_double, LL, P, P, P, P, P, P, P, LL, P, P, LL,
                                         P, LL]
        lib.fm_plan_rollout.restype = LL
        lib.fm_keyindex_upsert.argtypes = [P, P, P, LL]
        lib.fm_keyindex_upsert.restype = LL
        lib.fm_keyindex_retire.argtypes = [P, P, LL]
        lib.fm_keyindex_retire.restype = LL
        lib.fm_keyindex_lookup.argtypes = [P, P, LL, P]
        lib.fm_keyindex_lookup.restype = LL
        lib.fm_keyindex_new.argtypes = [P, P, LL]
        lib.fm_keyindex_new.restype = P
        lib.fm_keyindex_free.argtypes = [P]
        lib.fm_keyindex_free.restype = None
        lib.fm_prom_dense_indexed.argtypes = [C.c_char_p, LL, C.c_double, C.c_double, LL, P, LL, LL, C.c_char_p,
                                              C.c_char_p, P, P, P]
        lib.fm_prom_dense_indexed.restype = LL
        lib.fm_prom_decode_tick.argtypes = [C.c_int, P, P, P, C.c_char_p, C.c_char_p, C.c_double, C.c_double, LL,
                                            P, LL, LL, C.c_int, C.c_int, P]
        lib.fm_prom_decode_tick.restype = LL
        lib.fm_prom_decode_bodies.argtypes = [C.c_int, P, P, P, C.c_char_p, C.c_char_p, P, C.c_double, C.c_double, P,
                                              LL, P, P, LL, LL, C.c_int, C.c_int, P]
        lib.fm_prom_decode_bodies.restype = LL
        lib.fm_key_hashes.argtypes = [C.c_char_p, P, P, C.c_char_p, P, P, LL, P]
        lib.fm_key_hashes.restype = LL
        _lib = lib
        return lib


def default_threads() -> int:
    """Native decode threads of a rank: ``FOREMAST_DECODE_THREADS`` (at most 16), else 8.
    Measured on the MI355X box (16-CPU share): the 77 MB tick of the 100k-series node
    bench decodes in 1.40 ms on 8 threads and 1.41 ms on 16."""
    v = os.environ.get("FOREMAST_DECODE_THREADS", "")
    if v.isdigit() and int(v) > 0:
        return min(16, int(v))
    return 8


def available() -> bool:
    return _load() is not None


def _check_status(body: bytes) -> None:
    head = body[:256]
    if b'"status"' in head and b'"error"' in head and b'"success"' not in head:
        try:
            d = json.loads(body)
            raise ParseError(d.get("error", "prometheus error"))
        except ValueError:
            raise ParseError("prometheus error")


def parse_matrix(body: bytes) -> List[Tuple[Dict[str, str], np.ndarray, np.ndarray]]:
    if isinstance(body, str):
        body = body.encode()
    _check_status(body)
    lib = _load()
    if lib is None:
        return _parse_py(body)
    n = lib.fm_prom_scan(body, len(body), 0, None, None, None, None)
    if n < 0:
        raise ParseError(f"malformed query_range body (code {n})")
    off = np.zeros(n, dtype=np.int64)
    ln = np.zeros(n, dtype=np.int32)
    cnt = np.zeros(n, dtype=np.int64)
    tot = C.c_longlong(0)
    lib.fm_prom_scan(body, len(body), n, off.ctypes.data, ln.ctypes.data, cnt.ctypes.data, C.byref(tot))
    ts = np.empty(tot.value, dtype=np.float64)
    vals = np.empty(tot.value, dtype=np.float32)
    k = lib.fm_prom_fill(body, len(body), ts.ctypes.data, vals.ctypes.data, tot.value)
    if k < 0:
        raise ParseError(f"malformed query_range body (code {k})")
    out = []
    pos = 0
    for i in range(n):
        labels = json.loads(body[off[i]: off[i] + ln[i]]) if off[i] >= 0 and ln[i] > 0 else {}
        c = int(cnt[i])
        out.append((labels, ts[pos:pos + c], vals[pos:pos + c]))
        pos += c
    return out


def parse_dense(body: bytes, start: float, step: float, T: int, out: np.ndarray, row0: int = 0) -> Tuple[int, int]:
    """Scatter series into ``out[row0 + s, :]`` (float32, pre-filled with NaN).
    Returns (n_series, n_dropped_points)."""
    if isinstance(body, str):
        body = body.encode()
    _check_status(body)
    if out.dtype != np.float32 or out.ndim != 2 or out.shape[1] < T or not out.flags.c_contiguous:
        raise ValueError("out must be a C-contiguous float32 [rows, >=T] array")
    lib = _load()
    if lib is None:
        series = _parse_py(body)
        dropped = 0
        for s, (_, ts, v) in enumerate(series):
            if row0 + s >= out.shape[0]:
                dropped += len(ts)
                continue
            fi = (ts - start) / step
            i = np.rint(fi).astype(np.int64)
            ok = (i >= 0) & (i < T) & (np.abs(fi - i) < 1e-6)
            out[row0 + s, i[ok]] = v[ok]
            dropped += int((~ok).sum())
        return len(series), dropped
    dropped = C.c_longlong(0)
    n = lib.fm_prom_dense(body, len(body), float(start), float(step), int(T), out.ctypes.data, out.shape[1],
                          int(row0), out.shape[0], C.byref(dropped))
    if n < 0:
        raise ParseError(f"malformed query_range body (code {n})")
    return int(n), int(dropped.value)


_M64 = 0xFFFFFFFFFFFFFFFF


def key_hash(a: str, b: str) -> int:
    """64-bit key of ``a + 0x1f + b`` (UTF-8) — the row key of a series in
    :func:`parse_dense_keyed`; bit-identical to ``prom_parse.cpp series_key``
    (8-byte little-endian words, multiply/xorshift rounds, final avalanche)."""
    data = a.encode() + b"\x1f" + b.encode()
    h = 0x243F6A8885A308D3 ^ len(data)
    pad = data + b"\0" * (-len(data) % 8)
    for i in range(0, len(pad), 8):
        h = ((h ^ int.from_bytes(pad[i:i + 8], "little")) * 0x9E3779B97F4A7C15) & _M64
        h ^= h >> 29
    h ^= h >> 32
    h = (h * 0xD6E8FEB86659FD93) & _M64
    return h ^ (h >> 32)


def key_hashes(a_list, b_list) -> np.ndarray:
    """:func:`key_hash` of many ``(a[i], b[i])`` pairs (uint64), in one native call."""
    n = len(a_list)
    if len(b_list) != n:
        raise ValueError("a_list and b_list differ in length")
    lib = _load()
    if lib is None or n == 0:
        return np.array([key_hash(a, b) for a, b in zip(a_list, b_list)], dtype=np.uint64)
    ea = [x.encode() for x in a_list]
    eb = [x.encode() for x in b_list]
    la = np.fromiter((len(x) for x in ea), dtype=np.int64, count=n)
    lb = np.fromiter((len(x) for x in eb), dtype=np.int64, count=n)
    oa = np.zeros(n, dtype=np.int64)
    ob = np.zeros(n, dtype=np.int64)
    np.cumsum(la[:-1], out=oa[1:])
    np.cumsum(lb[:-1], out=ob[1:])
    out = np.empty(n, dtype=np.uint64)
    A, B = b"".join(ea) or b"\0", b"".join(eb) or b"\0"
    if lib.fm_key_hashes(A, oa.ctypes.data, la.ctypes.data, B, ob.ctypes.data, lb.ctypes.data, n,
                         out.ctypes.data) != n:
        raise RuntimeError("fm_key_hashes failed")
    return out


class KeyTable:
    """Sorted (hash → row) table of a shard's series keys for the keyed scatter."""

    def __init__(self, keys_rows, label_a: str = "namespace", label_b: str = "app") -> None:
        keys_rows = list(keys_rows)
        hs = key_hashes([a for (a, _), _ in keys_rows], [b for (_, b), _ in keys_rows]).tolist() if keys_rows else []
        given = [(h, int(r)) for h, (_, r) in zip(hs, keys_rows)]
        pairs = sorted(given)
        hs = [h for h, _ in pairs]
        if len(set(hs)) != len(hs):
            raise ValueError("series key hash collision")
        self.hash = np.array(hs, dtype=np.uint64)
        self.rows = np.array([r for _, r in pairs], dtype=np.int64)
        # the native index keeps the keys in the GIVEN order (ideally the order the
        # responses list them): a repeated response then walks it sequentially
        self._ix_hash = np.array([h for h, _ in given], dtype=np.uint64)
        self._ix_rows = np.array([r for _, r in given], dtype=np.int64)
        self.label_a, self.label_b = label_a.encode(), label_b.encode()

    @classmethod
    def indexed(cls, hashes: np.ndarray, rows: np.ndarray, label_a: str = "namespace",
                label_b: str = "app") -> "KeyTable":
        """A table for the native index only (no sorted copy): duplicate keys are
        reported when the index is built."""
        t = cls([], label_a, label_b)
        t._ix_hash = np.ascontiguousarray(hashes, dtype=np.uint64)
        t._ix_rows = np.ascontiguousarray(rows, dtype=np.int64)
        t.hash, t.rows = t._ix_hash, t._ix_rows
        return t

    @classmethod
    def from_hashes(cls, hashes: np.ndarray, rows: np.ndarray, label_a: str = "namespace",
                    label_b: str = "app") -> "KeyTable":
        t = cls([], label_a, label_b)
        order = np.argsort(hashes, kind="stable")
        t.hash = np.ascontiguousarray(hashes[order], dtype=np.uint64)
        t.rows = np.ascontiguousarray(np.asarray(rows, dtype=np.int64)[order])
        t._ix_hash = np.ascontiguousarray(hashes, dtype=np.uint64)
        t._ix_rows = np.ascontiguousarray(np.asarray(rows, dtype=np.int64))
        if len(t.hash) > 1 and bool((t.hash[1:] == t.hash[:-1]).any()):
            raise ValueError("series key hash collision")
        return t

    def __len__(self) -> int:
        return len(self.rows)

    @property
    def index(self) -> int:
        """Native open-addressing (hash → row) index of this table (built on
        first use; one probe per series instead of a binary search)."""
        ix = getattr(self, "_index", None)
        if ix is None:
            lib = _load()
            if lib is None:
                raise RuntimeError("native ingest library unavailable")
            ix = lib.fm_keyindex_new(self._ix_hash.ctypes.data, self._ix_rows.ctypes.data, len(self._ix_rows))
            if not ix:
                raise ValueError("series key hash collision or negative row")
            self._index = ix
            self._lib = lib
        return ix

    def __del__(self) -> None:
        ix = getattr(self, "_index", None)
        if ix:
            self._lib.fm_keyindex_free(ix)
            self._index = None


class LiveKeyIndex:
    """A native (hash -> row) index that is updated in place: keys are set or
    retired between decodes (a retired key is unmatched).  Usable wherever a
    :class:`KeyTable` is (``index``, ``label_a`` / ``label_b``), e.g. one pod index
    shared by every metric family's body of a tick."""

    def __init__(self, label_a: str = "namespace", label_b: str = "pod") -> None:
        self.label_a, self.label_b = label_a.encode(), label_b.encode()
        lib = _load()
        if lib is None:
            raise RuntimeError("native ingest library unavailable")
        self._lib = lib
        empty = np.zeros(1, dtype=np.uint64)
        self._index = lib.fm_keyindex_new(empty.ctypes.data, np.zeros(1, np.int64).ctypes.data, 0)
        if not self._index:
            raise RuntimeError("fm_keyindex_new failed")

    @property
    def index(self) -> int:
        return self._index

    def set(self, hashes: np.ndarray, rows: np.ndarray) -> None:
        h = np.ascontiguousarray(hashes, dtype=np.uint64)
        r = np.ascontiguousarray(rows, dtype=np.int64)
        if len(h) and self._lib.fm_keyindex_upsert(self._index, h.ctypes.data, r.ctypes.data, len(h)) != len(h):
            raise ValueError("key index update failed (negative row)")

    def retire(self, hashes: np.ndarray) -> None:
        h = np.ascontiguousarray(hashes, dtype=np.uint64)
        if len(h):
            self._lib.fm_keyindex_retire(self._index, h.ctypes.data, len(h))

    def lookup(self, hashes: np.ndarray) -> np.ndarray:
        h = np.ascontiguousarray(hashes, dtype=np.uint64)
        out = np.empty(len(h), dtype=np.int64)
        if len(h):
            self._lib.fm_keyindex_lookup(self._index, h.ctypes.data, len(h), out.ctypes.data)
        return out

    def __del__(self) -> None:
        ix = getattr(self, "_index", None)
        if ix:
            self._lib.fm_keyindex_free(ix)
            self._index = None


def series_keys(body: bytes, label_a: str = "namespace", label_b: str = "app") -> np.ndarray:
    """Key (:func:`key_hash`) of every series of a response, in response order (uint64)."""
    if isinstance(body, str):
        body = body.encode()
    lib = _load()
    if lib is None:
        return np.array([key_hash(l.get(label_a, ""), l.get(label_b, "")) for l, _, _ in _parse_py(body)],
                        dtype=np.uint64)
    n = lib.fm_prom_scan(body, len(body), 0, None, None, None, None)
    if n < 0:
        raise ParseError(f"malformed query_range body (code {n})")
    out = np.zeros(n, dtype=np.uint64)
    lib.fm_prom_keys(body, len(body), n, label_a.encode(), label_b.encode(), out.ctypes.data)
    return out


def parse_dense_keyed(body: bytes, start: float, step: float, T: int, out: np.ndarray, table: KeyTable,
                      col0: int = 0) -> Tuple[int, int, int]:
    """Scatter each series into ``out[row, col0 + (t - start)/step]`` where
    ``row`` is its (namespace, app) key's row in ``table`` (``out`` float32,
    pre-filled with NaN, unit column stride).  Returns (n_series,
    n_dropped_points, n_unmatched_series)."""
    if isinstance(body, str):
        body = body.encode()
    _check_status(body)
    if out.dtype != np.float32 or out.ndim != 2 or out.shape[1] < col0 + T or out.strides[1] != 4:
        raise ValueError("out must be float32 [rows, >= col0 + T] with unit column stride")
    lib = _load()
    if lib is None:
        lookup = dict(zip(table.hash.tolist(), table.rows.tolist()))
        dropped = unmatched = 0
        series = _parse_py(body)
        la, lb = table.label_a.decode(), table.label_b.decode()
        for labels, ts, v in series:
            row = lookup.get(key_hash(labels.get(la, ""), labels.get(lb, "")), -1)
            if row < 0 or row >= out.shape[0]:
                unmatched += 1
                dropped += len(ts)
                continue
            fi = (ts - start) / step
            i = np.rint(fi).astype(np.int64)
            ok = (i >= 0) & (i < T) & (np.abs(fi - i) < 1e-6)
            out[row, col0 + i[ok]] = v[ok]
            dropped += int((~ok).sum())
        return len(series), dropped, unmatched
    dropped, unmatched = C.c_longlong(0), C.c_longlong(0)
    ld = out.strides[0] // 4
    base = out.ctypes.data + 4 * col0
    n = lib.fm_prom_dense_indexed(body, len(body), float(start), float(step), int(T), base, ld, out.shape[0],
                                  table.label_a, table.label_b, table.index, C.byref(dropped), C.byref(unmatched))
    if n < 0:
        raise ParseError(f"malformed query_range body (code {n})")
    return int(n), int(dropped.value), int(unmatched.value)


def decode_tick(bodies, tables, start: float, step: float, T: int, out: np.ndarray, threads: int = 8,
                fill_nan: bool = True) -> List[Tuple[int, int, int]]:
    """Keyed scatter of a whole tick (body j through ``tables[j]``) into
    ``out`` (float32 ``[rows, >= T]``, unit column stride) by ``threads``
    native threads — each body split at series boundaries so the pool stays
    balanced — after a parallel NaN fill of the ``T`` columns.  One call,
    GIL released throughout.  Returns ``(series, dropped, unmatched)`` per body."""
    if len(bodies) != len(tables):
        raise ValueError(f"{len(bodies)} bodies for {len(tables)} key tables")
    if out.dtype != np.float32 or out.ndim != 2 or out.shape[1] < T or out.strides[1] != 4:
        raise ValueError("out must be float32 [rows, >= T] with unit column stride")
    bodies = [b.encode() if isinstance(b, str) else b for b in bodies]
    for b in bodies:
        _check_status(b)
    lib = _load()
    labels = {(t.label_a, t.label_b) for t in tables}
    if lib is None or len(labels) > 1:
        if fill_nan:
            out[:, :T] = np.nan
        return [parse_dense_keyed(b, start, step, T, out, t) for b, t in zip(bodies, tables)]
    nb = len(bodies)
    bufs = (C.c_char_p * nb)(*bodies)
    lens = (C.c_longlong * nb)(*[len(b) for b in bodies])
    idx = (C.c_void_p * nb)(*[t.index for t in tables])
    stats = np.zeros(3 * max(nb, 1), dtype=np.int64)
    la, lb = next(iter(labels)) if labels else (b"", b"")
    rc = lib.fm_prom_decode_tick(nb, C.cast(bufs, C.c_void_p), C.cast(lens, C.c_void_p), C.cast(idx, C.c_void_p),
                                 la, lb, float(start), float(step), int(T), out.ctypes.data, out.strides[0] // 4,
                                 out.shape[0], int(max(1, threads)), int(fill_nan), stats.ctypes.data)
    if rc < 0:
        bad = [j for j in range(nb) if stats[3 * j] < 0]
        raise ParseError(f"malformed query_range body {bad[:1]} (code {rc})")
    return [(int(stats[3 * j]), int(stats[3 * j + 1]), int(stats[3 * j + 2])) for j in range(nb)]


def decode_bodies(bodies, tables, starts, step: float, Ts, col0s, out: np.ndarray, threads: int = 8,
                  fill_nan: bool = False) -> List[Tuple[int, int, int]]:
    """Keyed scatter of many bodies in ONE native call on ``threads`` threads:
    body j through ``tables[j]`` into columns ``[col0s[j], col0s[j] + Ts[j])``
    of ``out`` on the ``(starts[j], step)`` grid (e.g. a history load: one
    body per (time chunk, app group) query).  Returns ``(series, dropped,
    unmatched)`` per body, ``series < 0`` marking a malformed body (the others
    are still decoded)."""
    n = len(bodies)
    if not (len(tables) == len(starts) == len(Ts) == len(col0s) == n):
        raise ValueError("one table, start, T and col0 per body")
    if out.dtype != np.float32 or out.ndim != 2 or out.strides[1] != 4:
        raise ValueError("out must be float32 [rows, cols] with unit column stride")
    if n and max(int(c) + int(t) for c, t in zip(col0s, Ts)) > out.shape[1]:
        raise ValueError("a body's column range exceeds out")
    bodies = [b.encode() if isinstance(b, str) else b for b in bodies]
    lib = _load()
    labels = {(t.label_a, t.label_b) for t in tables}
    res: List[Tuple[int, int, int]] = []
    if lib is None or len(labels) > 1:
        if fill_nan:
            out[:] = np.nan
        for b, t, st, T, c0 in zip(bodies, tables, starts, Ts, col0s):
            try:
                _check_status(b)
                res.append(parse_dense_keyed(b, st, step, int(T), out, t, col0=int(c0)))
            except ParseError:
                res.append((-1, 0, 0))
        return res
    ok = []
    for j, b in enumerate(bodies):
        try:
            _check_status(b)
            ok.append(j)
        except ParseError:
            pass
    m = len(ok)
    stats = np.zeros(3 * max(m, 1), dtype=np.int64)
    if m:
        bufs = (C.c_char_p * m)(*[bodies[j] for j in ok])
        lens = (C.c_longlong * m)(*[len(bodies[j]) for j in ok])
        idx = (C.c_void_p * m)(*[tables[j].index for j in ok])
        st = np.ascontiguousarray([float(starts[j]) for j in ok], dtype=np.float64)
        tt = np.ascontiguousarray([int(Ts[j]) for j in ok], dtype=np.int64)
        cc = np.ascontiguousarray([int(col0s[j]) for j in ok], dtype=np.int64)
        la, lb = next(iter(labels))
        lib.fm_prom_decode_bodies(m, C.cast(bufs, C.c_void_p), C.cast(lens, C.c_void_p), C.cast(idx, C.c_void_p),
                                  la, lb, st.ctypes.data, 0.0, float(step), tt.ctypes.data, 0, cc.ctypes.data,
                                  out.ctypes.data, out.strides[0] // 4, out.shape[0], int(max(1, threads)),
                                  int(fill_nan), stats.ctypes.data)
    by_j = {j: (int(stats[3 * i]), int(stats[3 * i + 1]), int(stats[3 * i + 2])) for i, j in enumerate(ok)}
    return [by_j.get(j, (-1, 0, 0)) for j in range(n)]


def _parse_py(body: bytes):
    d = json.loads(body)
    if d.get("status") != "success":
        raise ParseError(d.get("error", "prometheus error"))
    out = []
    for r in d.get("data", {}).get("result", []):
        pts = r.get("values") or ([r["value"]] if "value" in r else [])
        ts = np.array([float(p[0]) for p in pts], dtype=np.float64)
        vals = np.array([float(p[1]) for p in pts], dtype=np.float32)
        out.append((r.get("metric", {}), ts, vals))
    return out


def label_blob(labels: List[str]) -> Tuple[bytes, np.ndarray]:
    """Label objects (the text between the braces of ``"metric":{...}``) packed for
    :func:`render_matrix`: one blob and ``S + 1`` byte offsets."""
    enc = [x.encode() for x in labels]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum([len(e) for e in enc], out=off[1:])
    return b"".join(enc), off


def render_matrix(blob: Tuple[bytes, np.ndarray], vals: np.ndarray, ts0: float, step: float) -> bytes:
    """A ``query_range`` matrix body for S series x T points (``vals`` [S, T] float32,
    NaN = no sample) at ``ts0 + j * step`` — the encoder the benchmarks' Prometheus
    stand-in uses (native, ~20x a Python f-string renderer)."""
    lib = _load()
    if lib is None:
        raise RuntimeError("native ingest library unavailable")
    labels, off = blob
    v = np.ascontiguousarray(vals, dtype=np.float32)
    S, T = (v.shape[0], v.shape[1]) if v.ndim == 2 else (v.shape[0], 1)
    assert off.shape[0] == S + 1, "one label object per series"
    cap = int(S * (40 + 32 * T) + off[-1] + 256)
    while True:
        out = np.empty(cap, dtype=np.uint8)
        n = lib.fm_prom_render(labels, off.ctypes.data, S, v.ctypes.data, T, float(ts0), float(step),
                               out.ctypes.data, cap)
        if n >= 0:
            return out[:n].tobytes()
        cap = -n
