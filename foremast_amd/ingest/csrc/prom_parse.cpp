// Native Prometheus query_range matrix decoder (K10, host side).
//
// Parses the body of /api/v1/query_range:
//   {"status":"success","data":{"resultType":"matrix","result":[
//      {"metric":{...},"values":[[1700000000,"1.5"],[1700000060,"NaN"],...]}, ...]}}
// in one pass without building a DOM.  Two entry points:
//
//  * fm_prom_scan   — counts series and points (to size buffers) and records,
//                     per series, the byte span of its "metric" object and
//                     its point range;
//  * fm_prom_fill   — writes timestamps/values into caller arrays (columnar),
//  * fm_prom_dense  — scatters values straight into a NaN-initialised dense
//                     [S, T] float32 matrix on the (start, step) grid, which
//                     is what the GPU ring buffer ingests (pinned host memory
//                     → one H2D copy);
//  * fm_prom_dense_keyed — the same scatter, but each series goes to the row
//                     its (label_a, label_b) values map to (FNV-1a 64 key,
//                     binary search in the caller's sorted key table), so a
//                     response for any subset of a shard's series lands in
//                     place in one pass with no per-series Python work.
//
// Numbers are decoded with std::from_chars (locale independent).  Special
// values "NaN", "+Inf", "-Inf" are accepted.  Returns < 0 on malformed input.
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>

namespace {

struct Cursor {
  const char* p;
  const char* e;
  bool ok() const { return p < e; }
  void ws() {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool eat(char c) {
    ws();
    if (p < e && *p == c) { ++p; return true; }
    return false;
  }
};

// skip a JSON string (cursor at opening quote); returns false on error
bool skip_string(Cursor& c) {
  if (c.p >= c.e || *c.p != '"') return false;
  ++c.p;
  while (c.p < c.e) {
    if (*c.p == '\\') {  // escape: the escaped byte must exist
      if (c.e - c.p < 2) { c.p = c.e; return false; }
      c.p += 2;
      continue;
    }
    if (*c.p == '"') { ++c.p; return true; }
    ++c.p;
  }
  return false;
}

bool skip_value(Cursor& c);

bool skip_container(Cursor& c, char open, char close) {
  if (c.p >= c.e || *c.p != open) return false;
  int depth = 0;
  while (c.p < c.e) {
    const char ch = *c.p;
    if (ch == '"') { if (!skip_string(c)) return false; continue; }
    if (ch == open) ++depth;
    else if (ch == close) { --depth; if (depth == 0) { ++c.p; return true; } }
    ++c.p;
  }
  return false;
}

bool skip_value(Cursor& c) {
  c.ws();
  if (c.p >= c.e) return false;
  switch (*c.p) {
    case '"': return skip_string(c);
    case '{': return skip_container(c, '{', '}');
    case '[': return skip_container(c, '[', ']');
    default:
      while (c.p < c.e && *c.p != ',' && *c.p != '}' && *c.p != ']') ++c.p;
      return true;
  }
}

// read an object key (cursor before the quote) into [k0, k1)
bool read_key(Cursor& c, const char*& k0, const char*& k1) {
  c.ws();
  if (c.p >= c.e || *c.p != '"') return false;
  k0 = c.p + 1;
  if (!skip_string(c)) return false;
  k1 = c.p - 1;
  return c.eat(':');
}

bool key_is(const char* k0, const char* k1, const char* lit) {
  const size_t n = strlen(lit);
  return (size_t)(k1 - k0) == n && memcmp(k0, lit, n) == 0;
}

bool parse_number(const char* a, const char* b, double& out) {
  while (a < b && (*a == ' ' || *a == '"')) ++a;
  while (b > a && (b[-1] == ' ' || b[-1] == '"')) --b;
  if (a == b) return false;
  const size_t n = (size_t)(b - a);
  if ((n == 3 && memcmp(a, "NaN", 3) == 0)) { out = std::numeric_limits<double>::quiet_NaN(); return true; }
  if ((n == 4 && (memcmp(a, "+Inf", 4) == 0)) || (n == 3 && memcmp(a, "Inf", 3) == 0)) {
    out = std::numeric_limits<double>::infinity(); return true;
  }
  if (n == 4 && memcmp(a, "-Inf", 4) == 0) { out = -std::numeric_limits<double>::infinity(); return true; }
  if (*a == '+') ++a;
  auto r = std::from_chars(a, b, out);
  return r.ec == std::errc() && r.ptr == b;
}

// Visitor over the result array.  Calls on_series(metric0, metric1) then
// on_point(ts, value) for each pair, then on_end().
template <typename OnSeries, typename OnPoint>
long long walk(const char* buf, long long len, OnSeries on_series, OnPoint on_point) {
  Cursor c{buf, buf + len};
  // find "result":[
  const char* found = nullptr;
  for (const char* q = buf; q + 9 <= buf + len; ++q) {
    if (*q == '"' && memcmp(q, "\"result\"", 8) == 0) { found = q + 8; break; }
  }
  if (!found) return -1;
  c.p = found;
  if (!c.eat(':')) return -2;
  if (!c.eat('[')) return -3;
  long long nseries = 0;
  c.ws();
  if (c.eat(']')) return 0;
  while (true) {
    if (!c.eat('{')) return -4;
    const char* m0 = nullptr; const char* m1 = nullptr;
    bool started = false;
    while (true) {
      const char *k0, *k1;
      if (!read_key(c, k0, k1)) return -5;
      c.ws();
      if (key_is(k0, k1, "metric")) {
        m0 = c.p;
        if (!skip_container(c, '{', '}')) return -6;
        m1 = c.p;
      } else if (key_is(k0, k1, "values") || key_is(k0, k1, "value")) {
        const bool many = key_is(k0, k1, "values");
        if (!started) { on_series(nseries, m0, m1); started = true; }
        if (many && !c.eat('[')) return -7;
        c.ws();
        if (many && c.eat(']')) {
          // empty
        } else {
          while (true) {
            if (!c.eat('[')) return -8;
            c.ws();
            const char* a = c.p;
            while (c.p < c.e && *c.p != ',') ++c.p;
            double ts;
            if (!parse_number(a, c.p, ts)) return -9;
            if (!c.eat(',')) return -10;
            c.ws();
            const char* v0 = c.p;
            if (c.p >= c.e) return -11;
            if (*c.p == '"') { if (!skip_string(c)) return -11; } else { while (c.p < c.e && *c.p != ']') ++c.p; }
            double v;
            if (!parse_number(v0, c.p, v)) return -12;
            if (!c.eat(']')) return -13;
            on_point(nseries, ts, v);
            if (!many) break;
            if (c.eat(',')) continue;
            if (c.eat(']')) break;
            return -14;
          }
        }
      } else {
        if (!skip_value(c)) return -15;
      }
      if (c.eat(',')) continue;
      if (c.eat('}')) break;
      return -16;
    }
    if (!started) on_series(nseries, m0, m1);
    ++nseries;
    if (c.eat(',')) continue;
    if (c.eat(']')) break;
    return -17;
  }
  return nseries;
}

// FNV-1a 64 over a + 0x1f + b (foremast_amd/ingest/native.py key_hash must agree)
uint64_t fnv_key(const char* a0, const char* a1, const char* b0, const char* b1) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&h](unsigned char ch) { h ^= ch; h *= 1099511628211ull; };
  for (const char* q = a0; q < a1; ++q) mix((unsigned char)*q);
  mix(0x1f);
  for (const char* q = b0; q < b1; ++q) mix((unsigned char)*q);
  return h;
}

// raw bytes of the string value of `key` inside the metric object [m0, m1)
// (label values are plain DNS-style names; a value with escapes keeps them raw)
bool label_value(const char* m0, const char* m1, const char* key, const char*& v0, const char*& v1) {
  if (!m0) return false;
  Cursor c{m0, m1};
  if (!c.eat('{')) return false;
  c.ws();
  if (c.eat('}')) return false;
  while (true) {
    const char *k0, *k1;
    if (!read_key(c, k0, k1)) return false;
    c.ws();
    if (c.p < c.e && *c.p == '"') {
      const char* s0 = c.p + 1;
      if (!skip_string(c)) return false;
      if (key_is(k0, k1, key)) { v0 = s0; v1 = c.p - 1; return true; }
    } else if (!skip_value(c)) {
      return false;
    }
    if (c.eat(',')) continue;
    return false;
  }
}

}  // namespace

extern "C" {

// Count series / points; optional per-series outputs (arrays of size >= max_series).
long long fm_prom_scan(const char* buf, long long len, long long max_series, long long* label_off,
                       int* label_len, long long* point_count, long long* total_points) {
  long long total = 0;
  const long long r = walk(
      buf, len,
      [&](long long s, const char* m0, const char* m1) {
        if (s < max_series) {
          if (label_off) label_off[s] = m0 ? (long long)(m0 - buf) : -1;
          if (label_len) label_len[s] = m0 ? (int)(m1 - m0) : 0;
          if (point_count) point_count[s] = 0;
        }
      },
      [&](long long s, double, double) {
        ++total;
        if (s < max_series && point_count) point_count[s] += 1;
      });
  if (total_points) *total_points = total;
  return r;
}

// Columnar fill: ts/vals arrays of size >= total points, in series order.
long long fm_prom_fill(const char* buf, long long len, double* ts, float* vals, long long cap) {
  long long k = 0;
  const long long r = walk(
      buf, len, [&](long long, const char*, const char*) {},
      [&](long long, double t, double v) {
        if (k < cap) { ts[k] = t; vals[k] = (float)v; }
        ++k;
      });
  return r < 0 ? r : k;
}

// Dense scatter: out[row0 + s, (t - start)/step] = v for t on the grid
// (row stride ld); points off-grid or outside [0, T) are counted in *dropped.
long long fm_prom_dense(const char* buf, long long len, double start, double step, long long T, float* out,
                        long long ld, long long row0, long long max_rows, long long* dropped) {
  long long drop = 0;
  const long long r = walk(
      buf, len, [&](long long, const char*, const char*) {},
      [&](long long s, double t, double v) {
        const long long row = row0 + s;
        const double fi = (t - start) / step;
        const long long i = (long long)llround(fi);
        if (row >= max_rows || i < 0 || i >= T || std::fabs(fi - (double)i) > 1e-6) { ++drop; return; }
        out[row * ld + i] = (float)v;
      });
  if (dropped) *dropped = drop;
  return r;
}

// Key of every series in response order (FNV of its label_a / label_b values):
// builds the KeyTable of a known response layout without per-series Python.
long long fm_prom_keys(const char* buf, long long len, long long max_series, const char* label_a,
                       const char* label_b, uint64_t* out) {
  return walk(
      buf, len,
      [&](long long s, const char* m0, const char* m1) {
        const char *a0 = "", *a1 = a0, *b0 = a0, *b1 = a0;
        label_value(m0, m1, label_a, a0, a1);
        label_value(m0, m1, label_b, b0, b1);
        if (s < max_series) out[s] = fnv_key(a0, a1, b0, b1);
      },
      [&](long long, double, double) {});
}

// Keyed dense scatter: series s goes to row key_rows[j] where key_hash[j] is the
// FNV key of its (label_a, label_b) values (key_hash sorted ascending, n_keys
// entries); unmatched series are skipped and counted in *unmatched.
long long fm_prom_dense_keyed(const char* buf, long long len, double start, double step, long long T, float* out,
                              long long ld, long long max_rows, const char* label_a, const char* label_b,
                              const uint64_t* key_hash, const long long* key_rows, long long n_keys,
                              long long* dropped, long long* unmatched) {
  long long drop = 0, miss = 0, row = -1;
  const long long r = walk(
      buf, len,
      [&](long long, const char* m0, const char* m1) {
        const char *a0 = "", *a1 = a0, *b0 = a0, *b1 = a0;
        label_value(m0, m1, label_a, a0, a1);
        label_value(m0, m1, label_b, b0, b1);
        const uint64_t h = fnv_key(a0, a1, b0, b1);
        long long lo = 0, hi = n_keys;
        while (lo < hi) {
          const long long mid = (lo + hi) >> 1;
          if (key_hash[mid] < h) lo = mid + 1; else hi = mid;
        }
        row = (lo < n_keys && key_hash[lo] == h) ? key_rows[lo] : -1;
        if (row < 0 || row >= max_rows) { row = -1; ++miss; }
      },
      [&](long long, double t, double v) {
        const double fi = (t - start) / step;
        const long long i = (long long)llround(fi);
        if (row < 0 || i < 0 || i >= T || std::fabs(fi - (double)i) > 1e-6) { ++drop; return; }
        out[row * ld + i] = (float)v;
      });
  if (dropped) *dropped = drop;
  if (unmatched) *unmatched = miss;
  return r;
}

}  // extern "C"
