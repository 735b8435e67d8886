// Native decoder of rollout job documents into the resident engine's plan
// (brain/rollout.py: plan_rollout / _plan).
//
// A canary / rollingUpdate job arrives as the reference service's flattened
// strings (foremast-service/cmd/manager/main.go:28-31,49-127): per query kind
// "alias== <prometheus query_range URL>" entries joined by " ||", each URL
// "<endpoint>query_range?query=<escaped selector>&start=&end=&step="
// (prometheushelper.go:12-27) around the selectors barrelman writes
// (metricsquery.go:21-89): namespace_app_per_pod:<m>{namespace="ns",app="a"} for
// the 7-day history, namespace_pod:<m>{namespace="ns",pod=~"p1|p2"} for the
// current / baseline pods.  Python's general parser takes ~250 us per job; at
// a node's deploy bursts (thousands of jobs per tick) that is the admission
// bottleneck, so the common shape is decoded here in one pass per document.
//
// Contract: for every document this either produces exactly the plan the Python
// `_plan` produces (status 1), or declines (status 0) and the caller runs `_plan`
// -- anything unusual (general URL shapes, escapes that decode to non-ASCII,
// non-plain numbers, timezone offsets, duplicate aliases, regex pods, ...) is
// declined, never guessed.  The equivalence is property-tested against `_plan`
// (tests/test_job_plan.py).
//
// Outputs are spans (offset, length) into one caller-provided text buffer that
// holds every decoded string (selectors are percent-decoded), numeric columns per
// series, and 64-bit keys (series_key of prom_parse.cpp) of each pod (namespace,
// pod), of each history series and of each pod metric family, so the engine
// indexes slots / history rows / families without building Python strings.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

extern "C" uint64_t fm_series_key(const char* a0, const char* a1, const char* b0, const char* b1);  // prom_parse.cpp

namespace {

struct Span {
  const char* p;
  size_t n;
};

// Python str.isspace() over ASCII: \t \n \v \f \r, \x1c-\x1f and space
inline bool is_ws(char c) { return c == ' ' || (c >= '\t' && c <= '\r') || (c >= '\x1c' && c <= '\x1f'); }

inline Span strip(Span s) {
  while (s.n && is_ws(s.p[0])) { ++s.p; --s.n; }
  while (s.n && is_ws(s.p[s.n - 1])) --s.n;
  return s;
}

inline bool eq(Span s, const char* lit) {
  const size_t n = strlen(lit);
  return s.n == n && memcmp(s.p, lit, n) == 0;
}

inline bool starts_with(Span s, const char* lit) {
  const size_t n = strlen(lit);
  return s.n >= n && memcmp(s.p, lit, n) == 0;
}

inline bool ascii(Span s) {
  size_t i = 0;
  uint64_t acc = 0;
  for (; i + 8 <= s.n; i += 8) {
    uint64_t w;
    memcpy(&w, s.p + i, 8);
    acc |= w;
  }
  for (; i < s.n; ++i) acc |= (unsigned char)s.p[i];
  return (acc & 0x8080808080808080ull) == 0;
}

inline const char* find(Span s, const char* lit, size_t from = 0) {
  const size_t n = strlen(lit);
  if (s.n < n || from > s.n - n) return nullptr;
  const char* p = s.p + from;
  const char* last = s.p + s.n - n;  // last position a match can start at
  while (p <= last) {
    p = (const char*)memchr(p, lit[0], (size_t)(last - p) + 1);
    if (!p) return nullptr;
    if (memcmp(p + 1, lit + 1, n - 1) == 0) return p;
    ++p;
  }
  return nullptr;
}

// "alias== url" entries joined by " ||" (urls.parse_config); false on a malformed
// entry, duplicate alias or non-ASCII text (Python's str.strip / sort semantics
// then differ from the byte ones)
bool parse_config(Span cfg, std::vector<std::pair<Span, Span>>& out) {
  out.clear();
  if (!cfg.n) return true;
  if (!ascii(cfg)) return false;
  size_t pos = 0;
  while (true) {
    const char* sep = find(cfg, " ||", pos);
    Span e{cfg.p + pos, (size_t)((sep ? sep : cfg.p + cfg.n) - (cfg.p + pos))};
    e = strip(e);
    if (e.n) {
      const char* kv = find(e, "== ");
      if (!kv) return false;
      Span alias = strip(Span{e.p, (size_t)(kv - e.p)});
      Span url = strip(Span{kv + 3, (size_t)(e.p + e.n - kv - 3)});
      for (auto& x : out)
        if (x.first.n == alias.n && memcmp(x.first.p, alias.p, alias.n) == 0) return false;  // dict: last wins
      out.push_back({alias, url});
    }
    if (!sep) break;
    pos = (size_t)(sep - cfg.p) + 3;
  }
  return true;
}

inline int hexv(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// percent-decoding (urllib.parse.unquote on ASCII results; '+' stays '+', as in
// rollout._unquote); false when a decoded byte is not ASCII
bool unquote(Span s, std::string& out) {
  out.clear();
  out.reserve(s.n);
  for (size_t i = 0; i < s.n; ++i) {
    const char* pct = (const char*)memchr(s.p + i, '%', s.n - i);
    const size_t j = pct ? (size_t)(pct - s.p) : s.n;
    out.append(s.p + i, j - i);  // the literal run up to the next escape
    i = j;
    if (i >= s.n) break;
    char c = s.p[i];
    if (c == '%' && i + 2 < s.n) {
      const int h = hexv(s.p[i + 1]), l = hexv(s.p[i + 2]);
      if (h >= 0 && l >= 0) {
        const int v = h * 16 + l;
        if (v >= 0x80) return false;
        out.push_back((char)v);
        i += 2;
        continue;
      }
    }
    out.push_back(c);
  }
  return true;
}

// plain decimal [-]digits[.digits] (Python float() accepts more: those decline)
bool plain_number(Span s, double& v) {
  if (!s.n || s.n > 30) return false;
  size_t i = 0;
  bool neg = false;
  if (s.p[0] == '-') { neg = true; i = 1; }
  if (i >= s.n) return false;
  if (s.n - i <= 15) {  // the common case, an integer below 1e15: one pass, exact
    long long x = 0;
    size_t k = i;
    for (; k < s.n; ++k) {
      const unsigned d = (unsigned)(s.p[k] - '0');
      if (d > 9) break;
      x = x * 10 + (long long)d;
    }
    if (k == s.n) {
      v = neg ? -(double)x : (double)x;
      return true;
    }
  }
  bool digit = false, dot = false;
  for (size_t k = i; k < s.n; ++k) {
    const char c = s.p[k];
    if (c >= '0' && c <= '9') digit = true;
    else if (c == '.' && !dot) dot = true;
    else return false;
  }
  if (!digit) return false;
  if (!dot && s.n - i <= 15) {  // an integer below 1e15: exact, no strtod
    long long x = 0;
    for (size_t k = i; k < s.n; ++k) x = x * 10 + (s.p[k] - '0');
    v = neg ? -(double)x : (double)x;
    return true;
  }
  char t[32];
  memcpy(t, s.p, s.n);
  t[s.n] = 0;
  v = strtod(t, nullptr);  // correctly rounded, like Python float()
  (void)neg;
  return std::isfinite(v) && std::fabs(v) < 1e15;  // rounds into a long long below
}

struct Grid {
  Span ep;
  std::string sel;
  double start, end, step;
};

// rollout._grid fast shape: exactly the four parameters query / start / end / step
bool parse_grid(Span url, Grid& g) {
  const char* q = find(url, "query_range?");
  if (!q) return false;
  g.ep = Span{url.p, (size_t)(q - url.p)};
  Span qs{q + 12, (size_t)(url.p + url.n - q - 12)};
  Span vals[4];
  bool have[4] = {false, false, false, false};
  static const char* names[4] = {"query", "start", "end", "step"};
  size_t pos = 0;
  int count = 0;
  while (true) {
    const char* amp = (const char*)memchr(qs.p + pos, '&', qs.n - pos);
    Span kv{qs.p + pos, (size_t)((amp ? amp : qs.p + qs.n) - (qs.p + pos))};
    const char* eqp = (const char*)memchr(kv.p, '=', kv.n);
    Span k = eqp ? Span{kv.p, (size_t)(eqp - kv.p)} : kv;
    Span v = eqp ? Span{eqp + 1, (size_t)(kv.p + kv.n - eqp - 1)} : Span{kv.p + kv.n, 0};
    int idx = -1;
    for (int t = 0; t < 4; ++t)
      if (eq(k, names[t])) idx = t;
    if (idx < 0 || have[idx]) return false;
    have[idx] = true;
    vals[idx] = v;
    ++count;
    if (!amp) break;
    pos = (size_t)(amp - qs.p) + 1;
  }
  if (count != 4) return false;
  if (!unquote(vals[0], g.sel)) return false;
  return plain_number(vals[1], g.start) && plain_number(vals[2], g.end) && plain_number(vals[3], g.step);
}

struct Matcher {
  Span label, value;
  bool re;
};

inline bool name_start(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_' || c == ':'; }
inline bool name_char(char c) { return name_start(c) || (c >= '0' && c <= '9'); }
inline bool label_start(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_'; }
inline bool label_char(char c) { return label_start(c) || (c >= '0' && c <= '9'); }

// rollout._SIMPLE_SEL shape with a comma between matchers: name{l="v",l=~"v"}
bool parse_selector(const std::string& s, Span& name, std::vector<Matcher>& ms) {
  ms.clear();
  const char* p = s.data();
  const size_t n = s.size();
  size_t i = 0;
  if (!n || !name_start(p[0])) return false;
  while (i < n && name_char(p[i])) ++i;
  name = Span{p, i};
  if (i >= n || p[i] != '{') return false;
  ++i;
  if (n < 2 || p[n - 1] != '}') return false;
  const size_t close = n - 1;
  while (i < close) {
    if (!label_start(p[i])) return false;
    const size_t l0 = i;
    while (i < close && label_char(p[i])) ++i;
    Matcher m;
    m.label = Span{p + l0, i - l0};
    if (i + 1 < close && p[i] == '=' && p[i + 1] == '~') { m.re = true; i += 2; }
    else if (i < close && p[i] == '=') { m.re = false; i += 1; }
    else return false;
    if (i >= close || p[i] != '"') return false;
    ++i;
    const size_t v0 = i;
    while (i < close && p[i] != '"' && p[i] != '\\') ++i;
    if (i >= close || p[i] != '"') return false;
    m.value = Span{p + v0, i - v0};
    ++i;
    ms.push_back(m);
    if (i < close) {
      if (p[i] != ',') return false;
      ++i;
      if (i == close) break;  // trailing comma
    }
  }
  return true;
}

struct MetaTable {
  bool t[256] = {};
  MetaTable() {
    for (const char* c = "*+?()[]{}^$\\"; *c; ++c) t[(unsigned char)*c] = true;
  }
};
const MetaTable kMeta;

inline bool regex_meta(Span v) {
  bool any = false;
  for (size_t i = 0; i < v.n; ++i) any |= kMeta.t[(unsigned char)v.p[i]];
  return any;
}

// rollout._pods_of: (namespace, sorted distinct pods) of namespace= / pod= / pod=~ "a|b"
bool pods_of(const std::vector<Matcher>& ms, Span& ns, std::vector<Span>& pods) {
  bool have_ns = false, have_pods = false;
  pods.clear();
  for (const Matcher& m : ms) {
    if (eq(m.label, "namespace") && !m.re) { ns = m.value; have_ns = true; }
    else if (eq(m.label, "pod") && !m.re) { pods.assign(1, m.value); have_pods = true; }
    else if (eq(m.label, "pod") && m.re) {
      if (regex_meta(m.value)) return false;
      pods.clear();
      size_t a = 0;
      for (size_t k = 0; k <= m.value.n; ++k) {
        if (k == m.value.n || m.value.p[k] == '|') {
          if (k > a) pods.push_back(Span{m.value.p + a, k - a});
          a = k + 1;
        }
      }
      have_pods = true;
    } else {
      return false;
    }
  }
  if (!have_ns || !have_pods || pods.empty()) return false;
  std::sort(pods.begin(), pods.end(), [](const Span& x, const Span& y) {
    const int c = memcmp(x.p, y.p, std::min(x.n, y.n));
    return c < 0 || (c == 0 && x.n < y.n);
  });
  pods.erase(std::unique(pods.begin(), pods.end(),
                         [](const Span& x, const Span& y) { return x.n == y.n && memcmp(x.p, y.p, x.n) == 0; }),
             pods.end());
  return true;
}

inline long long days_from_civil(long long y, unsigned m, unsigned d) {
  y -= m <= 2;
  const long long era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = (unsigned)(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + (long long)doe - 719468;
}

// RFC3339 "YYYY-MM-DDTHH:MM:SS[.frac]Z" (utils/timeutil.parse_rfc3339; other zones decline)
bool rfc3339_utc(Span s, double& ts) {
  s = strip(s);
  auto dig = [&](size_t i, size_t k, int& v) {
    v = 0;
    for (size_t j = i; j < i + k; ++j) {
      if (j >= s.n || s.p[j] < '0' || s.p[j] > '9') return false;
      v = v * 10 + (s.p[j] - '0');
    }
    return true;
  };
  int y, mo, d, hh, mm, ss;
  if (s.n < 20 || !dig(0, 4, y) || s.p[4] != '-' || !dig(5, 2, mo) || s.p[7] != '-' || !dig(8, 2, d) ||
      (s.p[10] != 'T' && s.p[10] != 't') || !dig(11, 2, hh) || s.p[13] != ':' || !dig(14, 2, mm) ||
      s.p[16] != ':' || !dig(17, 2, ss))
    return false;
  size_t i = 19;
  long long us = 0;
  if (s.p[i] == '.') {
    ++i;
    int nd = 0;
    while (i < s.n && s.p[i] >= '0' && s.p[i] <= '9') {
      if (nd < 6) us = us * 10 + (s.p[i] - '0');
      ++nd;
      ++i;
    }
    if (!nd) return false;
    for (int k = nd; k < 6; ++k) us *= 10;
  }
  if (i + 1 != s.n || (s.p[i] != 'Z' && s.p[i] != 'z')) return false;
  static const int mdays[12] = {31, 29, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  if (y < 1 || mo < 1 || mo > 12 || d < 1 || d > mdays[mo - 1] || hh > 23 || mm > 59 || ss > 59) return false;
  const bool leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
  if (mo == 2 && d == 29 && !leap) return false;
  const long long secs = days_from_civil(y, (unsigned)mo, (unsigned)d) * 86400LL + hh * 3600LL + mm * 60LL + ss;
  ts = (double)(secs * 1000000LL + us) / 1e6;  // (exact integer) / 1e6: timedelta.total_seconds()
  return true;
}

struct Out {
  char* text;
  long long cap, used;
  bool overflow;
  long long put(Span s) {
    if (used + (long long)s.n > cap) { overflow = true; return 0; }
    memcpy(text + used, s.p, s.n);
    const long long off = used;
    used += (long long)s.n;
    return off;
  }
  // "a|b|c": the pods as one RE2 alternation (plain names: no metacharacters but '.')
  long long put_join(const std::vector<Span>& v, long long& len) {
    const long long off = used;
    for (size_t i = 0; i < v.size(); ++i) {
      if (i) put(Span{"|", 1});
      put(v[i]);
    }
    len = used - off;
    return off;
  }
};

inline uint64_t key2(Span a, Span b) { return fm_series_key(a.p, a.p + a.n, b.p, b.p + b.n); }

inline uint64_t key4(Span a, Span b, Span c, Span d) {
  thread_local std::string x, y;
  x.assign(a.p, a.n);
  x.push_back('\x1f');
  x.append(b.p, b.n);
  y.assign(c.p, c.n);
  y.push_back('\x1f');
  y.append(d.p, d.n);
  return fm_series_key(x.data(), x.data() + x.size(), y.data(), y.data() + y.size());
}

inline double pyround(double x) { return std::nearbyint(x); }  // round-half-even, like Python round()

}  // namespace

// Per document d (8 strings at str_off[8 d .. 8 d + 8]: strategy, endTime, current,
// baseline, historical configs, current / baseline / historical metric stores):
//   job_i32[d] = {status (1 planned, 0 decline), first series row, series count}
//   job_f64[d] = endTime (unix seconds)
//   job_span[d] = {app namespace off, len, app off, len}
// per series row s (aliases in sorted order, as _plan):
//   ser_f64[s] = {cur_start, base_start, hist_end}
//   ser_i32[s] = {cur_n, base_n, cur pod0, cur npod, base pod0, base npod, has_base}
//   ser_span[s] = {alias, hist endpoint, hist metric, hist namespace, hist app, cur metric,
//                  base endpoint, base metric, cur pods "a|b", base pods "c|d"} as (off, len) pairs
//   ser_u64[s] = {history key (endpoint\x1fmetric, namespace\x1fapp), family key
//                 (endpoint, cur metric), baseline family key (0 without baseline),
//                 history family key (endpoint, hist metric), app key (namespace, app),
//                 alias key (alias, hist metric): the threshold class of the row}
// per pod p: pod_span[p] = (off, len), pod_u64[p] = series_key(namespace, pod).
// Returns the number of series rows, or -1 when an output capacity was too small.
extern "C" long long fm_plan_rollout(const char* blob, const long long* str_off, long long n_docs, double step,
                                     long long window_cols, int* job_i32, double* job_f64, long long* job_span,
                                     double* ser_f64, int* ser_i32, long long* ser_span, uint64_t* ser_u64,
                                     long long ser_cap, long long* pod_span, uint64_t* pod_u64, long long pod_cap,
                                     char* text, long long text_cap) {
  Out out{text, text_cap, 0, false};
  long long ns_rows = 0, n_pods = 0;
  std::vector<std::pair<Span, Span>> cur, base, hist, store;
  std::vector<Matcher> mh, mc, mb;
  std::vector<Span> pc, pb;
  Grid gh, gc, gb;  // reused: their decoded selectors keep their capacity
  for (long long d = 0; d < n_docs; ++d) {
    int* ji = job_i32 + 3 * d;
    ji[0] = 0;
    ji[1] = (int)ns_rows;
    ji[2] = 0;
    job_f64[d] = 0.0;
    for (int k = 0; k < 4; ++k) job_span[4 * d + k] = 0;
    Span f[8];
    for (int k = 0; k < 8; ++k) f[k] = Span{blob + str_off[8 * d + k], (size_t)(str_off[8 * d + k + 1] - str_off[8 * d + k])};
    // strategy (case-insensitive canary / rollingupdate; anything else: Python decides)
    char strat[16];
    if (f[0].n >= sizeof(strat)) continue;
    for (size_t k = 0; k < f[0].n; ++k) {
      const char c = f[0].p[k];
      strat[k] = (char)((c >= 'A' && c <= 'Z') ? c - 'A' + 'a' : c);
    }
    strat[f[0].n] = 0;
    if (strcmp(strat, "canary") != 0 && strcmp(strat, "rollingupdate") != 0) continue;
    if (!parse_config(f[2], cur) || !parse_config(f[3], base) || !parse_config(f[4], hist)) continue;
    bool stores_ok = true;
    for (int k = 5; k < 8 && stores_ok; ++k) {
      if (!parse_config(f[k], store)) { stores_ok = false; break; }
      for (auto& e : store)
        if (e.second.n && !eq(e.second, "prometheus")) stores_ok = false;
    }
    if (!stores_ok || cur.empty()) continue;
    double end_ts;
    if (!rfc3339_utc(f[1], end_ts)) continue;
    std::sort(cur.begin(), cur.end(), [](const std::pair<Span, Span>& x, const std::pair<Span, Span>& y) {
      const int c = memcmp(x.first.p, y.first.p, std::min(x.first.n, y.first.n));
      return c < 0 || (c == 0 && x.first.n < y.first.n);
    });
    const long long row0 = ns_rows, pod0 = n_pods;
    const long long text0 = out.used;
    bool ok = true, first = true;
    long long app_ns_off = 0, app_ns_len = 0, app_off = 0, app_len = 0;
    for (auto& ce : cur) {
      const Span alias = ce.first;
      const std::pair<Span, Span>* he = nullptr;
      const std::pair<Span, Span>* be = nullptr;
      for (auto& x : hist)
        if (x.first.n == alias.n && memcmp(x.first.p, alias.p, alias.n) == 0) he = &x;
      for (auto& x : base)
        if (x.first.n == alias.n && memcmp(x.first.p, alias.p, alias.n) == 0) be = &x;
      if (!he) { ok = false; break; }
      if (!parse_grid(he->second, gh) || !parse_grid(ce.second, gc)) { ok = false; break; }
      Span nh, nc, nb;
      if (!parse_selector(gh.sel, nh, mh) || !parse_selector(gc.sel, nc, mc)) { ok = false; break; }
      // history: exactly namespace= and app= (the 2-matcher rule of _plan)
      Span hns{nullptr, 0}, happ{nullptr, 0};
      bool has_ns = false, has_app = false;
      for (auto& m : mh) {
        if (m.re) continue;
        if (eq(m.label, "namespace")) { hns = m.value; has_ns = true; }
        else if (eq(m.label, "app")) { happ = m.value; has_app = true; }
        else { has_ns = has_app = false; break; }
      }
      bool any_re = false;
      for (auto& m : mh) any_re |= m.re;
      if (mh.size() != 2 || any_re || !has_ns || !has_app || !nh.n || !nc.n) { ok = false; break; }
      static const char* split[6] = {"namespace_pod_caller:", "namespace_app_caller:", "namespace_app_caller_per_pod:",
                                     "namespace_pod_uri:", "namespace_app_uri:", "namespace_app_uri_per_pod:"};
      bool sp = false;
      for (auto* pre : split) sp |= starts_with(nh, pre) || starts_with(nc, pre);
      if (sp || gh.step != step || gc.step != step || gc.ep.n != gh.ep.n || memcmp(gc.ep.p, gh.ep.p, gh.ep.n) != 0) {
        ok = false;
        break;
      }
      Span cns;
      if (!pods_of(mc, cns, pc) || !(cns.n == hns.n && memcmp(cns.p, hns.p, hns.n) == 0)) { ok = false; break; }
      double b_start = 0.0;
      long long b_n = 0;
      Span bns{nullptr, 0};
      if (be) {
        if (!parse_grid(be->second, gb) || !parse_selector(gb.sel, nb, mb)) { ok = false; break; }
        if (!pods_of(mb, bns, pb) || !(nb.n == nc.n && memcmp(nb.p, nc.p, nc.n) == 0) || gb.step != step ||
            !(bns.n == cns.n && memcmp(bns.p, cns.p, cns.n) == 0)) {
          ok = false;
          break;
        }
        b_start = gb.start;
        const long long span_pts = (long long)pyround((gb.end - gb.start) / step) + 1;
        b_n = std::min(window_cols, span_pts);
        if (b_n > 0 && span_pts > window_cols) b_start = gb.end - (double)(window_cols - 1) * step;
      } else {
        pb.clear();
      }
      if (first) {  // copied now: the spans point into this series' decoded selector
        app_ns_off = out.put(hns);
        app_ns_len = (long long)hns.n;
        app_off = out.put(happ);
        app_len = (long long)happ.n;
        first = false;
      }
      if (ns_rows >= ser_cap || n_pods + (long long)(pc.size() + pb.size()) > pod_cap) return -1;
      const long long s = ns_rows++;
      double* sf = ser_f64 + 3 * s;
      int* si = ser_i32 + 7 * s;
      long long* ss = ser_span + 20 * s;
      uint64_t* su = ser_u64 + 6 * s;
      sf[0] = gc.start;
      sf[1] = b_start;
      sf[2] = gh.end;
      const long long cn = (long long)pyround((gc.end - gc.start) / step) + 1;
      si[0] = (int)std::max(0LL, std::min(window_cols, cn));
      si[1] = (int)b_n;
      si[2] = (int)n_pods;
      si[3] = (int)pc.size();
      for (auto& p : pc) {
        pod_span[2 * n_pods] = out.put(p);
        pod_span[2 * n_pods + 1] = (long long)p.n;
        pod_u64[n_pods] = key2(cns, p);
        ++n_pods;
      }
      si[4] = (int)n_pods;
      si[5] = (int)pb.size();
      for (auto& p : pb) {
        pod_span[2 * n_pods] = out.put(p);
        pod_span[2 * n_pods + 1] = (long long)p.n;
        pod_u64[n_pods] = key2(bns, p);
        ++n_pods;
      }
      si[6] = be ? 1 : 0;
      const Span parts[8] = {alias, gh.ep, nh, hns, happ, nc, be ? gb.ep : Span{"", 0}, be ? nb : Span{"", 0}};
      for (int k = 0; k < 8; ++k) {
        ss[2 * k] = out.put(parts[k]);
        ss[2 * k + 1] = (long long)parts[k].n;
      }
      ss[16] = out.put_join(pc, ss[17]);
      ss[18] = out.put_join(pb, ss[19]);
      su[0] = key4(gh.ep, nh, hns, happ);
      su[1] = key2(gc.ep, nc);
      su[2] = be ? key2(gb.ep, nb) : 0;
      su[3] = key2(gh.ep, nh);
      su[4] = key2(hns, happ);
      su[5] = key2(alias, nh);
    }
    if (out.overflow) return -1;
    if (!ok) {  // roll this document back: Python plans it
      ns_rows = row0;
      n_pods = pod0;
      out.used = text0;
      ji[1] = (int)row0;
      continue;
    }
    ji[0] = 1;
    ji[2] = (int)(ns_rows - row0);
    job_f64[d] = end_ts;
    job_span[4 * d] = app_ns_off;
    job_span[4 * d + 1] = app_ns_len;
    job_span[4 * d + 2] = app_off;
    job_span[4 * d + 3] = app_len;
  }
  return ns_rows;
}
