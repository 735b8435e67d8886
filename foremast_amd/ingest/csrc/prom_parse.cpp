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
//                     its (label_a, label_b) values map to (64-bit key,
//                     binary search in the caller's sorted key table), so a
//                     response for any subset of a shard's series lands in
//                     place in one pass with no per-series Python work.
//
//  * fm_prom_decode_tick — a whole tick: many bodies, each split at series
//                     boundaries into chunks that a pool of native threads
//                     decode in parallel (keyed scatter through open-addressing
//                     key indexes, fm_keyindex_new), after a parallel NaN fill.
//
// Hot-path details: strings are skipped 16 bytes at a time (SSE2 compare for
// '"' / '\\'), a series' label object is walked once for both key labels, and
// plain decimals (<= 19 digits, no exponent — every Prometheus sample value
// and timestamp in practice) take an exact fast path: an integer mantissa
// below 2^53 divided by an exact power of ten is one correctly rounded IEEE
// operation, i.e. the same double std::from_chars returns.  Anything else
// goes through std::from_chars (locale independent).  Special values "NaN",
// "+Inf", "-Inf" are accepted.  Returns < 0 on malformed input.
#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

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

// first '"' or '\\' in [p, e) (e if none), 16 bytes per step
inline const char* find_quote_or_bs(const char* p, const char* e) {
  const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\');
  while (e - p >= 16) {
    const __m128i v = _mm_loadu_si128((const __m128i*)p);
    const int m = _mm_movemask_epi8(_mm_or_si128(_mm_cmpeq_epi8(v, q), _mm_cmpeq_epi8(v, bs)));
    if (m) return p + __builtin_ctz((unsigned)m);
    p += 16;
  }
  while (p < e && *p != '"' && *p != '\\') ++p;
  return p;
}

// skip a JSON string (cursor at opening quote); returns false on error
bool skip_string(Cursor& c) {
  if (c.p >= c.e || *c.p != '"') return false;
  ++c.p;
  while (true) {
    c.p = find_quote_or_bs(c.p, c.e);
    if (c.p >= c.e) return false;
    if (*c.p == '"') { ++c.p; return true; }
    if (c.e - c.p < 2) { c.p = c.e; return false; }  // escape: the escaped byte must exist
    c.p += 2;
  }
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

constexpr double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                               1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// [-]digits[.digits], at most 19 digits, mantissa <= 2^53, <= 22 fraction digits:
// exact (see the header); false = use the general parser
inline bool fast_decimal(const char* p, const char* b, double& out) {
  bool neg = false;
  if (p < b && *p == '-') { neg = true; ++p; }
  uint64_t m = 0;
  int nd = 0, frac = 0;
  bool dot = false;
  for (; p < b; ++p) {
    const unsigned d = (unsigned)(*p - '0');
    if (d < 10) {
      if (++nd > 19) return false;
      m = m * 10 + d;
      frac += dot;
    } else if (*p == '.' && !dot) {
      dot = true;
    } else {
      return false;
    }
  }
  if (nd == 0 || m > (1ull << 53) || frac > 22) return false;
  double v = (double)m;
  if (frac) v /= kPow10[frac];
  out = neg ? -v : v;
  return true;
}

// ---- 8 digits at a time (SWAR) ------------------------------------------------
constexpr uint64_t kOnes = 0x0101010101010101ull;
constexpr uint64_t kPow10u[9] = {1, 10, 100, 1000, 10000, 100000, 1000000, 10000000, 100000000};

// k (1..8) ASCII digits ending at `end`, read as one 8-byte load from end - 8
// (the caller guarantees those bytes exist); false unless all k are digits.
inline bool digits8(const char* end, int k, uint64_t& out) {
  uint64_t x;
  memcpy(&x, end - 8, 8);
  const int sh = 8 * (8 - k);  // the leading 8 - k bytes (low bytes, little endian) read as '0'
  const uint64_t keep = sh ? ~0ull << sh : ~0ull;
  x = (x & keep) | (0x30 * kOnes & ~keep);
  // every byte in '0'..'9': high nibble 3, and adding 6 does not carry out of the low nibble
  if ((x & 0xF0 * kOnes) != 0x30 * kOnes || ((x + 6 * kOnes) & 0xF0 * kOnes) != 0x30 * kOnes) return false;
  x -= 0x30 * kOnes;
  x = x * 10 + (x >> 8);  // pairs
  x = (((x & 0x000000FF000000FFull) * (100 + (1000000ull << 32))) +
       (((x >> 16) & 0x000000FF000000FFull) * (1 + (10000ull << 32)))) >> 32;
  out = x;
  return true;
}

// fast_decimal for the common shape — [-]int[.frac] in <= 16 bytes, <= 8
// fraction digits — without a loop per digit: the same mantissa and power of
// ten, so the same double (one correctly rounded division).  Reads the 16
// bytes ending at b, so needs p - lo >= 16 (lo: start of the buffer); false =
// use fast_decimal / from_chars.
inline bool swar_decimal(const char* p, const char* b, const char* lo, double& out) {
  bool neg = false;
  if (p < b && *p == '-') { neg = true; ++p; }
  const long long n = b - p;
  if (n <= 0 || n > 16 || p - lo < 16) return false;
  // the dot among the last n of the 16 bytes ending at b
  const unsigned dm = (unsigned)_mm_movemask_epi8(
                          _mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)(b - 16)), _mm_set1_epi8('.'))) >>
                      (16 - n);
  if (dm & (dm - 1)) return false;  // two dots
  const char* dot = dm ? p + __builtin_ctz(dm) : nullptr;
  const char* ie = dot ? dot : b;
  const int ki = (int)(ie - p), kf = dot ? (int)(b - dot - 1) : 0;
  if (ki + kf == 0 || ki > 16 || kf > 8 || ki + kf > 18) return false;
  uint64_t ip = 0, fp = 0;
  if (ki > 8) {
    uint64_t hi, lo8;
    if (!digits8(ie - 8, ki - 8, hi) || !digits8(ie, 8, lo8)) return false;
    ip = hi * 100000000ull + lo8;
  } else if (ki > 0 && !digits8(ie, ki, ip)) {
    return false;
  }
  if (kf > 0 && !digits8(b, kf, fp)) return false;
  const uint64_t m = ip * kPow10u[kf] + fp;
  if (m > (1ull << 53)) return false;
  double v = (double)m;
  if (kf) v /= kPow10[kf];
  out = neg ? -v : v;
  return true;
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
  if (fast_decimal(a, b, out)) return true;
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

// Series key: a 64-bit word-at-a-time hash of the bytes a + 0x1f + b
// (little-endian 8-byte words, the last one zero-padded; multiply/xorshift
// rounds and a final avalanche).  foremast_amd/ingest/native.py key_hash must
// agree bit for bit.  ~4 multiply rounds for a typical (app, pod) key instead
// of FNV-1a's one serial multiply per byte.
constexpr uint64_t kKeyMul = 0x9E3779B97F4A7C15ull;
inline uint64_t key_round(uint64_t h, uint64_t w) {
  h = (h ^ w) * kKeyMul;
  return h ^ (h >> 29);
}
uint64_t series_key(const char* a0, const char* a1, const char* b0, const char* b1) {
  const size_t na = (size_t)(a1 - a0), nb = (size_t)(b1 - b0), n = na + 1 + nb;
  uint64_t h = 0x243F6A8885A308D3ull ^ (uint64_t)n;
  unsigned char tmp[256];
  std::vector<unsigned char> big;
  unsigned char* buf = tmp;
  if (n + 8 > sizeof(tmp)) { big.resize(n + 8); buf = big.data(); }
  memcpy(buf, a0, na);
  buf[na] = 0x1f;
  memcpy(buf + na + 1, b0, nb);
  memset(buf + n, 0, 8);
  for (size_t i = 0; i < n; i += 8) {
    uint64_t w;
    memcpy(&w, buf + i, 8);
    h = key_round(h, w);
  }
  h ^= h >> 32;
  h *= 0xD6E8FEB86659FD93ull;
  return h ^ (h >> 32);
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

// ---- keyed fast path ---------------------------------------------------------------

// Open-addressing (hash -> row) index of a shard's series keys: one probe per
// series in the common case, instead of a binary search over the sorted table.
//
// It also learns the response LAYOUT: a Prometheus response lists the same
// series in the same (label-sorted) order tick after tick, so for every key
// the index remembers the label object that FOLLOWED it last time (its length,
// a 64-bit hash of its bytes and its slot).  When the next element's label
// bytes hash to the remembered value, its row is known without parsing the
// labels, hashing the key or probing the table.  The remembered record is
// self-checking (the tag folds in the slot and length), so a record torn by a
// concurrent writer (possible only for a key repeated within one body) fails
// the check and falls back to the full path.
struct KeyIndex {
  // one 32-byte entry per key, stored in the order the keys were given (for a
  // table built from a response, the response order): the key, its row and
  // what followed it last time (`nx_*`: the next element's label-object
  // length, its row, its entry, and the self-checking tag).  A repeated
  // response therefore walks the entries sequentially — the prediction for the
  // next element is in the next cache line, which the hardware prefetcher has
  // already fetched — instead of chasing hash-ordered slots through DRAM.  The
  // open-addressing table maps key hash -> entry (int32, 4 bytes a slot: it
  // stays cache-resident) for chunk starts and mispredictions.
  struct Slot {
    uint64_t h;
    uint64_t nx_tag;
    int32_t row;
    int32_t nx_slot;
    int32_t nx_row;
    uint32_t nx_len; // 0: nothing learned
  };
  std::vector<Slot> slots;       // entries, build order
  std::vector<int32_t> table;    // hash slot -> entry (-1: empty)
  uint64_t mask = 0;
  static uint64_t mix(uint64_t h) { h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33; return h; }
  bool build(const uint64_t* hash, const long long* rows, long long n) {
    if (n > 0x3fffffffll) return false;
    uint64_t cap = 16;
    while (cap < (uint64_t)(2 * n)) cap <<= 1;
    table.assign(cap, -1);
    slots.resize((size_t)n);
    mask = cap - 1;
    for (long long j = 0; j < n; ++j) {
      if (rows[j] < 0 || rows[j] > 0x7fffffffll) return false;
      uint64_t i = mix(hash[j]) & mask;
      while (table[i] >= 0) {
        if (slots[table[i]].h == hash[j]) return false;  // duplicate key
        i = (i + 1) & mask;
      }
      table[i] = (int32_t)j;
      slots[j] = Slot{hash[j], 0, (int32_t)rows[j], -1, -1, 0};
    }
    return true;
  }
  // ---- live updates (single-threaded, between decodes) -----------------------------
  // A key's row can change or be retired (row -1: lookups miss, so a retired pod that
  // still reports is counted unmatched instead of landing in its reused slot).  The
  // predictions of `learn` carry entry indices, and a prediction is used only while
  // its entry still holds the predicted row (see keyed_elements), so updates need no
  // prediction reset; a compaction renumbers entries and forgets them all.
  long long dead = 0;
  void rehash(uint64_t cap) {
    table.assign(cap, -1);
    mask = cap - 1;
    for (size_t e = 0; e < slots.size(); ++e) {
      uint64_t i = mix(slots[e].h) & mask;
      while (table[i] >= 0) i = (i + 1) & mask;
      table[i] = (int32_t)e;
    }
  }
  bool upsert(uint64_t h, long long row) {
    if (row < 0 || row > 0x7fffffffll) return false;
    const long long e = find_slot(h);
    if (e >= 0) {
      if (slots[e].row < 0) --dead;
      __atomic_store_n(&slots[e].row, (int32_t)row, __ATOMIC_RELAXED);
      return true;
    }
    if (slots.size() >= 0x3fffffff) return false;
    slots.push_back(Slot{h, 0, (int32_t)row, -1, -1, 0});
    if (2 * slots.size() > table.size()) {
      rehash(table.size() * 2);
    } else {
      uint64_t i = mix(h) & mask;
      while (table[i] >= 0) i = (i + 1) & mask;
      table[i] = (int32_t)(slots.size() - 1);
    }
    return true;
  }
  void retire(uint64_t h) {
    const long long e = find_slot(h);
    if (e >= 0 && slots[e].row >= 0) {
      __atomic_store_n(&slots[e].row, (int32_t)-1, __ATOMIC_RELAXED);
      ++dead;
    }
  }
  void compact() {  // drop retired entries once they are half the index
    if (dead * 2 <= (long long)slots.size()) return;
    std::vector<Slot> keep;
    keep.reserve(slots.size() - (size_t)dead);
    for (const Slot& sl : slots)
      if (sl.row >= 0) keep.push_back(Slot{sl.h, 0, sl.row, -1, -1, 0});
    slots.swap(keep);
    dead = 0;
    uint64_t cap = 16;
    while (cap < 2 * slots.size()) cap <<= 1;
    rehash(cap);
  }
  void prefetch(uint64_t h) const { __builtin_prefetch(&table[mix(h) & mask]); }
  void prefetch_slot(long long i) const { __builtin_prefetch(&slots[i]); }
  long long find_slot(uint64_t h) const {
    uint64_t i = mix(h) & mask;
    while (true) {
      const int32_t e = table[i];
      if (e < 0) return -1;
      if (slots[e].h == h) return e;
      i = (i + 1) & mask;
    }
  }
  long long find(uint64_t h) const {
    const long long i = find_slot(h);
    return i < 0 ? -1 : slots[i].row;
  }
  static uint64_t tag_of(uint64_t bytes_hash, uint32_t len, int32_t slot, int32_t row) {
    return bytes_hash ^ mix(((uint64_t)len << 32) ^ (uint32_t)slot ^ ((uint64_t)(uint32_t)row << 20) ^ 0x5bd1e995ull);
  }
  // record / predict the element that follows the key in slot `prev`
  void learn(long long prev, uint64_t bytes_hash, uint32_t len, int32_t slot) {
    Slot& n = slots[prev];
    const int32_t row = slots[slot].row;
    __atomic_store_n(&n.nx_slot, slot, __ATOMIC_RELAXED);
    __atomic_store_n(&n.nx_row, row, __ATOMIC_RELAXED);
    __atomic_store_n(&n.nx_len, len, __ATOMIC_RELAXED);
    __atomic_store_n(&n.nx_tag, tag_of(bytes_hash, len, slot, row), __ATOMIC_RELAXED);
  }
  bool predict(long long prev, uint32_t& len, int32_t& slot, int32_t& row, uint64_t& tag) const {
    const Slot& n = slots[prev];
    tag = __atomic_load_n(&n.nx_tag, __ATOMIC_RELAXED);
    len = __atomic_load_n(&n.nx_len, __ATOMIC_RELAXED);
    slot = __atomic_load_n(&n.nx_slot, __ATOMIC_RELAXED);
    row = __atomic_load_n(&n.nx_row, __ATOMIC_RELAXED);
    return len > 0 && slot >= 0 && (size_t)slot < slots.size() && row >= 0;
  }
};

// 64-bit hash of a byte span (two independent multiply lanes, 16 bytes per round)
inline uint64_t bytes_hash(const char* p, size_t n) {
  uint64_t a = 0x9E3779B97F4A7C15ull ^ n, b = 0xC2B2AE3D27D4EB4Full;
  size_t i = 0;
  for (; i + 16 <= n; i += 16) {
    uint64_t w0, w1;
    memcpy(&w0, p + i, 8);
    memcpy(&w1, p + i + 8, 8);
    a = (a ^ w0) * 0x9E3779B97F4A7C15ull;
    b = (b ^ w1) * 0xC2B2AE3D27D4EB4Full;
    a ^= a >> 29;
    b ^= b >> 31;
  }
  if (i < n) {
    uint64_t w[2] = {0, 0};
    memcpy(w, p + i, n - i);
    a = (a ^ w[0]) * 0x9E3779B97F4A7C15ull;
    b = (b ^ w[1]) * 0xC2B2AE3D27D4EB4Full;
  }
  return KeyIndex::mix(a ^ ((b << 17) | (b >> 47)));
}

struct Label {
  const char* k;
  size_t n;
};

// Walk a flat label object {"k":"v",...} once (cursor at '{'), taking the raw
// value spans of labels `la` and `lb` (empty when absent).  False for anything
// else (a non-string value, malformed input): strings are skipped exactly as
// skip_container skips them and a flat object has no brace outside them, so
// when this succeeds it ends where brace matching would.
bool scan_labels(Cursor& c, const Label& la, const Label& lb, const char*& a0, const char*& a1, const char*& b0,
                 const char*& b1) {
  a0 = a1 = b0 = b1 = "";
  bool fa = false, fb = false;
  if (!c.eat('{')) return false;
  c.ws();
  if (c.p < c.e && *c.p == '}') { ++c.p; return true; }
  while (true) {
    const char *k0, *k1;
    if (!read_key(c, k0, k1)) return false;
    c.ws();
    if (c.p < c.e && *c.p == '"') {
      const char* v0 = c.p + 1;
      if (!skip_string(c)) return false;
      const size_t kn = (size_t)(k1 - k0);
      // first occurrence wins (as in label_value)
      if (!fa && kn == la.n && memcmp(k0, la.k, kn) == 0) { a0 = v0; a1 = c.p - 1; fa = true; }
      else if (!fb && kn == lb.n && memcmp(k0, lb.k, kn) == 0) { b0 = v0; b1 = c.p - 1; fb = true; }
    } else {
      return false;  // not a flat label object: the caller takes the general path
    }
    if (c.eat(',')) continue;
    if (c.eat('}')) return true;
    return false;
  }
}

struct KeyedOut {
  double start, step;
  long long T;
  float* out;
  long long ld, max_rows;
  Label la, lb;
  const char* lo;  // start of the body (swar_decimal reads up to 8 bytes before a number)
  bool skip_name;  // neither key label is __name__: predictions ignore a leading __name__
};

// Start of the span of a label object (cursor at its '{') that the layout prediction
// hashes: after a leading "__name__":"<metric>", when `skip` — the families of one
// tick (one body per metric, same series order, one shared index) then predict each
// other's elements; their label objects differ only in the metric name.  The label
// object itself otherwise (a name with an escape is not skipped).
inline const char* pred_span(const char* m0, const char* e, bool skip) {
  static const char kName[] = "{\"__name__\":\"";
  if (!skip || e - m0 < 14 || memcmp(m0, kName, 13) != 0) return m0;
  const char* q = find_quote_or_bs(m0 + 13, e);
  return (q + 1 < e && *q == '"' && q[1] == ',') ? q + 2 : m0;
}

// Timestamp text -> grid column by the sample's ordinal in its series: every
// series of a range response carries the same timestamps, so point j of a
// series almost always repeats the text of point j of the previous one.  One
// per decoding thread, reset per chunk (a chunk has one grid).
struct TsCache {
  struct Ent {
    char txt[23];
    uint8_t len;  // 0: empty
    int8_t ok;
    long long col;
  };
  static constexpr long long kCap = 1 << 14;
  std::vector<Ent> ents;
  long long used = 0;
  void reset() {
    for (long long i = 0; i < used; ++i) ents[i].len = 0;
    used = 0;
  }
  // point `j` of a series starting at `a`: on a hit, the column and the end of the text
  const Ent* hit(long long j, const char* a, const char* e) const {
    if (j >= used) return nullptr;
    const Ent& t = ents[j];
    if (!t.len || e - a <= t.len) return nullptr;
    if (t.len < 16 && e - a >= 16) {  // text and its ',' in one 16-byte compare
      const unsigned eq = (unsigned)_mm_movemask_epi8(
          _mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)a), _mm_loadu_si128((const __m128i*)t.txt)));
      const unsigned want = (2u << t.len) - 1;
      return (eq & want) == want ? &t : nullptr;
    }
    return a[t.len] == ',' && memcmp(a, t.txt, t.len) == 0 ? &t : nullptr;
  }
  void put(long long j, const char* a, long long n, long long col, bool ok) {
    if (j >= kCap || n <= 0 || n >= (long long)sizeof(Ent::txt)) return;
    if ((long long)ents.size() <= j) ents.resize((size_t)std::min(kCap, 2 * j + 64));
    while (used <= j) ents[used++].len = 0;
    Ent& t = ents[j];
    memcpy(t.txt, a, (size_t)n);
    t.txt[n] = ',';  // n < sizeof(txt): the separator that follows, compared with the text
    t.len = (uint8_t)n;
    t.ok = ok;
    t.col = col;
  }
};

TsCache& ts_cache() {
  thread_local TsCache c;
  return c;
}

struct KeyedCounts {
  long long series = 0, dropped = 0, unmatched = 0;
};

// Decode result-array elements starting at c.p (an element's '{') into the
// keyed dense matrix; stops after the element that ends the range (the next
// one would start at or past `stop`) or at the array's ']'.  < 0 on error.
// The label key's index slot is prefetched as soon as the key is hashed and
// probed only when the first sample is stored, so the (L3 / DRAM) miss
// overlaps the sample parsing.
long long keyed_elements(Cursor& c, const char* stop, const KeyedOut& o, KeyIndex& ix, KeyedCounts& k) {
  long long prev_slot = -1;  // slot of the previous element of this chunk (-1: unknown / not flat)
  TsCache& tsc = ts_cache();
  tsc.reset();
  const bool swar_ok = o.lo != nullptr;
  while (true) {
    if (!c.eat('{')) return -4;
    long long row = -1, cur_slot = -1;
    bool have_labels = false, resolved = false, flat = false;
    uint64_t key = 0;
    const char* lab0 = nullptr;
    uint32_t lab_len = 0;
    auto resolve = [&]() {
      if (resolved) return;
      resolved = true;
      cur_slot = ix.find_slot(key);
      row = cur_slot < 0 ? -1 : ix.slots[cur_slot].row;
      if (row >= o.max_rows) row = -1;
      if (row < 0) { ++k.unmatched; cur_slot = -1; return; }
      if (flat && prev_slot >= 0) ix.learn(prev_slot, bytes_hash(lab0, lab_len), lab_len, (int32_t)cur_slot);
    };
    // whole-element prediction: {"metric":<the label object that followed the previous
    // element last time>,"values": -- both key scans and the label branch skipped, the
    // same checks as the label branch's prediction below
    bool pre = false;
    if (prev_slot >= 0 && c.e - c.p >= 9 && memcmp(c.p, "\"metric\":", 9) == 0) {
      uint32_t plen;
      int32_t pslot, prow;
      uint64_t ptag;
      const char* m0 = pred_span(c.p + 9, c.e, o.skip_name);
      if (ix.predict(prev_slot, plen, pslot, prow, ptag) && (size_t)(c.e - m0) >= (size_t)plen + 10 &&
          m0[plen - 1] == '}' && memcmp(m0 + plen, ",\"values\":", 10) == 0 &&
          __atomic_load_n(&ix.slots[pslot].row, __ATOMIC_RELAXED) == prow &&
          KeyIndex::tag_of(bytes_hash(m0, plen), plen, pslot, prow) == ptag) {
        c.p = m0 + plen + 10;
        cur_slot = pslot;
        ix.prefetch_slot(pslot);
        row = prow;
        if (row >= o.max_rows) { row = -1; ++k.unmatched; cur_slot = -1; }
        resolved = flat = have_labels = pre = true;
      }
    }
    while (true) {
      const char *k0, *k1;
      static const char kValues[] = "values";
      if (pre) {  // positioned after "values":
        k0 = kValues;
        k1 = kValues + 6;
        pre = false;
      } else if (c.e - c.p >= 9 && c.p[0] == '"' && c.p[7] == '"' && c.p[8] == ':' &&
                 (memcmp(c.p + 1, "metric", 6) == 0 || memcmp(c.p + 1, "values", 6) == 0)) {
        // the two keys of every element, byte-exact and unspaced: no string scan
        k0 = c.p + 1;
        k1 = c.p + 7;
        c.p += 9;
      } else if (!read_key(c, k0, k1)) {
        return -5;
      }
      c.ws();
      const size_t kn = (size_t)(k1 - k0);
      if (kn == 6 && memcmp(k0, "metric", 6) == 0 && !have_labels) {
        const char *a0, *a1, *b0, *b1;
        const char* m0 = c.p;
        have_labels = true;
        // layout prediction: the label object that followed the previous key last time
        uint32_t plen;
        int32_t pslot, prow;
        uint64_t ptag;
        const char* s0 = pred_span(m0, c.e, o.skip_name);
        if (prev_slot >= 0 && ix.predict(prev_slot, plen, pslot, prow, ptag) && (size_t)(c.e - s0) >= plen &&
            s0[plen - 1] == '}' && __atomic_load_n(&ix.slots[pslot].row, __ATOMIC_RELAXED) == prow &&
            KeyIndex::tag_of(bytes_hash(s0, plen), plen, pslot, prow) == ptag) {
          c.p = s0 + plen;
          cur_slot = pslot;
          ix.prefetch_slot(pslot);  // the next element's prediction, needed after the samples
          row = prow;
          if (row >= o.max_rows) { row = -1; ++k.unmatched; cur_slot = -1; }
          resolved = true;
          flat = true;
        } else {
          if (scan_labels(c, o.la, o.lb, a0, a1, b0, b1)) {
            flat = true;  // learnable: the next tick can predict this label object
            lab0 = s0;
            lab_len = (uint32_t)(c.p - s0);
          } else {
            // not flat: brace matching for the extent, then the lenient lookup
            // of fm_prom_dense_keyed, so both decoders agree on any input
            c.p = m0;
            if (!skip_container(c, '{', '}')) return -6;
            a0 = a1 = b0 = b1 = "";
            label_value(m0, c.p, o.la.k, a0, a1);
            label_value(m0, c.p, o.lb.k, b0, b1);
          }
          key = series_key(a0, a1, b0, b1);
          ix.prefetch(key);
        }
      } else if ((kn == 6 && memcmp(k0, "values", 6) == 0) || (kn == 5 && memcmp(k0, "value", 5) == 0)) {
        const bool many = kn == 6;
        if (!have_labels) {  // values before the label object: key of an empty label set
          key = series_key("", "", "", "");
          have_labels = true;
        }
        if (many && !c.eat('[')) return -7;
        c.ws();
        if (!(many && c.eat(']'))) {
          for (long long pt = 0;; ++pt) {
            // every series of a response carries the same timestamps: point pt
            // reuses the grid column of point pt of the previous series when the
            // bytes repeat
            long long gi;
            bool on_grid;
            double v;
            const TsCache::Ent* t;
            const char* q1;
            if (c.e - c.p > 1 && c.p[0] == '[' && (t = tsc.hit(pt, c.p + 1, c.e)) && c.e - c.p > t->len + 3 &&
                c.p[t->len + 2] == '"' && (q1 = find_quote_or_bs(c.p + t->len + 3, c.e)) < c.e - 1 &&
                *q1 == '"' && q1[1] == ']') {
              // compact [ts,"v"] with a known timestamp: no whitespace or token walk
              const char* q0 = c.p + t->len + 3;
              gi = t->col;
              on_grid = t->ok;
              if (!((swar_ok && swar_decimal(q0, q1, o.lo, v)) || parse_number(q0 - 1, q1 + 1, v))) return -12;
              c.p = q1 + 2;
            } else {
              if (!c.eat('[')) return -8;
              c.ws();
              const char* a = c.p;
              if ((t = tsc.hit(pt, a, c.e))) {
                gi = t->col;
                on_grid = t->ok;
                c.p = a + t->len;
              } else {
                while (c.p < c.e && *c.p != ',') ++c.p;
                double ts;
                if (!((swar_ok && swar_decimal(a, c.p, o.lo, ts)) || parse_number(a, c.p, ts))) return -9;
                const double fi = (ts - o.start) / o.step;
                gi = (long long)llround(fi);
                on_grid = !(gi < 0 || gi >= o.T || std::fabs(fi - (double)gi) > 1e-6);
                tsc.put(pt, a, c.p - a, gi, on_grid);
              }
              if (!c.eat(',')) return -10;
              c.ws();
              const char* v0 = c.p;
              if (c.p >= c.e) return -11;
              if (*c.p == '"') {
                if (!skip_string(c)) return -11;
                if (!((swar_ok && swar_decimal(v0 + 1, c.p - 1, o.lo, v)) || parse_number(v0, c.p, v))) return -12;
              } else {
                while (c.p < c.e && *c.p != ']') ++c.p;
                if (!parse_number(v0, c.p, v)) return -12;
              }
              if (!c.eat(']')) return -13;
            }
            resolve();
            if (row < 0 || !on_grid) ++k.dropped;
            else o.out[row * o.ld + gi] = (float)v;
            if (!many) break;
            if (c.p < c.e && *c.p == ',') { ++c.p; continue; }
            if (c.eat(',')) continue;
            if (c.eat(']')) break;
            return -14;
          }
        }
      } else if (!skip_value(c)) {
        return -15;
      }
      if (c.eat(',')) continue;
      if (c.eat('}')) break;
      return -16;
    }
    if (!have_labels) key = series_key("", "", "", "");
    resolve();
    // an unmatched series (a pod the node does not watch, e.g. of a job not admitted yet)
    // keeps the chain: the next element is predicted from the last matched one, so only
    // the unmatched element itself takes the full parse
    if (!flat) prev_slot = -1;
    else if (cur_slot >= 0) prev_slot = cur_slot;
    ++k.series;
    if (c.eat(',')) {
      c.ws();
      if (c.p >= stop) return k.series;
      continue;
    }
    if (c.eat(']')) return k.series;
    return -17;
  }
}

// Position just after `"result":[` (ws allowed), or null.
const char* result_array(const char* buf, long long len) {
  const char* end = buf + len;
  for (const char* q = buf; q + 9 <= end; ++q) {
    q = (const char*)memchr(q, '"', (size_t)(end - q));
    if (!q || q + 9 > end) return nullptr;
    if (memcmp(q, "\"result\"", 8) == 0) {
      Cursor c{q + 8, end};
      if (!c.eat(':') || !c.eat('[')) return nullptr;
      return c.p;
    }
  }
  return nullptr;
}

// Up to `parts` series-aligned chunk starts of a body's result array (cut[0] =
// the first element); returns the count (0: empty array, < 0: malformed).  A
// later cut is the first `{"metric"` at or after an even byte split preceded
// (spaces aside) by `},` — a quote inside a JSON string is always escaped, so
// that byte sequence cannot occur inside a label value.
long long split_elements(const char* buf, long long len, int parts, const char** cut) {
  const char* p = result_array(buf, len);
  if (!p) return -1;
  const char* end = buf + len;
  Cursor c{p, end};
  c.ws();
  if (c.p >= end) return -3;
  if (*c.p == ']') return 0;
  cut[0] = c.p;
  long long n = 1;
  static const char pat[] = "{\"metric\"";
  for (int k = 1; k < parts; ++k) {
    const char* q = cut[0] + (end - cut[0]) * (long long)k / parts;
    if (q <= cut[n - 1]) q = cut[n - 1] + 1;
    while (q + 9 <= end) {
      q = (const char*)memchr(q, '{', (size_t)(end - q));
      if (!q || q + 9 > end) { q = end; break; }
      if (memcmp(q, pat, 9) == 0) {
        const char* b = q - 1;
        while (b > cut[0] && (*b == ' ' || *b == '\n' || *b == '\r' || *b == '\t')) --b;
        if (*b == ',' && b > cut[0]) {
          const char* b2 = b - 1;  // the previous element's closing brace
          while (b2 > cut[0] && (*b2 == ' ' || *b2 == '\n' || *b2 == '\r' || *b2 == '\t')) --b2;
          if (*b2 == '}') break;
        }
      }
      ++q;
    }
    if (q + 9 > end) break;
    cut[n++] = q;
  }
  return n;
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

// Key of every series in response order (series_key of its label_a / label_b values):
// builds the KeyTable of a known response layout without per-series Python.
long long fm_prom_keys(const char* buf, long long len, long long max_series, const char* label_a,
                       const char* label_b, uint64_t* out) {
  return walk(
      buf, len,
      [&](long long s, const char* m0, const char* m1) {
        const char *a0 = "", *a1 = a0, *b0 = a0, *b1 = a0;
        label_value(m0, m1, label_a, a0, a1);
        label_value(m0, m1, label_b, b0, b1);
        if (s < max_series) out[s] = series_key(a0, a1, b0, b1);
      },
      [&](long long, double, double) {});
}

// Keyed dense scatter: series s goes to row key_rows[j] where key_hash[j] is the
// series_key of its (label_a, label_b) values (key_hash sorted ascending, n_keys
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
        const uint64_t h = series_key(a0, a1, b0, b1);
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

// ---- key index + parallel tick decode -----------------------------------------------

void* fm_keyindex_new(const uint64_t* key_hash, const long long* key_rows, long long n_keys) {
  KeyIndex* ix = new KeyIndex();
  if (!ix->build(key_hash, key_rows, n_keys)) { delete ix; return nullptr; }
  return ix;
}

void fm_keyindex_free(void* ix) { delete (KeyIndex*)ix; }

// Live index updates: set (insert or re-row) / retire keys; returns n or -1.
long long fm_keyindex_upsert(void* index, const uint64_t* key_hash, const long long* key_rows, long long n) {
  KeyIndex* ix = (KeyIndex*)index;
  if (!ix || n < 0) return -1;
  for (long long j = 0; j < n; ++j)
    if (!ix->upsert(key_hash[j], key_rows[j])) return -1;
  return n;
}

long long fm_keyindex_retire(void* index, const uint64_t* key_hash, long long n) {
  KeyIndex* ix = (KeyIndex*)index;
  if (!ix || n < 0) return -1;
  for (long long j = 0; j < n; ++j) ix->retire(key_hash[j]);
  ix->compact();
  return n;
}

// rows of keys (-1: absent or retired)
long long fm_keyindex_lookup(void* index, const uint64_t* key_hash, long long n, long long* rows) {
  KeyIndex* ix = (KeyIndex*)index;
  if (!ix || n < 0) return -1;
  for (long long j = 0; j < n; ++j) rows[j] = ix->find(key_hash[j]);
  return n;
}

// Keyed dense scatter of one body through a KeyIndex (same outputs as
// fm_prom_dense_keyed).
long long fm_prom_dense_indexed(const char* buf, long long len, double start, double step, long long T, float* out,
                                long long ld, long long max_rows, const char* label_a, const char* label_b,
                                void* index, long long* dropped, long long* unmatched) {
  KeyIndex* ix = (KeyIndex*)index;
  const char* p = result_array(buf, len);
  if (!p || !ix) return -1;
  Cursor c{p, buf + len};
  c.ws();
  KeyedCounts k;
  long long r = 0;
  if (c.eat(']')) {
    r = 0;
  } else {
    const KeyedOut o{start, step, T, out, ld, max_rows, {label_a, strlen(label_a)}, {label_b, strlen(label_b)},
                     buf, strcmp(label_a, "__name__") != 0 && strcmp(label_b, "__name__") != 0};
    r = keyed_elements(c, buf + len + 1, o, *ix, k);
  }
  if (dropped) *dropped = k.dropped;
  if (unmatched) *unmatched = k.unmatched;
  return r;
}

// Persistent decode workers.  A tick's bodies decode in ~2 ms on 16 threads; creating and
// joining 15 std::threads per call (stacks mapped and unmapped every time) cost a 10-15 ms
// stall every few ticks on the GPU hosts.  run() executes fn on n threads (the caller and
// n - 1 workers) and returns when every one has finished; calls are serialised.  The pool is
// rebuilt in a forked child (its workers do not exist there) and never joined (process exit).
namespace {
class DecodePool {
 public:
  void run(int n, const std::function<void()>& fn) {
    std::lock_guard<std::mutex> call(call_mu_);
    if (n <= 1) {
      fn();
      return;
    }
    ensure(n - 1);
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &fn;
      want_ = n - 1;
      started_ = 0;
      done_ = 0;
      ++gen_;
    }
    cv_.notify_all();
    fn();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return done_ == want_; });
    job_ = nullptr;
  }

 private:
  void ensure(int k) {
    std::lock_guard<std::mutex> lk(mu_);
    // a new worker joins from the NEXT call: it starts from the generation current now (read
    // at its own start, a call issued meanwhile would be missed and never completed)
    while ((int)workers_.size() < k) workers_.emplace_back([this, g = gen_] { loop(g); });
  }
  void loop(unsigned long long seen) {
    std::unique_lock<std::mutex> lk(mu_);
    while (true) {
      cv_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      if (started_ >= want_) continue;  // this call needs fewer workers than the pool has
      ++started_;
      const std::function<void()>* f = job_;
      lk.unlock();
      (*f)();
      lk.lock();
      if (++done_ == want_) done_cv_.notify_one();
    }
  }
  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  const std::function<void()>* job_ = nullptr;
  int want_ = 0, started_ = 0, done_ = 0;
  unsigned long long gen_ = 0;
};

DecodePool& decode_pool() {
  static std::mutex mu;
  static DecodePool* pool = nullptr;
  static pid_t owner = 0;
  std::lock_guard<std::mutex> lk(mu);
  if (!pool || owner != getpid()) {  // first use, or a forked child: a fresh pool (the old one leaks)
    pool = new DecodePool();
    owner = getpid();
  }
  return *pool;
}
}  // namespace

// Many bodies at once: body j (keyed by index[j]) is scattered into columns
// [col0s[j], col0s[j] + Ts[j]) of `out` ([max_rows, ld] float32) on the
// (starts[j], step) grid (null arrays: start / T / column 0 for every body) by
// `threads` native threads.  With fill_nan those columns of every row are
// first set to NaN (in parallel); otherwise the caller pre-fills them.  Each
// body is split at series boundaries into chunks sized so the pool stays
// balanced; stats[3j..3j+2] = (series, dropped points, unmatched series) of
// body j, or stats[3j] < 0 when body j is malformed.  Returns 0, or the first
// negative code.
long long fm_prom_decode_bodies(int nb, const char* const* bufs, const long long* lens, void* const* index,
                                const char* label_a, const char* label_b, const double* starts, double start,
                                double step, const long long* Ts, long long T, const long long* col0s, float* out,
                                long long ld, long long max_rows, int threads, int fill_nan, long long* stats) {
  if (nb < 0 || threads < 1) return -1;
  threads = std::min(threads, 256);
  auto st_of = [&](int j) { return starts ? starts[j] : start; };
  auto T_of = [&](int j) { return Ts ? Ts[j] : T; };
  auto c0_of = [&](int j) { return col0s ? col0s[j] : 0ll; };
  for (int j = 0; j < nb; ++j)
    if (T_of(j) < 0 || c0_of(j) < 0 || c0_of(j) + T_of(j) > ld) return -1;
  struct Task { int body; const char* p; const char* stop; const char* end = nullptr; };
  std::vector<Task> tasks;
  long long total = 0;
  for (int j = 0; j < nb; ++j) total += std::max(0ll, lens[j]);
  const long long target = std::max(1ll, total / (4ll * threads));  // ~4 chunks per thread
  std::vector<long long> code(nb, 0);
  for (int j = 0; j < nb; ++j) {
    if (!index[j]) { code[j] = -1; continue; }
    const int parts = (int)std::min<long long>(4096, std::max(1ll, lens[j] / target));
    std::vector<const char*> cut(parts + 1);
    const long long n = split_elements(bufs[j], lens[j], parts, cut.data());
    if (n < 0) { code[j] = n; continue; }
    for (long long i = 0; i < n; ++i)
      tasks.push_back(Task{j, cut[i], i + 1 < n ? cut[i + 1] : bufs[j] + lens[j] + 1});
  }
  const Label la{label_a, strlen(label_a)}, lb{label_b, strlen(label_b)};
  const bool skip_name = strcmp(label_a, "__name__") != 0 && strcmp(label_b, "__name__") != 0;
  std::vector<std::atomic<long long>> acc(3 * (size_t)std::max(nb, 1));
  for (auto& a : acc) a.store(0);
  std::vector<std::atomic<long long>> err(std::max(nb, 1));
  for (auto& a : err) a.store(0);
  std::atomic<long long> next{0};
  std::atomic<long long> fill_next{0};
  const long long rows_per = 4096;
  // the column span every body covers (fill_nan)
  long long fc0 = ld, fc1 = 0;
  for (int j = 0; j < nb; ++j) { fc0 = std::min(fc0, c0_of(j)); fc1 = std::max(fc1, c0_of(j) + T_of(j)); }
  auto work = [&]() {
    const float nan = std::numeric_limits<float>::quiet_NaN();
    while (true) {
      const long long r0 = fill_next.fetch_add(rows_per);
      if (r0 >= max_rows) break;
      const long long r1 = std::min(max_rows, r0 + rows_per);
      for (long long r = r0; r < r1; ++r) std::fill(out + r * ld + fc0, out + r * ld + fc1, nan);
    }
  };
  auto parse = [&]() {
    while (true) {
      const long long t = next.fetch_add(1);
      if (t >= (long long)tasks.size()) break;
      Task& tk = tasks[t];
      const int j = tk.body;
      KeyIndex* ix = (KeyIndex*)index[j];
      Cursor c{tk.p, bufs[j] + lens[j]};
      KeyedCounts k;
      const KeyedOut o{st_of(j), step, T_of(j), out + c0_of(j), ld, max_rows, la, lb, bufs[j], skip_name};
      const long long r = keyed_elements(c, tk.stop, o, *ix, k);
      if (r < 0) { err[j].store(1); continue; }
      tk.end = c.p;
      acc[3 * j].fetch_add(k.series);
      acc[3 * j + 1].fetch_add(k.dropped);
      acc[3 * j + 2].fetch_add(k.unmatched);
    }
  };
  auto run = [&](auto fn) {
    const std::function<void()> f = fn;
    decode_pool().run(threads, f);
  };
  if (fill_nan && fc1 > fc0) run(work);
  if (!tasks.empty()) run(parse);
  // Every chunk but a body's last must have stopped exactly at the next cut.
  // A failed chunk, or one that did not (a cut that was not an element of the
  // result array — impossible in a Prometheus body, possible in malformed or
  // foreign JSON), makes the body's result that of a sequential decode, after
  // its cells (its column range of every row its key index maps to: the only
  // cells a chunk can write) are reset to NaN — unless another body of this
  // call shares the index (its rows may hold that body's data).
  for (size_t t = 0; t + 1 < tasks.size(); ++t) {
    const int j = tasks[t].body;
    if (tasks[t + 1].body == j && tasks[t].end != tasks[t + 1].p) err[j].store(1);
  }
  const float nanf = std::numeric_limits<float>::quiet_NaN();
  for (int j = 0; j < nb; ++j) {
    if (err[j].load() != 1) continue;
    bool shared = false;
    for (int q = 0; q < nb; ++q) shared |= (q != j && index[q] == index[j]);
    if (!shared)
      for (const auto& sl : ((const KeyIndex*)index[j])->slots)
        if (sl.row >= 0 && sl.row < max_rows)
          std::fill(out + sl.row * ld + c0_of(j), out + sl.row * ld + c0_of(j) + T_of(j), nanf);
    long long dr = 0, um = 0;
    const long long r = fm_prom_dense_indexed(bufs[j], lens[j], st_of(j), step, T_of(j), out + c0_of(j), ld,
                                              max_rows, label_a, label_b, index[j], &dr, &um);
    err[j].store(r < 0 ? r : 0);
    acc[3 * j].store(r < 0 ? 0 : r);
    acc[3 * j + 1].store(dr);
    acc[3 * j + 2].store(um);
  }
  long long rc = 0;
  for (int j = 0; j < nb; ++j) {
    const long long s0 = code[j] < 0 ? code[j] : (err[j].load() < 0 ? err[j].load() : acc[3 * j].load());
    if (stats) { stats[3 * j] = s0; stats[3 * j + 1] = acc[3 * j + 1].load(); stats[3 * j + 2] = acc[3 * j + 2].load(); }
    if (s0 < 0 && rc == 0) rc = s0;
  }
  return rc;
}

// One tick: every body on the same (start, step) grid, columns [0, T).
long long fm_prom_decode_tick(int nb, const char* const* bufs, const long long* lens, void* const* index,
                              const char* label_a, const char* label_b, double start, double step, long long T,
                              float* out, long long ld, long long max_rows, int threads, int fill_nan,
                              long long* stats) {
  return fm_prom_decode_bodies(nb, bufs, lens, index, label_a, label_b, nullptr, start, step, nullptr, T, nullptr,
                               out, ld, max_rows, threads, fill_nan, stats);
}

}  // extern "C"

// Batch form of series_key for host-side tables: key i hashes a[i] + 0x1f + b[i]
// where a[i] is A[a_off[i] .. a_off[i] + a_len[i]) (same for b): the rollout
// engine keys tens of thousands of (namespace, pod) pairs per admission batch.
extern "C" long long fm_key_hashes(const char* A, const long long* a_off, const long long* a_len, const char* B,
                                   const long long* b_off, const long long* b_len, long long n, uint64_t* out) {
  if (n < 0 || (n > 0 && (!A || !B || !a_off || !a_len || !b_off || !b_len || !out))) return -1;
  for (long long i = 0; i < n; ++i) {
    const char* a = A + a_off[i];
    const char* b = B + b_off[i];
    out[i] = series_key(a, a + a_len[i], b, b + b_len[i]);
  }
  return n;
}

// Encoder of the same wire format (the Prometheus side of the node benchmarks and
// tests): series s is {"metric":{<labels[lab_off[s] .. lab_off[s + 1])>},"values":[[t,"v"],...]}
// with T points at ts0 + j * step; NaN values are omitted (Prometheus returns no
// sample for a missing scrape).  Values print as the shortest decimal that reads back
// as the same float (std::to_chars).  Returns the bytes written, or -(bytes needed)
// when `cap` is too small.
extern "C" long long fm_prom_render(const char* labels, const long long* lab_off, long long S, const float* vals,
                                    long long T, double ts0, double step, char* out, long long cap) {
  if (S < 0 || T < 0) return 0;
  static const char head[] = "{\"status\":\"success\",\"data\":{\"resultType\":\"matrix\",\"result\":[";
  static const char tail[] = "]}}";
  std::string buf;
  buf.reserve((size_t)(S * (64 + 28 * T)) + 128);
  buf.append(head);
  char num[64];
  for (long long s = 0; s < S; ++s) {
    if (s) buf.push_back(',');
    buf.append("{\"metric\":{");
    buf.append(labels + lab_off[s], (size_t)(lab_off[s + 1] - lab_off[s]));
    buf.append("},\"values\":[");
    bool first = true;
    for (long long j = 0; j < T; ++j) {
      const float v = vals[s * T + j];
      if (std::isnan(v)) continue;
      if (!first) buf.push_back(',');
      first = false;
      buf.push_back('[');
      const double t = ts0 + (double)j * step;
      auto r = std::to_chars(num, num + sizeof(num), (long long)std::llround(t));
      buf.append(num, r.ptr);
      buf.append(",\"");
      r = std::to_chars(num, num + sizeof(num), v);
      buf.append(num, r.ptr);
      buf.append("\"]");
    }
    buf.append("]}");
  }
  buf.append(tail);
  if ((long long)buf.size() > cap) return -(long long)buf.size();
  std::memcpy(out, buf.data(), buf.size());
  return (long long)buf.size();
}

// series_key for the other translation units of this library (job_plan.cpp)
extern "C" uint64_t fm_series_key(const char* a0, const char* a1, const char* b0, const char* b1) {
  return series_key(a0, a1, b0, b1);
}
