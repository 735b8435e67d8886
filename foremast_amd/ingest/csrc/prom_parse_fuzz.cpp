// Sanitizer harness for the native Prometheus matrix decoder (prom_parse.cpp).
//
// Built by tests/test_sanitizers.py with
//   g++ -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all
// and run on the CPU: seed bodies (well-formed matrices, vectors, special
// values, error bodies) and deterministic mutations of them (byte flips,
// truncation, duplication, insertion of JSON punctuation) go through every
// entry point exactly as ingest/native.py calls them — scan to size, scan with
// per-series outputs, fill, dense scatter into a guarded matrix.  Each input
// is copied into an exactly-sized heap buffer so any read past `len` is an
// ASan report.  Exit status 0 = no sanitizer finding and consistent counts.
#include <algorithm>
#include <cstdio>
#include <limits>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "prom_parse.cpp"

namespace {

struct Rng {
  unsigned long long s;
  unsigned next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return (unsigned)(s >> 11);
  }
  unsigned below(unsigned n) { return n ? next() % n : 0; }
};

const char* kSeeds[] = {
    R"({"status":"success","data":{"resultType":"matrix","result":[{"metric":{"__name__":"x","pod":"a-1"},"values":[[1700000000,"1.5"],[1700000060,"NaN"],[1700000120,"+Inf"]]},{"metric":{},"values":[[1700000000.5,"-Inf"],[1700000060,"2e-3"]]}]}})",
    R"({"status":"success","data":{"resultType":"vector","result":[{"metric":{"app":"demo"},"value":[1700000000,"3"]}]}})",
    R"({"status":"success","data":{"resultType":"matrix","result":[]}})",
    R"({"status":"error","errorType":"bad_data","error":"parse error"})",
    R"({"data":{"result":[{"values":[[1,"1"],[2,"2"],[3,"3"]],"metric":{"a":"\"q\\\"","b":[1,{"c":null}]}}]},"status":"success"})",
    R"({"status":"success","data":{"resultType":"matrix","result":[{"metric":{"x":"y"},"values":[[1e300,"1"],[-1e300,"2"],[1700000000,"1e400"]]}]}})",
};

void run_one(const std::string& body, long long& checks) {
  // exactly-sized heap copy: no terminator, so an over-read hits the redzone
  char* buf = (char*)std::malloc(body.size() ? body.size() : 1);
  std::memcpy(buf, body.data(), body.size());
  const long long len = (long long)body.size();
  const long long n = fm_prom_scan(buf, len, 0, nullptr, nullptr, nullptr, nullptr);
  if (n >= 0) {
    std::vector<long long> off(n + 1), cnt(n + 1);
    std::vector<int> ln(n + 1);
    long long tot = -1;
    const long long n2 = fm_prom_scan(buf, len, n, off.data(), ln.data(), cnt.data(), &tot);
    if (n2 != n) { std::fprintf(stderr, "scan count mismatch %lld vs %lld\n", n, n2); std::exit(3); }
    long long sum = 0;
    for (long long i = 0; i < n; ++i) {
      sum += cnt[i];
      if (off[i] >= 0 && (off[i] + ln[i] > len || ln[i] < 0)) { std::fprintf(stderr, "label span out of body\n"); std::exit(3); }
    }
    if (sum != tot) { std::fprintf(stderr, "point count mismatch\n"); std::exit(3); }
    std::vector<double> ts(tot + 1);
    std::vector<float> vals(tot + 1);
    const long long k = fm_prom_fill(buf, len, ts.data(), vals.data(), tot);
    if (k != tot) { std::fprintf(stderr, "fill count %lld vs %lld\n", k, tot); std::exit(3); }
    // dense scatter into a matrix with a guard row on each side
    const long long T = 4, rows = 3, ld = 5;
    std::vector<float> dense((rows + 2) * ld, -7.f);
    long long dropped = 0;
    fm_prom_dense(buf, len, 1700000000.0, 60.0, T, dense.data() + ld, ld, 0, rows, &dropped);
    for (long long j = 0; j < ld; ++j)
      if (dense[j] != -7.f || dense[(rows + 1) * ld + j] != -7.f) { std::fprintf(stderr, "dense guard hit\n"); std::exit(3); }
    // keyed paths: binary-search table, key index, threaded tick decode (the body
    // twice, so it is split into chunks) must agree on a guarded matrix
    if (n > 0) {
      std::vector<uint64_t> keys(n);
      fm_prom_keys(buf, len, n, "__name__", "pod", keys.data());
      std::vector<uint64_t> hs;
      std::vector<long long> rws;
      for (long long i = 0; i < n; ++i)
        if (std::find(hs.begin(), hs.end(), keys[i]) == hs.end()) { hs.push_back(keys[i]); rws.push_back((long long)hs.size() - 1); }
      std::vector<size_t> ord(hs.size());
      for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
      std::sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return hs[x] < hs[y]; });
      std::vector<uint64_t> sh;
      std::vector<long long> sr;
      for (size_t i : ord) { sh.push_back(hs[i]); sr.push_back(rws[i]); }
      const long long kr = (long long)hs.size();
      void* ix = fm_keyindex_new(sh.data(), sr.data(), kr);
      if (!ix) { std::fprintf(stderr, "key index build failed\n"); std::exit(3); }
      // guard rows -7, body rows NaN (the tick decoder resets a re-decoded body's rows to NaN)
      std::vector<float> m1((kr + 2) * ld, -7.f), m2((kr + 2) * ld, -7.f), m3((kr + 2) * ld, -7.f);
      for (long long q = ld; q < (kr + 1) * ld; ++q) m1[q] = m2[q] = m3[q] = std::numeric_limits<float>::quiet_NaN();
      long long d1 = 0, u1 = 0, d2 = 0, u2 = 0;
      const long long r1 = fm_prom_dense_keyed(buf, len, 1700000000.0, 60.0, T, m1.data() + ld, ld, kr, "__name__",
                                               "pod", sh.data(), sr.data(), kr, &d1, &u1);
      const long long r2 = fm_prom_dense_indexed(buf, len, 1700000000.0, 60.0, T, m2.data() + ld, ld, kr, "__name__",
                                                 "pod", ix, &d2, &u2);
      // the body twice, keyed to disjoint row blocks [0, kr) and [kr, 2kr)
      std::vector<long long> sr2(sr);
      for (auto& x : sr2) x += kr;
      void* ix2 = fm_keyindex_new(sh.data(), sr2.data(), kr);
      m3.assign((2 * kr + 2) * ld, std::numeric_limits<float>::quiet_NaN());
      for (long long j = 0; j < ld; ++j) m3[j] = m3[(2 * kr + 1) * ld + j] = -7.f;
      const char* bufs[2] = {buf, buf};
      const long long lens[2] = {len, len};
      void* ixs[2] = {ix, ix2};
      long long st[6];
      // twice: the second decode runs on the layout the first one taught the indexes
      for (int pass = 0; pass < 2; ++pass)
        fm_prom_decode_tick(2, bufs, lens, ixs, "__name__", "pod", 1700000000.0, 60.0, T, m3.data() + ld, ld, 2 * kr,
                            3, 0, st);
      for (long long j = 0; j < ld; ++j)
        if (m2[j] != -7.f || m2[(kr + 1) * ld + j] != -7.f || m3[j] != -7.f || m3[(2 * kr + 1) * ld + j] != -7.f) {
          std::fprintf(stderr, "keyed guard hit\n"); std::exit(3);
        }
      // a key that occurs twice in one body may land in two chunks: which of its
      // values survives is then unspecified, so bodies with repeated keys only
      // get the guard and error-code checks
      const bool unique = kr == n;
      if (r1 >= 0 && (r2 != r1 || d2 != d1 || u2 != u1 || std::memcmp(m1.data(), m2.data(), m1.size() * 4) != 0)) {
        std::fprintf(stderr, "indexed decode disagrees with the table decode\n"); std::exit(3);
      }
      if (r2 >= 0 && (st[0] != r2 || st[3] != r2 || st[1] != d2 || st[2] != u2 ||
                      (unique && (std::memcmp(m2.data() + ld, m3.data() + ld, kr * ld * 4) != 0 ||
                                  std::memcmp(m2.data() + ld, m3.data() + (kr + 1) * ld, kr * ld * 4) != 0)))) {
        std::fprintf(stderr, "tick decode disagrees with the indexed decode\n"); std::exit(3);
      }
      fm_keyindex_free(ix);
      fm_keyindex_free(ix2);
    }
    ++checks;
  }
  std::free(buf);
}

std::string mutate(const std::string& s, Rng& r) {
  std::string t = s;
  const int ops = 1 + (int)r.below(4);
  static const char punct[] = "{}[],:\"\\ 0123456789.eE+-naNIf";
  for (int o = 0; o < ops && !t.empty(); ++o) {
    const size_t i = r.below((unsigned)t.size());
    switch (r.below(5)) {
      case 0: t[i] = (char)(t[i] ^ (1u << r.below(8))); break;
      case 1: t.resize(i); break;
      case 2: t.insert(i, 1, punct[r.below(sizeof(punct) - 1)]); break;
      case 3: t.erase(i, 1 + r.below(8)); break;
      default: t.insert(i, t.substr(i, 1 + r.below(16))); break;
    }
  }
  return t;
}

}  // namespace

int main(int argc, char** argv) {
  const long long iters = argc > 1 ? std::atoll(argv[1]) : 20000;
  Rng r{0x9E3779B97F4A7C15ull};
  long long checks = 0;
  std::vector<std::string> seeds(kSeeds, kSeeds + sizeof(kSeeds) / sizeof(kSeeds[0]));
  // a body with enough series that the tick decoder splits it into chunks
  std::string many = R"({"status":"success","data":{"resultType":"matrix","result":[)";
  for (int i = 0; i < 24; ++i) {
    if (i) many += (i % 5 == 0) ? ",\n " : ",";
    many += R"({"metric":{"__name__":"m","pod":"p-)" + std::to_string(i) + R"("},"values":[[1700000000,")" +
            std::to_string(i) + R"(.25"],[1700000060,")" + std::to_string(2 * i) + R"("]]})";
  }
  many += "]}}";
  seeds.push_back(many);
  for (const auto& s : seeds) run_one(s, checks);
  const unsigned nseeds = (unsigned)seeds.size();
  for (long long it = 0; it < iters; ++it) run_one(mutate(seeds[r.below(nseeds)], r), checks);
  std::printf("fuzz OK: %lld inputs, %lld parsed\n", iters + (long long)nseeds, checks);
  return 0;
}
