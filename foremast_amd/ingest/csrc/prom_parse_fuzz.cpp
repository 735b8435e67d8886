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
#include <cstdio>
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
  for (const char* s : kSeeds) run_one(s, checks);
  const int nseeds = (int)(sizeof(kSeeds) / sizeof(kSeeds[0]));
  for (long long it = 0; it < iters; ++it) run_one(mutate(kSeeds[r.below(nseeds)], r), checks);
  std::printf("fuzz OK: %lld inputs, %lld parsed\n", iters + nseeds, checks);
  return 0;
}
