// Sanitizer driver for the host C++ runtime (ops/csrc/host_text.cpp, host_pav.cpp).
// Built by tests/test_native_sanitizers.py with -fsanitize=address,undefined (and
// separately -fsanitize=thread around a multi-threaded caller) and run on the CPU: every
// entry point is driven over random and edge-case inputs, including the tokenizer's
// capacity-overflow path, and PAV is checked against a quadratic reference.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void o3s_host_murmur3(const int64_t* offs, const uint8_t* bytes, int64_t n, uint32_t seed,
                      int64_t num_buckets, int32_t* hash_out, int64_t* bucket_out);
int64_t o3s_host_tokenize(const int64_t* offs, const uint8_t* bytes, int64_t n, uint8_t* out_bytes,
                          int64_t* tok_start, int64_t* tok_end, int64_t cap, int64_t* counts);
int64_t o3s_host_pav(const double* xlo, const double* xhi, const double* y, const double* w, int64_t n,
                     double* oxlo, double* oxhi, double* oy, double* ow);
}

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) { fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } \
  } while (0)

static void pack(const std::vector<std::string>& v, std::vector<int64_t>& offs, std::vector<uint8_t>& bytes) {
  offs.assign(1, 0);
  bytes.clear();
  for (const auto& s : v) {
    bytes.insert(bytes.end(), s.begin(), s.end());
    offs.push_back((int64_t)bytes.size());
  }
  if (bytes.empty()) bytes.push_back(0);   // valid pointer for the empty corpus
}

static void text_checks(uint32_t seed) {
  std::mt19937 rng(seed);
  const char alpha[] = "aB c\tD\nEf  gh ";
  std::vector<std::string> v;
  for (int i = 0; i < 500; ++i) {
    std::string s;
    const int len = (int)(rng() % 40);
    for (int j = 0; j < len; ++j) s.push_back(alpha[rng() % (sizeof(alpha) - 1)]);
    v.push_back(s);
  }
  v.push_back("");
  v.push_back("   ");
  std::vector<int64_t> offs;
  std::vector<uint8_t> bytes;
  pack(v, offs, bytes);
  const int64_t n = (int64_t)v.size();
  std::vector<int32_t> h(n), h2(n);
  std::vector<int64_t> b(n), b2(n);
  o3s_host_murmur3(offs.data(), bytes.data(), n, 42u, 1 << 18, h.data(), b.data());
  o3s_host_murmur3(offs.data(), bytes.data(), n, 42u, 1 << 18, h2.data(), b2.data());
  for (int64_t i = 0; i < n; ++i) {
    CHECK(h[i] == h2[i]);
    CHECK(b[i] >= 0 && b[i] < (1 << 18));
  }
  // tokenizer: exact-capacity run, then a too-small capacity (must report failure, not overflow)
  std::vector<uint8_t> out(bytes.size());
  int64_t cap = (int64_t)bytes.size() + n + 1;      // Spark split: <= one token per byte + one per string
  std::vector<int64_t> ts(cap), te(cap), counts(n);
  const int64_t k = o3s_host_tokenize(offs.data(), bytes.data(), n, out.data(), ts.data(), te.data(), cap,
                                      counts.data());
  CHECK(k >= 0);
  int64_t total = 0;
  for (int64_t i = 0; i < n; ++i) total += counts[i];
  CHECK(total == k);
  for (int64_t q = 0; q < k; ++q) {
    CHECK(ts[q] <= te[q]);                           // empty tokens are legal (Spark split("\\s"))
    CHECK(te[q] <= (int64_t)out.size());
    for (int64_t p = ts[q]; p < te[q]; ++p) CHECK(out[p] != ' ' && !(out[p] >= 'A' && out[p] <= 'Z'));
  }
  if (k > 1) {
    std::vector<int64_t> ts2(k - 1), te2(k - 1);
    const int64_t k2 = o3s_host_tokenize(offs.data(), bytes.data(), n, out.data(), ts2.data(), te2.data(),
                                         k - 1, counts.data());
    CHECK(k2 < 0);
  }
}

static void pav_checks(uint32_t seed) {
  std::mt19937 rng(seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  for (int trial = 0; trial < 200; ++trial) {
    const int n = 1 + (int)(rng() % 60);
    std::vector<double> x(n), y(n), w(n);
    double cur = 0.0;
    for (int i = 0; i < n; ++i) {
      cur += (rng() % 3 == 0) ? 0.0 : U(rng);      // ties in x
      x[i] = cur;
      y[i] = U(rng) * 10.0;
      w[i] = (rng() % 7 == 0) ? 0.0 : 0.1 + U(rng);
    }
    std::vector<double> oxlo(n), oxhi(n), oy(n), ow(n);
    const int64_t m = o3s_host_pav(x.data(), x.data(), y.data(), w.data(), n, oxlo.data(), oxhi.data(),
                                   oy.data(), ow.data());
    CHECK(m >= 0 && m <= n);
    double wsum = 0.0, wy = 0.0, osum = 0.0, owy = 0.0;
    for (int i = 0; i < n; ++i) { wsum += w[i]; wy += w[i] * y[i]; }
    for (int64_t j = 0; j < m; ++j) {
      osum += ow[j];
      owy += ow[j] * oy[j];
      if (j) CHECK(oy[j] > oy[j - 1] - 1e-12);     // isotonic
      CHECK(oxlo[j] <= oxhi[j]);
    }
    CHECK(fabs(wsum - osum) < 1e-9 * (1 + wsum));   // weight and weighted mean preserved
    CHECK(fabs(wy - owy) < 1e-8 * (1 + fabs(wy)));
  }
}

int main(int argc, char** argv) {
  const bool threaded = argc > 1 && strcmp(argv[1], "threads") == 0;
  if (threaded) {     // concurrent callers (widgets run fits on worker threads): must be re-entrant
    std::vector<std::thread> th;
    for (int t = 0; t < 4; ++t) th.emplace_back([t] { text_checks(100 + t); pav_checks(200 + t); });
    for (auto& t : th) t.join();
  } else {
    text_checks(1);
    pav_checks(2);
  }
  if (fails) { fprintf(stderr, "%d checks failed\n", fails); return 1; }
  printf("host sanitizer driver ok (%s)\n", threaded ? "threads" : "serial");
  return 0;
}
