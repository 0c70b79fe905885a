// Host-only driver of the CPU oracle (oracle/gs_oracle.cpp) for sanitizer builds:
// tests/test_oracle.py compiles both files with -fsanitize=address,undefined and runs
// this. It exercises every oracle entry point the tests and the bench use -- the
// reference's pin vectors (DisjointSetTest, ConnectedComponentsTest's default stream,
// BipartitenessCheckTest's triangle orders), windowed/partitioned dataflows, a
// growth stream, the parity truth, the quirk Candidates on a generated stream, the
// text edge codec and the CPU baselines -- and exits non-zero on a wrong result.
// (Sanitizer findings abort the process on their own: -fno-sanitize-recover=all.)
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
void or_rmat_edges(uint64_t seed, int scale, uint64_t start, uint64_t count, int scramble, int64_t* src, int64_t* dst);
void or_bip_edges(uint64_t seed, int logside, uint64_t start, uint64_t count, const uint64_t* inject, size_t ninject,
                  int64_t* src, int64_t* dst);
size_t or_cc_labels(const int64_t* src, const int64_t* dst, size_t n, int64_t* out_v, int64_t* out_l, size_t cap);
int or_cc_dataflow(const int64_t* src, const int64_t* dst, const int64_t* win, const int32_t* part, size_t n,
                   int transient_state, char* out, size_t cap, size_t* len);
int or_bip_dataflow(const int64_t* src, const int64_t* dst, const int64_t* win, const int32_t* part, size_t n,
                    int transient_state, char* out, size_t cap, size_t* len);
size_t or_bip_truth(const int64_t* src, const int64_t* dst, size_t n, int* ok, int64_t* out_comp, int64_t* out_v,
                    uint8_t* out_sign, size_t cap);
int64_t or_bip_first_failure(const int64_t* src, const int64_t* dst, size_t n);
int or_disjointset_unit_test();
double or_cpu_baseline_cc(const int64_t* src, const int64_t* dst, size_t n, size_t window);
double or_cpu_baseline_cc_threads(const int64_t* src, const int64_t* dst, size_t n, size_t window, int p);
size_t or_format_edges(const int64_t* src, const int64_t* dst, size_t n, int sep, char* out, size_t cap);
int or_parse_edges(const char* text, size_t len, int sep, int64_t* src, int64_t* dst, size_t cap, uint64_t* n_lines,
                   int64_t* bad_line);
double or_cpu_baseline_bip(const int64_t* src, const int64_t* dst, size_t n);
}

static int failures = 0;
#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      fprintf(stderr, "FAILED %s:%d %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                             \
    }                                                         \
  } while (0)

static std::string dataflow(bool bip, const std::vector<int64_t>& s, const std::vector<int64_t>& d,
                            const std::vector<int64_t>& w, const std::vector<int32_t>& p) {
  std::vector<char> out(1 << 22);
  size_t len = 0;
  const int rc = bip ? or_bip_dataflow(s.data(), d.data(), w.data(), p.data(), s.size(), 0, out.data(), out.size(), &len)
                     : or_cc_dataflow(s.data(), d.data(), w.data(), p.data(), s.size(), 0, out.data(), out.size(), &len);
  CHECK(rc == 0);
  return std::string(out.data(), len);
}

static std::string last_line(const std::string& x) {
  const size_t k = x.rfind('\n');
  return k == std::string::npos ? x : x.substr(k + 1);
}

int main() {
  CHECK(or_disjointset_unit_test() == 0);  // DisjointSetTest.java:37-77

  {  // ConnectedComponentsExample default stream: (k, k+2), 1000-ms windows of ts 100k
    std::vector<int64_t> s, d, w;
    std::vector<int32_t> p;
    for (int k = 1; k <= 100; ++k) {
      s.push_back(k);
      d.push_back(k + 2);
      w.push_back(100 * k / 1000);
      p.push_back(k % 3);
    }
    const std::string out = dataflow(false, s, d, w, p);
    CHECK(!out.empty());
    std::vector<int64_t> v(128), l(128);
    const size_t nv = or_cc_labels(s.data(), d.data(), s.size(), v.data(), l.data(), v.size());
    CHECK(nv == 102);
    for (size_t i = 0; i < nv && i < v.size(); ++i) CHECK(l[i] == ((v[i] & 1) ? 1 : 2));
  }

  {  // BipartitenessCheck triangle orders: quirk (true,...) vs (false,{})
    const std::vector<int64_t> s1{2, 1, 1}, d1{3, 2, 3}, s2{1, 2, 1}, d2{2, 3, 3}, w{0, 0, 0};
    const std::vector<int32_t> p{0, 0, 0};
    CHECK(dataflow(true, s1, d1, w, p).rfind("(true", 0) == 0);
    CHECK(dataflow(true, s2, d2, w, p) == "(false,{})");
  }

  {  // growth stream: RMAT-14 prefix, windowed + partitioned == one window (CC is window-free)
    const size_t n = 1 << 16;
    std::vector<int64_t> s(n), d(n), w(n), w1(n, 0);
    std::vector<int32_t> p(n), p1(n, 0);
    or_rmat_edges(0x5EED0014ull, 14, 0, n, 1, s.data(), d.data());
    for (size_t i = 0; i < n; ++i) {
      w[i] = (int64_t)(i / 4096);
      p[i] = (int32_t)(i % 5);
    }
    CHECK(last_line(dataflow(false, s, d, w, p)) == dataflow(false, s, d, w1, p1));
    std::vector<int64_t> v(n * 2), l(n * 2);
    CHECK(or_cc_labels(s.data(), d.data(), n, v.data(), l.data(), v.size()) > 0);
    CHECK(or_cpu_baseline_cc(s.data(), d.data(), n, 4096) > 0);
    CHECK(or_cpu_baseline_cc_threads(s.data(), d.data(), n, 4096, 4) > 0);
    // text codec round trip
    std::vector<char> text(n * 48);
    const size_t len = or_format_edges(s.data(), d.data(), n, 0, text.data(), text.size());
    std::vector<int64_t> s2(n), d2(n);
    uint64_t lines = 0;
    int64_t bad = 0;
    CHECK(or_parse_edges(text.data(), len, 0, s2.data(), d2.data(), n, &lines, &bad) == 0);
    CHECK(lines == n && bad == -1 && s2 == s && d2 == d);
  }

  {  // bipartite stream with an odd cycle: truth, first failure, quirk Candidates on a prefix
    const size_t n = 1 << 12;
    const uint64_t inject[1] = {n / 2};
    std::vector<int64_t> s(n), d(n), w(n, 0);
    std::vector<int32_t> p(n, 0);
    or_bip_edges(0x5EED0B1Bull, 9, 0, n, inject, 1, s.data(), d.data());
    int ok = -1;
    std::vector<int64_t> comp(2 * n), v(2 * n);
    std::vector<uint8_t> sign(2 * n);
    or_bip_truth(s.data(), d.data(), n / 2, &ok, comp.data(), v.data(), sign.data(), comp.size());
    CHECK(ok == 1);
    const int64_t first = or_bip_first_failure(s.data(), d.data(), n);
    CHECK(first == -1 || first >= (int64_t)(n / 2));
    const std::vector<int64_t> ps(s.begin(), s.begin() + 512), pd(d.begin(), d.begin() + 512), pw(512, 0);
    const std::vector<int32_t> pp(512, 0);
    CHECK(!dataflow(true, ps, pd, pw, pp).empty());
    CHECK(or_cpu_baseline_bip(ps.data(), pd.data(), ps.size()) > 0);
  }

  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("oracle sanitizer driver: all checks passed\n");
  return 0;
}
