// Config-5 latency through the C ABI alone, as a JNI caller would drive it (no
// Python): ER G(2^logn, 2^loge) in 2^logw-edge windows, per window one
// gs_fold_take_device (fold + delta rows + count + completion), steady clock around
// the call. Prints one JSON line with p50 / p99 / max in microseconds.
// Usage: window_latency [logn 22] [loge 26] [logw 16] [mode launch|server]
//   launch: one fused k_fold launch per window; server: the resident window server
//   (gs_set_window_server)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gs_gen.h"
#include "gs_summary.h"

int main(int argc, char** argv) {
  const int logn = argc > 1 ? atoi(argv[1]) : 22, loge = argc > 2 ? atoi(argv[2]) : 26, logw = argc > 3 ? atoi(argv[3]) : 16;
  const bool server = argc > 4 && std::string(argv[4]) == "server";
  const uint64_t E = 1ull << loge, B = 1ull << logw, cap = 3 * B + 16;
  int64_t *src = nullptr, *dst = nullptr, *rec = nullptr;
  uint64_t* cnt = nullptr;
  if (hipMalloc(&src, E * 8) != hipSuccess || hipMalloc(&dst, E * 8) != hipSuccess ||
      hipMalloc(&rec, cap * 24) != hipSuccess || hipMalloc(&cnt, 8) != hipSuccess)
    return 3;
  if (gs_gen_er(nullptr, src, dst, 0, E, logn, 0x5EED00E5ull, 1) != GS_OK) return 3;
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  gs_handle h = nullptr;
  if (gs_create(&h, 0, GS_KIND_CC, 1ull << logn) != GS_OK || gs_set_delta_tracking(h, 1) != GS_OK ||
      gs_set_window_server(h, server ? 1 : 0) != GS_OK) {
    std::fprintf(stderr, "%s\n", gs_last_error());
    return 4;
  }
  std::vector<double> lat;
  uint64_t records = 0;
  for (int pass = 0; pass < 2; ++pass) {  // pass 0 warms up
    if (gs_reset(h) != GS_OK || gs_sync(h) != GS_OK) return 4;
    lat.clear();
    records = 0;
    for (uint64_t o = 0; o < E; o += B) {
      uint64_t k = 0;
      const auto t0 = std::chrono::steady_clock::now();
      const int rc = gs_fold_take_device(h, src + o, dst + o, B, rec, cap, cnt, &k);
      lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
      if (rc != GS_OK) {
        std::fprintf(stderr, "%s\n", gs_last_error());
        return 5;
      }
      records += k;
    }
  }
  std::vector<double> s = lat;
  std::sort(s.begin(), s.end());
  const auto pct = [&](double q) { return s[std::min(s.size() - 1, (size_t)(q * (double)s.size()))]; };
  std::printf("{\"mode\": \"%s\", \"windows\": %zu, \"window_edges\": %llu, \"p50_us\": %.2f, \"p99_us\": %.2f, \"max_us\": %.2f, "
              "\"delta_records\": %llu}\n",
              server ? "server" : "launch", lat.size(), (unsigned long long)B, pct(0.5), pct(0.99), s.back(), (unsigned long long)records);
  gs_destroy(h);
  return 0;
}
