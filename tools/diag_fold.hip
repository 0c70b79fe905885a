// diag_fold.hip -- per-wave timing of k_fold on the first RMAT-26 batches
// (is a slow batch a long tail of a few waves, or uniformly slow?).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -DGS_DIAG_WAVES -Iinclude -Igelly-streaming_amd/csrc \
//          tools/diag_fold.hip gelly-streaming_amd/csrc/gs_kernels.hip gelly-streaming_amd/csrc/gs_gen.hip \
//          -o tools/diag_fold
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "gs_gen.h"
#include "gs_kernels.hpp"

namespace gs {
void diag_copy(uint64_t* w, uint32_t* m, size_t nw, uint32_t* cnt, size_t nt);
void diag_clear(size_t nt);
}

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));              \
      return 1;                                                           \
    }                                                                     \
  } while (0)

int main(int argc, char** argv) {
  const int scale = 26, logb = 20;
  const uint32_t B = 1u << logb;
  const int nb = argc > 1 ? atoi(argv[1]) : 4;
  const int inline_max = argc > 2 ? atoi(argv[2]) : 64;  // 0: append every active edge, hook in k_hook
  const int report_from = argc > 3 ? atoi(argv[3]) : 0;    // fold earlier batches silently
  const uint64_t cap = 1ull << 27;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  gs::Slot* tab;
  uint32_t* ctr;
  uint2* act;
  CK(hipMalloc(&tab, (cap + 2) * sizeof(gs::Slot)));
  CK(hipMalloc(&ctr, gs::CTR_COUNT * gs::kCtrStride * 4));
  CK(hipMemset(ctr, 0, gs::CTR_COUNT * gs::kCtrStride * 4));
  const uint32_t act_cap = ((B / 256 + gs::kShards - 1) / gs::kShards) * 256;
  CK(hipMalloc(&act, sizeof(uint2) * gs::kActSets * gs::kShards * act_cap));
  gs::launch_init(tab, cap + 2, st);
  int64_t *src, *dst;
  CK(hipMalloc(&src, (size_t)nb * B * 8));
  CK(hipMalloc(&dst, (size_t)nb * B * 8));
  if (gs_gen_rmat(st, src, dst, 0, (uint64_t)nb * B, scale, 0x5EED0026, 1)) return 1;
  CK(hipStreamSynchronize(st));
  gs::Table t{};
  t.tab = tab;
  t.ctr = ctr;
  t.cap = (uint32_t)cap;
  t.mask = (uint32_t)(cap - 1);
  t.shift = 64 - 27;
  t.r0 = (uint32_t)cap;
  gs::Lists L{};
  L.act = act;
  L.act_shard_cap = act_cap;
  L.dctr = gs::CTR_DELTA;
  const uint32_t nw = B / 64;
  std::vector<uint64_t> w(2 * nw);
  std::vector<uint32_t> m(nw);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<uint32_t> cnt((size_t)B * 5);
  std::vector<int64_t> hs((size_t)B), hd((size_t)B);
  for (int b = 0; b < nb; ++b) {
    if (b < report_from) {
      gs::launch_fold(false, false, 1, t, L, src + (size_t)b * B, dst + (size_t)b * B, nullptr, B, 1, 1, (int)(b % 3),
                      -1, (int)((b + 1) % 3), 64, 0, -1, nullptr, 0, st);
      continue;
    }
    gs::diag_clear(B);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, st));
    gs::launch_fold(false, false, 1, t, L, src + (size_t)b * B, dst + (size_t)b * B, nullptr, B, 1, 1,
                    (int)(b % 3), -1, (int)((b + 1) % 3), inline_max, 0, -1, nullptr, 0, st);
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (inline_max < 64) {
      float hms;
      std::vector<uint32_t> hc(gs::CTR_COUNT * gs::kCtrStride);
      CK(hipMemcpy(hc.data(), ctr, hc.size() * 4, hipMemcpyDeviceToHost));
      uint64_t nact = 0;
      for (int q = 0; q < gs::kShards; ++q) nact += hc[gs::ctr_index(gs::CTR_ACT + (b % 3) * gs::kShards + q)];
      CK(hipEventRecord(e0, st));
      gs::launch_hook(false, false, t, L, b % 3, gs::kShards * 16, st);
      CK(hipEventRecord(e1, st));
      CK(hipStreamSynchronize(st));
      CK(hipEventElapsedTime(&hms, e0, e1));
      printf("batch %d: k_hook over %llu active edges: %.1f us\n", b, (unsigned long long)nact, hms * 1e3);
    }
    gs::diag_copy(w.data(), m.data(), nw, cnt.data(), B);
    CK(hipMemcpy(hs.data(), src + (size_t)b * B, B * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hd.data(), dst + (size_t)b * B, B * 8, hipMemcpyDeviceToHost));
    {
      const char* nm[5] = {"find_steps", "hook_iters", "cas_fail", "probe_steps", "settles"};
      for (int k = 0; k < 5; ++k) {
        std::vector<uint32_t> v(B);
        uint64_t tot = 0;
        for (uint32_t i = 0; i < B; ++i) {
          v[i] = cnt[(size_t)i * 5 + k];
          tot += v[i];
        }
        std::vector<uint32_t> sv = v;
        std::sort(sv.begin(), sv.end());
        printf("  %-11s total %9llu  p50 %u p99 %u p99.9 %u max %u\n", nm[k], (unsigned long long)tot, sv[B / 2],
               sv[B * 99 / 100], sv[B * 999 / 1000], sv[B - 1]);
      }
      // the thread with the most find steps + hook iterations
      uint32_t worst = 0, wv = 0;
      for (uint32_t i = 0; i < B; ++i) {
        const uint32_t x = cnt[(size_t)i * 5] + cnt[(size_t)i * 5 + 1];
        if (x > wv) wv = x, worst = i;
      }
      printf("  worst thread %u: find %u hook %u casfail %u probe %u settle %u  edge (%lld, %lld)\n", worst,
             cnt[(size_t)worst * 5], cnt[(size_t)worst * 5 + 1], cnt[(size_t)worst * 5 + 2], cnt[(size_t)worst * 5 + 3],
             cnt[(size_t)worst * 5 + 4], (long long)hs[worst], (long long)hd[worst]);
    }
    uint64_t t0 = ~0ull, t1 = 0;
    for (uint32_t i = 0; i < nw; ++i) {
      t0 = std::min(t0, w[2 * i]);
      t1 = std::max(t1, w[2 * i + 1]);
    }
    std::vector<double> dur(nw);
    for (uint32_t i = 0; i < nw; ++i) dur[i] = (w[2 * i + 1] - w[2 * i]) * 0.01;  // us
    std::vector<double> sd = dur;
    std::sort(sd.begin(), sd.end());
    printf("batch %d: event %.1f us, waves span %.1f us; wave duration us p50 %.1f p90 %.1f p99 %.1f p99.9 %.1f max %.1f\n",
           b, ms * 1e3, (t1 - t0) * 0.01, sd[nw / 2], sd[nw * 9 / 10], sd[nw * 99 / 100], sd[nw * 999 / 1000],
           sd[nw - 1]);
    // timeline: how many waves end in each 5% of the span; start of the 10 slowest waves
    int hist[20] = {0};
    for (uint32_t i = 0; i < nw; ++i) {
      int k = (int)((w[2 * i + 1] - t0) * 20 / (t1 - t0 + 1));
      hist[std::min(k, 19)]++;
    }
    printf("  wave ends per 5%% of span:");
    for (int k = 0; k < 20; ++k) printf(" %d", hist[k]);
    printf("\n");
    std::vector<uint32_t> idx(nw);
    for (uint32_t i = 0; i < nw; ++i) idx[i] = i;
    std::partial_sort(idx.begin(), idx.begin() + 8, idx.end(), [&](uint32_t a, uint32_t c) { return dur[a] > dur[c]; });
    printf("  slowest waves (start us, dur us, block, xcc):");
    for (int k = 0; k < 8; ++k)
      printf(" (%.1f, %.1f, %u, %u)", (w[2 * idx[k]] - t0) * 0.01, dur[idx[k]], m[idx[k]] >> 4, m[idx[k]] & 15);
    printf("\n");
    int xh[8] = {0};
    for (uint32_t i = 0; i < nw; ++i) xh[m[i] & 7]++;
    printf("  waves per xcc: %d %d %d %d %d %d %d %d\n", xh[0], xh[1], xh[2], xh[3], xh[4], xh[5], xh[6], xh[7]);
  }
  return 0;
}
