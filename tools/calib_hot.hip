// Hot-index calibration (gfx950): can an L2-sized table of the stream's heavy
// hitters cut k_fold's fabric requests per endpoint?
// Real RMAT-26 micro-batches (gs_gen_rmat), a 2 GiB main table of 16-B slots filled
// with every endpoint of the first `fill` edges. A hot table of 2^logH slots holds the
// keys seen >= T times in the stream's FIRST micro-batch (T picked so that at most
// 5/8 of its slots fill). Per endpoint of 32 later micro-batches:
//   A : main-table probe only (what k_fold does today)
//   B : hot probe first; main probe only on a hot miss
//   C : B with non-temporal main-table loads (leave the L2 to hot lines)
//   D : A with non-temporal main loads (reference for C)
// Build: hipcc -O3 --offload-arch=gfx950 -Iinclude tools/calib_hot.hip
//          -Lgelly-streaming_amd/lib -lgs_summary -Wl,-rpath,$PWD/gelly-streaming_amd/lib -o tools/bin/calib_hot
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "gs_gen.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
constexpr int64_t kEmpty = INT64_MIN;

__device__ __forceinline__ uint32_t hmain(int64_t k, int sh) { return (uint32_t)(((uint64_t)k * 0x9E3779B97F4A7C15ull) >> sh); }
__device__ __forceinline__ uint32_t hhot(int64_t k, int sh) { return (uint32_t)(((uint64_t)k * 0xD6E8FEB86659FD93ull) >> sh); }

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4* p) {
  if (NT) {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    uint4 r;
    r.x = v.x;
    r.y = v.y;
    r.z = v.z;
    r.w = v.w;
    return r;
  }
  return *p;
}
__device__ __forceinline__ int64_t key_of(uint4 v) { return (int64_t)(((uint64_t)v.y << 32) | v.x); }

// insert (or count) every endpoint; cnt != 0: slots are {key, count} and counts are added
__global__ void k_insert(uint4* tab, uint32_t mask, int sh, const int64_t* src, const int64_t* dst, uint32_t n, int cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t ks[2] = {src[i], dst[i]};
  for (int j = 0; j < 2; ++j) {
    const int64_t key = ks[j];
    uint32_t h = hmain(key, sh);
    for (uint32_t p = 0; p <= mask; ++p) {
      unsigned long long* kp = reinterpret_cast<unsigned long long*>(tab + h);
      unsigned long long k = __hip_atomic_load(kp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (k == (unsigned long long)kEmpty) k = atomicCAS(kp, (unsigned long long)kEmpty, (unsigned long long)key);
      if (k == (unsigned long long)kEmpty || k == (unsigned long long)key) {
        if (cnt) atomicAdd(kp + 1, 1ull);
        else tab[h].z = h << 1;
        break;
      }
      h = (h + 1) & mask;
    }
  }
}

__global__ void k_hist(const uint4* cnt, uint64_t n, unsigned long long* hist) {
  __shared__ unsigned long long sh[64];
  if (threadIdx.x < 64) sh[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = cnt[s];
    if (key_of(v) == kEmpty) continue;
    const unsigned long long c = ((unsigned long long)v.w << 32) | v.z;
    atomicAdd(&sh[c < 63 ? c : 63], 1ull);
  }
  __syncthreads();
  if (threadIdx.x < 64) atomicAdd(&hist[threadIdx.x], sh[threadIdx.x]);
}

__global__ void k_select(const uint4* cnt, uint64_t n, uint64_t T, uint4* hot, uint32_t hmask, int hsh,
                         unsigned long long* nsel) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = cnt[s];
    const int64_t key = key_of(v);
    if (key == kEmpty) continue;
    const unsigned long long c = ((unsigned long long)v.w << 32) | v.z;
    if (c < T) continue;
    uint32_t h = hhot(key, hsh);
    for (uint32_t p = 0; p <= hmask; ++p) {
      unsigned long long* kp = reinterpret_cast<unsigned long long*>(hot + h);
      const unsigned long long k = atomicCAS(kp, (unsigned long long)kEmpty, (unsigned long long)key);
      if (k == (unsigned long long)kEmpty) {
        hot[h].z = h << 1;
        atomicAdd(nsel, 1ull);
        break;
      }
      h = (h + 1) & hmask;
    }
  }
}

// direct-mapped hot table: slot hhot(key) holds the candidate with the highest count
__global__ void k_dm_max(const uint4* cnt, uint64_t n, uint64_t T, unsigned long long* best, int hsh) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = cnt[s];
    const int64_t key = key_of(v);
    const unsigned long long c = ((unsigned long long)v.w << 32) | v.z;
    if (key == kEmpty || c < T) continue;
    atomicMax(best + hhot(key, hsh), c);
  }
}
__global__ void k_dm_place(const uint4* cnt, uint64_t n, uint64_t T, const unsigned long long* best, uint4* hot, int hsh,
                           unsigned long long* nsel) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = cnt[s];
    const int64_t key = key_of(v);
    const unsigned long long c = ((unsigned long long)v.w << 32) | v.z;
    if (key == kEmpty || c < T) continue;
    const uint32_t h = hhot(key, hsh);
    if (best[h] != c) continue;
    if (atomicCAS(reinterpret_cast<unsigned long long*>(hot + h), (unsigned long long)kEmpty, (unsigned long long)key) ==
        (unsigned long long)kEmpty) {
      hot[h].z = h << 1;
      atomicAdd(nsel, 1ull);
    }
  }
}

template <bool NT>
__device__ __forceinline__ uint32_t probe_main(const uint4* tab, uint32_t mask, int sh, int64_t key, uint32_t h, uint4 v) {
  for (uint32_t p = 0; p <= mask; ++p) {
    const int64_t k = key_of(v);
    if (k == key) return v.z;
    if (k == kEmpty) return 0u;
    h = (h + 1) & mask;
    v = ld<NT>(tab + h);
  }
  return 0u;
}

// hot probe: the key's link if it lives in the hot table, else ~0u
__device__ __forceinline__ uint32_t probe_hot(const uint4* hot, uint32_t hmask, int64_t key, uint32_t h, uint4 v) {
  for (uint32_t p = 0; p <= hmask; ++p) {
    const int64_t k = key_of(v);
    if (k == key) return v.z;
    if (k == kEmpty) return ~0u;
    h = (h + 1) & hmask;
    v = hot[h];
  }
  return ~0u;
}

template <int MODE>  // 0 A, 1 B, 2 C, 3 D
__global__ __launch_bounds__(256) void k_probe(const uint4* tab, uint32_t mask, int sh, const uint4* hot, uint32_t hmask,
                                               int hsh, const int64_t* src, const int64_t* dst, uint32_t n,
                                               uint32_t* sink, unsigned long long* hits) {
  constexpr bool NT = MODE >= 2;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t ku = __builtin_nontemporal_load(src + i), kv = __builtin_nontemporal_load(dst + i);
  uint32_t lu = ~0u, lv = ~0u;
  if (MODE == 1 || MODE == 2) {
    const uint32_t hu = hhot(ku, hsh), hv = hhot(kv, hsh);
    const uint4 a = hot[hu], b = hot[hv];
    lu = probe_hot(hot, hmask, ku, hu, a);
    lv = probe_hot(hot, hmask, kv, hv, b);
    if (hits) {
      const unsigned long long c = (lu != ~0u) + (lv != ~0u);
      if (c) atomicAdd(hits, c);
    }
  }
  const uint32_t hu = hmain(ku, sh), hv = hmain(kv, sh);
  uint4 a{}, b{};
  if (lu == ~0u) a = ld<NT>(tab + hu);
  if (lv == ~0u) b = ld<NT>(tab + hv);
  if (lu == ~0u) lu = probe_main<NT>(tab, mask, sh, ku, hu, a);
  if (lv == ~0u) lv = probe_main<NT>(tab, mask, sh, kv, hv, b);
  if ((lu ^ lv) == 0x12345671u) sink[0] = lu;
}

// K edges per thread (edges i, i + n/K, ...): every probe round of all 2K endpoints
// is issued together (memory-level parallelism across edges).
template <bool HOT, int K, bool DM = false>
__global__ __launch_bounds__(256) void k_probe_k(const uint4* tab, uint32_t mask, int sh, const uint4* hot,
                                                 uint32_t hmask, int hsh, const int64_t* src, const int64_t* dst,
                                                 uint32_t n, uint32_t* sink) {
  const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x, m = n / K;
  if (i0 >= m) return;
  int64_t key[2 * K];
  uint32_t l[2 * K];
  uint4 v[2 * K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    key[2 * j] = __builtin_nontemporal_load(src + i0 + j * m);
    key[2 * j + 1] = __builtin_nontemporal_load(dst + i0 + j * m);
  }
#pragma unroll
  for (int j = 0; j < 2 * K; ++j) l[j] = ~0u;
  if (HOT) {
#pragma unroll
    for (int j = 0; j < 2 * K; ++j) v[j] = hot[hhot(key[j], hsh)];
#pragma unroll
    for (int j = 0; j < 2 * K; ++j)
      l[j] = DM ? (key_of(v[j]) == key[j] ? v[j].z : ~0u) : probe_hot(hot, hmask, key[j], hhot(key[j], hsh), v[j]);
  }
#pragma unroll
  for (int j = 0; j < 2 * K; ++j)
    if (l[j] == ~0u) v[j] = tab[hmain(key[j], sh)];
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < 2 * K; ++j) {
    if (l[j] == ~0u) l[j] = probe_main<false>(tab, mask, sh, key[j], hmain(key[j], sh), v[j]);
    acc ^= l[j];
  }
  if (acc == 0x12345671u) sink[0] = acc;
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int logs = 27, scale = 26;
  const uint64_t fill = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 28);
  const uint64_t slots = 1ull << logs;
  const int sh = 64 - logs;
  const uint32_t B = 1u << 20, NB = 32, first = 500;
  const uint64_t seed = 0x5EED0026ull;
  uint4 *tab, *cnt, *hot;
  int64_t *src, *dst, *fs, *fd;
  uint32_t* sink;
  unsigned long long *hist, *nsel, *hits;
  const int logc = 22;
  const uint64_t cslots = 1ull << logc;
  CK(hipMalloc(&tab, slots * 16));
  CK(hipMalloc(&cnt, cslots * 16));
  CK(hipMalloc(&hot, (1ull << 20) * 16));
  CK(hipMalloc(&src, (size_t)NB * B * 8));
  CK(hipMalloc(&dst, (size_t)NB * B * 8));
  const uint64_t FC = 1ull << 24;
  CK(hipMalloc(&fs, FC * 8));
  CK(hipMalloc(&fd, FC * 8));
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&hist, 64 * 8));
  CK(hipMalloc(&nsel, 8));
  CK(hipMalloc(&hits, 8));
  // main table: {EMPTY, ...}
  CK(hipMemset(tab, 0, slots * 16));
  // key words := INT64_MIN (byte 7 of every slot = 0x80)
  CK(hipMemset2D(reinterpret_cast<char*>(tab) + 7, 16, 0x80, 1, slots));
  printf("filling the main table with the endpoints of the first %llu edges...\n", (unsigned long long)fill);
  for (uint64_t off = 0; off < fill; off += FC) {
    if (gs_gen_rmat(nullptr, fs, fd, off, FC, scale, seed, 1)) return 1;
    k_insert<<<FC / 256, 256>>>(tab, (uint32_t)(slots - 1), sh, fs, fd, (uint32_t)FC, 0);
  }
  CK(hipDeviceSynchronize());
  // heavy hitters of micro-batch 0
  CK(hipMemset(cnt, 0, cslots * 16));
  CK(hipMemset2D(reinterpret_cast<char*>(cnt) + 7, 16, 0x80, 1, cslots));
  if (gs_gen_rmat(nullptr, fs, fd, 0, B, scale, seed, 1)) return 1;
  k_insert<<<B / 256, 256>>>(cnt, (uint32_t)(cslots - 1), 64 - logc, fs, fd, B, 1);
  CK(hipMemset(hist, 0, 64 * 8));
  k_hist<<<2048, 256>>>(cnt, cslots, hist);
  std::vector<unsigned long long> hh(64);
  CK(hipMemcpy(hh.data(), hist, 64 * 8, hipMemcpyDeviceToHost));
  printf("batch-0 occurrence histogram (count: keys):");
  for (int c = 1; c < 64; ++c)
    if (hh[c]) printf(" %d:%llu", c, hh[c]);
  printf("\n");
  if (gs_gen_rmat(nullptr, src, dst, (uint64_t)first * B, (uint64_t)NB * B, scale, seed, 1)) return 1;
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](int mode, int logH, const char* name) -> int {
    const uint32_t hmask = (1u << logH) - 1;
    const int hsh = 64 - logH;
    float best = 1e9f;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (uint32_t b = 0; b < NB; ++b) {
        const int64_t* s = src + (size_t)b * B;
        const int64_t* d = dst + (size_t)b * B;
        if (mode == 0) k_probe<0><<<B / 256, 256>>>(tab, (uint32_t)(slots - 1), sh, hot, hmask, hsh, s, d, B, sink, nullptr);
        if (mode == 1) k_probe<1><<<B / 256, 256>>>(tab, (uint32_t)(slots - 1), sh, hot, hmask, hsh, s, d, B, sink, nullptr);
        if (mode == 2) k_probe<2><<<B / 256, 256>>>(tab, (uint32_t)(slots - 1), sh, hot, hmask, hsh, s, d, B, sink, nullptr);
        if (mode == 3) k_probe<3><<<B / 256, 256>>>(tab, (uint32_t)(slots - 1), sh, hot, hmask, hsh, s, d, B, sink, nullptr);
        if (mode == 12) k_probe_k<false, 2><<<B / 512, 256>>>(tab, (uint32_t)(slots - 1), sh, hot, hmask, hsh, s, d, B, sink);
        if (mode == 14) k_probe_k<false, 4><<<B / 1024, 256>>>(tab, (uint32_t)(slots - 1), sh, hot, hmask, hsh, s, d, B, sink);
        if (mode == 22) k_probe_k<true, 2><<<B / 512, 256>>>(tab, (uint32_t)(slots - 1), sh, hot, hmask, hsh, s, d, B, sink);
        if (mode == 24) k_probe_k<true, 4><<<B / 1024, 256>>>(tab, (uint32_t)(slots - 1), sh, hot, hmask, hsh, s, d, B, sink);
        if (mode == 31) k_probe_k<true, 1, true><<<B / 256, 256>>>(tab, (uint32_t)(slots - 1), sh, hot, hmask, hsh, s, d, B, sink);
        if (mode == 32) k_probe_k<true, 2, true><<<B / 512, 256>>>(tab, (uint32_t)(slots - 1), sh, hot, hmask, hsh, s, d, B, sink);
        if (mode == 34) k_probe_k<true, 4, true><<<B / 1024, 256>>>(tab, (uint32_t)(slots - 1), sh, hot, hmask, hsh, s, d, B, sink);
        if (mode == 28) k_probe_k<true, 8><<<B / 2048, 256>>>(tab, (uint32_t)(slots - 1), sh, hot, hmask, hsh, s, d, B, sink);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    printf("  %-34s %8.2f us/batch -> %6.1f G endpoints/s\n", name, best * 1e3 / NB, 2.0 * B * NB / (best * 1e6));
    return 0;
  };
  if (run(0, 16, "A  main only")) return 1;
  if (run(3, 16, "D  main only, NT loads")) return 1;
  if (run(12, 16, "A2 main only, 2 edges/thread")) return 1;
  if (run(14, 16, "A4 main only, 4 edges/thread")) return 1;
  for (int logH : {15, 16, 17, 18}) {
    const uint64_t H = 1ull << logH;
    // smallest T with sum_{c>=T} keys <= 5/8 H
    uint64_t T = 63, acc = 0;
    for (int c = 63; c >= 2; --c) {
      if (acc + hh[c] > H * 5 / 8) break;
      acc += hh[c];
      T = c;
    }
    CK(hipMemset(hot, 0, H * 16));
    CK(hipMemset2D(reinterpret_cast<char*>(hot) + 7, 16, 0x80, 1, H));
    CK(hipMemset(nsel, 0, 8));
    k_select<<<2048, 256>>>(cnt, cslots, T, hot, (uint32_t)(H - 1), 64 - logH, nsel);
    unsigned long long ns = 0, nh = 0;
    CK(hipMemcpy(&ns, nsel, 8, hipMemcpyDeviceToHost));
    CK(hipMemset(hits, 0, 8));
    for (uint32_t b = 0; b < NB; ++b)
      k_probe<1><<<B / 256, 256>>>(tab, (uint32_t)(slots - 1), sh, hot, (uint32_t)(H - 1), 64 - logH, src + (size_t)b * B,
                                   dst + (size_t)b * B, B, sink, hits);
    CK(hipMemcpy(&nh, hits, 8, hipMemcpyDeviceToHost));
    printf("hot 2^%d slots (%llu KiB): T=%llu, %llu keys, hot share of test endpoints %.3f\n", logH,
           (unsigned long long)(H * 16 >> 10), (unsigned long long)T, ns, (double)nh / (2.0 * B * NB));
    if (run(1, logH, "B  hot first")) return 1;
    if (run(22, logH, "B2 hot first, 2 edges/thread")) return 1;
  }
  unsigned long long* best;
  CK(hipMalloc(&best, (1ull << 20) * 8));
  for (int logH : {15, 16, 17, 18}) {
    const uint64_t H = 1ull << logH;
    for (uint64_t frac8 : {4ull, 8ull}) {  // candidates <= frac8/8 H
      uint64_t T = 63, acc = 0;
      for (int c = 63; c >= 2; --c) {
        if (acc + hh[c] > H * frac8 / 8) break;
        acc += hh[c];
        T = c;
      }
      CK(hipMemset(hot, 0, H * 16));
      CK(hipMemset2D(reinterpret_cast<char*>(hot) + 7, 16, 0x80, 1, H));
      CK(hipMemset(best, 0, H * 8));
      CK(hipMemset(nsel, 0, 8));
      k_dm_max<<<2048, 256>>>(cnt, cslots, T, best, 64 - logH);
      k_dm_place<<<2048, 256>>>(cnt, cslots, T, best, hot, 64 - logH, nsel);
      unsigned long long ns = 0;
      CK(hipMemcpy(&ns, nsel, 8, hipMemcpyDeviceToHost));
      printf("direct-mapped hot 2^%d slots (%llu KiB): T=%llu, %llu keys placed\n", logH,
             (unsigned long long)(H * 16 >> 10), (unsigned long long)T, ns);
      if (run(31, logH, "M1 direct-mapped hot, 1 edge/thread")) return 1;
      if (run(32, logH, "M2 direct-mapped hot, 2 edges/thread")) return 1;
      if (run(34, logH, "M4 direct-mapped hot, 4 edges/thread")) return 1;
    }
  }
  return 0;
}
