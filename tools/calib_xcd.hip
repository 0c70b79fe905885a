// XCD-locality calibration (gfx950): do relabel probes hit the per-XCD L2 more
// often when every XCD only probes its own 1/8 of the table?
// Real RMAT-26 micro-batches (gs_gen_rmat), a 2 GiB table of 16-B slots, one load
// per endpoint at slot = fib_hash(key) (the k_fold first probe).
//   A  : edge order (thread i probes src[i] and dst[i]) -- what k_fold does today
//   B  : endpoints pre-bucketed by table region (top 3 slot bits); a block reads
//        its XCC_ID and grabs chunks of ITS region's bucket (dynamic, atomic cursor)
//   B' : same buckets, block b takes bucket b % 8 regardless of where it runs
// Build: hipcc -O3 --offload-arch=gfx950 -I../include calib_xcd.hip
//          -L../gelly-streaming_amd/lib -lgs_summary -o calib_xcd
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "gs_gen.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
__constant__ int kShift;     // 64 - log2(table slots) (argv[1], default 27)
__constant__ int kRegionShift;  // log2(slots) - 3: the top 3 slot bits pick the region
__device__ __forceinline__ uint32_t slot_of(int64_t k) { return (uint32_t)(((uint64_t)k * 0x9E3779B97F4A7C15ull) >> kShift); }
__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 15u; }

__global__ void k_edge_order(const uint4* tab, const int64_t* src, const int64_t* dst, uint32_t n, uint32_t* sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 a = tab[slot_of(src[i])];
  const uint4 b = tab[slot_of(dst[i])];
  if ((a.x ^ b.x) == 0x12345678u) sink[0] = a.y;
}

__global__ void k_bucket(const int64_t* src, const int64_t* dst, uint32_t n, int64_t* bk, uint32_t bcap, uint32_t* bn) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t k[2] = {src[i], dst[i]};
  for (int j = 0; j < 2; ++j) {
    const uint32_t r = slot_of(k[j]) >> kRegionShift;
    const uint32_t p = atomicAdd(&bn[r], 1u);
    if (p < bcap) bk[(size_t)r * bcap + p] = k[j];
  }
}

template <bool BY_XCC>
__global__ void k_bucketed(const uint4* tab, const int64_t* bk, uint32_t bcap, const uint32_t* bn, uint32_t* cursor,
                           uint32_t* sink) {
  __shared__ uint32_t base;
  const uint32_t r = BY_XCC ? xcc_id() : (blockIdx.x & 7u);
  const uint32_t n = min(bn[r], bcap);
  constexpr uint32_t CH = 512;
  uint32_t acc = 0;
  while (true) {
    if (threadIdx.x == 0) base = atomicAdd(&cursor[r], CH);
    __syncthreads();
    const uint32_t b0 = base;
    __syncthreads();
    if (b0 >= n) break;
    constexpr uint32_t PER = CH / 256;  // all of a thread's probes in flight together
    uint32_t v[PER];
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
      const uint32_t j = b0 + q * 256 + threadIdx.x;
      v[q] = j < n ? tab[slot_of(bk[(size_t)r * bcap + j])].x : 0u;
    }
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) acc ^= v[q];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// static: block b takes region b % 8, chunk b / 8 (no atomics); records its XCC_ID
__global__ void k_static(const uint4* tab, const int64_t* bk, uint32_t bcap, const uint32_t* bn, uint32_t* sink,
                         uint32_t* xcc_of_block) {
  const uint32_t r = blockIdx.x & 7u, c = blockIdx.x >> 3;
  const uint32_t n = min(bn[r], bcap);
  const uint32_t j0 = c * 512 + threadIdx.x, j1 = j0 + 256;
  const uint32_t a = j0 < n ? tab[slot_of(bk[(size_t)r * bcap + j0])].x : 0u;
  const uint32_t b = j1 < n ? tab[slot_of(bk[(size_t)r * bcap + j1])].x : 0u;
  if ((a ^ b) == 0x12345678u) sink[0] = a;
  if (threadIdx.x == 0) xcc_of_block[blockIdx.x] = xcc_id();
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int logs = argc > 1 ? atoi(argv[1]) : 27, scale = argc > 2 ? atoi(argv[2]) : 26;
  const uint64_t slots = 1ull << logs;
  const int sh = 64 - logs, rsh = logs - 3;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(kShift), &sh, sizeof(int)));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(kRegionShift), &rsh, sizeof(int)));
  printf("table 2^%d slots (%llu MiB), RMAT-%d micro-batches\n", logs, (unsigned long long)(slots * 16 >> 20), scale);
  const uint32_t B = 1u << 20, NB = 16, first = 500;
  uint4* tab;
  int64_t *src, *dst, *bk;
  uint32_t *bn, *cur, *sink;
  const uint32_t bcap = (2 * B) / 8 + (2 * B) / 16;
  CK(hipMalloc(&tab, slots * 16));
  CK(hipMemset(tab, 0, slots * 16));
  CK(hipMalloc(&src, (size_t)NB * B * 8));
  CK(hipMalloc(&dst, (size_t)NB * B * 8));
  CK(hipMalloc(&bk, (size_t)NB * 8 * bcap * 8));
  CK(hipMalloc(&bn, NB * 8 * 4));
  CK(hipMalloc(&cur, NB * 8 * 4));
  CK(hipMalloc(&sink, 64));
  if (gs_gen_rmat(nullptr, src, dst, (uint64_t)(scale >= 24 ? first : 0) * B, (uint64_t)NB * B, scale,
                  scale == 26 ? 0x5EED0026ull : 0x5EED0020ull, 1))
    return 1;
  CK(hipMemset(bn, 0, NB * 8 * 4));
  for (uint32_t b = 0; b < NB; ++b)
    k_bucket<<<B / 256, 256>>>(src + (size_t)b * B, dst + (size_t)b * B, B, bk + (size_t)b * 8 * bcap, bcap, bn + b * 8);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> hn(NB * 8);
  CK(hipMemcpy(hn.data(), bn, NB * 32, hipMemcpyDeviceToHost));
  printf("bucket sizes of batch %u:", first);
  for (int r = 0; r < 8; ++r) printf(" %u", hn[r]);
  printf(" (cap %u)\n", bcap);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = B / 256;  // as many blocks as mode A
  uint32_t* xob;
  CK(hipMalloc(&xob, 8192 * 4));
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemset(cur, 0, NB * 32));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (uint32_t b = 0; b < NB; ++b) {
        if (mode == 0)
          k_edge_order<<<B / 256, 256>>>(tab, src + (size_t)b * B, dst + (size_t)b * B, B, sink);
        else if (mode == 1)
          k_bucketed<true><<<grid, 256>>>(tab, bk + (size_t)b * 8 * bcap, bcap, bn + b * 8, cur + b * 8, sink);
        else if (mode == 3)
          k_static<<<(2 * B) / 512 + 8 * 64, 256>>>(tab, bk + (size_t)b * 8 * bcap, bcap, bn + b * 8, sink, xob);
        else
          k_bucketed<false><<<grid, 256>>>(tab, bk + (size_t)b * 8 * bcap, bcap, bn + b * 8, cur + b * 8, sink);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%-28s %8.2f us/batch (2^21 probes) -> %6.1f G probes/s\n",
             mode == 0 ? "A  edge order" : (mode == 1 ? "B  region bucket by XCC_ID" : (mode == 2 ? "B' region bucket by block" : "S  static region b%8")),
             ms * 1e3 / NB, 2.0 * B * NB / (ms * 1e6));
    }
  }
  std::vector<uint32_t> hx(8192);
  CK(hipMemcpy(hx.data(), xob, 8192 * 4, hipMemcpyDeviceToHost));
  int hist[8] = {0};
  const int nblk = (2 * B) / 512 + 8 * 64;
  for (int b = 0; b < nblk; ++b) hist[(hx[b] - (b & 7) + 8) & 7]++;
  printf("static mode, last launch: blocks per (xcc - block%%8) offset:");
  for (int o = 0; o < 8; ++o) printf(" %d", hist[o]);
  printf("\n");
  return 0;
}
