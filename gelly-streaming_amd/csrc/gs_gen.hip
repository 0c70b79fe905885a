// gs_gen.hip -- counter-based synthetic stream generators (spec: DESIGN.md "Workloads").
// Each edge is a pure function of (seed, absolute edge index), so every GPU writes
// its own shard straight into HBM and any sub-range can be regenerated for checks.
#include <hip/hip_runtime.h>

#include <string>

#include "gs_gen.h"

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

constexpr uint32_t TA = 37356, TB = 12452, TC = 12452;  // (0.57, 0.19, 0.19, 0.05) * 2^16

__global__ __launch_bounds__(256) void k_rmat(int64_t* __restrict__ src, int64_t* __restrict__ dst, uint64_t start,
                                              uint64_t count, int scale, uint64_t base, uint64_t idkey, int scramble) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < count; k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = start + k;
    uint64_t s = 0, d = 0, r = 0;
    for (int l = 0; l < scale; ++l) {
      if ((l & 3) == 0) r = mix64(base ^ (i * 8 + (uint64_t)(l >> 2)));
      const uint32_t u = (uint32_t)(r >> (16 * (l & 3))) & 0xFFFFu;
      const uint64_t sb = u >= TA + TB;
      const uint64_t db = (u >= TA && u < TA + TB) || (u >= TA + TB + TC);
      s = (s << 1) | sb;
      d = (d << 1) | db;
    }
    src[k] = scramble ? (int64_t)mix64(s ^ idkey) : (int64_t)s;
    dst[k] = scramble ? (int64_t)mix64(d ^ idkey) : (int64_t)d;
  }
}

__global__ __launch_bounds__(256) void k_er(int64_t* __restrict__ src, int64_t* __restrict__ dst, uint64_t start,
                                            uint64_t count, int logn, uint64_t base, uint64_t idkey, int scramble) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < count; k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = start + k;
    const uint64_t a = mix64(base ^ (2 * i)) >> (64 - logn);
    const uint64_t b = mix64(base ^ (2 * i + 1)) >> (64 - logn);
    src[k] = scramble ? (int64_t)mix64(a ^ idkey) : (int64_t)a;
    dst[k] = scramble ? (int64_t)mix64(b ^ idkey) : (int64_t)b;
  }
}

__global__ __launch_bounds__(256) void k_bip(int64_t* __restrict__ src, int64_t* __restrict__ dst, uint64_t start,
                                             uint64_t count, int logside, uint64_t base, const uint64_t* inj, int ninj) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < count; k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = start + k;
    const uint64_t a = mix64(base ^ (2 * i)) >> (64 - logside);
    const uint64_t b = mix64(base ^ (2 * i + 1)) >> (64 - logside);
    bool same = false;
    for (int q = 0; q < ninj; ++q) same |= inj[q] == i;
    src[k] = (int64_t)(2 * a);
    dst[k] = same ? (int64_t)(2 * b) : (int64_t)(2 * b + 1);
  }
}

uint64_t host_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

unsigned grid_for(uint64_t count) {
  const uint64_t b = (count + 255) / 256;
  return (unsigned)(b < 16384 ? (b ? b : 1) : 16384);
}

}  // namespace

extern "C" {

int gs_gen_rmat(void* stream, int64_t* src, int64_t* dst, uint64_t start, uint64_t count, int scale, uint64_t seed,
                int scramble) {
  if (scale < 1 || scale > 32) return -1;
  if (!count) return 0;
  const uint64_t idkey = host_mix64(seed ^ 0x5CA3B1E5D00DFEEDull);
  hipLaunchKernelGGL(k_rmat, dim3(grid_for(count)), dim3(256), 0, (hipStream_t)stream, src, dst, start, count, scale,
                     host_mix64(seed), idkey, scramble);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int gs_gen_er(void* stream, int64_t* src, int64_t* dst, uint64_t start, uint64_t count, int logn, uint64_t seed,
              int scramble) {
  if (logn < 1 || logn > 63) return -1;
  if (!count) return 0;
  const uint64_t idkey = host_mix64(seed ^ 0x5CA3B1E5D00DFEEDull);
  hipLaunchKernelGGL(k_er, dim3(grid_for(count)), dim3(256), 0, (hipStream_t)stream, src, dst, start, count, logn,
                     host_mix64(seed), idkey, scramble);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int gs_gen_bip(void* stream, int64_t* src, int64_t* dst, uint64_t start, uint64_t count, int logside, uint64_t seed,
               const uint64_t* inject, size_t ninject) {
  if (logside < 1 || logside > 62) return -1;
  if (!count) return 0;
  uint64_t* dinj = nullptr;
  hipStream_t st = (hipStream_t)stream;
  if (ninject) {
    if (hipMalloc(&dinj, ninject * 8) != hipSuccess) return -2;
    if (hipMemcpyAsync(dinj, inject, ninject * 8, hipMemcpyHostToDevice, st) != hipSuccess) return -2;
  }
  hipLaunchKernelGGL(k_bip, dim3(grid_for(count)), dim3(256), 0, st, src, dst, start, count, logside,
                     host_mix64(seed), dinj, (int)ninject);
  hipError_t e = hipGetLastError();
  if (dinj) {
    (void)hipStreamSynchronize(st);
    (void)hipFree(dinj);
  }
  return e == hipSuccess ? 0 : -2;
}

}  // extern "C"
