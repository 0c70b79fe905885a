// Is the random-probe rate bound by address translation or by the caches? (gfx950)
// Uniform random 16-B loads (2^25 per launch, 8 in flight per thread) over:
//   contig F     one contiguous footprint of F bytes (F / 2 MiB pages)
//   spread F     the same F bytes of data as 2^k equal chunks, one at the start of each
//                2 MiB page of a 2 GiB allocation (1024 pages touched, same lines)
// Equal rates for equal F => caches decide; spread << contig => translation (TLB) decides.
// Build: hipcc -O3 --offload-arch=gfx950 calib_tlb.hip -o bin/calib_tlb
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// slot index of probe i: `chunk_slots` slots at the start of each of `pages` strided
// chunks `stride_slots` apart (contiguous footprint: pages = 1, chunk = footprint)
__global__ __launch_bounds__(256) void k_probe(const uint4* tab, uint64_t pages, uint64_t chunk_slots,
                                               uint64_t stride_slots, uint64_t seed, uint32_t* sink) {
  constexpr int PER = 8;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  uint4 v[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint64_t r = mix(seed ^ (t * PER + j));
    const uint64_t p = (r >> 32) % pages, o = (r & 0xffffffffull) % chunk_slots;
    v[j] = tab[p * stride_slots + o];
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) acc ^= v[j].x;
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const uint64_t total = 2ull << 30, page = 2ull << 20, slots_per_page = page / 16;
  uint4* tab;
  uint32_t* sink;
  CK(hipMalloc(&tab, total));
  CK(hipMemset(tab, 1, total));
  CK(hipMalloc(&sink, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint64_t probes = 1ull << 25;
  const unsigned grid = (unsigned)(probes / 8 / 256);
  const uint64_t foot[] = {4ull << 20, 32ull << 20, 256ull << 20, 2048ull << 20};
  for (uint64_t f : foot) {
    for (int spread = 0; spread < 2; ++spread) {
      uint64_t pages, chunk, stride;
      if (!spread || f == total) {
        pages = 1;
        chunk = f / 16;
        stride = 0;
      } else {
        pages = total / page;  // 1024 pages, f / 1024 bytes at the start of each
        chunk = f / pages / 16;
        stride = slots_per_page;
      }
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_probe, dim3(grid), dim3(256), 0, 0, tab, pages, chunk, stride, 0x1234ull + rep, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep && ms < best) best = ms;
      }
      printf("%-7s footprint %5llu MiB over %4llu pages: %6.1f G loads/s\n", spread ? "spread" : "contig",
             (unsigned long long)(f >> 20), (unsigned long long)(spread ? pages : (f + page - 1) / page),
             probes / (best * 1e6));
      if (f == total) break;
    }
  }
  return 0;
}
