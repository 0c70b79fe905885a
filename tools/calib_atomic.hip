// Atomic-throughput calibration on MI355X (gfx950): random device-scope 64/32-bit CAS
// over a 2 GiB table, random plain loads for comparison, and same-address contention
// (n ops on ONE address). Build: hipcc -O3 --offload-arch=gfx950 calib_atomic.hip -o calib_atomic
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x;
}
__global__ void k_cas64(unsigned long long* t, uint64_t mask, uint32_t n, uint64_t seed, unsigned long long* sink) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t h = mix(i + seed) & mask;
  unsigned long long o = atomicCAS(&t[h * 2], 0ull, (unsigned long long)i + 1);
  if (o == 0xdeadull) sink[0] = o;
}
__global__ void k_cas32(uint32_t* t, uint64_t mask, uint32_t n, uint64_t seed, unsigned long long* sink) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t h = mix(i + seed) & mask;
  uint32_t o = atomicCAS(&t[h * 4 + 2], 0u, i + 1);
  if (o == 0xdeadu) sink[0] = o;
}
__global__ void k_load(const uint4* t, uint64_t mask, uint32_t n, uint64_t seed, unsigned long long* sink) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t h = mix(i + seed) & mask;
  uint4 v = t[h];
  if (v.x == 0xdeadu) sink[0] = v.y;
}
__global__ void k_hot_cas(uint32_t* a, uint32_t n, unsigned long long* sink) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t o = atomicCAS(a, i, i + 1);  // mostly fails: one address, n attempts
  if (o == 0xdeadbeefu) sink[0] = o;
}
__global__ void k_hot_cas_spread(uint32_t* a, uint32_t n, uint32_t naddr, unsigned long long* sink) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t o = atomicCAS(a + (i % naddr) * 32, i, i + 1);
  if (o == 0xdeadbeefu) sink[0] = o;
}
__global__ void k_hot_load_fresh(uint32_t* a, uint32_t n, unsigned long long* sink) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t o = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (o == 0xdeadbeefu) sink[0] = o;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const uint64_t slots = 1ull << 27;  // 16-B slots: 2 GiB
  void* tab;
  unsigned long long* sink;
  CK(hipMalloc(&tab, slots * 16));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(tab, 0, slots * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint32_t n = 1u << 21;
  float ms;
  auto timeit = [&](const char* name, auto launch, double ops) {
    launch(); hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1000.0 / 5;
    printf("%-34s %9.2f us/launch  %8.2f G ops/s\n", name, us, ops / us / 1e3);
  };
  uint64_t seed = 1;
  timeit("random load 16B (2 GiB)", [&] { k_load<<<n / 256, 256>>>((const uint4*)tab, slots - 1, n, seed++, sink); }, n);
  timeit("random CAS64 (2 GiB)", [&] { k_cas64<<<n / 256, 256>>>((unsigned long long*)tab, slots - 1, n, seed++, sink); }, n);
  timeit("random CAS32 (2 GiB)", [&] { k_cas32<<<n / 256, 256>>>((uint32_t*)tab, slots - 1, n, seed++, sink); }, n);
  for (uint32_t m : {1u << 10, 1u << 14, 1u << 16, 1u << 18}) {
    char nm[64];
    snprintf(nm, 64, "CAS32 one address x%u", m);
    timeit(nm, [&] { k_hot_cas<<<(m + 255) / 256, 256>>>((uint32_t*)tab, m, sink); }, m);
    snprintf(nm, 64, "fresh load one address x%u", m);
    timeit(nm, [&] { k_hot_load_fresh<<<(m + 255) / 256, 256>>>((uint32_t*)tab, m, sink); }, m);
  }
  for (uint32_t na : {8u, 64u, 512u}) {
    char nm[64];
    snprintf(nm, 64, "CAS32 2^18 ops on %u lines", na);
    timeit(nm, [&] { k_hot_cas_spread<<<(1 << 18) / 256, 256>>>((uint32_t*)tab, 1 << 18, na, sink); }, 1 << 18);
  }
  return 0;
}
