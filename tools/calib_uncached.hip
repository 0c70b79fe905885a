// Calibration: is a random 16-B probe of a 2 GiB table bound by HBM bytes (128-B L2
// lines) or by the fabric request rate? Same access stream over three allocations:
//   cached      hipMalloc (coarse-grained, L2-cached: every miss fetches a 128-B line)
//   uncached    hipExtMallocWithFlags(hipDeviceMallocUncached) (L2 bypassed)
//   finegrained hipExtMallocWithFlags(hipDeviceMallocFinegrained)
// Kernels: random 16-B loads (2 per thread, independent), random 16-B loads with 4
// in flight per thread, random 64-bit CAS (expected-value mismatch: no store).
// If uncached loads run much faster than cached ones, the fold's probes are byte-bound
// and a smaller fetch granule would raise its rate.
//   calib_uncached [log2 loads = 25]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ void k_rand2(const uint4* __restrict__ tab, uint64_t mask, uint64_t n, uint64_t seed, uint32_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i >= n) return;
  const uint64_t a = mix64(seed ^ (2 * i)) & mask, b = mix64(seed ^ (2 * i + 1)) & mask;
  const uint4 x = tab[a], y = tab[b];
  if ((x.x ^ y.z) == 0x12345678u) out[0] = 1;
}

__global__ void k_rand4(const uint4* __restrict__ tab, uint64_t mask, uint64_t n, uint64_t seed, uint32_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (4 * i >= n) return;
  uint4 x[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) x[k] = tab[mix64(seed ^ (4 * i + k)) & mask];
  if ((x[0].x ^ x[1].y ^ x[2].z ^ x[3].w) == 0x12345678u) out[0] = 1;
}

__global__ void k_cas(unsigned long long* tab, uint64_t mask, uint64_t n, uint64_t seed, uint32_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t a = (mix64(seed ^ i) & mask) * 2;  // 16-B slots, CAS the first 8 B
  const unsigned long long old = atomicCAS(tab + a, 0x7777777777777777ull, 1ull);  // never matches
  if (old == 0x12345678ull) out[0] = 1;
}

int main(int argc, char** argv) {
  const int logn = argc > 1 ? atoi(argv[1]) : 25;
  const uint64_t n = 1ull << logn;
  const uint64_t tbytes = 2ull << 30, nslots = tbytes / 16;
  uint32_t* out;
  CK(hipMalloc(&out, 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* names[3] = {"cached", "uncached", "finegrained"};
  for (int m = 0; m < 3; ++m) {
    void* tab = nullptr;
    if (m == 0) CK(hipMalloc(&tab, tbytes));
    if (m == 1) CK(hipExtMallocWithFlags(&tab, tbytes, hipDeviceMallocUncached));
    if (m == 2) CK(hipExtMallocWithFlags(&tab, tbytes, hipDeviceMallocFinegrained));
    CK(hipMemset(tab, 1, tbytes));
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 2; ++rep) {
      float ms2 = 0, ms4 = 0, msc = 0;
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(k_rand2, dim3((n / 2 + 255) / 256), dim3(256), 0, nullptr, (const uint4*)tab, nslots - 1, n,
                         11 + rep, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms2, a, b));
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(k_rand4, dim3((n / 4 + 255) / 256), dim3(256), 0, nullptr, (const uint4*)tab, nslots - 1, n,
                         23 + rep, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms4, a, b));
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(k_cas, dim3((n / 4 + 255) / 256), dim3(256), 0, nullptr, (unsigned long long*)tab,
                         nslots - 1, n / 4, 37 + rep, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&msc, a, b));
      printf("%-11s rand2 %6.1f G loads/s  rand4 %6.1f G loads/s  cas %6.1f G/s\n", names[m], n / (ms2 * 1e6),
             n / (ms4 * 1e6), n / 4 / (msc * 1e6));
    }
    CK(hipFree(tab));
  }
  return 0;
}
