// Calibration: what does a random 16-B load cost in fabric bytes / time on MI355X?
// Reads N random 16-B slots of a table of T bytes (uniform), plus a streaming
// baseline. Run under rocprofv3 --pmc FETCH_SIZE / TCC_EA0_RDREQ_sum to map
// requests -> bytes for this access pattern (MI355X_MICROARCH.md: calibrate
// non-streaming widths on a known byte count).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ void k_random16(const uint4* __restrict__ tab, uint64_t mask, uint64_t n, uint64_t seed, uint32_t* out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t a = mix64(seed ^ (2 * i)) & mask, b = mix64(seed ^ (2 * i + 1)) & mask;
  uint4 x = tab[a], y = tab[b];
  if ((x.x ^ y.z) == 0x12345678u) out[0] = 1;
}

__global__ void k_random64(const uint4* __restrict__ tab, uint64_t mask, uint64_t n, uint64_t seed, uint32_t* out) {
  // 4 lanes read one 64-B line (16 B each): n/4 random lines
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t line = mix64(seed ^ (i >> 2)) & (mask >> 2);
  uint4 x = tab[line * 4 + (i & 3)];
  if (x.x == 0x12345678u) out[0] = 1;
}

__global__ void k_stream(const uint4* __restrict__ tab, uint64_t n, uint32_t* out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint4 x = tab[i];
  if (x.x == 0x12345678u) out[0] = 1;
}

int main(int argc, char** argv) {
  const uint64_t tbytes = 2ull << 30;  // 2 GiB table (RMAT-26 slot table size)
  const uint64_t nslots = tbytes / 16;
  uint4* tab;
  uint32_t* out;
  hipMalloc(&tab, tbytes);
  hipMalloc(&out, 4);
  hipMemset(tab, 1, tbytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const uint64_t n = 1ull << 21;  // 2M random loads (~ one 1M-edge batch's probes)
  for (int rep = 0; rep < 3; ++rep) {
    float ms;
    hipEventRecord(a);
    k_random16<<<(n + 255) / 256, 256>>>(tab, nslots - 1, n, 42 + rep, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("random16: %llu loads in %.2f us -> %.1f G loads/s, %.1f GB/s useful, %.1f GB/s if 64B, %.1f GB/s if 128B\n",
           (unsigned long long)n, ms * 1e3, n / (ms * 1e6), n * 16 / (ms * 1e6), n * 64 / (ms * 1e6),
           n * 128 / (ms * 1e6));
    hipEventRecord(a);
    k_random64<<<(n + 255) / 256, 256>>>(tab, nslots - 1, n, 77 + rep, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("random64: %llu lines in %.2f us -> %.1f G lines/s, %.1f GB/s\n", (unsigned long long)(n / 4), ms * 1e3,
           n / 4 / (ms * 1e6), n * 16 / (ms * 1e6));
    const uint64_t ns = 1ull << 24;  // 256 MiB streaming
    hipEventRecord(a);
    k_stream<<<(ns + 255) / 256, 256>>>(tab, ns, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("stream16: %.1f MiB in %.2f us -> %.1f GB/s\n", ns * 16 / 1048576.0, ms * 1e3, ns * 16 / (ms * 1e6));
  }
  return 0;
}
