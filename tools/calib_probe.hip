// calib_probe.hip -- ceiling of the relabel-probe pattern on MI355X.
// Measures back-to-back launches (like the 1024 fold launches of one bench step) of
//   rand  : P independent random 16-B loads per thread from a table of T bytes
//   chain : 16-B edge load (streamed) -> 2 random 16-B probes -> 2 dependent 16-B loads
// for table sizes from L2-resident to 2 GiB. Output: G loads/s (and requests/edge).
// Build: hipcc -O3 --offload-arch=gfx950 tools/calib_probe.hip -o tools/calib_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

template <int P>
__global__ __launch_bounds__(256) void k_rand(const uint4* __restrict__ tab, uint64_t mask, uint32_t n, uint64_t seed,
                                              uint32_t* out) {
  const uint32_t i0 = blockIdx.x * (256u * P) + threadIdx.x;
  uint4 x[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const uint32_t i = i0 + p * 256u;
    const uint64_t a = mix64(seed ^ i) & mask;
    x[p] = i < n ? tab[a] : make_uint4(0, 0, 0, 0);
  }
  uint32_t acc = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) acc ^= x[p].x ^ x[p].z;
  if (acc == 0x12345678u) out[0] = acc;
}

// edge -> 2 probes -> 2 dependent loads (addresses taken from the probe results)
__global__ __launch_bounds__(256) void k_chain(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                               const uint4* __restrict__ tab, uint64_t mask, uint32_t n,
                                               uint32_t* out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t u = (uint64_t)src[i], v = (uint64_t)dst[i];
  const uint4 a = tab[(u * 0x9E3779B97F4A7C15ull >> 20) & mask];
  const uint4 b = tab[(v * 0x9E3779B97F4A7C15ull >> 20) & mask];
  const uint4 c = tab[(a.z ^ (uint32_t)u) & mask];
  const uint4 d = tab[(b.z ^ (uint32_t)v) & mask];
  if ((c.x ^ d.y) == 0x12345678u) out[0] = 1;
}

__global__ void k_fill(uint4* tab, uint64_t n) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (uint64_t)gridDim.x * blockDim.x)
    tab[s] = make_uint4((uint32_t)mix64(s), (uint32_t)(s >> 32), (uint32_t)mix64(s + 7), 0);
}

__global__ void k_fill_edges(int64_t* s, int64_t* d, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    s[i] = (int64_t)mix64(2 * i + 1);
    d[i] = (int64_t)mix64(2 * i + 2);
  }
}

int main() {
  const uint64_t maxbytes = 2ull << 30;
  uint4* tab;
  uint32_t* out;
  hipMalloc(&tab, maxbytes);
  hipMalloc(&out, 4);
  k_fill<<<8192, 256>>>(tab, maxbytes / 16);
  const uint64_t ne = 1ull << 26;  // 64M edges = 1 GiB of pairs, cycled through per launch
  int64_t *es, *ed;
  hipMalloc(&es, ne * 8);
  hipMalloc(&ed, ne * 8);
  k_fill_edges<<<8192, 256>>>(es, ed, ne);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const uint64_t sizes[] = {4ull << 20, 16ull << 20, 64ull << 20, 192ull << 20, 512ull << 20, 2ull << 30};
  const uint32_t batch = 1u << 20;  // edges per launch (2^21 probes)
  const int reps = 256;
  for (uint64_t T : sizes) {
    const uint64_t mask = T / 16 - 1;
    float ms;
    // rand: 2^21 loads per launch
    for (int P : {1, 2, 4}) {
      const uint32_t n = 2 * batch;
      const uint32_t g = (n + 256 * P - 1) / (256 * P);
      hipEventRecord(e0);
      for (int r = 0; r < reps; ++r) {
        if (P == 1) k_rand<1><<<g, 256>>>(tab, mask, n, 1000 + r, out);
        if (P == 2) k_rand<2><<<g, 256>>>(tab, mask, n, 1000 + r, out);
        if (P == 4) k_rand<4><<<g, 256>>>(tab, mask, n, 1000 + r, out);
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
      printf("T=%5llu MiB rand P=%d: %.2f us/launch (2^21 loads) -> %.1f G loads/s\n",
             (unsigned long long)(T >> 20), P, ms * 1e3 / reps, (double)n * reps / (ms * 1e6));
    }
    // rand with a big launch (2^26 loads)
    {
      const uint32_t n = 1u << 26;
      hipEventRecord(e0);
      for (int r = 0; r < 8; ++r) k_rand<2><<<n / 512, 256>>>(tab, mask, n, 77 + r, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
      printf("T=%5llu MiB rand P=2 big: %.1f G loads/s\n", (unsigned long long)(T >> 20), (double)n * 8 / (ms * 1e6));
    }
    // chain
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) {
      const uint64_t off = ((uint64_t)r * batch) % ne;
      k_chain<<<batch / 256, 256>>>(es + off, ed + off, tab, mask, batch, out);
    }
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("T=%5llu MiB chain: %.2f us/launch (2^20 edges) -> %.1f G edges/s, %.1f G random loads/s\n",
           (unsigned long long)(T >> 20), ms * 1e3 / reps, (double)batch * reps / (ms * 1e6),
           4.0 * batch * reps / (ms * 1e6));
  }
  return 0;
}
