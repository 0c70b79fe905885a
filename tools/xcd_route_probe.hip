// Price of routing edges to per-XCD table regions ("a routing cost shown
// first"). A stable-free radix partition of an edge stream (two int64 arrays, 16 B per edge)
// into 8 buckets by the region of the source's hash, as a per-XCD fold would need before its
// launches:
//   k_route_hist    per 4096-edge tile, the count of each bucket (reads src: 8 B/edge)
//   k_route_scan    bucket-major exclusive scan of the tile counts (one block)
//   k_route_scatter the tile sorted by bucket in LDS, each bucket's run written contiguously at
//                   its scanned offset (reads 16 B, writes 16 B per edge)
// Checked on 2^22 edges against a host partition count and checksum, then timed on 2^28 edges
// beside a device-to-device copy of the same 32 B/edge. Build:
//   hipcc --offload-arch=gfx950 -O3 tools/xcd_route_probe.hip -o tools/xcd_route_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

constexpr int kBS = 256, kPer = 16, kTile = kBS * kPer, kBuckets = 8;

__host__ __device__ inline unsigned bucket_of(uint64_t v) {
  v ^= v >> 33;
  v *= 0xff51afd7ed558ccdull;
  v ^= v >> 33;
  v *= 0xc4ceb9fe1a85ec53ull;
  v ^= v >> 33;
  return (unsigned)(v >> 61);
}

__global__ __launch_bounds__(kBS) void k_route_hist(const uint64_t* __restrict__ src, uint32_t* __restrict__ hist,
                                                    uint32_t nblocks) {
  __shared__ uint32_t cnt[kBuckets];
  if (threadIdx.x < kBuckets) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kTile;
#pragma unroll
  for (int i = 0; i < kPer; ++i) atomicAdd(&cnt[bucket_of(src[base + i * kBS + threadIdx.x])], 1u);
  __syncthreads();
  if (threadIdx.x < kBuckets) hist[(uint64_t)threadIdx.x * nblocks + blockIdx.x] = cnt[threadIdx.x];
}

// exclusive scan of m = 8 * nblocks counts in place (bucket-major: each bucket's runs contiguous)
__global__ __launch_bounds__(1024) void k_route_scan(uint32_t* __restrict__ hist, uint32_t m) {
  __shared__ uint32_t part[1024];
  const uint32_t per = (m + 1023) / 1024;
  const uint32_t lo = min(m, threadIdx.x * per), hi = min(m, lo + per);
  uint32_t s = 0;
  for (uint32_t i = lo; i < hi; ++i) s += hist[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t v = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - s;
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t c = hist[i];
    hist[i] = run;
    run += c;
  }
}

__global__ __launch_bounds__(kBS) void k_route_scatter(const uint64_t* __restrict__ src, const uint64_t* __restrict__ dst,
                                                       const uint32_t* __restrict__ off, uint32_t nblocks,
                                                       uint64_t* __restrict__ osrc, uint64_t* __restrict__ odst) {
  __shared__ uint64_t ls[kTile], ld[kTile];
  __shared__ uint32_t cnt[kBuckets], start[kBuckets + 1], goff[kBuckets];
  if (threadIdx.x < kBuckets) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kTile;
  uint64_t s[kPer], d[kPer];
  unsigned b[kPer], pos[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    s[i] = src[base + i * kBS + threadIdx.x];
    d[i] = dst[base + i * kBS + threadIdx.x];
    b[i] = bucket_of(s[i]);
    pos[i] = atomicAdd(&cnt[b[i]], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t r = 0;
    for (int k = 0; k < kBuckets; ++k) {
      start[k] = r;
      r += cnt[k];
    }
    start[kBuckets] = r;
  }
  if (threadIdx.x < kBuckets) goff[threadIdx.x] = off[(uint64_t)threadIdx.x * nblocks + blockIdx.x];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const uint32_t j = start[b[i]] + pos[i];
    ls[j] = s[i];
    ld[j] = d[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const uint32_t j = i * kBS + threadIdx.x;
    unsigned k = 0;
    while (k + 1 < kBuckets && start[k + 1] <= j) ++k;
    const uint64_t o = (uint64_t)goff[k] + (j - start[k]);
    osrc[o] = ls[j];
    odst[o] = ld[j];
  }
}

static void route(const uint64_t* s, const uint64_t* d, uint32_t* hist, uint64_t* os, uint64_t* od, uint64_t n,
                  hipStream_t st) {
  const uint32_t nb = (uint32_t)(n / kTile);
  hipLaunchKernelGGL(k_route_hist, dim3(nb), dim3(kBS), 0, st, s, hist, nb);
  hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, st, hist, nb * kBuckets);
  hipLaunchKernelGGL(k_route_scatter, dim3(nb), dim3(kBS), 0, st, s, d, hist, nb, os, od);
}

__global__ void k_fill(uint64_t* a, uint64_t* b, uint64_t n, uint64_t seed) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    x ^= x >> 29;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 32;
    a[i] = x & ((1ull << 26) - 1);
    b[i] = (x >> 26) & ((1ull << 26) - 1);
  }
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const uint64_t nmax = 1ull << 28;
  uint64_t *s, *d, *os, *od;
  uint32_t* hist;
  CK(hipMalloc(&s, nmax * 8));
  CK(hipMalloc(&d, nmax * 8));
  CK(hipMalloc(&os, nmax * 8));
  CK(hipMalloc(&od, nmax * 8));
  CK(hipMalloc(&hist, (nmax / kTile) * kBuckets * 4));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, st, s, d, nmax, 0x5EEDull);
  CK(hipStreamSynchronize(st));

  // 1. check on 2^22 edges
  {
    const uint64_t n = 1ull << 22;
    route(s, d, hist, os, od, n, st);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(st));
    std::vector<uint64_t> hs(n), hd(n), ho(n), hod(n);
    CK(hipMemcpy(hs.data(), s, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hd.data(), d, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ho.data(), os, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hod.data(), od, n * 8, hipMemcpyDeviceToHost));
    uint64_t c[kBuckets] = {}, ck_in = 0, ck_out = 0;
    for (uint64_t i = 0; i < n; ++i) {
      ++c[bucket_of(hs[i])];
      ck_in += hs[i] * 0x9E3779B97F4A7C15ull + hd[i];
      ck_out += ho[i] * 0x9E3779B97F4A7C15ull + hod[i];
    }
    uint64_t at = 0;
    bool ok = ck_in == ck_out;
    for (int k = 0; k < kBuckets && ok; ++k) {
      for (uint64_t i = at; i < at + c[k]; ++i)
        if (bucket_of(ho[i]) != (unsigned)k) {
          ok = false;
          break;
        }
      at += c[k];
    }
    std::printf("check 2^22 edges: %s (bucket sizes %llu..)\n", ok ? "ok" : "FAILED", (unsigned long long)c[0]);
    if (!ok) return 1;
  }
  // 2. time on 2^28 edges
  hipEvent_t e0, e1, e2, e3;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  CK(hipEventCreate(&e3));
  const uint32_t nb = (uint32_t)(nmax / kTile);
  double th = 0, tsc = 0, tsp = 0, tc = 0;
  const int reps = 10;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipEventRecord(e0, st));
    hipLaunchKernelGGL(k_route_hist, dim3(nb), dim3(kBS), 0, st, s, hist, nb);
    CK(hipEventRecord(e1, st));
    hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, st, hist, nb * kBuckets);
    CK(hipEventRecord(e2, st));
    hipLaunchKernelGGL(k_route_scatter, dim3(nb), dim3(kBS), 0, st, s, d, hist, nb, os, od);
    CK(hipEventRecord(e3, st));
    CK(hipEventSynchronize(e3));
    float a, b, c;
    CK(hipEventElapsedTime(&a, e0, e1));
    CK(hipEventElapsedTime(&b, e1, e2));
    CK(hipEventElapsedTime(&c, e2, e3));
    CK(hipMemcpyAsync(os, s, nmax * 8, hipMemcpyDeviceToDevice, st));  // the copy baseline
    CK(hipMemcpyAsync(od, d, nmax * 8, hipMemcpyDeviceToDevice, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float cp;
    CK(hipEventElapsedTime(&cp, e3, e1));
    if (r >= 2) {
      th += a;
      tsc += b;
      tsp += c;
      tc += cp;
    }
  }
  th /= reps;
  tsc /= reps;
  tsp /= reps;
  tc /= reps;
  const double gb = 32.0 * nmax / 1e9;
  std::printf("2^28 edges: hist %.3f ms, scan %.3f ms, scatter %.3f ms, total %.3f ms (%.0f GB/s of 32 B/edge);"
              " device copy of the same bytes %.3f ms (%.0f GB/s)\n",
              th, tsc, tsp, th + tsc + tsp, gb / ((th + tsc + tsp) * 1e-3), tc, gb / (tc * 1e-3));
  std::printf("per 2^30-edge pass (x4): routing %.2f ms, copy %.2f ms\n", 4 * (th + tsc + tsp), 4 * tc);
  return 0;
}
