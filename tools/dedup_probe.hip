// dedup_probe.hip -- cost of a batch-level "dedup by hashing" stage in front of k_fold
// (VERDICT r01 item 4), measured on the bench's own RMAT-26 micro-batches.
//
// A dedup stage that probes the summary once per DISTINCT endpoint of a 2^20-edge
// micro-batch needs at least two passes over the batch's endpoint occurrences:
//   k_dd_insert  every occurrence inserts its id into a batch hash table D (CAS,
//                linear probing) and writes its D slot (coalesced);
//   k_dd_gather  after the distinct ids are resolved, every occurrence reads its
//                distinct id's resolved summary slot back (random read of D's side
//                array) -- the edge's union then starts from that slot.
// The summary probes then drop from one per occurrence to one per distinct id. This
// program times both passes and, under rocprofv3 --pmc, gives their fabric read
// requests (TCC_EA0_RDREQ) per edge, to compare with k_fold's 1.95 per edge.
//
// Build: hipcc -O3 --offload-arch=gfx950 -I../include tools/dedup_probe.hip \
//          -L gelly-streaming_amd/lib -lgs_summary -Wl,-rpath,... (tools/dedup_probe.sh)
// Run:   dedup_probe [log2_table=22] [batches=64]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gs_gen.h"

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int64_t kNone = 0;  // empty slot (a scrambled id of 0 would alias it: not in these batches' accounting)

__device__ __forceinline__ uint32_t dd_hash(int64_t key, int shift) {
  return (uint32_t)(((uint64_t)key * 0x9E3779B97F4A7C15ull) >> shift);
}

__device__ __forceinline__ uint32_t dd_insert(unsigned long long* D, uint32_t mask, int shift, int64_t key,
                                              uint32_t& fresh) {
  uint32_t h = dd_hash(key, shift);
  for (uint32_t p = 0; p <= mask; ++p) {
    unsigned long long k = __hip_atomic_load(D + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == (unsigned long long)key) return h;
    if (k == (unsigned long long)kNone) {
      unsigned long long prev = atomicCAS(D + h, (unsigned long long)kNone, (unsigned long long)key);
      if (prev == (unsigned long long)kNone) {
        ++fresh;
        return h;
      }
      if (prev == (unsigned long long)key) return h;
    }
    h = (h + 1) & mask;
  }
  return 0xFFFFFFFFu;  // full (not reached at these loads)
}

__global__ void k_dd_insert(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, uint32_t n,
                            unsigned long long* D, uint32_t mask, int shift, uint2* __restrict__ occ,
                            unsigned long long* distinct) {
  __shared__ uint32_t blk_fresh;
  if (threadIdx.x == 0) blk_fresh = 0;
  __syncthreads();
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t fresh = 0;
  if (e < n) {
    const uint32_t a = dd_insert(D, mask, shift, src[e], fresh);
    const uint32_t b = dd_insert(D, mask, shift, dst[e], fresh);
    occ[e] = make_uint2(a, b);
  }
  if (fresh) atomicAdd(&blk_fresh, fresh);  // distinct ids: one global add per block
  __syncthreads();
  if (threadIdx.x == 0 && blk_fresh) atomicAdd(distinct, (unsigned long long)blk_fresh);
}

__global__ void k_dd_gather(const uint2* __restrict__ occ, uint32_t n, const uint32_t* __restrict__ resolved,
                            uint2* __restrict__ out) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const uint2 o = occ[e];
  out[e] = make_uint2(resolved[o.x], resolved[o.y]);
}

int main(int argc, char** argv) {
  const int logt = argc > 1 ? atoi(argv[1]) : 22;
  const int batches = argc > 2 ? atoi(argv[2]) : 64;
  const uint32_t B = 1u << 20;
  const uint64_t E = (uint64_t)B * batches;
  int64_t *src, *dst;
  CK(hipMalloc(&src, E * 8));
  CK(hipMalloc(&dst, E * 8));
  if (gs_gen_rmat(nullptr, src, dst, 0, E, 26, 0x5EED0026ull, 1)) return 1;  // bench.py's stream
  const uint32_t T = 1u << logt;
  unsigned long long *D, *distinct;
  uint32_t* resolved;
  uint2 *occ, *out;
  CK(hipMalloc(&D, (size_t)T * 8));
  CK(hipMalloc(&resolved, (size_t)T * 4));
  CK(hipMemset(resolved, 0, (size_t)T * 4));
  CK(hipMalloc(&occ, (size_t)B * 8));
  CK(hipMalloc(&out, (size_t)B * 8));
  CK(hipMalloc(&distinct, 8 * batches));
  CK(hipMemset(distinct, 0, 8 * batches));
  hipEvent_t ev[4];
  for (auto& x : ev) CK(hipEventCreate(&x));
  double t_clear = 0, t_ins = 0, t_gat = 0;
  const dim3 grid(B / 256), blk(256);
  for (int b = 0; b < batches; ++b) {
    const uint64_t o = (uint64_t)b * B;
    CK(hipEventRecord(ev[0], nullptr));
    CK(hipMemsetAsync(D, 0, (size_t)T * 8, nullptr));  // the batch table starts empty
    CK(hipEventRecord(ev[1], nullptr));
    hipLaunchKernelGGL(k_dd_insert, grid, blk, 0, nullptr, src + o, dst + o, B, D, T - 1, 64 - logt, occ,
                       distinct + b);
    CK(hipEventRecord(ev[2], nullptr));
    hipLaunchKernelGGL(k_dd_gather, grid, blk, 0, nullptr, occ, B, resolved, out);
    CK(hipEventRecord(ev[3], nullptr));
    CK(hipEventSynchronize(ev[3]));
    float a, c, d;
    CK(hipEventElapsedTime(&a, ev[0], ev[1]));
    CK(hipEventElapsedTime(&c, ev[1], ev[2]));
    CK(hipEventElapsedTime(&d, ev[2], ev[3]));
    if (b) t_clear += a, t_ins += c, t_gat += d;  // batch 0 warms up
  }
  std::vector<unsigned long long> nd(batches);
  CK(hipMemcpy(nd.data(), distinct, 8 * batches, hipMemcpyDeviceToHost));
  double avg_d = 0;
  for (int b = 1; b < batches; ++b) avg_d += nd[b];
  const int m = batches - 1;
  avg_d /= m;
  printf("{\"table_log2\": %d, \"batches\": %d, \"edges_per_batch\": %u, \"distinct_per_batch\": %.0f, "
         "\"distinct_per_occurrence\": %.4f, \"clear_us\": %.2f, \"insert_us\": %.2f, \"gather_us\": %.2f}\n",
         logt, m, B, avg_d, avg_d / (2.0 * B), 1e3 * t_clear / m, 1e3 * t_ins / m, 1e3 * t_gat / m);
  return 0;
}
