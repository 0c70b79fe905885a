// gs_changes_k.hip -- kernels of per-window change emission (gs_changes.cpp).
//
// Sinks of the reference consume, per window, every (vertex, component) pair of the
// cumulative summary: FlattenSet (ConnectedComponentsExample.java:143-156) emits
// (v, find(v)) for all of getMatches(), keyed downstream, and DisjointSet.toString
// (DisjointSet.java:134-150) groups all vertices. Emitting only what changed gives
// the keyed sink the same state. A vertex's canonical label (its component's
// minimum id) changes exactly when its component's old root is hooked under a
// smaller key -- each hook record names that root -- and a vertex is new when it was
// inserted since the last emission (kAuxNew, set at insertion).
//
// Members are enumerated through circular member lists nxt[] (one u32 per slot),
// spliced in O(1) per hook at emission time: for a hooked old root hi whose final
// root is R, swap(nxt[hi], nxt[R]) by atomic exchange on nxt[R] -- nxt[hi] is only
// written by the thread that owns the record of hi (each root is hooked once), and
// R is never hooked, so concurrent splices into one R compose into one circle and
// no walked list changes while it is walked.
#include "gs_device.hpp"

namespace gs {

__global__ __launch_bounds__(256) void k_iota(uint32_t* nxt, uint64_t n) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (uint64_t)gridDim.x * blockDim.x)
    nxt[s] = (uint32_t)s;
}

// Rebuild the member lists of the current forest (after iota): every non-root
// occupied slot is spliced after its root.
__global__ __launch_bounds__(256) void k_relist(Table t, uint32_t* nxt) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= t.r0; s += (uint64_t)gridDim.x * blockDim.x) {
    int64_t k;
    uint32_t l, acc;
    load_slot(t.tab + s, k, l);
    const bool present = (s == t.r0) ? ((t.tab[s].aux & kAuxPresent) != 0) : (k != kEmpty);
    if (!present || (l >> 1) == s) continue;
    int64_t kr = k;
    const uint32_t r = find_ro(t, (uint32_t)s, l, kr, acc);
    nxt[s] = atomicExch(&nxt[r], (uint32_t)s);
  }
}

__device__ __forceinline__ void emit_row(uint32_t* ctr, uint64_t pos, int64_t v, int64_t lab, uint8_t par, int64_t* ov,
                                         int64_t* ol, uint8_t* op, uint64_t cap) {
  (void)ctr;
  if (pos < cap) {
    ov[pos] = v;
    ol[pos] = lab;
    if (op) op[pos] = par;
  }
}

// Parity of slot x relative to its final root (read-only find).
__device__ __forceinline__ uint32_t parity_to_root(const Table& t, uint32_t x) {
  int64_t k;
  uint32_t l, acc;
  load_slot(t.tab + x, k, l);
  find_ro(t, x, l, k, acc);
  return acc;
}

// One thread per delta record {hi key, lo key, w}; two phases. Phase 0: a hooked
// OLD root hi (not new since the last emission) has a list of exactly its old
// component; if it is longer than walk_max, hi's final root R is flagged (kAuxBig)
// and every vertex under R is emitted by k_emit_scan instead. Phase 1: the members
// of every other hooked old root get R's key; then hi's circle is spliced into R's.
__global__ __launch_bounds__(256) void k_emit_records(Table t, uint32_t* nxt, const int64_t* __restrict__ rec,
                                                      const unsigned long long* nrec, uint32_t walk_max,
                                                      int64_t* __restrict__ ov, int64_t* __restrict__ ol,
                                                      uint8_t* __restrict__ op, uint64_t cap, uint32_t* big,
                                                      int phase) {
  const uint64_t n = *nrec;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t a = rec[i * 3], b = rec[i * 3 + 1];
    if (a == b) continue;  // a self-loop's new vertex: emitted by k_emit_new
    uint32_t l;
    const uint32_t hi = lookup_find(t, a, l);
    if (hi == kNoSlot) continue;
    int64_t kr = a;
    uint32_t acc;
    const uint32_t R = find_ro(t, hi, l, kr, acc);
    if (R == hi) continue;  // cannot happen for a hook record (hi was hooked)
    const bool fresh = (t.tab[hi].aux & kAuxNew) != 0;
    if (phase == 0) {
      if (fresh) continue;
      uint32_t len = 1;
      for (uint32_t m = nxt[hi]; m != hi && len <= walk_max; m = nxt[m]) ++len;
      if (len > walk_max && (atomicOr(&t.tab[R].aux, kAuxBig) & kAuxBig) == 0) {
        const uint32_t q = atomicAdd(&t.ctr[ctr_index(CTR_BIG)], 1u);
        big[q] = R;
      }
      continue;
    }
    if (!fresh && !(t.tab[R].aux & kAuxBig)) {
      uint32_t len = 1;
      for (uint32_t m = nxt[hi]; m != hi; m = nxt[m]) ++len;
      const unsigned long long pos =
          atomicAdd(reinterpret_cast<unsigned long long*>(&t.ctr[ctr_index(CTR_EMIT)]), (unsigned long long)len);
      uint32_t m = hi;
      for (uint32_t j = 0; j < len; ++j, m = nxt[m]) {
        int64_t km;
        uint32_t lm;
        load_slot(t.tab + m, km, lm);
        km = settle_key(t, m, km);
        const uint32_t par = op ? parity_to_root(t, m) : 0u;
        emit_row(t.ctr, pos + j, km, kr, (uint8_t)par, ov, ol, op, cap);
      }
    }
    const uint32_t after_hi = nxt[hi];
    nxt[hi] = atomicExch(&nxt[R], after_hi);
  }
}

// Components too large to walk: every occupied vertex whose final root is flagged
// and that is not new (new vertices are k_emit_new's) is emitted. This includes the
// unchanged old members of the absorbing root -- idempotent rows for a keyed sink.
// all = 1: every vertex (first emission after a rebuild), new bits cleared.
__global__ __launch_bounds__(256) void k_emit_scan(Table t, int64_t* __restrict__ ov, int64_t* __restrict__ ol,
                                                   uint8_t* __restrict__ op, uint64_t cap, int all) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= t.r0; s += (uint64_t)gridDim.x * blockDim.x) {
    int64_t k;
    uint32_t l, acc;
    load_slot(t.tab + s, k, l);
    const uint32_t aux = t.tab[s].aux;
    const bool present = (s == t.r0) ? ((aux & kAuxPresent) != 0) : (k != kEmpty);
    if (!present || (!all && (aux & kAuxNew))) continue;
    const int64_t v = settle_key(t, (uint32_t)s, k);
    int64_t kr = v;
    const uint32_t R = find_ro(t, (uint32_t)s, l, kr, acc);
    if (!all && !(t.tab[R].aux & kAuxBig)) continue;
    if (all && (aux & kAuxNew)) atomicAnd(&t.tab[s].aux, ~kAuxNew);  // a full emission covers the new vertices
    const unsigned long long pos =
        atomicAdd(reinterpret_cast<unsigned long long*>(&t.ctr[ctr_index(CTR_EMIT)]), 1ull);
    emit_row(t.ctr, pos, v, kr, (uint8_t)acc, ov, ol, op, cap);
  }
}

__global__ __launch_bounds__(256) void k_clear_big(Table t, const uint32_t* big) {
  const uint32_t n = t.ctr[ctr_index(CTR_BIG)];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    atomicAnd(&t.tab[big[i]].aux, ~kAuxBig);
}

// New vertices since the last emission: the vertex-list entries past each shard's
// mark. Emitted with their final label (emit = 0: a full emission already covered
// them) and their kAuxNew bit cleared; k_set_marks then advances the marks.
__global__ __launch_bounds__(256) void k_emit_new(Table t, const uint32_t* vmark, int64_t* __restrict__ ov,
                                                  int64_t* __restrict__ ol, uint8_t* __restrict__ op, uint64_t cap,
                                                  int emit) {
  __shared__ uint32_t lo[kShards], hi[kShards];
  __shared__ uint64_t pre[kShards + 1];
  if (threadIdx.x < (uint32_t)kShards) {
    lo[threadIdx.x] = min(vmark[threadIdx.x], t.vshard_cap);
    hi[threadIdx.x] = min(t.ctr[ctr_index(CTR_NV + threadIdx.x)], t.vshard_cap);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t o = 0;
    for (int q = 0; q < kShards; ++q) {
      pre[q] = o;
      o += hi[q] > lo[q] ? hi[q] - lo[q] : 0;
    }
    pre[kShards] = o;
  }
  __syncthreads();
  const uint64_t total = pre[kShards];
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += (uint64_t)gridDim.x * blockDim.x) {
    int q = 0, r = kShards - 1;
    while (q < r) {
      const int mid = (q + r + 1) >> 1;
      if (pre[mid] <= g) q = mid;
      else r = mid - 1;
    }
    const uint32_t s = t.vlist[(size_t)q * t.vshard_cap + lo[q] + (g - pre[q])];
    if (emit) {
      int64_t k;
      uint32_t l, acc;
      load_slot(t.tab + s, k, l);
      const int64_t v = settle_key(t, s, k);
      int64_t kr = v;
      find_ro(t, s, l, kr, acc);
      const unsigned long long pos =
          atomicAdd(reinterpret_cast<unsigned long long*>(&t.ctr[ctr_index(CTR_EMIT)]), 1ull);
      emit_row(t.ctr, pos, v, kr, (uint8_t)acc, ov, ol, op, cap);
    }
    atomicAnd(&t.tab[s].aux, ~kAuxNew);
  }
}

__global__ void k_set_marks(const uint32_t* ctr, uint32_t* vmark) {
  if (threadIdx.x < (uint32_t)kShards) vmark[threadIdx.x] = ctr[ctr_index(CTR_NV + threadIdx.x)];
}

static unsigned grid_for(uint64_t n) {
  const uint64_t b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}

void launch_iota(uint32_t* nxt, uint64_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n)), dim3(256), 0, st, nxt, (unsigned long long)n);
}
void launch_relist(const Table& t, uint32_t* nxt, hipStream_t st) {
  hipLaunchKernelGGL(k_relist, dim3(grid_for((uint64_t)t.r0 + 1)), dim3(256), 0, st, t, nxt);
}
void launch_emit_records(const Table& t, uint32_t* nxt, const int64_t* rec, const unsigned long long* nrec,
                         uint64_t nrec_bound, uint32_t walk_max, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap,
                         uint32_t* big, hipStream_t st) {
  for (int phase = 0; phase < 2; ++phase)
    hipLaunchKernelGGL(k_emit_records, dim3(grid_for(nrec_bound)), dim3(256), 0, st, t, nxt, rec, nrec, walk_max, ov,
                       ol, op, (unsigned long long)cap, big, phase);
}
void launch_emit_scan(const Table& t, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap, bool all,
                      hipStream_t st) {
  hipLaunchKernelGGL(k_emit_scan, dim3(grid_for((uint64_t)t.r0 + 1)), dim3(256), 0, st, t, ov, ol, op,
                     (unsigned long long)cap, all ? 1 : 0);
}
void launch_clear_big(const Table& t, const uint32_t* big, uint64_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_clear_big, dim3(grid_for(n)), dim3(256), 0, st, t, big);
}
void launch_emit_new(const Table& t, uint32_t* vmark, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap,
                     uint64_t bound, bool emit, hipStream_t st) {
  hipLaunchKernelGGL(k_emit_new, dim3(grid_for(bound)), dim3(256), 0, st, t, (const uint32_t*)vmark, ov, ol, op,
                     (unsigned long long)cap, emit ? 1 : 0);
  hipLaunchKernelGGL(k_set_marks, dim3(1), dim3(64), 0, st, (const uint32_t*)t.ctr, vmark);
}

}  // namespace gs
