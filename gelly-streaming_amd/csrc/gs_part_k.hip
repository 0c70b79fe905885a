// gs_part_k.hip -- kernels of a group's owner-partitioned combine (gs_part.hpp,
// include/gs_group.h gs_group_create_partitioned).
//
// The combine runs with the rank's own folds joined (they queue behind it), so every
// root found here is the local forest's current root: the finds walk with plain loads
// and then confirm the root with an agent-scope load of its link (a root a block has
// confirmed once is remembered in LDS: the giant component's root is read once per
// block, not once per vertex).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gs_part.hpp"

namespace gs {

namespace {

constexpr uint32_t kPartBS = 256;
constexpr int kPartPer = (int)(kPartRowsPB / kPartBS);  // rows per thread (8)
constexpr uint32_t kRootCache = 256;                    // LDS: roots this block has confirmed

__device__ __forceinline__ uint64_t part_prefix(const Table& t, const uint32_t* mark, const uint32_t* snap, int full,
                                                uint32_t* lm, uint64_t* pre) {
  __shared__ uint32_t cnt[kShards];
  if (threadIdx.x < (uint32_t)kShards) {
    const uint32_t m = full ? 0u : mark[threadIdx.x], c = snap[threadIdx.x];
    lm[threadIdx.x] = m;
    cnt[threadIdx.x] = c > m ? c - m : 0u;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t o = 0;
    for (int q = 0; q < kShards; ++q) {
      pre[q] = o;
      o += cnt[q];
    }
    pre[kShards] = o;
  }
  __syncthreads();
  return pre[kShards];
}

// the g-th new vertex (slot id) since the marks
__device__ __forceinline__ uint32_t part_new_at(const Table& t, const uint32_t* lm, const uint64_t* pre, uint64_t g) {
  int lo = 0, hi = kShards - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pre[mid] <= g) lo = mid;
    else hi = mid - 1;
  }
  return t.vlist[(size_t)lo * t.vshard_cap + lm[lo] + (g - pre[lo])];
}

// Current root of slot x (link lx): the plain walk reaches an ancestor; its link is then
// re-read at the agent scope (another XCD's L2 may hold an older line) and the walk
// continues fresh until a root. kx = the root's key, acc ^= the parity on the way.
__device__ __forceinline__ uint32_t find_current(const Table& t, uint32_t x, uint32_t lx, int64_t& kx, uint32_t& acc,
                                                 uint32_t* cache, bool* cached = nullptr) {
  while ((lx >> 1) != x) {
    acc ^= lx & 1u;
    x = lx >> 1;
    load_slot(t.tab + x, kx, lx);
  }
  if (cache && cache[x & (kRootCache - 1)] == x) {  // confirmed (and marked) by this block
    kx = settle_key(t, x, kx);
    if (cached) *cached = true;
    return x;
  }
  uint32_t lf = load_link_fresh(t.tab + x);
  const bool moved = (lf >> 1) != x;
  while ((lf >> 1) != x) {
    acc ^= lf & 1u;
    x = lf >> 1;
    lf = load_link_fresh(t.tab + x);
  }
  if (moved) {
    uint32_t l;
    load_slot(t.tab + x, kx, l);
  }
  kx = settle_key(t, x, kx);
  if (cache) cache[x & (kRootCache - 1)] = x;
  return x;
}

// Mark a root handed out as a label (the marking block remembers it in the root cache: a
// confirmed root is marked by then).
__device__ __forceinline__ void mark_exported(const Table& t, uint32_t x) {
  const uint32_t aux = __hip_atomic_load(&t.tab[x].aux, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!(aux & kAuxExported)) atomicOr(&t.tab[x].aux, kAuxExported);
}

__global__ __launch_bounds__(256) void k_part_init(OwnerSlot* tab, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    OwnerSlot s;
    s.key = kEmpty;
    s.anchor = 0;
    s.aw = 0;
    s.pad0 = 0;
    s.pad1 = 0;
    tab[i] = s;
  }
}

__global__ __launch_bounds__(64) void k_part_snap(Table t, const uint32_t* mark, uint32_t* snap, int full, uint32_t dctr,
                                                  uint32_t shard_cap, unsigned long long* out) {
  const uint32_t s = threadIdx.x;
  const uint32_t c = min(t.ctr[ctr_index(CTR_NV + s)], t.vshard_cap);
  const uint32_t m = full ? 0u : mark[s];
  snap[s] = c;
  unsigned long long nv = c > m ? c - m : 0u;
  unsigned long long nr = min(t.ctr[ctr_index(dctr + s)], shard_cap);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    nv += __shfl_xor(nv, o, 64);
    nr += __shfl_xor(nr, o, 64);
  }
  if (s == 0) {
    out[0] = nv;
    out[1] = nr;
    out[2] = t.ctr[ctr_index(CTR_VOVF)];
  }
}

template <bool SIGNED>
__global__ __launch_bounds__(kPartBS) void k_part_export(Table t, const uint32_t* mark, const uint32_t* snap, int full,
                                                         uint64_t total, int64_t* __restrict__ stage, int width,
                                                         uint32_t* __restrict__ bcnt, int nranks, uint32_t nblocks) {
  __shared__ uint32_t lm[kShards];
  __shared__ uint64_t pre[kShards + 1];
  __shared__ uint32_t lcnt[kPartMaxRanks];
  __shared__ uint32_t cache[kRootCache];
  part_prefix(t, mark, snap, full, lm, pre);
  if (threadIdx.x < (uint32_t)nranks) lcnt[threadIdx.x] = 0;
  cache[threadIdx.x] = kNoSlot;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kPartRowsPB;
  uint32_t s[kPartPer], l[kPartPer];
  int64_t k[kPartPer];
#pragma unroll
  for (int j = 0; j < kPartPer; ++j) {  // every slot load of the thread in flight together
    const uint64_t g = base + (uint64_t)j * kPartBS + threadIdx.x;
    s[j] = kNoSlot;
    if (g < total) {
      s[j] = part_new_at(t, lm, pre, g);
      load_slot(t.tab + s[j], k[j], l[j]);
    }
  }
  int64_t kq[kPartPer];
  uint32_t lq[kPartPer];
#pragma unroll
  for (int j = 0; j < kPartPer; ++j) {  // the first hops together
    kq[j] = 0;
    lq[j] = 0;
    if (s[j] != kNoSlot && (l[j] >> 1) != s[j]) load_slot(t.tab + (l[j] >> 1), kq[j], lq[j]);
  }
#pragma unroll
  for (int j = 0; j < kPartPer; ++j) {
    if (s[j] == kNoSlot) continue;
    const uint64_t g = base + (uint64_t)j * kPartBS + threadIdx.x;
    const int64_t v = settle_key(t, s[j], k[j]);
    int64_t kx = v;
    uint32_t acc = 0, x;
    bool cached = false;
    if ((l[j] >> 1) == s[j]) {
      x = find_current(t, s[j], l[j], kx, acc, cache, &cached);
    } else {
      acc = l[j] & 1u;
      kx = kq[j];
      x = find_current(t, l[j] >> 1, lq[j], kx, acc, cache, &cached);
    }
    if (!cached) mark_exported(t, x);
    int64_t* r = stage + g * (uint64_t)width;
    r[0] = v;
    r[1] = kx;
    if (SIGNED) r[2] = (int64_t)(acc & 1u);
    atomicAdd(&lcnt[part_owner(v, nranks)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < (uint32_t)nranks) bcnt[(size_t)threadIdx.x * nblocks + blockIdx.x] = lcnt[threadIdx.x];
}

// wave-aggregated append of label pairs (one atomic per wave); wave-uniform control flow
__device__ __forceinline__ void append_pair(bool has, int64_t a, int64_t b, uint32_t w, int64_t* pairs, int width,
                                            unsigned long long* npairs, uint64_t pair_cap) {
  const unsigned long long m = __ballot(has);
  if (!m) return;
  const int lane = (int)(threadIdx.x & 63u);
  const int leader = __ffsll((long long)m) - 1;
  unsigned long long basep = 0;
  if (lane == leader) basep = atomicAdd(npairs, (unsigned long long)__popcll(m));
  basep = __shfl(basep, leader, 64);
  if (!has) return;
  const uint64_t pos = basep + (uint64_t)__popcll(m & ((1ull << lane) - 1ull));
  if (pos < pair_cap) {
    int64_t* r = pairs + pos * (uint64_t)width;
    r[0] = a;
    r[1] = b;
    if (width == 3) r[2] = (int64_t)w;
  }
}

// Records of the window (delta set D): a root hooked away whose label was handed out
// becomes the pair (a, its root now, parity). Grid: one block per delta shard.
template <bool SIGNED>
__global__ __launch_bounds__(256) void k_part_records(Table t, Delta D, int64_t* pairs, int width,
                                                      unsigned long long* npairs, uint64_t pair_cap) {
  __shared__ uint32_t cache[kRootCache];
  cache[threadIdx.x] = kNoSlot;
  __syncthreads();
  const uint32_t sh = blockIdx.x;
  const uint32_t n = min(t.ctr[ctr_index(D.dctr + sh)], D.shard_cap);
  const uint32_t rounds = (n + 255u) / 256u;  // wave-uniform loop
  for (uint32_t q = 0; q < rounds; ++q) {
    const uint32_t i = q * 256u + threadIdx.x;
    bool has = false;
    int64_t a = 0, kx = 0;
    uint32_t acc = 0;
    if (i < n) {
      const int64_t* rec = D.drec + ((size_t)sh * D.shard_cap + i) * 3;
      a = rec[0];
      const int64_t b = rec[1];
      if (a != b) {
        uint32_t la;
        const uint32_t sa = lookup_find(t, a, la);
        if (sa != kNoSlot &&
            (__hip_atomic_load(&t.tab[sa].aux, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kAuxExported)) {
          kx = a;
          const uint32_t x = find_current(t, sa, la, kx, acc, cache);
          if (x != sa) {
            mark_exported(t, x);
            has = true;
          }
        }
      }
    }
    append_pair(has, a, kx, acc & 1u, pairs, width, npairs, pair_cap);
  }
}

// Per-owner exclusive offsets of the export blocks: one block, a scan per owner column.
__global__ __launch_bounds__(1024) void k_part_scan(uint32_t* bcnt, uint32_t nblocks, int nranks,
                                                    unsigned long long* send_counts) {
  __shared__ uint32_t wsum[16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int o = 0; o < nranks; ++o) {
    uint32_t* col = bcnt + (size_t)o * nblocks;
    unsigned long long carry = 0;
    for (uint32_t c0 = 0; c0 < nblocks; c0 += 1024) {
      const uint32_t b = c0 + threadIdx.x;
      const uint32_t v = b < nblocks ? col[b] : 0u;
      uint32_t x = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
      }
      if (lane == 63) wsum[wid] = x;
      __syncthreads();
      uint32_t wb = 0, tot = 0;
      for (int q = 0; q < 16; ++q) {
        if (q < wid) wb += wsum[q];
        tot += wsum[q];
      }
      if (b < nblocks) col[b] = (uint32_t)(carry + wb + (x - v));
      carry += tot;
      __syncthreads();
    }
    if (threadIdx.x == 0) send_counts[o] = carry;
  }
}

__global__ __launch_bounds__(kPartBS) void k_part_scatter(const int64_t* __restrict__ stage, uint64_t total, int width,
                                                          const uint32_t* __restrict__ bcnt, uint32_t nblocks,
                                                          const unsigned long long* __restrict__ send_counts,
                                                          int nranks, int64_t* __restrict__ sendbuf) {
  __shared__ unsigned long long obase[kPartMaxRanks];
  __shared__ uint32_t opos[kPartMaxRanks];
  if (threadIdx.x == 0) {
    unsigned long long o = 0;
    for (int q = 0; q < nranks; ++q) {
      obase[q] = o + bcnt[(size_t)q * nblocks + blockIdx.x];
      o += send_counts[q];
    }
  }
  if (threadIdx.x < (uint32_t)nranks) opos[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kPartRowsPB;
#pragma unroll
  for (int j = 0; j < kPartPer; ++j) {
    const uint64_t g = base + (uint64_t)j * kPartBS + threadIdx.x;
    if (g >= total) continue;
    const int64_t* r = stage + g * (uint64_t)width;
    const int64_t v = r[0];
    const int o = part_owner(v, nranks);
    const uint64_t pos = obase[o] + atomicAdd(&opos[o], 1u);
    int64_t* d = sendbuf + pos * (uint64_t)width;
    d[0] = v;
    d[1] = r[1];
    if (width == 3) d[2] = r[2];
  }
}

__device__ __forceinline__ uint32_t owner_hash(int64_t v, int shift) {
  return (uint32_t)(((uint64_t)v * 0x9E3779B97F4A7C15ull) >> shift);
}

// Insert-or-find of an owned vertex. `inserted`: this row's key CAS created the slot -- its
// row sets the anchor (no claim atomic of its own).
__device__ __forceinline__ uint32_t owner_insert(const OwnerTable& ot, int64_t v, bool& inserted) {
  inserted = false;
  if (v == kEmpty) {
    inserted = !(atomicOr(&ot.tab[ot.r0].aw, kAncPresent) & kAncPresent);
    return ot.r0;
  }
  uint32_t h = owner_hash(v, ot.shift);
  for (uint32_t probes = 0; probes <= ot.mask; ++probes) {
    const int64_t k = ot.tab[h].key;
    if (k == v) return h;
    if (k == kEmpty) {
      const unsigned long long old =
          atomicCAS((unsigned long long*)&ot.tab[h].key, (unsigned long long)kEmpty, (unsigned long long)v);
      if (old == (unsigned long long)kEmpty) {
        inserted = true;
        return h;
      }
      if ((int64_t)old == v) return h;
    }
    h = (h + 1) & ot.mask;
  }
  atomicOr(ot.err, 1u);
  return kNoSlot;
}

// Pair-set insert, phase 1 (per lane, no waiting): the slot this pair claimed (*win) or whose
// fingerprint it met (*win false), or kNoSlot when it met neither within the probe bound (the
// pair is then emitted: a repeat is harmless, the label forest's fold drops it).
__device__ __forceinline__ unsigned long long pair_fp(int64_t a, int64_t b, uint32_t w) {
  unsigned long long z = (unsigned long long)a * 0x9E3779B97F4A7C15ull ^ ((unsigned long long)b + 0x632BE59BD9B4E019ull);
  z ^= (unsigned long long)w << 63;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z | 1ull;  // never 0 (empty)
}
constexpr uint32_t kPairProbes = 32;
__device__ __forceinline__ uint32_t pairset_probe(const PairSet& ps, unsigned long long fp, bool& win) {
  win = false;
  uint32_t h = (uint32_t)(fp >> 32) & ps.mask;
  for (uint32_t k = 0; k < kPairProbes; ++k, h = (h + 1) & ps.mask) {
    unsigned long long cur = __hip_atomic_load(&ps.tab[h].fp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == 0ull) {
      cur = atomicCAS(&ps.tab[h].fp, 0ull, fp);
      if (cur == 0ull) {
        win = true;
        return h;
      }
    }
    if (cur == fp) return h;
  }
  return kNoSlot;
}
// Phases 2 and 3, in this order for the whole wave (a lane that met a fingerprint waits for its
// inserter, which is resident and publishes here without waiting on anyone): inserters publish
// their pair (write-through, drained, then the ready bit); the others wait for ready and compare.
// Returns whether the pair is new (to be emitted).
__device__ __forceinline__ bool pairset_settle(const PairSet& ps, uint32_t h, bool win, bool active, int64_t a,
                                               int64_t b, uint32_t w) {
  if (active && h != kNoSlot && win) {
    __hip_atomic_store(&ps.tab[h].a, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ps.tab[h].b, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    atomicOr(&ps.tab[h].state, 1u | (w << 1));
  }
  bool fresh = active;
  if (active && h != kNoSlot && !win) {
    uint32_t st = __hip_atomic_load(&ps.tab[h].state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (!(st & 1u)) {
      __builtin_amdgcn_s_sleep(1);
      st = __hip_atomic_load(&ps.tab[h].state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const int64_t a2 = __hip_atomic_load(&ps.tab[h].a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t b2 = __hip_atomic_load(&ps.tab[h].b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    fresh = !(a2 == a && b2 == b && ((st >> 1) & 1u) == w);  // (a different pair: a fingerprint collision)
  }
  return fresh;
}
__device__ __forceinline__ bool pairset_new(const PairSet& ps, bool active, int64_t a, int64_t b, uint32_t w) {
  if (!ps.tab) return active;
  bool win = false;
  const uint32_t h = active ? pairset_probe(ps, pair_fp(a, b, w), win) : kNoSlot;
  return pairset_settle(ps, h, win, active, a, b, w);
}

// The owner step: every received row (v, l[, p]) claims or reads v's anchor; a row whose
// label differs from the anchor (or, signed, whose parity does) becomes the label pair
// (anchor, l, p ^ parity(anchor)). A row whose label equals the anchor with the other
// parity is an odd cycle: `fail`. The block collects its pairs in an LDS table keyed by a
// hash of the pair: per round of 256 rows the claimers of empty entries write theirs, a
// block barrier, then a pair that finds its own entry is a repeat (dropped) and one that
// finds another pair there goes out at once; the table's pairs go out at the block's end
// with ONE reservation (the giant component's (anchor, label) pairs repeat thousands of
// times per block: one append atomic per pair would queue on a single address).
constexpr uint32_t kOwnerTab = 1024;
template <bool SIGNED>
__global__ __launch_bounds__(kPartBS) void k_part_owner(OwnerTable ot, PairSet ps, const int64_t* __restrict__ rows,
                                                        uint64_t nrows, int width, int64_t* pairs,
                                                        unsigned long long* npairs, uint64_t pair_cap, uint32_t* fail) {
  __shared__ uint32_t dflag[kOwnerTab];  // 0 empty, 1 claimed, 2 | w << 2 ready
  __shared__ int64_t da[kOwnerTab], db[kOwnerTab];
  __shared__ uint32_t lwave[kPartBS / 64];
  __shared__ unsigned long long lbase;
  for (uint32_t i = threadIdx.x; i < kOwnerTab; i += kPartBS) dflag[i] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kPartRowsPB;
  for (int j = 0; j < kPartPer; ++j) {  // block-uniform
    const uint64_t i = base + (uint64_t)j * kPartBS + threadIdx.x;
    const bool valid = i < nrows;
    int64_t v = 0, l = 0;
    uint32_t p = 0;
    if (valid) {
      const int64_t* r = rows + i * (uint64_t)width;
      v = r[0];
      l = r[1];
      if (SIGNED) p = (uint32_t)r[2] & 1u;
    }
    uint32_t aw = 0, s = kNoSlot;
    int64_t anchor = 0;
    bool claimer = false;
    if (valid) s = owner_insert(ot, v, claimer);
    const bool live = valid && s != kNoSlot;
    // Publish without a fence (a release fence is an L2 write-back + invalidate: one per claim
    // made this step 24 ms at one rank): the anchor goes out write-through (agent scope), its
    // acknowledgement is awaited, then the published bit -- a memory-side atomic -- follows.
    // A reader sees the bit at the memory side and only then reads the anchor there.
    if (claimer) {
      __hip_atomic_store(&ot.tab[s].anchor, l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      atomicOr(&ot.tab[s].aw, kAncPublished | (p ? kAncParity : 0u));
    }
    bool has = false;
    int64_t A = 0;
    uint32_t w = 0;
    if (live && !claimer) {
      // the claimer (a resident wave past its key CAS) publishes without waiting on anyone
      aw = __hip_atomic_load(&ot.tab[s].aw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while (!(aw & kAncPublished)) {
        __builtin_amdgcn_s_sleep(1);
        aw = __hip_atomic_load(&ot.tab[s].aw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      anchor = __hip_atomic_load(&ot.tab[s].anchor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      A = anchor;
      const uint32_t pa = (aw & kAncParity) ? 1u : 0u;
      w = SIGNED ? (p ^ pa) : 0u;
      if (l == A) {
        if (SIGNED && w) atomicOr(fail, 1u);  // v on both sides of one label: an odd cycle
      } else {
        has = true;
      }
    }
    uint32_t e = 0;
    bool mine = false;
    if (has) {
      const unsigned long long hsh =
          ((unsigned long long)A * 0x9E3779B97F4A7C15ull) ^ ((unsigned long long)l * 0xC2B2AE3D27D4EB4Full) ^ w;
      e = (uint32_t)(hsh >> 40) & (kOwnerTab - 1);
      if (atomicCAS(&dflag[e], 0u, 1u) == 0u) {
        da[e] = A;
        db[e] = l;
        dflag[e] = 2u | (w << 2);
        mine = true;
      }
    }
    __syncthreads();  // every claimed entry of this round is ready
    bool direct = false;
    if (has && !mine) {
      const uint32_t g = dflag[e];
      direct = !((g >> 2) == w && da[e] == A && db[e] == l);  // another pair holds the entry
    }
    append_pair(pairset_new(ps, direct, A, l, w), A, l, w, pairs, width, npairs, pair_cap);
  }
  __syncthreads();
  // the table's pairs not emitted by another block yet (the pair set): one reservation per block
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t keep = 0, cnt = 0;  // bit q: entry threadIdx.x + q * kPartBS goes out
#pragma unroll
  for (uint32_t q = 0; q < kOwnerTab / kPartBS; ++q) {
    const uint32_t e = threadIdx.x + q * kPartBS;
    const uint32_t f = dflag[e];
    const bool ready = (f & 3u) == 2u;
    if (pairset_new(ps, ready, da[e], db[e], f >> 2)) {
      keep |= 1u << q;
      ++cnt;
    }
  }
  uint32_t x = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) lwave[wid] = x;
  __syncthreads();
  uint32_t wb = 0, tot = 0;
  for (int q = 0; q < (int)(kPartBS / 64); ++q) {
    if (q < wid) wb += lwave[q];
    tot += lwave[q];
  }
  if (threadIdx.x == 0) lbase = tot ? atomicAdd(npairs, (unsigned long long)tot) : 0ull;
  __syncthreads();
  uint64_t pos = lbase + wb + (x - cnt);
#pragma unroll
  for (uint32_t q = 0; q < kOwnerTab / kPartBS; ++q) {
    if (!((keep >> q) & 1u)) continue;
    const uint32_t e = threadIdx.x + q * kPartBS;
    if (pos < pair_cap) {
      int64_t* r = pairs + pos * (uint64_t)width;
      r[0] = da[e];
      r[1] = db[e];
      if (width == 3) r[2] = (int64_t)(dflag[e] >> 2);
    }
    ++pos;
  }
}

__global__ void k_part_count_word(const unsigned long long* npairs, const uint32_t* local_fail,
                                  const uint32_t* part_fail, unsigned long long* word) {
  const bool f = (local_fail && *local_fail) || (part_fail && *part_fail);
  *word = *npairs | (f ? kFailBit : 0ull);
}

// owned vertices -> (v, label, parity). Each thread reads kLabPer slots of a block tile (32-B
// slots, coalesced), and the block reserves its tile's output with ONE atomic: one per wave
// put 2^21 same-address atomics into the one-rank pass (11.4 ns each at the memory side:
// 25 ms for a 2^27-slot owner table).
constexpr int kLabPer = 8;
constexpr uint32_t kLabBS = 256;
__global__ __launch_bounds__(kLabBS) void k_part_labels(OwnerTable ot, Table G, int64_t* __restrict__ ov,
                                                        int64_t* __restrict__ ol, uint8_t* __restrict__ op,
                                                        uint64_t cap_out, unsigned long long* count) {
  __shared__ uint32_t wsum[kLabBS / 64];
  __shared__ unsigned long long base_sh;
  const uint64_t n = (uint64_t)ot.cap + 1;
  const int lane = (int)(threadIdx.x & 63u), wid = (int)(threadIdx.x >> 6);
  for (uint64_t tile = (uint64_t)blockIdx.x * (kLabBS * kLabPer); tile < n;
       tile += (uint64_t)gridDim.x * (kLabBS * kLabPer)) {  // block-uniform
    int64_t vk[kLabPer], lk[kLabPer];
    uint32_t pk = 0, occ = 0, cnt = 0;
#pragma unroll
    for (int j = 0; j < kLabPer; ++j) {  // every slot of the thread in flight together
      const uint64_t s = tile + (uint64_t)j * kLabBS + threadIdx.x;
      vk[j] = kEmpty;
      lk[j] = 0;
      uint32_t aw = 0;
      if (s < n) {
        const uint4 lo = *reinterpret_cast<const uint4*>(ot.tab + s);
        aw = (reinterpret_cast<const uint4*>(ot.tab + s) + 1)->x;
        vk[j] = (int64_t)(((uint64_t)lo.y << 32) | lo.x);
        lk[j] = (int64_t)(((uint64_t)lo.w << 32) | lo.z);
        const bool present = (s == ot.r0) ? ((aw & kAncPresent) != 0) : (vk[j] != kEmpty);
        if (present) {
          occ |= 1u << j;
          ++cnt;
          if (aw & kAncParity) pk |= 1u << j;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kLabPer; ++j) {
      if (!((occ >> j) & 1u)) continue;
      const int64_t A = lk[j];
      uint32_t la;
      const uint32_t sa = lookup_find(G, A, la);
      if (sa != kNoSlot) {  // the anchor took part in a union: G's canonical label, parities composed
        int64_t kx = A;
        uint32_t acc = 0;
        find_ro(G, sa, la, kx, acc);
        lk[j] = kx;
        pk ^= (acc & 1u) << j;
      }
    }
    // block exclusive scan of cnt: wave inclusive scan + wave totals in LDS
    uint32_t x = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
#pragma unroll
    for (int q = 0; q < (int)(kLabBS / 64); ++q) {
      if (q < wid) wbase += wsum[q];
      total += wsum[q];
    }
    if (threadIdx.x == 0) base_sh = total ? atomicAdd(count, (unsigned long long)total) : 0ull;
    __syncthreads();
    uint64_t pos = base_sh + wbase + (x - cnt);
#pragma unroll
    for (int j = 0; j < kLabPer; ++j) {
      if (!((occ >> j) & 1u)) continue;
      if (pos < cap_out) {
        const uint64_t s = tile + (uint64_t)j * kLabBS + threadIdx.x;
        ov[pos] = (s == ot.r0) ? kEmpty : vk[j];
        ol[pos] = lk[j];
        if (op) op[pos] = (uint8_t)((pk >> j) & 1u);
      }
      ++pos;
    }
    __syncthreads();  // (wsum and base_sh are rewritten by the next tile)
  }
}

uint32_t grid_for(uint64_t n, uint32_t bs, uint32_t cap = 65535u) {
  const uint64_t g = (n + bs - 1) / bs;
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(g, cap));
}

}  // namespace

void launch_part_init(OwnerSlot* tab, uint64_t nslots, hipStream_t st) {
  hipLaunchKernelGGL(k_part_init, dim3(grid_for(nslots, 256, 8192)), dim3(256), 0, st, tab, nslots);
}

void launch_part_snap(const Table& t, const uint32_t* mark, uint32_t* snap, int full, uint32_t dctr,
                      uint32_t shard_cap, unsigned long long* out, hipStream_t st) {
  hipLaunchKernelGGL(k_part_snap, dim3(1), dim3(64), 0, st, t, mark, snap, full, dctr, shard_cap, out);
}

void launch_part_export(bool sign, const Table& t, const uint32_t* mark, const uint32_t* snap, int full,
                        uint64_t total, int64_t* stage, int width, uint32_t* bcnt, int nranks, hipStream_t st) {
  if (!total) return;
  const uint32_t nb = (uint32_t)((total + kPartRowsPB - 1) / kPartRowsPB);
  if (sign)
    hipLaunchKernelGGL(k_part_export<true>, dim3(nb), dim3(kPartBS), 0, st, t, mark, snap, full, total, stage, width,
                       bcnt, nranks, nb);
  else
    hipLaunchKernelGGL(k_part_export<false>, dim3(nb), dim3(kPartBS), 0, st, t, mark, snap, full, total, stage, width,
                       bcnt, nranks, nb);
}

void launch_part_records(bool sign, const Table& t, const Delta& D, int64_t* pairs, int width,
                         unsigned long long* npairs, uint64_t pair_cap, hipStream_t st) {
  if (sign)
    hipLaunchKernelGGL(k_part_records<true>, dim3(kShards), dim3(256), 0, st, t, D, pairs, width, npairs, pair_cap);
  else
    hipLaunchKernelGGL(k_part_records<false>, dim3(kShards), dim3(256), 0, st, t, D, pairs, width, npairs, pair_cap);
}

void launch_part_scan(uint32_t* bcnt, uint32_t nblocks, int nranks, unsigned long long* send_counts, hipStream_t st) {
  hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(1024), 0, st, bcnt, nblocks, nranks, send_counts);
}

void launch_part_scatter(const int64_t* stage, uint64_t total, int width, const uint32_t* bcnt, uint32_t nblocks,
                         const unsigned long long* send_counts, int nranks, int64_t* sendbuf, hipStream_t st) {
  if (!total) return;
  hipLaunchKernelGGL(k_part_scatter, dim3(nblocks), dim3(kPartBS), 0, st, stage, total, width, bcnt, nblocks,
                     send_counts, nranks, sendbuf);
}

void launch_part_owner(bool sign, const OwnerTable& ot, const PairSet& ps, const int64_t* rows, uint64_t nrows,
                       int width, int64_t* pairs, unsigned long long* npairs, uint64_t pair_cap, uint32_t* fail,
                       hipStream_t st) {
  if (!nrows) return;
  const uint32_t nb = (uint32_t)((nrows + kPartRowsPB - 1) / kPartRowsPB);
  if (sign)
    hipLaunchKernelGGL(k_part_owner<true>, dim3(nb), dim3(kPartBS), 0, st, ot, ps, rows, nrows, width, pairs, npairs,
                       pair_cap, fail);
  else
    hipLaunchKernelGGL(k_part_owner<false>, dim3(nb), dim3(kPartBS), 0, st, ot, ps, rows, nrows, width, pairs, npairs,
                       pair_cap, fail);
}

void launch_part_count_word(const unsigned long long* npairs, const uint32_t* local_fail, const uint32_t* part_fail,
                            unsigned long long* word, hipStream_t st) {
  hipLaunchKernelGGL(k_part_count_word, dim3(1), dim3(1), 0, st, npairs, local_fail, part_fail, word);
}

void launch_part_labels(const OwnerTable& ot, const Table& G, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap_out,
                        unsigned long long* count, hipStream_t st) {
  hipLaunchKernelGGL(k_part_labels, dim3(grid_for((uint64_t)ot.cap + 1, kLabBS * kLabPer, 16384)), dim3(kLabBS), 0, st,
                     ot, G, ov, ol, op, cap_out, count);
}

}  // namespace gs
