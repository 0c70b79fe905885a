// gs_device.hpp -- device-side data layout and union-find primitives (gfx950).
//
// HBM layout (DESIGN.md "Data layout"): ONE open-addressing table of 16-byte slots
//   slot s = { int64 key | uint32 link | uint32 aux }
// that is at the same time the sparse-64-bit -> dense relabel table (the slot index
// IS the dense vertex id) and the union-find forest (link = parent slot << 1 |
// parity-to-parent). A relabel probe therefore returns the vertex's parent in the
// same 16-byte load, and a root's key (needed to hook by minimum id) arrives in the
// same load that proves it is a root. Slot `cap` (one past the hashed range) is
// reserved for the one id that collides with the empty marker, INT64_MIN.
//
// Concurrency model (MI355X: per-CU L1 and per-XCD L2 are not coherent inside a
// launch). Correctness never depends on a plain load being fresh:
//   * a key changes once, EMPTY -> k, by 64-bit CAS; a stale EMPTY read is settled by
//     the CAS (insert) or by an atomic re-read (hook path);
//   * links only move "up": every parent pointer points to a strictly smaller key,
//     so any historical link is still an ancestor and finds terminate;
//   * only roots are hooked (32-bit CAS expecting `self<<1`); a failed CAS returns
//     the live link and the hook loop continues from it, so each failure strictly
//     lowers that side's key -> the loop terminates without re-reading stale lines;
//   * path halving writes only to non-roots (never CAS targets) and only writes
//     ancestors with the composed parity -> benign races.
// Reference semantics replaced: DisjointSet.union/find (DisjointSet.java:66-118),
// Candidates.merge (Candidates.java:77-192) -- see DESIGN.md for the contract.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gs {

constexpr int64_t kEmpty = INT64_MIN;
constexpr int64_t kSealed = INT64_MIN + 1;  // hot-level slot closed to inserts (the id itself lives in slot r0 + 1)
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
#ifndef GS_HOT_BUCKET
#define GS_HOT_BUCKET 4
#endif
constexpr uint32_t kHotBucket = GS_HOT_BUCKET;  // hot-level bucket: slots loaded in one round trip
#ifndef GS_FOLD_BS
#define GS_FOLD_BS 256
#endif
constexpr uint32_t kFoldBS = GS_FOLD_BS;  // k_fold threads per block
#ifndef GS_INSERT_TTAS
#define GS_INSERT_TTAS 1
#endif
constexpr bool kInsertTTAS = GS_INSERT_TTAS != 0;  // fresh key load before an insert CAS (lookup_resolve)
constexpr int kShards = 64;      // sharded append counters (one 128-B line each)
constexpr int kCtrStride = 32;   // u32 per counter line
constexpr int kActSets = 3;     // active-edge lists: appended at epoch e, drained at e+1, zeroed at e+2
enum CounterBlock : int {
  CTR_NV = 0,                    // [kShards] new-vertex counts
  CTR_ACT = kShards,             // [kActSets][kShards] active-edge counts
  CTR_DELTA = (1 + kActSets) * kShards,  // [2][kShards] delta counts (two delta sets)
  CTR_FAIL = (3 + kActSets) * kShards,   // sticky bipartiteness failure
  CTR_ERR,                       // device-side error (table overflow)
  CTR_EXPORT,                    // export append counter
  CTR_OVF,                       // delta / active list overflow
  CTR_STAGE_N,                   // records staged by the running k_stage (u32 pair = u64)
  CTR_STAGE_N_HI,
  CTR_STAGE_DONE,                // k_stage block ticket
  CTR_SENT,                      // records sent by all stages since reset (u64)
  CTR_EDONE,                     // edges of completed folds since reset (u64, k_report)
  CTR_DBG_HOOKS,                 // debug build (-DGS_DEBUG_COUNTERS): hook calls,
  CTR_DBG_ITERS,                 //   hook-loop iterations,
  CTR_DBG_CASFAIL,               //   failed hook CASes
  CTR_COUNT
};
__host__ __device__ constexpr int ctr_index(int c) { return c * kCtrStride; }

#ifdef GS_DIAG_WAVES
// Diagnostic build only (tools/diag_fold.hip): per-thread event counts of k_fold
// {find steps, hook iterations, failed hook CASes, probe steps, key settles}.
constexpr uint32_t kDiagThreads = 1u << 22;
extern __device__ uint32_t gs_diag_cnt[kDiagThreads * 5];
#define GS_DIAG(k)                                                              \
  do {                                                                          \
    const uint32_t dtid_ = blockIdx.x * blockDim.x + threadIdx.x;               \
    if (dtid_ < kDiagThreads) gs_diag_cnt[dtid_ * 5 + (k)]++;                   \
  } while (0)
#else
#define GS_DIAG(k) ((void)0)
#endif

struct alignas(16) Slot {
  int64_t key;
  uint32_t link;  // parent slot << 1 | parity(v) ^ parity(parent)
  uint32_t aux;   // bit 0: reserved slot present
};

// Slot index space: [0, hotcap) hot level | [hotcap, hotcap + cap) cold level |
// r0 = hotcap + cap (id INT64_MIN) | r0 + 1 (id INT64_MIN + 1). The hot level holds
// the vertices inserted while it is open -- in a skewed stream the early, high-
// degree ones -- densely enough to stay resident in the Infinity Cache.
struct Table {
  Slot* tab;
  uint32_t* ctr;
  uint32_t hotcap;  // 0: no hot level
  uint32_t hotmask;
  int hotshift;
  int hot_open;     // inserts may go to the hot level
  uint32_t cap;     // cold level size (power of two)
  uint32_t mask;    // cap - 1
  int shift;        // 64 - log2(cap)
  uint32_t r0;      // reserved slots r0 (INT64_MIN) and r0 + 1 (INT64_MIN + 1)
};

struct Lists {
  uint2* act;            // active (root<<1|parity, root) entries, [kActSets][kShards][act_shard_cap]
  uint32_t act_shard_cap;
  int64_t* drec;         // delta records {a, b, parity} of this set, [kShards][delta_shard_cap][3]
  uint32_t delta_shard_cap;
  uint32_t dctr;         // counter index of this set's shard 0 (CTR_DELTA + set * kShards)
};

__device__ __forceinline__ uint32_t hash_slot(int64_t key, int shift) {
  return (uint32_t)(((uint64_t)key * 0x9E3779B97F4A7C15ull) >> shift);
}

// Slot of a key's first probe: its hot bucket's first slot if there is a hot level
// (buckets are kHotBucket aligned slots), else the cold level.
__device__ __forceinline__ uint32_t first_probe_slot(const Table& t, int64_t key) {
  return t.hotcap ? (hash_slot(key, t.hotshift) & ~(kHotBucket - 1)) : hash_slot(key, t.shift);
}

__device__ __forceinline__ bool is_reserved_key(int64_t key) { return key == kEmpty || key == kSealed; }

__device__ __forceinline__ void load_slot(const Slot* p, int64_t& key, uint32_t& link) {
  // one 16-B load (global_load_dwordx4): key + link in the same request
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  key = (int64_t)(((uint64_t)v.y << 32) | v.x);
  link = v.z;
}

__device__ __forceinline__ uint32_t load_link_fresh(const Slot* p) {
  return __hip_atomic_load(&p->link, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A key read as EMPTY for an occupied slot is a stale line: settle it at the
// memory-side atomic unit (rare path).
__device__ __forceinline__ int64_t settle_key(const Table& t, uint32_t s, int64_t k) {
  if (k == kEmpty && s != t.r0) {
    GS_DIAG(4);
    k = (int64_t)atomicOr((unsigned long long*)&t.tab[s].key, 0ull);
  }
  return k;
}

// Hot level: a key lives in its bucket (kHotBucket aligned slots) or not at all.
// The whole bucket is read at once (independent 16-B loads, one round trip) and
// scanned in registers. While the level is open an EMPTY slot is claimed by CAS;
// once closed, the first EMPTY slot of the bucket is sealed (CAS EMPTY -> kSealed)
// so nothing can be inserted there later: a lookup that meets a seal, or a full
// bucket of other keys, continues in the cold level. A key is therefore in at most
// one level. Returns the slot, or kNoSlot to continue in the cold level.
struct HotBucket {
  int64_t k[kHotBucket];
  uint32_t l[kHotBucket];
};

__device__ __forceinline__ void load_bucket(const Table& t, uint32_t b0, HotBucket& hb) {
#pragma unroll
  for (uint32_t i = 0; i < kHotBucket; ++i) load_slot(t.tab + b0 + i, hb.k[i], hb.l[i]);
}

// (the bucket at b0 was loaded into hb by the caller)
__device__ __forceinline__ uint32_t hot_resolve(const Table& t, int64_t key, uint32_t b0, const HotBucket& hb,
                                                uint32_t& link, bool& fresh) {
  const int64_t* k = hb.k;
  const uint32_t* l = hb.l;
#pragma unroll
  for (uint32_t i = 0; i < kHotBucket; ++i) {
    if (k[i] == key) {
      link = l[i];
      return b0 + i;
    }
  }
  for (uint32_t i = 0; i < kHotBucket; ++i) {
    int64_t ki = k[i];
    if (ki == kEmpty) {
      const int64_t want = t.hot_open ? key : kSealed;
      const unsigned long long old = atomicCAS((unsigned long long*)&t.tab[b0 + i].key, (unsigned long long)kEmpty,
                                               (unsigned long long)want);
      if (old == (unsigned long long)kEmpty) {
        if (!t.hot_open) return kNoSlot;
        fresh = true;
        link = (b0 + i) << 1;
        return b0 + i;
      }
      ki = (int64_t)old;
      if (ki == key) {
        link = t.tab[b0 + i].link;
        return b0 + i;
      }
    }
    if (ki == kSealed) return kNoSlot;
  }
  return kNoSlot;  // bucket full of other keys
}

// Insert-or-find of one id. Its first probe was already loaded by the caller
// (callers issue both endpoints' first loads back to back so they overlap): with a
// hot level the bucket at h into hb, else the cold slot h into (k, l). Returns the
// slot (dense id), its observed link and whether this call inserted it.
__device__ __forceinline__ uint32_t lookup_resolve(const Table& t, int64_t key, uint32_t h, int64_t k, uint32_t l,
                                                   const HotBucket& hb, uint32_t& link, bool& fresh) {
  fresh = false;
  if (is_reserved_key(key)) {
    const uint32_t r = t.r0 + (key == kSealed ? 1u : 0u);
    const uint32_t old = atomicOr(&t.tab[r].aux, 1u);
    fresh = (old & 1u) == 0;
    link = t.tab[r].link;
    return r;
  }
  if (t.hotcap) {
    const uint32_t s = hot_resolve(t, key, h, hb, link, fresh);
    if (s != kNoSlot) return s;
    h = t.hotcap + hash_slot(key, t.shift);
    load_slot(t.tab + h, k, l);
  }
  for (uint32_t probes = 0; probes <= t.mask; ++probes) {
    GS_DIAG(3);
    if (k == key) {
      link = l;
      return h;
    }
    if (k == kEmpty && kInsertTTAS) {
      // test-and-test-and-set: an EMPTY read may be a stale line of a hub's slot that
      // another XCD has filled; a fresh load settles it without queueing a CAS on
      // that address (all of a hub's occurrences in a batch would otherwise CAS it)
      k = (int64_t)__hip_atomic_load((unsigned long long*)&t.tab[h].key, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
      if (k == key) {
        link = load_link_fresh(t.tab + h);
        return h;
      }
    }
    if (k == kEmpty) {
      const unsigned long long old =
          atomicCAS((unsigned long long*)&t.tab[h].key, (unsigned long long)kEmpty, (unsigned long long)key);
      if (old == (unsigned long long)kEmpty) {
        fresh = true;
        link = h << 1;  // table init: every slot is its own root
        return h;
      }
      if ((int64_t)old == key) {
        link = t.tab[h].link;
        return h;
      }
    }
    h = t.hotcap + ((h - t.hotcap + 1) & t.mask);
    load_slot(t.tab + h, k, l);
  }
  atomicOr(&t.ctr[ctr_index(CTR_ERR)], 1u);
  return kNoSlot;
}

__device__ __forceinline__ uint32_t lookup_insert(const Table& t, int64_t key, uint32_t& link, bool& fresh) {
  const uint32_t h = first_probe_slot(t, key);
  int64_t k = 0;
  uint32_t l = 0;
  HotBucket hb;
  if (t.hotcap)
    load_bucket(t, h, hb);
  else
    load_slot(t.tab + h, k, l);
  return lookup_resolve(t, key, h, k, l, hb, link, fresh);
}

// Read-only lookup (no insert, no seal): slot or kNoSlot.
__device__ __forceinline__ uint32_t lookup_find(const Table& t, int64_t key, uint32_t& link) {
  if (is_reserved_key(key)) {
    const uint32_t r = t.r0 + (key == kSealed ? 1u : 0u);
    link = t.tab[r].link;
    return (t.tab[r].aux & 1u) ? r : kNoSlot;
  }
  int64_t k;
  if (t.hotcap) {
    const uint32_t b0 = hash_slot(key, t.hotshift) & ~(kHotBucket - 1);
    for (uint32_t i = 0; i < kHotBucket; ++i) {
      load_slot(t.tab + b0 + i, k, link);
      if (k == key) return b0 + i;
      if (k == kEmpty || k == kSealed) break;
    }
  }
  uint32_t h = t.hotcap + hash_slot(key, t.shift);
  for (uint32_t probes = 0; probes <= t.mask; ++probes) {
    load_slot(t.tab + h, k, link);
    if (k == key) return h;
    if (k == kEmpty) return kNoSlot;
    h = t.hotcap + ((h - t.hotcap + 1) & t.mask);
  }
  return kNoSlot;
}

// One step of a find with path splitting. (x, lx, kx): current slot, its link and
// key; (kp, lp): the loaded slot of p = parent(x). Moves x to p; when p is not a
// root, x is re-pointed at its grandparent with the composed parity first (x is a
// non-root forever and the grandparent is an ancestor: a benign race).
__device__ __forceinline__ void find_step(const Table& t, uint32_t& x, uint32_t& lx, int64_t& kx, uint32_t& acc,
                                          bool& done, int64_t kp, uint32_t lp) {
  GS_DIAG(0);
  const uint32_t p = lx >> 1;
  const uint32_t gp = lp >> 1;
  acc ^= lx & 1u;
  if (gp != p) t.tab[x].link = (gp << 1) | ((lx ^ lp) & 1u);
  else done = true;
  x = p;
  lx = lp;
  kx = kp;
}

// Find of one slot: on return x is the (believed) root, acc the parity from the
// start, kx the root's key. FRESH: read links with agent-scope loads (hook phase).
template <bool FRESH>
__device__ __forceinline__ void find_root1(const Table& t, uint32_t& x, uint32_t& lx, int64_t& kx, uint32_t& acc) {
  bool done = (lx >> 1) == x;
  while (!done) {
    int64_t kp;
    uint32_t lp;
    load_slot(t.tab + (lx >> 1), kp, lp);
    if (FRESH) lp = load_link_fresh(t.tab + (lx >> 1));
    find_step(t, x, lx, kx, acc, done, kp, lp);
  }
  kx = settle_key(t, x, kx);
}

// Two finds advanced in lockstep so that their dependent loads overlap.
template <bool FRESH>
__device__ __forceinline__ void find_root2(const Table& t, uint32_t& xa, uint32_t& la, int64_t& ka, uint32_t& acca,
                                           uint32_t& xb, uint32_t& lb, int64_t& kb, uint32_t& accb) {
  bool da = (la >> 1) == xa, db = (lb >> 1) == xb;
  while (!(da && db)) {
    int64_t kpa = 0, kpb = 0;
    uint32_t lpa = 0, lpb = 0;
    if (!da) load_slot(t.tab + (la >> 1), kpa, lpa);
    if (!db) load_slot(t.tab + (lb >> 1), kpb, lpb);
    if (FRESH) {
      if (!da) lpa = load_link_fresh(t.tab + (la >> 1));
      if (!db) lpb = load_link_fresh(t.tab + (lb >> 1));
    }
    if (!da) find_step(t, xa, la, ka, acca, da, kpa, lpa);
    if (!db) find_step(t, xb, lb, kb, accb, db, kpb, lpb);
  }
  ka = settle_key(t, xa, ka);
  kb = settle_key(t, xb, kb);
}

// Compatibility wrapper: (root, parity, key) of slot x with observed link lx.
template <bool FRESH>
__device__ __forceinline__ void find_root(const Table& t, uint32_t x, uint32_t lx, int64_t kx, uint32_t& root,
                                          uint32_t& par, int64_t& rkey) {
  uint32_t acc = 0;
  find_root1<FRESH>(t, x, lx, kx, acc);
  root = x;
  par = acc;
  rkey = kx;
}

// Hook loop: make a and b one set with colour(a) ^ colour(b) == need (SIGNED).
// The larger-key root is hooked under the smaller key, so every root is the
// minimum id of its tree (the canonical label) at all times.
#ifdef GS_DEBUG_COUNTERS
#define GS_DBG(c) atomicAdd(&t.ctr[ctr_index(c)], 1u)
#else
#define GS_DBG(c) ((void)0)
#endif

// Wave-level combining of hooks that target the same root (the hub of a skewed
// stream: while a giant component forms, most active edges of a wave are
// (hub root H, smaller root lo_i) and every one of them would CAS H's link --
// same-address atomics serialise at the memory side). For up to `rounds` groups of
// active lanes sharing the larger-key root H, the lane with the smallest lo_m keeps
// (H, lo_m) and every other lane rewrites its edge to (lo_i, lo_m) with parity
// need_i ^ need_m -- the same partition (and colouring): H ~ lo_m and lo_i ~ lo_m
// instead of H ~ lo_i, but CASes on lo_i's own link. Call in wave-uniform control
// flow; `active` marks the lanes holding an edge.
__device__ __forceinline__ int64_t wave_min_i64(int64_t x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const int64_t y = __shfl_xor(x, o, 64);
    x = y < x ? y : x;
  }
  return x;
}

__device__ __forceinline__ void combine_hooks(bool active, uint32_t& a, int64_t& ka, uint32_t& b, int64_t& kb,
                                              uint32_t& need, int rounds) {
  const int lane = (int)(threadIdx.x & 63u);
  const bool alo = ka < kb;
  const uint32_t hi = alo ? b : a, lo = alo ? a : b;
  const int64_t klo = alo ? ka : kb;
  unsigned long long pending = __ballot(active);
  for (int r = 0; r < rounds && __popcll(pending) >= 2; ++r) {
    const int leader = __ffsll((long long)pending) - 1;
    const uint32_t H = __shfl(hi, leader, 64);
    const bool in = active && ((pending >> lane) & 1ull) && hi == H;
    const unsigned long long grp = __ballot(in);
    pending &= ~grp;
    if (__popcll(grp) < 2) continue;
    const int64_t m = wave_min_i64(in ? klo : INT64_MAX);
    const int ml = __ffsll((long long)__ballot(in && klo == m)) - 1;
    const uint32_t lo_m = __shfl(lo, ml, 64);
    const uint32_t need_m = __shfl(need, ml, 64);
    if (in && lane != ml) {
      a = lo;
      ka = klo;
      b = lo_m;
      kb = m;
      need ^= need_m;
    }
  }
}

// Hook-loop finds with agent-scope (memory-side) link loads, or plain L2-cached
// loads: a stale root only costs a failed CAS, which returns the live link.
#ifndef GS_HOOK_FRESH
#define GS_HOOK_FRESH 1
#endif
constexpr bool kHookFresh = GS_HOOK_FRESH != 0;
#ifndef GS_HOOK_TTAS
#define GS_HOOK_TTAS 1
#endif
constexpr bool kHookTTAS = GS_HOOK_TTAS != 0;

template <bool SIGNED, bool TRACK>
__device__ __forceinline__ void hook(const Table& t, const Lists& L, int shard, uint32_t a, uint32_t la, int64_t ka,
                                     uint32_t b, uint32_t lb, int64_t kb, uint32_t need) {
  GS_DBG(CTR_DBG_HOOKS);
  while (true) {
    GS_DBG(CTR_DBG_ITERS);
    GS_DIAG(1);
    uint32_t pa = 0, pb = 0;
    find_root2<kHookFresh>(t, a, la, ka, pa, b, lb, kb, pb);
    la = a << 1;
    lb = b << 1;
    need ^= pa ^ pb;
    if (a == b) {
      if (SIGNED && (need & 1u)) atomicOr(&t.ctr[ctr_index(CTR_FAIL)], 1u);
      return;
    }
    const bool a_lo = ka < kb;
    const uint32_t hi = a_lo ? b : a;
    const uint32_t lo = a_lo ? a : b;
    const uint32_t expect = hi << 1;
    const uint32_t desired = (lo << 1) | (SIGNED ? (need & 1u) : 0u);
    // test-and-test-and-set: a root that a concurrent hook already moved (the hub
    // root while a giant component forms) is seen by a cheap fresh load instead of
    // a CAS that would queue behind every other CAS on that address
    const uint32_t seen = kHookTTAS ? load_link_fresh(t.tab + hi) : expect;
    const uint32_t old = seen == expect ? atomicCAS(&t.tab[hi].link, expect, desired) : seen;
    if (old == expect) {
      if (TRACK) {
        const uint32_t pos = atomicAdd(&t.ctr[ctr_index(L.dctr + shard)], 1u);
        if (pos < L.delta_shard_cap) {
          int64_t* r = L.drec + ((size_t)shard * L.delta_shard_cap + pos) * 3;
          r[0] = a_lo ? kb : ka;
          r[1] = a_lo ? ka : kb;
          r[2] = (int64_t)(SIGNED ? (need & 1u) : 0u);
        } else {
          atomicOr(&t.ctr[ctr_index(CTR_OVF)], 1u);
        }
      }
      return;
    }
    // hi was hooked meanwhile: continue that side from its live link
    GS_DBG(CTR_DBG_CASFAIL);
    GS_DIAG(2);
    if (a_lo)
      lb = old;
    else
      la = old;
  }
}

}  // namespace gs
