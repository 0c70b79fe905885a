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
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
constexpr int kShards = 64;      // sharded append counters (one 128-B line each)
constexpr int kCtrStride = 32;   // u32 per counter line
enum CounterBlock : int {
  CTR_NV = 0,                    // [kShards] new-vertex counts
  CTR_ACT0 = kShards,            // [kShards] active-edge counts, set 0
  CTR_ACT1 = 2 * kShards,        // [kShards] active-edge counts, set 1
  CTR_DELTA = 3 * kShards,       // [kShards] delta counts
  CTR_FAIL = 4 * kShards,        // sticky bipartiteness failure
  CTR_ERR,                       // device-side error (table overflow)
  CTR_EXPORT,                    // export append counter
  CTR_OVF,                       // delta / active list overflow
  CTR_COUNT
};
__host__ __device__ constexpr int ctr_index(int c) { return c * kCtrStride; }

struct alignas(16) Slot {
  int64_t key;
  uint32_t link;  // parent slot << 1 | parity(v) ^ parity(parent)
  uint32_t aux;   // bit 0: reserved slot present
};

struct Table {
  Slot* tab;
  uint32_t* ctr;
  uint32_t capidx;  // == cap: index of the reserved INT64_MIN slot
  uint32_t mask;    // cap - 1
  int shift;        // 64 - log2(cap)
};

struct Lists {
  uint2* act;            // active (root, root, parity) entries, [2][kShards][act_shard_cap]
  uint32_t act_shard_cap;
  int64_t* da;           // delta triples, [kShards][delta_shard_cap]
  int64_t* db;
  uint8_t* dw;
  uint32_t delta_shard_cap;
};

__device__ __forceinline__ uint32_t hash_slot(int64_t key, int shift) {
  return (uint32_t)(((uint64_t)key * 0x9E3779B97F4A7C15ull) >> shift);
}

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
  if (k == kEmpty && s != t.capidx) {
    k = (int64_t)atomicOr((unsigned long long*)&t.tab[s].key, 0ull);
  }
  return k;
}

// Insert-or-find of one id. Returns the slot (dense id), the slot's observed link
// and whether this call inserted it. Linear probing over 16-B slots (4 per 64-B line).
__device__ __forceinline__ uint32_t lookup_insert(const Table& t, int64_t key, uint32_t& link, bool& fresh) {
  fresh = false;
  if (key == kEmpty) {
    const uint32_t old = atomicOr(&t.tab[t.capidx].aux, 1u);
    fresh = (old & 1u) == 0;
    link = t.capidx << 1;  // the minimum id is always a root
    return t.capidx;
  }
  uint32_t h = hash_slot(key, t.shift);
  for (uint32_t probes = 0; probes <= t.mask; ++probes) {
    int64_t k;
    uint32_t l;
    load_slot(t.tab + h, k, l);
    if (k == key) {
      link = l;
      return h;
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
    h = (h + 1) & t.mask;
  }
  atomicOr(&t.ctr[ctr_index(CTR_ERR)], 1u);
  return kNoSlot;
}

// Find with path halving. (x, lx, kx) = start slot, its observed link and key.
// Returns the (believed) root, the parity x->root and the root's key.
// FRESH: read links with agent-scope loads (hook phase, where roots move).
template <bool FRESH>
__device__ __forceinline__ void find_root(const Table& t, uint32_t x, uint32_t lx, int64_t kx, uint32_t& root,
                                          uint32_t& par, int64_t& rkey) {
  uint32_t acc = 0;
  while (true) {
    const uint32_t p = lx >> 1;
    if (p == x) break;
    int64_t kp;
    uint32_t lp;
    load_slot(t.tab + p, kp, lp);
    if (FRESH) lp = load_link_fresh(t.tab + p);
    const uint32_t gp = lp >> 1;
    if (gp == p) {  // parent is the root
      acc ^= lx & 1u;
      x = p;
      kx = kp;
      break;
    }
    const uint32_t nl = (gp << 1) | ((lx ^ lp) & 1u);
    t.tab[x].link = nl;  // halving: x is a non-root forever, gp is an ancestor
    acc ^= nl & 1u;
    x = gp;
    load_slot(t.tab + gp, kx, lx);
    if (FRESH) lx = load_link_fresh(t.tab + gp);
  }
  root = x;
  par = acc;
  rkey = settle_key(t, x, kx);
}

// Hook loop: make a and b one set with colour(a) ^ colour(b) == need (SIGNED).
// The larger-key root is hooked under the smaller key, so every root is the
// minimum id of its tree (the canonical label) at all times.
template <bool SIGNED, bool TRACK>
__device__ __forceinline__ void hook(const Table& t, const Lists& L, int shard, uint32_t a, uint32_t la, int64_t ka,
                                     uint32_t b, uint32_t lb, int64_t kb, uint32_t need) {
  while (true) {
    uint32_t pa, pb;
    find_root<true>(t, a, la, ka, a, pa, ka);
    find_root<true>(t, b, lb, kb, b, pb, kb);
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
    const uint32_t old = atomicCAS(&t.tab[hi].link, expect, desired);
    if (old == expect) {
      if (TRACK) {
        const uint32_t pos = atomicAdd(&t.ctr[ctr_index(CTR_DELTA + shard)], 1u);
        if (pos < L.delta_shard_cap) {
          const size_t o = (size_t)shard * L.delta_shard_cap + pos;
          L.da[o] = a_lo ? kb : ka;
          L.db[o] = a_lo ? ka : kb;
          L.dw[o] = (uint8_t)(SIGNED ? (need & 1u) : 0u);
        } else {
          atomicOr(&t.ctr[ctr_index(CTR_OVF)], 1u);
        }
      }
      return;
    }
    // hi was hooked meanwhile: continue that side from its live link
    if (a_lo)
      lb = old;
    else
      la = old;
  }
}

}  // namespace gs
