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
// Beside the table: the VERTEX LIST (the dense ids in insertion order, 64 shards,
// so exports, resets and combines cost O(vertices) instead of O(table) on sparse
// tables), the sharded delta-record lists (multi-GPU exchange, change emission) and
// the member lists of change tracking (gs_changes.hip).
//
// Concurrency model (MI355X: per-CU L1 and per-XCD L2 are not coherent inside a
// launch). Correctness never depends on a plain load being fresh:
//   * a key changes once, EMPTY -> k, by 64-bit CAS; a stale EMPTY read is settled by
//     the CAS itself (it returns the key that won the slot);
//   * links only move "up": every parent pointer points to a strictly smaller key,
//     so any historical link is still an ancestor and finds terminate;
//   * only roots are hooked (32-bit CAS expecting `self<<1`); a failed CAS returns
//     the live link and the hook loop continues from it, so each failure strictly
//     lowers that side's key -> the loop terminates without re-reading stale lines;
//   * path splitting writes only to non-roots (never CAS targets) and only writes
//     ancestors with the composed parity -> benign races.
// Reference semantics replaced: DisjointSet.union/find (DisjointSet.java:66-118),
// Candidates.merge (Candidates.java:77-192) -- see DESIGN.md for the contract.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gs {

constexpr int64_t kEmpty = INT64_MIN;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
constexpr uint32_t kFoldBS = 256;  // k_fold threads per block (one edge per thread)
constexpr int kShards = 64;        // sharded append counters (one 128-B line each)
constexpr int kCtrStride = 32;     // u32 per counter line
constexpr uint64_t kFailBit = 1ull << 62;  // exchange count word: the sender's verdict failed
// Delta sets: tracked folds of a group's exchange b record into set b mod kDeltaSets, so
// they wait only for the stage of exchange b - kDeltaSets (which emptied that set).
#ifndef GS_DELTA_SETS
#define GS_DELTA_SETS 4
#endif
constexpr int kDeltaSets = GS_DELTA_SETS;
// experiment switches (make variant VFLAGS=...): hook's first CAS on a root the thread
// just inserted skips the re-read; throughput folds re-read an EMPTY slot before the key CAS
#ifndef GS_FRESH_HOOK_SKIP
#define GS_FRESH_HOOK_SKIP 1
#endif
#ifndef GS_WAVE_APPEND
#define GS_WAVE_APPEND 1  // 0: one append atomic per record (experiment switch)
#endif
#ifndef GS_INSERT_TTAS
// The agent-scope re-read of an EMPTY-looking slot before its key CAS (test-and-test-and-set)
// in throughput folds. Off since the paired key CASes: with both endpoints' CASes in flight
// together the re-read costs more than the hub CASes it avoids (serialised k_fold -4.7 %
// on RMAT-26, -4 % on RMAT-20; steps -0.5 / -1.9 / -0.5 % on configs 3 / 2 / 4 over three
// interleaved rounds, profiles/r04_insert_path_ab.txt). Before them it was the other way
// round (RMAT-20 0.656 vs 0.690 ms, profiles/r04_hook_ttas_ab.txt). The exchange's tracked
// own folds keep it regardless (fold_block: GS_INSERT_TTAS || TRACK).
#define GS_INSERT_TTAS 0
#endif
enum CounterBlock : int {
  CTR_NV = 0,                    // [kShards] new-vertex counts (= vertex-list fill per shard)
  CTR_DELTA = kShards,           // [kDeltaSets][kShards] delta-record counts
  CTR_FAIL = (1 + kDeltaSets) * kShards,  // sticky bipartiteness failure
  CTR_ERR,                       // device-side error (table overflow)
  CTR_EXPORT,                    // export append counter
  CTR_OVF,                       // delta list overflow
  CTR_VOVF,                      // vertex list overflow (exports / resets fall back to table scans)
  CTR_STAGE_DONE,                // k_stage block ticket
  CTR_SENT,                      // records staged since reset (u64)
  CTR_SENT_HI,
  CTR_EDONE,                     // edges of completed folds since reset (u64, k_report)
  CTR_EDONE_HI,
  CTR_EMIT,                      // change-emission output rows (u64)
  CTR_EMIT_HI,
  CTR_BIG,                       // change emission: hooked roots too large to walk
  CTR_SCAN_ALL,                  // change emission: emit every vertex (after a table rebuild)
  CTR_TAKE,                      // fused window take (k_fold TAKE): output rows reserved (u64)
  CTR_TAKE_HI,
  CTR_TAKE_DONE,                 //   block ticket, top level: shards whose blocks are all done
  CTR_DBG_HOOKS,                 // debug build (-DGS_DEBUG_COUNTERS): hook calls,
  CTR_DBG_ITERS,                 //   hook-loop iterations,
  CTR_DBG_CASFAIL,               //   failed hook CASes
  CTR_TAKE_SHARD,                // [kTicketShards] block tickets, first level (block b -> shard b mod 16)
  CTR_SRV_NV = CTR_TAKE_SHARD + 16,  // resident window server: vertices after its last window (u64)
  CTR_SRV_NV_HI,
  // debug build only (-DGS_DEBUG_COUNTERS, gs_debug_counters): where a fold's memory operations go
  CTR_DBG_EDGES,                 // valid edges / rows folded
  CTR_DBG_KCAS,                  // key CASes issued (inserts)
  CTR_DBG_KCAS_LOST,             //   ... that found the slot taken (another id, or this id by another lane)
  CTR_DBG_TTAS,                  // agent-scope re-reads of an EMPTY-looking slot before its key CAS
  CTR_DBG_SHORT,                 // edges settled by the shared-parent shortcut (no find)
  CTR_DBG_SAME,                  // edges whose finds met one root (no hook)
  CTR_DBG_FINDLD,                // parent loads of the finds (fold phase, before the hook)
  CTR_DBG_HOOKOK,                // hooks whose CAS joined two trees
  CTR_DBG_PROBES,                // extra linear-probe loads (beyond each endpoint's first)
  CTR_DBG_LAST_,
  CTR_COUNT
};
__host__ __device__ constexpr int ctr_index(int c) { return c * kCtrStride; }

#ifdef GS_DEBUG_COUNTERS
#define GS_DBG(c) atomicAdd(&t.ctr[ctr_index(c)], 1u)
#else
#define GS_DBG(c) ((void)0)
#endif

// aux bits of a slot
constexpr uint32_t kAuxPresent = 1u;  // reserved slot only: INT64_MIN is a vertex
constexpr uint32_t kAuxNew = 2u;      // change tracking: inserted since the last emission
constexpr uint32_t kAuxBig = 4u;      // change emission: a root whose absorbed list is too long to walk

struct alignas(16) Slot {
  int64_t key;
  uint32_t link;  // parent slot << 1 | parity(v) ^ parity(parent)
  uint32_t aux;
};

struct Table {
  Slot* tab;
  uint32_t* ctr;
  uint32_t cap;        // hashed slots (power of two)
  uint32_t mask;       // cap - 1
  int shift;           // 64 - log2(cap)
  uint32_t r0;         // reserved slot of INT64_MIN (== cap)
  uint32_t* vlist;     // vertex list [kShards][vshard_cap] (dense ids), or null
  uint32_t vshard_cap;
  int mark_new;        // change tracking: fresh inserts set kAuxNew
  uint32_t* hflags;    // host-mapped mirror of the rare flags: [0] CTR_ERR, [1] CTR_OVF, [2] CTR_VOVF
};

// Raise a rare flag: the device counter (read by later kernels) and its host-mapped
// mirror, so the host checks flags after a stream sync without a device-to-host copy.
__device__ __forceinline__ void raise_flag(const Table& t, int ctr_id, int mirror) {
  atomicOr(&t.ctr[ctr_index(ctr_id)], 1u);
  // a flag only goes 0 -> 1: a system-scope store (as k_report's), no PCIe atomic needed
  if (t.hflags) __hip_atomic_store(t.hflags + mirror, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Delta {
  int64_t* drec;       // records {a, b, parity} of one delta set [kShards][shard_cap][3], or null
  uint32_t shard_cap;
  uint32_t dctr;       // counter index of that set's shard 0 (CTR_DELTA + set * kShards)
  // fused window take (k_fold TAKE): the block's records go to an LDS buffer instead
  int64_t* lrec = nullptr;   // [kFoldBS][3] (LDS)
  uint32_t* lcnt = nullptr;  // its fill (LDS)
  uint32_t* lnv = nullptr;   // resident window server: the block's new vertices of the window (LDS)
};

// Home slot of an id. Ids that differ only in their low 3 bits share one 128-B line of 8
// slots: the line from a Fibonacci hash of key >> 3, the slot within it from key & 7. Dense
// id ranges (config 4's first-appearance ids, ids assigned in order) then fill whole lines,
// and the table's working set is their 16 B per id instead of a line per id: config 4
// 0.893-0.902 -> 0.774-0.802 ms/step; random 64-bit ids (configs 2, 3, 5) place as before
// (profiles/r05_hash_line_ab.txt). GS_HASH_LINE=0: the plain Fibonacci hash of the id.
#ifndef GS_HASH_LINE
#define GS_HASH_LINE 1
#endif
__device__ __forceinline__ uint32_t hash_slot(int64_t key, int shift) {
#if GS_HASH_LINE
  return ((uint32_t)((((uint64_t)key >> 3) * 0x9E3779B97F4A7C15ull) >> (shift + 3)) << 3) | (uint32_t)(key & 7);
#else
  return (uint32_t)(((uint64_t)key * 0x9E3779B97F4A7C15ull) >> shift);
#endif
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
  if (k == kEmpty && s != t.r0) k = (int64_t)atomicOr((unsigned long long*)&t.tab[s].key, 0ull);
  return k;
}

// Insert-or-find of one id. Its first probe (slot h, loaded into k, l) was issued by
// the caller (callers issue both endpoints' first loads back to back so they
// overlap). Returns the slot (dense id), its observed link and whether this call
// inserted it. TTAS: re-read an EMPTY-looking slot with an agent-scope load before the
// key CAS (throughput folds; the window takes CAS at once, below).
template <bool TTAS = true>
__device__ __forceinline__ uint32_t lookup_resolve(const Table& t, int64_t key, uint32_t h, int64_t k, uint32_t l,
                                                   uint32_t& link, bool& fresh) {
  fresh = false;
  if (key == kEmpty) {
    const uint32_t old = atomicOr(&t.tab[t.r0].aux, kAuxPresent);
    fresh = (old & kAuxPresent) == 0;
    if (fresh && t.mark_new) atomicOr(&t.tab[t.r0].aux, kAuxNew);
    link = t.tab[t.r0].link;
    return t.r0;
  }
  for (uint32_t probes = 0; probes <= t.mask; ++probes) {
    if (k == key) {
      link = l;
      return h;
    }
    // An EMPTY read may be a stale line of a slot another XCD has filled; the CAS settles
    // it (it returns the winner's key). With TTAS (GS_INSERT_TTAS, off by default since
    // the paired key CASes) a throughput fold first re-reads the slot with an agent-scope
    // load, so that a hub's occurrences in a young table's batch do not queue CASes on
    // its slot. The window takes (TAKE) never re-read: one round trip less per insert
    // (config 5 p50 13.6 -> 12.9 us, p99 27.1 -> 25.5; profiles/r03_insert_ab.txt).
    if (TTAS && k == kEmpty) {
      GS_DBG(CTR_DBG_TTAS);
      k = (int64_t)__hip_atomic_load((unsigned long long*)&t.tab[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (k == key) {
        link = load_link_fresh(t.tab + h);
        return h;
      }
    }
    if (k == kEmpty) {
      GS_DBG(CTR_DBG_KCAS);
      const unsigned long long old =
          atomicCAS((unsigned long long*)&t.tab[h].key, (unsigned long long)kEmpty, (unsigned long long)key);
      if (old != (unsigned long long)kEmpty) GS_DBG(CTR_DBG_KCAS_LOST);
      if (old == (unsigned long long)kEmpty) {
        fresh = true;
        if (t.mark_new) t.tab[h].aux = kAuxNew;  // only the inserting thread writes a fresh slot's aux
        link = h << 1;  // table init: every slot is its own root
        return h;
      }
      if ((int64_t)old == key) {
        link = load_link_fresh(t.tab + h);
        return h;
      }
    }
    h = (h + 1) & t.mask;
    GS_DBG(CTR_DBG_PROBES);
    load_slot(t.tab + h, k, l);
  }
  raise_flag(t, CTR_ERR, 0);
  return kNoSlot;
}

// The end of an insert attempt at slot h: `old` is the key the slot held (the CAS's
// return when `tried`, else an agent-scope read). Slot won, found, or -- held by another
// id -- the probe continues at h + 1.
template <bool TTAS>
__device__ __forceinline__ uint32_t insert_finish(const Table& t, int64_t key, uint32_t h, unsigned long long old,
                                                  bool tried, uint32_t& link, bool& fresh) {
  fresh = false;
  if (tried && old != (unsigned long long)kEmpty) GS_DBG(CTR_DBG_KCAS_LOST);
  if (tried && old == (unsigned long long)kEmpty) {
    fresh = true;
    if (t.mark_new) t.tab[h].aux = kAuxNew;
    link = h << 1;
    return h;
  }
  if ((int64_t)old == key) {
    link = load_link_fresh(t.tab + h);
    return h;
  }
  h = (h + 1) & t.mask;
  int64_t k;
  uint32_t l;
  GS_DBG(CTR_DBG_PROBES);
  load_slot(t.tab + h, k, l);
  return lookup_resolve<TTAS>(t, key, h, k, l, link, fresh);
}

// Both endpoints' first probes read EMPTY (a young table: config 5's first windows,
// config 4's insert phase): their key CASes (and, TTAS, the re-reads before them) go out
// together instead of one endpoint's chain after the other's -- one dependent atomic
// round trip less per edge that inserts both ends. Precondition: ku != kv, hu != hv,
// neither id is kEmpty.
#ifndef GS_PAIR_INSERT
#define GS_PAIR_INSERT 1  // 0: endpoints inserted one after the other (experiment switch)
#endif
template <bool TTAS, bool TTAS_V = TTAS>
__device__ __forceinline__ void insert_pair(const Table& t, int64_t ku, uint32_t hu, int64_t kv, uint32_t hv,
                                            uint32_t& su, uint32_t& lu, bool& nu, uint32_t& sv, uint32_t& lv,
                                            bool& nv) {
  unsigned long long ou = (unsigned long long)kEmpty, ov = (unsigned long long)kEmpty;
  if (TTAS) {
    GS_DBG(CTR_DBG_TTAS);
    ou = __hip_atomic_load((unsigned long long*)&t.tab[hu].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (TTAS_V) {
    GS_DBG(CTR_DBG_TTAS);
    ov = __hip_atomic_load((unsigned long long*)&t.tab[hv].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const bool tu = ou == (unsigned long long)kEmpty, tv = ov == (unsigned long long)kEmpty;
  // Both tests before either CAS, and no use of the first CAS's result before the second
  // is issued (left to itself the compiler tested the second re-read after the first CAS
  // and waited for that CAS). A slot the re-read found taken gets no CAS: a hub's slot
  // must not queue same-address atomics (RMAT-20: 0.69 -> 0.745 ms/step with no-op CASes).
  const uint32_t tv32 = tv ? 1u : 0u;
  asm volatile("" ::"v"(tv32) : "memory");  // the second test is materialised here, before either CAS
  __builtin_amdgcn_sched_barrier(0);
  if (tu) GS_DBG(CTR_DBG_KCAS);
  if (tv32) GS_DBG(CTR_DBG_KCAS);
  if (tu) ou = atomicCAS((unsigned long long*)&t.tab[hu].key, (unsigned long long)kEmpty, (unsigned long long)ku);
  if (tv32) ov = atomicCAS((unsigned long long*)&t.tab[hv].key, (unsigned long long)kEmpty, (unsigned long long)kv);
  __builtin_amdgcn_sched_barrier(0);
  su = insert_finish<TTAS>(t, ku, hu, ou, tu, lu, nu);
  sv = insert_finish<TTAS_V>(t, kv, hv, ov, tv, lv, nv);
}

__device__ __forceinline__ uint32_t lookup_insert(const Table& t, int64_t key, uint32_t& link, bool& fresh) {
  const uint32_t h = hash_slot(key, t.shift);
  int64_t k;
  uint32_t l;
  load_slot(t.tab + h, k, l);
  return lookup_resolve(t, key, h, k, l, link, fresh);
}

// Read-only lookup (no insert): slot or kNoSlot.
__device__ __forceinline__ uint32_t lookup_find(const Table& t, int64_t key, uint32_t& link) {
  if (key == kEmpty) {
    link = t.tab[t.r0].link;
    return (t.tab[t.r0].aux & kAuxPresent) ? t.r0 : kNoSlot;
  }
  int64_t k;
  uint32_t h = hash_slot(key, t.shift);
  for (uint32_t probes = 0; probes <= t.mask; ++probes) {
    load_slot(t.tab + h, k, link);
    if (k == key) return h;
    if (k == kEmpty) return kNoSlot;
    h = (h + 1) & t.mask;
  }
  return kNoSlot;
}

// Register fresh inserts: the shard's new-vertex count (capacity tracking) doubles
// as the append position of the vertex list; change tracking needs nothing more
// (lookup_resolve marked the slots). The fold reserves the positions right after its
// probes and writes the ids after its finds and hook, so that the returning atomic
// overlaps the find loads instead of preceding them (config 5 with the CAS-only
// insert: p50 13.4 -> 12.5 us, p99 27.2 -> 24.8; profiles/r03_insert_ab.txt).
// The reservation is wave-aggregated: one atomic per wave for the wave's new vertices
// (a wave scan of the per-lane counts gives each lane its offset). One per inserting lane
// serialised on the shard's counter while a young table fills: ~1 K same-address
// atomics per shard per 2^16-edge window of config 5, ~16 K per 2^20-edge batch of
// config 4's insert phase (11 ns each at the memory side, profiles/r01_calib_atomic.log).
// Both calls are made in wave-uniform control flow.
#ifndef GS_WAVE_RESERVE
#define GS_WAVE_RESERVE 1  // 0: one reservation atomic per inserting lane (experiment switch)
#endif
struct NewVertices {
  uint32_t k = 0, pos = 0, su = 0, sv = 0;
  bool nu = false;
};

// lnv (optional, LDS): the block's count of new vertices, for the window server's tickets
__device__ __forceinline__ NewVertices reserve_new_vertices(const Table& t, int shard, bool nu, uint32_t su, bool nv,
                                                            uint32_t sv, uint32_t* lnv = nullptr) {
  NewVertices r;
  r.k = (nu ? 1u : 0u) + ((nv && sv != su) ? 1u : 0u);
  r.nu = nu;
  r.su = su;
  r.sv = sv;
  if (!GS_WAVE_RESERVE) {
    if (r.k) r.pos = atomicAdd(&t.ctr[ctr_index(CTR_NV + shard)], r.k);
    if (lnv && r.k) atomicAdd(lnv, r.k);
    return r;
  }
  const int lane = (int)(threadIdx.x & 63u);
  uint32_t x = r.k;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  const uint32_t total = __shfl(x, 63, 64);
  // until write_new_vertices: lane 0 holds the wave's base (the returning atomic overlaps
  // the finds), every lane its exclusive offset
  r.pos = x - r.k;
  if (total && lane == 0) {
    r.pos = atomicAdd(&t.ctr[ctr_index(CTR_NV + shard)], total);
    if (lnv) atomicAdd(lnv, total);
  }
  return r;
}

__device__ __forceinline__ void write_new_vertices(const Table& t, int shard, NewVertices r) {
  if (GS_WAVE_RESERVE) {
    const uint32_t excl = r.pos;
    const uint32_t base = __shfl(r.pos, 0, 64);
    // lane 0's own offset is 0: its pos became the base
    r.pos = base + ((threadIdx.x & 63u) == 0 ? 0u : excl);
  }
  if (!r.k || !t.vlist) return;
  if (r.pos + r.k > t.vshard_cap) {
    raise_flag(t, CTR_VOVF, 2);
    return;
  }
  uint32_t* vl = t.vlist + (size_t)shard * t.vshard_cap + r.pos;
  if (r.nu) *vl++ = r.su;
  if (r.k == 2u || !r.nu) *vl = r.sv;
}

// One step of a find with path splitting. (x, lx, kx): current slot, its link and
// key; (kp, lp): the loaded slot of p = parent(x). Moves x to p; when p is not a
// root, x is re-pointed at its grandparent with the composed parity first (x is a
// non-root forever and the grandparent is an ancestor: a benign race).
__device__ __forceinline__ void find_step(const Table& t, uint32_t& x, uint32_t& lx, int64_t& kx, uint32_t& acc,
                                          bool& done, int64_t kp, uint32_t lp) {
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
    if (!FRESH && !da) GS_DBG(CTR_DBG_FINDLD);
    if (!FRESH && !db) GS_DBG(CTR_DBG_FINDLD);
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

// Read-only find (no path splitting): root slot, key and parity of slot x.
__device__ __forceinline__ uint32_t find_ro(const Table& t, uint32_t x, uint32_t lx, int64_t& kx, uint32_t& acc) {
  acc = 0;
  while ((lx >> 1) != x) {
    acc ^= lx & 1u;
    x = lx >> 1;
    load_slot(t.tab + x, kx, lx);
  }
  kx = settle_key(t, x, kx);
  return x;
}


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

// Append one delta record {a, b, w} to shard `shard` of the delta list, or (TAKE) to
// the block's LDS buffer: a lane appends at most one record per edge it folds (a
// self-loop's new vertex or one successful hook), so kFoldBS rows always suffice.
template <bool TAKE = false>
__device__ __forceinline__ void append_record(const Table& t, const Delta& D, int shard, int64_t a, int64_t b,
                                              int64_t w) {
  if (TAKE) {
    const uint32_t p = atomicAdd(D.lcnt, 1u);
    if (p < kFoldBS) {
      D.lrec[p * 3] = a;
      D.lrec[p * 3 + 1] = b;
      D.lrec[p * 3 + 2] = w;
    }
    return;
  }
  const uint32_t pos = atomicAdd(&t.ctr[ctr_index(D.dctr + shard)], 1u);
  if (pos < D.shard_cap) {
    int64_t* r = D.drec + ((size_t)shard * D.shard_cap + pos) * 3;
    r[0] = a;
    r[1] = b;
    r[2] = w;
  } else {
    raise_flag(t, CTR_OVF, 1);
  }
}

// Wave-aggregated append (the tracked folds of a group's exchange): the lanes of a wave
// holding a record take one range of the shard with ONE atomic and write their rows
// contiguously (coalesced 24-B rows), instead of one same-address atomic and a scattered
// row per record. Call in wave-uniform control flow.
__device__ __forceinline__ void append_record_wave(const Table& t, const Delta& D, int shard, bool has, int64_t a,
                                                   int64_t b, int64_t w) {
  const unsigned long long m = __ballot(has);
  if (!m) return;
  const int lane = (int)(threadIdx.x & 63u);
  const int leader = __ffsll((long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(&t.ctr[ctr_index(D.dctr + shard)], (uint32_t)__popcll(m));
  base = __shfl(base, leader, 64);
  if (!has) return;
  const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
  if (pos < D.shard_cap) {
    int64_t* r = D.drec + ((size_t)shard * D.shard_cap + pos) * 3;
    r[0] = a;
    r[1] = b;
    r[2] = w;
  } else {
    raise_flag(t, CTR_OVF, 1);
  }
}

// Hook loop: make a and b one set with colour(a) ^ colour(b) == need (SIGNED).
// The larger-key root is hooked under the smaller key, so every root is the
// minimum id of its tree (the canonical label) at all times. Finds read links with
// agent-scope loads; before its CAS the loop re-reads the target root's link
// (test-and-test-and-set): a root a concurrent hook already moved -- the hub root
// while a giant component forms -- is followed without queueing a CAS on its address.
// fresh0 / fresh1: slots this thread has just inserted (kNoSlot: none). A root this
// thread created itself is not a hub other lanes queue on: its first CAS goes out without
// the re-read (one dependent round trip less for every edge that hooks a new vertex --
// the young table's windows of config 5 and the first micro-batches of configs 2 and 4).
// Returns whether this call's CAS joined two trees; with TRACK the join's record
// {hi key, lo key, parity} goes to rec (appended by the caller).
template <bool SIGNED, bool TRACK>
__device__ __forceinline__ bool hook(const Table& t, uint32_t a, uint32_t la, int64_t ka, uint32_t b, uint32_t lb,
                                     int64_t kb, uint32_t need, uint32_t fresh0, uint32_t fresh1, int64_t* rec) {
  GS_DBG(CTR_DBG_HOOKS);
  bool first = true;
  while (true) {
    GS_DBG(CTR_DBG_ITERS);
    uint32_t pa = 0, pb = 0;
    find_root2<true>(t, a, la, ka, pa, b, lb, kb, pb);
    la = a << 1;
    lb = b << 1;
    need ^= pa ^ pb;
    if (a == b) {
      if (SIGNED && (need & 1u)) atomicOr(&t.ctr[ctr_index(CTR_FAIL)], 1u);
      return false;
    }
    const bool a_lo = ka < kb;
    const uint32_t hi = a_lo ? b : a;
    const uint32_t lo = a_lo ? a : b;
    const uint32_t expect = hi << 1;
    const uint32_t desired = (lo << 1) | (SIGNED ? (need & 1u) : 0u);
    const bool own = GS_FRESH_HOOK_SKIP && first && (hi == fresh0 || hi == fresh1);
    first = false;
    const uint32_t seen = own ? expect : load_link_fresh(t.tab + hi);
    const uint32_t old = seen == expect ? atomicCAS(&t.tab[hi].link, expect, desired) : seen;
    if (old == expect) {
      GS_DBG(CTR_DBG_HOOKOK);
      if (TRACK) {
        rec[0] = a_lo ? kb : ka;
        rec[1] = a_lo ? ka : kb;
        rec[2] = (int64_t)(SIGNED ? (need & 1u) : 0u);
      }
      return true;
    }
    // hi was hooked meanwhile: continue that side from its live link
    GS_DBG(CTR_DBG_CASFAIL);
    if (a_lo)
      lb = old;
    else
      la = old;
  }
}

}  // namespace gs
