// gs_kernels.hip -- HIP kernels of the summary fold (gfx950, wave64).
//
//   k_init    : table reset (slot s := {EMPTY, s<<1, 0})              -- HBM write-bound
//   k_fold    : per edge: 2 relabel probes + 2 finds, drop edges whose roots are
//               already equal, append the rest (root, root, parity) to the sharded
//               active list (wave-aggregated appends)                  -- HBM/latency-bound
//   k_hook    : lock-free CAS hooking of the compacted active edges    -- latency-bound
//   k_export  : (vertex, min-id label, parity) of every occupied slot, block-aggregated
//   k_pack    : contiguous copy of the sharded delta list (multi-GPU exchange)
// Reference: DisjointSet.union (DisjointSet.java:92-118) / Candidates.merge
// (Candidates.java:77-139) folded once per edge by PartialAgg.fold
// (SummaryBulkAggregation.java:121-123).
#include "gs_device.hpp"
#include "gs_kernels.hpp"

namespace gs {

#ifdef GS_DIAG_WAVES
// Diagnostic build only (tools/diag_fold.hip): per-wave {start, end, block, xcc}
// of k_fold in 100 MHz wall-clock ticks.
constexpr uint32_t kDiagWaves = 1u << 16;
__device__ uint64_t gs_diag_waves[kDiagWaves * 2];
__device__ uint32_t gs_diag_meta[kDiagWaves];
__device__ uint32_t gs_diag_cnt[kDiagThreads * 5];
void diag_copy(uint64_t* w, uint32_t* m, size_t nw, uint32_t* cnt, size_t nt) {
  (void)hipMemcpyFromSymbol(w, HIP_SYMBOL(gs_diag_waves), nw * 16);
  (void)hipMemcpyFromSymbol(m, HIP_SYMBOL(gs_diag_meta), nw * 4);
  if (cnt) (void)hipMemcpyFromSymbol(cnt, HIP_SYMBOL(gs_diag_cnt), nt * 20);
}
void diag_clear(size_t nt) {
  static uint32_t* z = nullptr;
  if (!z) z = (uint32_t*)calloc(kDiagThreads * 5, 4);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(gs_diag_cnt), z, nt * 20);
}
#endif

// slot s := {EMPTY, s << 1, 0}; the second reserved slot carries its id INT64_MIN + 1
__global__ __launch_bounds__(256) void k_init(Slot* tab, uint64_t nslots) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < nslots;
       s += (uint64_t)gridDim.x * blockDim.x) {
    uint4 v;
    v.x = (s == nslots - 1) ? 1u : 0u;
    v.y = 0x80000000u;  // INT64_MIN (+1 for the last slot)
    v.z = (uint32_t)(s << 1);
    v.w = 0u;
#ifdef GS_INIT_NT
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const v4u nv = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(nv, reinterpret_cast<v4u*>(tab + s));
#else
    *reinterpret_cast<uint4*>(tab + s) = v;
#endif
  }
}

// Hook every entry of one shard slice of active set `set` (entries j = j0, j0+step, ...).
template <bool SIGNED, bool TRACK>
__device__ __forceinline__ void drain_entries(const Table& t, const Lists& L, int set, int s, uint32_t j0,
                                              uint32_t step) {
  const uint32_t cnt = min(t.ctr[ctr_index(CTR_ACT + set * kShards + s)], L.act_shard_cap);
  const uint2* act = L.act + ((size_t)set * kShards + s) * L.act_shard_cap;
  for (uint32_t j = j0; j < cnt; j += step) {
    const uint2 e = act[j];
    const uint32_t a = e.x >> 1, b = e.y;
    int64_t ka, kb;
    uint32_t la, lb;
    load_slot(t.tab + a, ka, la);
    load_slot(t.tab + b, kb, lb);
    la = load_link_fresh(t.tab + a);
    lb = load_link_fresh(t.tab + b);
    hook<SIGNED, TRACK>(t, L, s, a, la, settle_key(t, a, ka), b, lb, settle_key(t, b, kb), e.x & 1u);
  }
}

// Drain a whole active set with the current grid (any size).
template <bool SIGNED, bool TRACK>
__device__ __forceinline__ void drain_set(const Table& t, const Lists& L, int set) {
  const uint32_t G = gridDim.x;
  if (G >= (uint32_t)kShards) {
    const uint32_t nparts = G / kShards, part = blockIdx.x / kShards;
    if (part < nparts) drain_entries<SIGNED, TRACK>(t, L, set, blockIdx.x % kShards, part * blockDim.x + threadIdx.x, nparts * blockDim.x);
  } else {
    for (uint32_t s = blockIdx.x; s < (uint32_t)kShards; s += G)
      drain_entries<SIGNED, TRACK>(t, L, set, (int)s, threadIdx.x, blockDim.x);
  }
}

// k_fold: EPT edges per thread (edge i = block*256*EPT + e*256 + tid: coalesced).
// For every edge: both relabel probes issued back to back, shortcut on a shared
// parent, lockstep finds of the two roots; an edge whose roots differ is hooked
// in place when its wave has <= a.inline_max such edges, otherwise appended to
// active set a.cur (drained by the next launch, or by k_hook on a flush).
// The block also drains its slice of set a.drain and block 0 zeroes set a.zero.
struct FoldArgs {
  const int64_t* src;
  const int64_t* dst;
  const uint8_t* w;   // per edge: bit 0 = required parity (SIGNED), bit 7 = skip (padding record)
  uint32_t n;
  uint32_t stride;    // elements between consecutive src (and dst) entries
  uint32_t w_stride;  // bytes between consecutive w entries
  uint32_t rows;      // > 0: exchange layout, `rows` records per rank, row 0 = header {sent, ...}
  int skip_rank;      // rank whose rows are skipped (the caller's own)
  const int64_t* hdr; // exchange layout: start of the gathered buffer (rank r header at hdr[r * rows * stride])
  uint32_t base;      // exchange layout: index of this launch's first record in the gathered buffer
  int cur;
  int drain;
  int zero;
  int inline_max;
};

#ifndef GS_COMBINE_ROUNDS
#define GS_COMBINE_ROUNDS 2
#endif
constexpr int kCombineRounds = GS_COMBINE_ROUNDS;  // wave-level hook combining (combine_hooks)

template <bool SIGNED, bool TRACK, int EPT, bool HOT>
__global__ __launch_bounds__(kFoldBS) void k_fold(Table t, Lists L, FoldArgs a) {
  if (!HOT) t.hotcap = 0;  // compile-time: the plain path carries no hot-level code
#ifdef GS_DIAG_WAVES
  const uint64_t diag_t0 = wall_clock64();
  struct DiagEnd {
    uint64_t t0;
    __device__ ~DiagEnd() {
      const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) / 64u;
      if ((threadIdx.x & 63u) == 0 && w < kDiagWaves) {
        gs_diag_waves[2 * w] = t0;
        gs_diag_waves[2 * w + 1] = wall_clock64();
        gs_diag_meta[w] = (blockIdx.x << 4) | (__builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 15u);
      }
    }
  } diag_end{diag_t0};
#endif
  if (SIGNED && __builtin_amdgcn_readfirstlane(t.ctr[ctr_index(CTR_FAIL)]) != 0) return;
  const int shard = blockIdx.x & (kShards - 1);
  if (a.zero >= 0 && blockIdx.x == 0 && threadIdx.x < kShards)
    t.ctr[ctr_index(CTR_ACT + a.zero * kShards + threadIdx.x)] = 0u;

  bool valid[EPT], act[EPT];
  int64_t ks[EPT], kd[EPT];
  uint32_t need[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const uint32_t i = blockIdx.x * (kFoldBS * EPT) + e * kFoldBS + threadIdx.x;
    valid[e] = i < a.n;
    act[e] = false;
    if (valid[e] && a.rows) {  // exchange layout: per-rank header gives the live row count
      const uint32_t ig = a.base + i, r = ig / a.rows, j = ig - r * a.rows;
      valid[e] = j >= 1 && (int)r != a.skip_rank && (int64_t)j <= a.hdr[(size_t)r * a.rows * a.stride];
    }
    const uint32_t wi = (valid[e] && a.w) ? a.w[(size_t)i * a.w_stride] : 1u;
    if (wi & 0x80u) valid[e] = false;
#ifdef GS_NT_EDGES
    ks[e] = valid[e] ? __builtin_nontemporal_load(&a.src[(size_t)i * a.stride]) : 0;
    kd[e] = valid[e] ? __builtin_nontemporal_load(&a.dst[(size_t)i * a.stride]) : 0;
#else
    ks[e] = valid[e] ? a.src[(size_t)i * a.stride] : 0;
    kd[e] = valid[e] ? a.dst[(size_t)i * a.stride] : 0;
#endif
    need[e] = SIGNED ? (wi & 1u) : 0u;
  }
  // all first relabel probes of the thread in flight together
  uint32_t hu[EPT], hv[EPT], l0u[EPT], l0v[EPT];
  int64_t k0u[EPT], k0v[EPT];
  HotBucket hbu[HOT ? EPT : 1], hbv[HOT ? EPT : 1];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    hu[e] = first_probe_slot(t, ks[e]);
    hv[e] = first_probe_slot(t, kd[e]);
    k0u[e] = k0v[e] = 0;
    l0u[e] = l0v[e] = 0;
    if (valid[e]) {
      if (HOT) {  // both endpoints' hot buckets in one round trip
        load_bucket(t, hu[e], hbu[HOT ? e : 0]);
        load_bucket(t, hv[e], hbv[HOT ? e : 0]);
      } else {
        load_slot(t.tab + hu[e], k0u[e], l0u[e]);
        load_slot(t.tab + hv[e], k0v[e], l0v[e]);
      }
    }
  }
  uint32_t ru[EPT], rv[EPT], lu[EPT], lv[EPT];
  int64_t kru[EPT], krv[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    if (!valid[e]) continue;
    bool nu, nv;
    const uint32_t su = lookup_resolve(t, ks[e], hu[e], k0u[e], l0u[e], hbu[HOT ? e : 0], lu[e], nu);
    const uint32_t sv = lookup_resolve(t, kd[e], hv[e], k0v[e], l0v[e], hbv[HOT ? e : 0], lv[e], nv);
    if (nu || nv) atomicAdd(&t.ctr[ctr_index(CTR_NV + shard)], (nu ? 1u : 0u) + (nv && sv != su ? 1u : 0u));
    // Delta: a new vertex with an edge to another vertex is always named by a hook
    // record (as the hooked root or as the new parent: its singleton tree can only
    // change through a CAS on it or onto it), so only a new vertex seen through a
    // self-loop needs a record of its own.
    if (TRACK && nu && su == sv) {
      const uint32_t pos = atomicAdd(&t.ctr[ctr_index(L.dctr + shard)], 1u);
      if (pos < L.delta_shard_cap) {
        int64_t* r = L.drec + ((size_t)shard * L.delta_shard_cap + pos) * 3;
        r[0] = ks[e];
        r[1] = ks[e];
        r[2] = 0;
      } else {
        atomicOr(&t.ctr[ctr_index(CTR_OVF)], 1u);
      }
    }
    ru[e] = su;
    rv[e] = sv;
    if (su == kNoSlot || sv == kNoSlot || su == sv) continue;  // self-loop: vertex added, never a conflict
    // shortcut: shared parent (the common case once trees are flat) or parent/child
    const uint32_t pu = lu[e] >> 1, pv = lv[e] >> 1;
    if (pu == pv || pu == sv || pv == su) {
      if (SIGNED) {
        const uint32_t par = (pu == pv) ? ((lu[e] ^ lv[e]) & 1u) : (pu == sv ? (lu[e] & 1u) : (lv[e] & 1u));
        if ((need[e] ^ par) & 1u) atomicOr(&t.ctr[ctr_index(CTR_FAIL)], 1u);
      }
      continue;
    }
    uint32_t pru = 0, prv = 0;
    kru[e] = ks[e];
    krv[e] = kd[e];
    find_root2<false>(t, ru[e], lu[e], kru[e], pru, rv[e], lv[e], krv[e], prv);
    need[e] ^= pru ^ prv;
    if (ru[e] == rv[e]) {
      if (SIGNED && (need[e] & 1u)) atomicOr(&t.ctr[ctr_index(CTR_FAIL)], 1u);
      continue;
    }
    act[e] = true;
  }
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const unsigned long long m = __ballot(act[e]);
    const bool in_place = __popcll(m) <= (unsigned)a.inline_max;
    if (in_place && kCombineRounds > 0 && __popcll(m) >= 2)  // wave-uniform
      combine_hooks(act[e], ru[e], kru[e], rv[e], krv[e], need[e], kCombineRounds);
    if (!act[e]) continue;
    if (in_place) {
      hook<SIGNED, TRACK>(t, L, shard, ru[e], ru[e] << 1, kru[e], rv[e], rv[e] << 1, krv[e], need[e]);
    } else {
      const uint32_t pos = atomicAdd(&t.ctr[ctr_index(CTR_ACT + a.cur * kShards + shard)], 1u);
      if (pos < L.act_shard_cap) {
        L.act[((size_t)a.cur * kShards + shard) * L.act_shard_cap + pos] =
            make_uint2((ru[e] << 1) | (SIGNED ? (need[e] & 1u) : 0u), rv[e]);
      } else {
        atomicOr(&t.ctr[ctr_index(CTR_OVF)], 1u);
      }
    }
  }
  if (a.drain >= 0) drain_set<SIGNED, TRACK>(t, L, a.drain);
}

// Flush / compacted mode: drain active set `set` with a dedicated launch.
template <bool SIGNED, bool TRACK>
__global__ __launch_bounds__(256) void k_hook(Table t, Lists L, int set) {
  if (SIGNED && __builtin_amdgcn_readfirstlane(t.ctr[ctr_index(CTR_FAIL)]) != 0) return;
  drain_set<SIGNED, TRACK>(t, L, set);
}

// Export (vertex, label, parity) of every occupied slot. Each thread owns 16 slots
// of a 16 x kExportBS-slot tile (slot = tile + j*kExportBS + tid: coalesced 16-B loads); the block
// reserves its output range with ONE atomic per tile.
#ifndef GS_EXPORT_BS
#define GS_EXPORT_BS 1024
#endif
constexpr uint32_t kExportBS = GS_EXPORT_BS;  // one output-reservation atomic per kExportPer x kExportBS slots
#ifndef GS_EXPORT_PER
#define GS_EXPORT_PER 16
#endif
constexpr int kExportPer = GS_EXPORT_PER;  // slots per thread per tile

template <bool SIGNED>
__global__ __launch_bounds__(kExportBS) void k_export(Table t, int64_t* __restrict__ ov, int64_t* __restrict__ ol,
                                                uint8_t* __restrict__ op, uint64_t cap_out, uint64_t s_begin,
                                                uint64_t s_end) {
  constexpr int PER = kExportPer;
  __shared__ uint32_t wsum[kExportBS / 64];
  __shared__ uint32_t base_sh;
  const uint64_t nslots = s_end;  // slots [s_begin, s_end) of [0, r0 + 2)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (uint64_t tile = s_begin + (uint64_t)blockIdx.x * (kExportBS * PER); tile < nslots;
       tile += (uint64_t)gridDim.x * (kExportBS * PER)) {
    int64_t vk[PER], lk[PER];
    uint32_t pp[PER];
    uint32_t occ = 0, cnt = 0;
    // 1) all of the thread's slots in flight together (coalesced 16-B loads)
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint64_t s = tile + (uint64_t)j * kExportBS + threadIdx.x;
      vk[j] = 0;
      pp[j] = 0;
      if (s < nslots) {
        load_slot(t.tab + s, vk[j], pp[j]);
        const bool present = (s >= t.r0) ? ((t.tab[s].aux & 1u) != 0)
                                         : (vk[j] != kEmpty && !(s < t.hotcap && vk[j] == kSealed));
        if (present) {
          occ |= 1u << j;
          ++cnt;
        }
      }
    }
    // 2) read-only finds (the label pass does not compress: no stores between loads)
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      lk[j] = vk[j];
      if (!((occ >> j) & 1u)) continue;
      uint32_t x = (uint32_t)(tile + (uint64_t)j * kExportBS + threadIdx.x), lx = pp[j], acc = 0;
      int64_t kx = vk[j];
      while ((lx >> 1) != x) {
        acc ^= lx & 1u;
        x = lx >> 1;
        load_slot(t.tab + x, kx, lx);
      }
      lk[j] = kx;
      pp[j] = acc;
    }
    // block exclusive scan of cnt: wave inclusive scan + 4 wave totals in LDS
    uint32_t x = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
    for (int q = 0; q < (int)(kExportBS / 64); ++q) {
      if (q < wid) wbase += wsum[q];
      total += wsum[q];
    }
    if (threadIdx.x == 0) base_sh = total ? atomicAdd(&t.ctr[ctr_index(CTR_EXPORT)], total) : 0u;
    __syncthreads();
    uint64_t pos = (uint64_t)base_sh + wbase + (x - cnt);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (occ & (1u << j)) {
        if (pos < cap_out) {
          ov[pos] = vk[j];
          ol[pos] = lk[j];
          if (op) op[pos] = (uint8_t)pp[j];
        }
        ++pos;
      }
    }
    __syncthreads();
  }
}

// One exchange stage, one launch. Every delta record -- first the backlog q_in
// (qn_in records left over from the previous stage), then the sharded delta list --
// takes a position from one counter (block-aggregated): positions < cap go to send rows 1..cap,
// the rest to the backlog q_out. Send rows are `width` int64 wide ({a, b} or
// {a, b, w}); the backlog is always {a, b, w}. The last block to finish writes the
// header row {sent, queued[, skip]}, *qn_out, and resets the counters it consumed. The receiver
// reads `sent` from the header, so unused send rows need no padding.
// cap == 0 with send == nullptr: everything goes to q_out (gs_take_delta_records).
__device__ __forceinline__ void stage_write(const Table& t, unsigned long long pos, int64_t a, int64_t b, int64_t w,
                                            int64_t* send, uint64_t cap, int64_t* q_out, uint64_t qcap, bool plain,
                                            int width) {
  int64_t* r;
  if (pos < cap) {  // send rows are `width` int64 wide: {a, b} (CC) or {a, b, w}
    r = send + (pos + (plain ? 0 : 1)) * width;
    r[0] = a;
    r[1] = b;
    if (width == 3) r[2] = w;
    return;
  } else if (plain) {
    return;  // take: records past cap are dropped (the caller sees the total count)
  } else if (pos - cap < qcap) {
    r = q_out + (pos - cap) * 3;
  } else {
    atomicOr(&t.ctr[ctr_index(CTR_OVF)], 1u);
    return;
  }
  r[0] = a;
  r[1] = b;
  r[2] = w;
}

// grid = kShards blocks: block s copies backlog slice s and delta shard s to
// deterministic positions (backlog first, then shards in order: a prefix of the
// 64 shard counts, no append atomics); the last block (64-way ticket) resets the
// counters the others read.
__global__ __launch_bounds__(256) void k_stage(Table t, Lists L, const int64_t* __restrict__ q_in,
                                               unsigned long long* qn_in, int64_t* __restrict__ q_out,
                                               unsigned long long* qn_out, uint64_t qcap, int64_t* __restrict__ send,
                                               uint64_t cap, unsigned long long* count_out, int width) {
  const bool plain = count_out != nullptr;  // take: rows from 0, no header, total -> *count_out
  __shared__ uint32_t cnt[kShards];
  __shared__ uint64_t off_sh, total_sh;
  const uint32_t s = blockIdx.x;
  const uint64_t backlog = min((unsigned long long)*qn_in, (unsigned long long)qcap);
  if (threadIdx.x < kShards) cnt[threadIdx.x] = min(t.ctr[ctr_index(L.dctr + threadIdx.x)], L.delta_shard_cap);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t off = backlog, tot = backlog;
    for (uint32_t q = 0; q < kShards; ++q) {
      if (q < s) off += cnt[q];
      tot += cnt[q];
    }
    off_sh = off;
    total_sh = tot;
  }
  __syncthreads();
  const uint64_t total = total_sh;
  // backlog slice s
  const uint64_t per = (backlog + kShards - 1) / kShards;
  const uint64_t b0 = (uint64_t)s * per, b1 = min(backlog, b0 + per);
  for (uint64_t i = b0 + threadIdx.x; i < b1; i += 256) stage_write(t, i, q_in[i * 3], q_in[i * 3 + 1], q_in[i * 3 + 2], send, cap, q_out, qcap, plain, width);
  // delta shard s
  const int64_t* in = L.drec + (size_t)s * L.delta_shard_cap * 3;
  const uint64_t off = off_sh;
  for (uint32_t j = threadIdx.x; j < cnt[s]; j += 256)
    stage_write(t, off + j, in[(size_t)j * 3], in[(size_t)j * 3 + 1], in[(size_t)j * 3 + 2], send, cap, q_out, qcap,
                plain, width);
  if (s == 0 && threadIdx.x == 0 && plain) {
    *count_out = total;
    *qn_out = 0ull;
  } else if (s == 0 && threadIdx.x == 0) {
    const uint64_t sent = total < cap ? total : cap;
    if (send) {
      send[0] = (int64_t)sent;
      send[1] = (int64_t)total;
      if (width == 3) send[2] = 0x80;
      atomicAdd((unsigned long long*)&t.ctr[ctr_index(CTR_SENT)], (unsigned long long)sent);
    }
    *qn_out = total - sent;
  }
  // the last block resets what every block has read
  __shared__ uint32_t last;
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(&t.ctr[ctr_index(CTR_STAGE_DONE)], 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  if (threadIdx.x < kShards) t.ctr[ctr_index(L.dctr + threadIdx.x)] = 0u;
  if (threadIdx.x == 0) {
    *qn_in = 0ull;
    atomicExch(&t.ctr[ctr_index(CTR_STAGE_DONE)], 0u);
  }
}

// Capacity report, queued behind a fold on its stream: adds the fold's edge count
// to the completed-edges counter, then reads the new-vertex count and writes both,
// packed into one 64-bit word (count << 33 | edges mod 2^33), to host-coherent
// memory. Every fold whose report preceded this one (by the atomic order of the
// adds) had completed before this read, so count + 2 x (edges launched - edges
// done) bounds the vertex count without a host synchronisation.
__global__ __launch_bounds__(64) void k_report(uint32_t* ctr, unsigned long long n, unsigned long long* out) {
  __shared__ unsigned long long done_sh;
  if (threadIdx.x == 0)
    done_sh = atomicAdd(reinterpret_cast<unsigned long long*>(ctr + ctr_index(CTR_EDONE)), n) + n;
  __syncthreads();
  uint32_t c = threadIdx.x < (uint32_t)kShards
                   ? __hip_atomic_load(ctr + ctr_index(CTR_NV + threadIdx.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : 0u;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
  if (threadIdx.x == 0) {
    const unsigned long long w = ((unsigned long long)c << 33) | (done_sh & ((1ull << 33) - 1));
    __hip_atomic_store(out, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

void launch_report(uint32_t* ctr, uint64_t n, unsigned long long* out, hipStream_t st) {
  hipLaunchKernelGGL(k_report, dim3(1), dim3(64), 0, st, ctr, (unsigned long long)n, out);
}

// Single-vertex lookup (gs_find): label and presence.
__global__ void k_find_one(Table t, int64_t key, int64_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  out[0] = 0;
  out[1] = 0;
  uint32_t l = 0;
  const uint32_t s = lookup_find(t, key, l);
  if (s == kNoSlot) return;
  uint32_t r, p;
  int64_t rk;
  find_root<false>(t, s, l, key, r, p, rk);
  out[0] = 1;
  out[1] = rk;
}

// ---------------------------------------------------------------- launchers
void launch_init(Slot* tab, uint64_t nslots, hipStream_t st) {
  const uint64_t blocks = (nslots + 255) / 256;
#ifndef GS_INIT_BLOCKS
#define GS_INIT_BLOCKS (1u << 22)  // one slot per thread: 2 GiB in 0.30 ms vs 0.48 ms with 8192 grid-strided blocks
#endif
  const unsigned g = (unsigned)(blocks < GS_INIT_BLOCKS ? blocks : GS_INIT_BLOCKS);
  hipLaunchKernelGGL(k_init, dim3(g), dim3(256), 0, st, tab, nslots);
}

void launch_fold(bool sign, bool track, int ept, const Table& t, const Lists& L, const int64_t* src,
                 const int64_t* dst, const uint8_t* w, uint32_t n, uint32_t stride, uint32_t w_stride, int cur,
                 int drain, int zero, int inline_max, uint32_t rows, int skip_rank, const int64_t* hdr,
                 uint32_t base, hipStream_t st) {
  FoldArgs a{src, dst, w, n, stride, w_stride, rows, skip_rank, hdr, base, cur, drain, zero, inline_max};
  const uint32_t per_block = kFoldBS * (uint32_t)ept;
  const dim3 g((n + per_block - 1) / per_block), b(kFoldBS);
  const bool hot = t.hotcap != 0;
  static const size_t lds = getenv("GS_FOLD_LDS") ? (size_t)atoi(getenv("GS_FOLD_LDS")) : 0;  // occupancy experiment
#define GS_FOLD(S, T, E, H)                                                       \
  if (sign == S && track == T && ept == E && hot == H) {                          \
    hipLaunchKernelGGL((k_fold<S, T, E, H>), g, b, lds, st, t, L, a);             \
    return;                                                                       \
  }
#define GS_FOLD_H(S, T, E) GS_FOLD(S, T, E, false) GS_FOLD(S, T, E, true)
  GS_FOLD_H(false, false, 1)
  GS_FOLD_H(false, true, 1)
  GS_FOLD_H(true, false, 1)
  GS_FOLD_H(true, true, 1)
  GS_FOLD_H(false, false, 2)
  GS_FOLD_H(false, true, 2)
  GS_FOLD_H(true, false, 2)
  GS_FOLD_H(true, true, 2)
#undef GS_FOLD_H
#undef GS_FOLD
}

void launch_hook(bool sign, bool track, const Table& t, const Lists& L, int set, int blocks, hipStream_t st) {
  const dim3 g(blocks), b(256);
  if (!sign && !track) hipLaunchKernelGGL((k_hook<false, false>), g, b, 0, st, t, L, set);
  if (!sign && track) hipLaunchKernelGGL((k_hook<false, true>), g, b, 0, st, t, L, set);
  if (sign && !track) hipLaunchKernelGGL((k_hook<true, false>), g, b, 0, st, t, L, set);
  if (sign && track) hipLaunchKernelGGL((k_hook<true, true>), g, b, 0, st, t, L, set);
}

void launch_export(bool sign, const Table& t, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap_out, hipStream_t st,
                   int part, int nparts) {
  const uint64_t all = (uint64_t)t.r0 + 2;
  const uint64_t s0 = all * (uint64_t)part / (uint64_t)nparts, s1 = all * (uint64_t)(part + 1) / (uint64_t)nparts;
  const uint64_t nslots = s1 - s0;
  const uint64_t tile = (uint64_t)kExportPer * kExportBS;
  const uint64_t tiles = (nslots + tile - 1) / tile;
  const uint64_t cap_blocks = 4096ull * 256 / kExportBS;
  const unsigned g = (unsigned)(tiles < cap_blocks ? tiles : cap_blocks);
  if (sign)
    hipLaunchKernelGGL((k_export<true>), dim3(g), dim3(kExportBS), 0, st, t, ov, ol, op, cap_out, s0, s1);
  else
    hipLaunchKernelGGL((k_export<false>), dim3(g), dim3(kExportBS), 0, st, t, ov, ol, op, cap_out, s0, s1);
}

void launch_stage(const Table& t, const Lists& L, const int64_t* q_in, unsigned long long* qn_in, int64_t* q_out,
                  unsigned long long* qn_out, uint64_t qcap, int64_t* send, uint64_t cap, hipStream_t st,
                  unsigned long long* count_out, int width) {
  hipLaunchKernelGGL(k_stage, dim3(kShards), dim3(256), 0, st, t, L, q_in, qn_in, q_out, qn_out, qcap, send, cap,
                     count_out, width);
}

// Exchange headers -> host-mapped memory: row 0 ({sent, queued}) of every rank's block
// of a gathered exchange buffer, one thread per rank, system-scope stores. Replaces a
// 2-D device-to-host copy whose host-side cost (~110 us per call) bounded the
// exchange loop. Then out[2] = seq (release): the host polls that word instead of
// synchronising on an event.
__global__ __launch_bounds__(64) void k_headers(const int64_t* __restrict__ recv, uint64_t rank_stride, int nranks,
                                                long long* out, long long seq) {
  for (int r = threadIdx.x; r < nranks; r += 64) {
    const int64_t* hd = recv + (size_t)r * rank_stride;
    __hip_atomic_store(out + r * 3, (long long)hd[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(out + r * 3 + 1, (long long)hd[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(out + 2, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

void launch_headers(const int64_t* recv, uint64_t rank_stride, int nranks, long long* out, long long seq,
                    hipStream_t st) {
  hipLaunchKernelGGL(k_headers, dim3(1), dim3(64), 0, st, recv, (unsigned long long)rank_stride, nranks, out, seq);
}

void launch_find_one(const Table& t, int64_t key, int64_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_find_one, dim3(1), dim3(64), 0, st, t, key, out);
}

}  // namespace gs
