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

__global__ __launch_bounds__(256) void k_init(Slot* tab, uint64_t nslots) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < nslots;
       s += (uint64_t)gridDim.x * blockDim.x) {
    uint4 v;
    v.x = 0u;
    v.y = 0x80000000u;  // INT64_MIN
    v.z = (uint32_t)(s << 1);
    v.w = 0u;
    *reinterpret_cast<uint4*>(tab + s) = v;
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
    if (part < nparts) drain_entries<SIGNED, TRACK>(t, L, set, blockIdx.x % kShards, part * 256u + threadIdx.x, nparts * 256u);
  } else {
    for (uint32_t s = blockIdx.x; s < (uint32_t)kShards; s += G)
      drain_entries<SIGNED, TRACK>(t, L, set, (int)s, threadIdx.x, 256u);
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
  const uint8_t* w;
  uint32_t n;
  uint32_t stride;
  int cur;
  int drain;
  int zero;
  int inline_max;
};

template <bool SIGNED, bool TRACK, int EPT>
__global__ __launch_bounds__(256) void k_fold(Table t, Lists L, FoldArgs a) {
  if (SIGNED && __builtin_amdgcn_readfirstlane(t.ctr[ctr_index(CTR_FAIL)]) != 0) return;
  const int shard = blockIdx.x & (kShards - 1);
  if (a.zero >= 0 && blockIdx.x == 0 && threadIdx.x < kShards)
    t.ctr[ctr_index(CTR_ACT + a.zero * kShards + threadIdx.x)] = 0u;

  bool valid[EPT], act[EPT];
  int64_t ks[EPT], kd[EPT];
  uint32_t need[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const uint32_t i = blockIdx.x * (256u * EPT) + e * 256u + threadIdx.x;
    valid[e] = i < a.n;
    act[e] = false;
    ks[e] = valid[e] ? a.src[(size_t)i * a.stride] : 0;
    kd[e] = valid[e] ? a.dst[(size_t)i * a.stride] : 0;
    need[e] = SIGNED ? ((valid[e] && a.w) ? (a.w[i] & 1u) : 1u) : 0u;
  }
  // all first relabel probes of the thread in flight together
  uint32_t hu[EPT], hv[EPT], l0u[EPT], l0v[EPT];
  int64_t k0u[EPT], k0v[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    hu[e] = hash_slot(ks[e], t.shift);
    hv[e] = hash_slot(kd[e], t.shift);
    if (valid[e]) {
      load_slot(t.tab + hu[e], k0u[e], l0u[e]);
      load_slot(t.tab + hv[e], k0v[e], l0v[e]);
    }
  }
  uint32_t ru[EPT], rv[EPT], lu[EPT], lv[EPT];
  int64_t kru[EPT], krv[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    if (!valid[e]) continue;
    bool nu, nv;
    const uint32_t su = lookup_resolve(t, ks[e], hu[e], k0u[e], l0u[e], lu[e], nu);
    const uint32_t sv = lookup_resolve(t, kd[e], hv[e], k0v[e], l0v[e], lv[e], nv);
    if (nu || nv) {
      const uint32_t cnt = (nu ? 1u : 0u) + (nv && sv != su ? 1u : 0u);
      atomicAdd(&t.ctr[ctr_index(CTR_NV + shard)], cnt);
      if (TRACK) {
        const uint32_t pos = atomicAdd(&t.ctr[ctr_index(CTR_DELTA + shard)], cnt);
        if (pos + cnt <= L.delta_shard_cap) {
          const size_t o = (size_t)shard * L.delta_shard_cap + pos;
          if (nu) {
            L.da[o] = ks[e];
            L.db[o] = ks[e];
            L.dw[o] = 0;
          }
          if (nv && sv != su) {
            const size_t o2 = o + (nu ? 1 : 0);
            L.da[o2] = kd[e];
            L.db[o2] = kd[e];
            L.dw[o2] = 0;
          }
        } else {
          atomicOr(&t.ctr[ctr_index(CTR_OVF)], 1u);
        }
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
// of a 4096-slot tile (slot = tile + j*256 + tid: coalesced 16-B loads); the block
// reserves its output range with ONE atomic per tile.
template <bool SIGNED>
__global__ __launch_bounds__(256) void k_export(Table t, int64_t* __restrict__ ov, int64_t* __restrict__ ol,
                                                uint8_t* __restrict__ op, uint64_t cap_out) {
  constexpr int PER = 16;
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t base_sh;
  const uint64_t nslots = (uint64_t)t.capidx + 1;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (uint64_t tile = (uint64_t)blockIdx.x * (256 * PER); tile < nslots; tile += (uint64_t)gridDim.x * (256 * PER)) {
    int64_t vk[PER], lk[PER];
    uint32_t pp[PER];
    uint32_t occ = 0, cnt = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint64_t s = tile + (uint64_t)j * 256 + threadIdx.x;
      vk[j] = 0;
      lk[j] = 0;
      pp[j] = 0;
      if (s < nslots) {
        int64_t k;
        uint32_t l;
        load_slot(t.tab + s, k, l);
        const bool present = (s == t.capidx) ? ((t.tab[s].aux & 1u) != 0) : (k != kEmpty);
        if (present) {
          uint32_t r, p;
          int64_t rk;
          find_root<false>(t, (uint32_t)s, l, k, r, p, rk);
          vk[j] = k;
          lk[j] = rk;
          pp[j] = p;
          occ |= 1u << j;
          ++cnt;
        }
      }
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
    for (int q = 0; q < 4; ++q) {
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

// Copy the sharded delta list into contiguous arrays. grid = kShards * sub.
__global__ __launch_bounds__(256) void k_pack(Table t, Lists L, int64_t* __restrict__ oa, int64_t* __restrict__ ob,
                                              uint8_t* __restrict__ ow, uint64_t cap_out, int sub) {
  const int shard = blockIdx.x & (kShards - 1);
  const int part = blockIdx.x / kShards;
  uint64_t base = 0;
  for (int s = 0; s < shard; ++s) base += min(t.ctr[ctr_index(CTR_DELTA + s)], L.delta_shard_cap);
  const uint32_t cnt = min(t.ctr[ctr_index(CTR_DELTA + shard)], L.delta_shard_cap);
  const size_t in0 = (size_t)shard * L.delta_shard_cap;
  for (uint32_t j = part * 256u + threadIdx.x; j < cnt; j += (uint32_t)sub * 256u) {
    const uint64_t o = base + j;
    if (o < cap_out) {
      oa[o] = L.da[in0 + j];
      ob[o] = L.db[in0 + j];
      ow[o] = L.dw[in0 + j];
    }
  }
}

// Single-vertex lookup (gs_find): label and presence.
__global__ void k_find_one(Table t, int64_t key, int64_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  out[0] = 0;
  out[1] = 0;
  uint32_t s = kNoSlot, l = 0;
  if (key == kEmpty) {
    if (t.tab[t.capidx].aux & 1u) s = t.capidx;
    l = t.capidx << 1;
  } else {
    uint32_t h = hash_slot(key, t.shift);
    for (uint32_t probes = 0; probes <= t.mask; ++probes) {
      int64_t k;
      load_slot(t.tab + h, k, l);
      if (k == key) {
        s = h;
        break;
      }
      if (k == kEmpty) break;
      h = (h + 1) & t.mask;
    }
  }
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
  const unsigned g = (unsigned)(blocks < 8192 ? blocks : 8192);
  hipLaunchKernelGGL(k_init, dim3(g), dim3(256), 0, st, tab, nslots);
}

void launch_fold(bool sign, bool track, int ept, const Table& t, const Lists& L, const int64_t* src,
                 const int64_t* dst, const uint8_t* w, uint32_t n, uint32_t stride, int cur, int drain, int zero,
                 int inline_max, hipStream_t st) {
  FoldArgs a{src, dst, w, n, stride, cur, drain, zero, inline_max};
  const uint32_t per_block = 256u * (uint32_t)ept;
  const dim3 g((n + per_block - 1) / per_block), b(256);
#define GS_FOLD(S, T, E)                                                          \
  if (sign == S && track == T && ept == E) {                                      \
    hipLaunchKernelGGL((k_fold<S, T, E>), g, b, 0, st, t, L, a);                  \
    return;                                                                       \
  }
  GS_FOLD(false, false, 1)
  GS_FOLD(false, true, 1)
  GS_FOLD(true, false, 1)
  GS_FOLD(true, true, 1)
  GS_FOLD(false, false, 2)
  GS_FOLD(false, true, 2)
  GS_FOLD(true, false, 2)
  GS_FOLD(true, true, 2)
#undef GS_FOLD
}

void launch_hook(bool sign, bool track, const Table& t, const Lists& L, int set, int blocks, hipStream_t st) {
  const dim3 g(blocks), b(256);
  if (!sign && !track) hipLaunchKernelGGL((k_hook<false, false>), g, b, 0, st, t, L, set);
  if (!sign && track) hipLaunchKernelGGL((k_hook<false, true>), g, b, 0, st, t, L, set);
  if (sign && !track) hipLaunchKernelGGL((k_hook<true, false>), g, b, 0, st, t, L, set);
  if (sign && track) hipLaunchKernelGGL((k_hook<true, true>), g, b, 0, st, t, L, set);
}

void launch_export(bool sign, const Table& t, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap_out, hipStream_t st) {
  const uint64_t nslots = (uint64_t)t.capidx + 1;
  const uint64_t tiles = (nslots + 4095) / 4096;
  const unsigned g = (unsigned)(tiles < 4096 ? tiles : 4096);
  if (sign)
    hipLaunchKernelGGL((k_export<true>), dim3(g), dim3(256), 0, st, t, ov, ol, op, cap_out);
  else
    hipLaunchKernelGGL((k_export<false>), dim3(g), dim3(256), 0, st, t, ov, ol, op, cap_out);
}

void launch_pack(const Table& t, const Lists& L, int64_t* oa, int64_t* ob, uint8_t* ow, uint64_t cap_out, int sub,
                 hipStream_t st) {
  hipLaunchKernelGGL(k_pack, dim3(kShards * sub), dim3(256), 0, st, t, L, oa, ob, ow, cap_out, sub);
}

void launch_find_one(const Table& t, int64_t key, int64_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_find_one, dim3(1), dim3(64), 0, st, t, key, out);
}

}  // namespace gs
