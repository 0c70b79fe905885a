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

template <bool SIGNED, bool FUSED, bool TRACK>
__global__ __launch_bounds__(256) void k_fold(Table t, Lists L, const int64_t* __restrict__ src,
                                              const int64_t* __restrict__ dst, const uint8_t* __restrict__ w,
                                              uint32_t n, uint32_t stride, int actset) {
  if (SIGNED && __builtin_amdgcn_readfirstlane(t.ctr[ctr_index(CTR_FAIL)]) != 0) return;
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  const int shard = blockIdx.x & (kShards - 1);
  if (i >= n) return;
  const int64_t ks = src[(size_t)i * stride];
  const int64_t kd = dst[(size_t)i * stride];
  uint32_t need = 0;
  if (SIGNED) need = w ? (w[i] & 1u) : 1u;

  // both first relabel probes in flight together
  const uint32_t hu = hash_slot(ks, t.shift), hv = hash_slot(kd, t.shift);
  int64_t k0u, k0v;
  uint32_t l0u, l0v;
  load_slot(t.tab + hu, k0u, l0u);
  load_slot(t.tab + hv, k0v, l0v);
  uint32_t lu, lv;
  bool nu, nv;
  const uint32_t su = lookup_resolve(t, ks, hu, k0u, l0u, lu, nu);
  const uint32_t sv = lookup_resolve(t, kd, hv, k0v, l0v, lv, nv);
  if (nu || nv) {
    const uint32_t cnt = (nu ? 1u : 0u) + (nv && sv != su ? 1u : 0u);
    atomicAdd(&t.ctr[ctr_index(CTR_NV + shard)], cnt);
    if (TRACK) {
      uint32_t pos = atomicAdd(&t.ctr[ctr_index(CTR_DELTA + shard)], cnt);
      if (pos + cnt <= L.delta_shard_cap) {
        const size_t o = (size_t)shard * L.delta_shard_cap + pos;
        if (nu) {
          L.da[o] = ks;
          L.db[o] = ks;
          L.dw[o] = 0;
        }
        if (nv && sv != su) {
          const size_t o2 = o + (nu ? 1 : 0);
          L.da[o2] = kd;
          L.db[o2] = kd;
          L.dw[o2] = 0;
        }
      } else {
        atomicOr(&t.ctr[ctr_index(CTR_OVF)], 1u);
      }
    }
  }
  if (su == kNoSlot || sv == kNoSlot || su == sv) return;  // self-loop: vertex added, never a conflict

  // shortcut: a shared parent (the common case once trees are flat) or a direct
  // parent/child pair decides the edge without touching a root
  const uint32_t pu = lu >> 1, pv = lv >> 1;
  if (pu == pv || pu == sv || pv == su) {
    if (SIGNED) {
      const uint32_t par = (pu == pv) ? ((lu ^ lv) & 1u) : (pu == sv ? (lu & 1u) : (lv & 1u));
      if ((need ^ par) & 1u) atomicOr(&t.ctr[ctr_index(CTR_FAIL)], 1u);
    }
    return;
  }

  uint32_t ru = su, rv = sv, pru = 0, prv = 0;
  int64_t kru = ks, krv = kd;
  find_root2<false>(t, ru, lu, kru, pru, rv, lv, krv, prv);
  need ^= pru ^ prv;
  if (ru == rv) {
    if (SIGNED && (need & 1u)) atomicOr(&t.ctr[ctr_index(CTR_FAIL)], 1u);
    return;
  }
  if (FUSED) {
    hook<SIGNED, TRACK>(t, L, shard, ru, ru << 1, kru, rv, rv << 1, krv, need);
  } else {
    const uint32_t pos = atomicAdd(&t.ctr[ctr_index((actset ? CTR_ACT1 : CTR_ACT0) + shard)], 1u);
    if (pos < L.act_shard_cap) {
      L.act[((size_t)actset * kShards + shard) * L.act_shard_cap + pos] =
          make_uint2((ru << 1) | (SIGNED ? (need & 1u) : 0u), rv);
    } else {
      atomicOr(&t.ctr[ctr_index(CTR_OVF)], 1u);
    }
  }
}

// grid = kShards * sub blocks; block b drains shard b % kShards of active set `actset`
// and zeroes the other set's counters (it is free: its k_hook has finished and the
// next k_fold that uses it has not started -- same-stream order).
template <bool SIGNED, bool TRACK>
__global__ __launch_bounds__(256) void k_hook(Table t, Lists L, int actset, int sub) {
  const int shard = blockIdx.x & (kShards - 1);
  const int part = blockIdx.x / kShards;
  if (blockIdx.x == 0 && threadIdx.x < kShards)
    t.ctr[ctr_index((actset ? CTR_ACT0 : CTR_ACT1) + threadIdx.x)] = 0u;
  if (SIGNED && __builtin_amdgcn_readfirstlane(t.ctr[ctr_index(CTR_FAIL)]) != 0) return;
  const uint32_t cnt = min(t.ctr[ctr_index((actset ? CTR_ACT1 : CTR_ACT0) + shard)], L.act_shard_cap);
  const uint2* act = L.act + ((size_t)actset * kShards + shard) * L.act_shard_cap;
  for (uint32_t j = part * 256u + threadIdx.x; j < cnt; j += (uint32_t)sub * 256u) {
    const uint2 e = act[j];
    const uint32_t a = e.x >> 1, b = e.y;
    int64_t ka, kb;
    uint32_t la, lb;
    load_slot(t.tab + a, ka, la);
    load_slot(t.tab + b, kb, lb);
    la = load_link_fresh(t.tab + a);
    lb = load_link_fresh(t.tab + b);
    hook<SIGNED, TRACK>(t, L, shard, a, la, settle_key(t, a, ka), b, lb, settle_key(t, b, kb), e.x & 1u);
  }
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

void launch_fold(bool sign, bool fused, bool track, const Table& t, const Lists& L, const int64_t* src,
                 const int64_t* dst, const uint8_t* w, uint32_t n, uint32_t stride, int actset, hipStream_t st) {
  const dim3 g((n + 255) / 256), b(256);
#define GS_FOLD(S, F, T)                                                                         \
  if (sign == S && fused == F && track == T) {                                                   \
    hipLaunchKernelGGL((k_fold<S, F, T>), g, b, 0, st, t, L, src, dst, w, n, stride, actset);    \
    return;                                                                                      \
  }
  GS_FOLD(false, false, false)
  GS_FOLD(false, false, true)
  GS_FOLD(false, true, false)
  GS_FOLD(false, true, true)
  GS_FOLD(true, false, false)
  GS_FOLD(true, false, true)
  GS_FOLD(true, true, false)
  GS_FOLD(true, true, true)
#undef GS_FOLD
}

void launch_hook(bool sign, bool track, const Table& t, const Lists& L, int actset, int sub, hipStream_t st) {
  const dim3 g(kShards * sub), b(256);
  if (!sign && !track) hipLaunchKernelGGL((k_hook<false, false>), g, b, 0, st, t, L, actset, sub);
  if (!sign && track) hipLaunchKernelGGL((k_hook<false, true>), g, b, 0, st, t, L, actset, sub);
  if (sign && !track) hipLaunchKernelGGL((k_hook<true, false>), g, b, 0, st, t, L, actset, sub);
  if (sign && track) hipLaunchKernelGGL((k_hook<true, true>), g, b, 0, st, t, L, actset, sub);
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
