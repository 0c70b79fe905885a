// gs_kernels.hip -- HIP kernels of the summary fold (gfx950, wave64).
//
//   k_init        : table reset (slot s := {EMPTY, s<<1, 0})                 -- HBM write-bound
//   k_reset_list  : the same for the listed (touched) slots only            -- O(vertices)
//   k_fold        : per edge: 2 relabel probes + 2 finds, shortcut on equal roots,
//                   wave-combined lock-free CAS hook in place               -- HBM request-bound
//   k_export      : (vertex, min-id label, parity) of every occupied slot (table scan)
//   k_export_list : the same over the vertex list (sparse tables)
//   k_stage       : sharded delta lists -> contiguous records + count word
//   k_report      : asynchronous vertex-count bound for the host (capacity tracking)
//   k_headers     : gathered exchange counts -> host-mapped memory
//   k_find_one / k_find_batch : canonical labels of given ids
// Reference: DisjointSet.union (DisjointSet.java:92-118) / Candidates.merge
// (Candidates.java:77-139) folded once per edge by PartialAgg.fold
// (SummaryBulkAggregation.java:121-123).
#include "gs_device.hpp"
#include "gs_kernels.hpp"

namespace gs {

// slot s := {EMPTY, s << 1, 0} (the reserved slot's key field IS its id, INT64_MIN).
// ctr (optional): block 0 also zeroes the counters -- the first 16 B of every counter line
// (nothing reads them during a reset: no fill launch of its own).
__global__ __launch_bounds__(256) void k_init(Slot* tab, uint64_t nslots, uint32_t* ctr) {
  if (ctr && blockIdx.x == 0)
    for (uint32_t i = threadIdx.x; i < (uint32_t)CTR_COUNT; i += blockDim.x)
      *reinterpret_cast<uint4*>(ctr + ctr_index((int)i)) = make_uint4(0, 0, 0, 0);
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

// Per-shard fill of the vertex list, clamped, and its exclusive prefix (LDS).
__device__ __forceinline__ uint64_t vlist_prefix(const Table& t, uint32_t* cnt, uint64_t* pre) {
  if (threadIdx.x < (uint32_t)kShards) cnt[threadIdx.x] = min(t.ctr[ctr_index(CTR_NV + threadIdx.x)], t.vshard_cap);
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

// Dense id of vertex-list entry g (g < total): binary search of the shard prefix.
__device__ __forceinline__ uint32_t vlist_at(const Table& t, const uint64_t* pre, uint64_t g) {
  int lo = 0, hi = kShards - 1;
  while (lo < hi) {  // last shard q with pre[q] <= g
    const int mid = (lo + hi + 1) >> 1;
    if (pre[mid] <= g) lo = mid;
    else hi = mid - 1;
  }
  return t.vlist[(size_t)lo * t.vshard_cap + (g - pre[lo])];
}

// Reset only the listed slots (and the reserved one): a slot is only ever written
// after its insertion (key CAS, links of occupied slots), so this restores the
// initial table exactly. nxt (change tracking member lists) is reset alongside.
// If the list overflowed (CTR_VOVF) the kernel resets every slot instead.
__device__ __forceinline__ void reset_slot(const Table& t, uint32_t* nxt, uint32_t s) {
  uint4 v;
  v.x = 0u;
  v.y = 0x80000000u;
  v.z = s << 1;
  v.w = 0u;
  *reinterpret_cast<uint4*>(t.tab + s) = v;
  if (nxt) nxt[s] = s;
}

// The block that finishes last (a ticket) zeroes the whole counter block: every other
// block has read the list counts and CTR_VOVF by then, and the reset needs no fill launch
// of its own after it (config 2: a 5 us fill + its gap per step).
__global__ __launch_bounds__(256) void k_reset_list(Table t, uint32_t* nxt) {
  __shared__ uint32_t cnt[kShards];
  __shared__ uint64_t pre[kShards + 1];
  __shared__ uint32_t last;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t.ctr[ctr_index(CTR_VOVF)]) {  // rare (block-uniform): the list is incomplete
    for (uint64_t s = g0; s <= t.r0; s += stride) reset_slot(t, nxt, (uint32_t)s);
  } else {
    const uint64_t total = vlist_prefix(t, cnt, pre);
    for (uint64_t g = g0; g < total; g += stride) reset_slot(t, nxt, vlist_at(t, pre, g));
    if (g0 == 0) reset_slot(t, nxt, t.r0);
  }
  __syncthreads();  // the block's reads of the counters have returned (their values are in LDS)
  // (no fence: the slot stores need no order against the zeroing, only the counter reads
  // do, and every block's reads precede its ticket; the next kernel sees both). Two-level
  // ticket: same-address atomics serialise at the memory side (11.4 ns each), and one counter
  // for config 2's 2.5 K blocks cost the reset ~29 us. The window take's ticket counters serve
  // (zero at rest: a take leaves them zeroed, no take runs beside a reset, and this kernel's
  // last block zeroes them again).
  if (threadIdx.x == 0) {
    constexpr uint32_t kTS = 16;
    bool l = true;
    if (gridDim.x > kTS) {
      const uint32_t shard = blockIdx.x % kTS;
      const uint32_t in_shard = (gridDim.x - shard + kTS - 1) / kTS;
      l = atomicAdd(&t.ctr[ctr_index(CTR_TAKE_SHARD + (int)shard)], 1u) == in_shard - 1;
      if (l) l = atomicAdd(&t.ctr[ctr_index(CTR_TAKE_DONE)], 1u) == kTS - 1;
    } else {
      l = atomicAdd(&t.ctr[ctr_index(CTR_TAKE_DONE)], 1u) == gridDim.x - 1;
    }
    last = l;
  }
  __syncthreads();
  if (!last) return;
  // (a counter is word 0, or words 0-1, of its 128-B line: the first 16 B of every line; a
  // memset of all 48 KB from one block made the reset 25 -> 36 us)
  for (uint32_t i = threadIdx.x; i < (uint32_t)CTR_COUNT; i += blockDim.x)
    *reinterpret_cast<uint4*>(t.ctr + ctr_index((int)i)) = make_uint4(0, 0, 0, 0);
}

// k_fold: one edge per thread (edge i = block*256 + tid: coalesced 8-B loads of src
// and dst). Both relabel probes issued back to back, shortcut when the two slots
// share a parent (the common case once trees are flat), lockstep finds of the two
// roots, then the wave's hooks are combined per target root and CASed in place.
struct FoldArgs {
  const int64_t* src;
  const int64_t* dst;
  const uint8_t* w;   // per edge: bit 0 = required parity (SIGNED), bit 7 = skip (padding record)
  uint32_t n;
  uint32_t stride;    // elements between consecutive src (and dst) entries
  uint32_t w_stride;  // bytes between consecutive w entries
  uint32_t rows;      // > 0: exchange layout, world blocks of `rows` records
  int skip_rank;      // block whose rows are skipped (the caller's own)
  const unsigned long long* counts;  // exchange layout: live rows of block r (| kFailBit)
  uint32_t base;      // index of this launch's first element (chunked launches)
  const unsigned long long* n_dev;   // optional: device count word (valid: base + i < low 62 bits;
                                     // bit 62 = kFailBit, a failed verdict the SIGNED fold ANDs in)
  const uint32_t* fail_in;           // optional: failure flag of a combined summary (SIGNED)
  uint32_t shard0;    // first shard of this launch (rotates per launch: balanced shard fill)
  // fused window take (TAKE): rows -> take_out[take_cap][3], count -> *take_count; the
  // last block writes {seq, vertices, rows} to the host-mapped completion word `done`
  int64_t* take_out;
  unsigned long long take_cap;
  unsigned long long* take_count;
  unsigned long long* done;
  unsigned long long seq;
  bool server = false;  // resident window server: vertices carried by the tickets (take_tail)
  // capacity report carried by this launch for the chunks queued before it on its stream
  // (k_report's work in block 0's first wave: no launch of its own)
  unsigned long long* rep_out = nullptr;
  unsigned long long rep_claim = 0;
  unsigned rep_epoch = 0;
};

// The capacity report (k_report below) by one wave: edges covered += n, then the
// new-vertex count of the 64 shards and the covered edges into one host-mapped word.
__device__ __forceinline__ void report_wave(uint32_t* ctr, unsigned long long n, unsigned long long* out,
                                            unsigned epoch) {
  unsigned long long done = 0;
  if (threadIdx.x == 0)
    done = atomicAdd(reinterpret_cast<unsigned long long*>(ctr + ctr_index(CTR_EDONE)), n) + n;
  done = __shfl(done, 0, 64);
  uint32_t c = threadIdx.x < (uint32_t)kShards
                   ? __hip_atomic_load(ctr + ctr_index(CTR_NV + threadIdx.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : 0u;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
  if (threadIdx.x == 0) {
    const unsigned long long w = ((unsigned long long)c << 34) | ((unsigned long long)(epoch & 7u) << 31) |
                                 (done & ((1ull << 31) - 1));
    __hip_atomic_store(out, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

#ifndef GS_ROWS_TTAS
#define GS_ROWS_TTAS 3  // other replicas' rows: re-read before the key CAS on both sides (experiment switch)
#endif
#ifndef GS_COMBINE_ROUNDS
#define GS_COMBINE_ROUNDS 2
#endif
constexpr int kCombineRounds = GS_COMBINE_ROUNDS;  // wave-level hook combining (combine_hooks)

#ifdef GS_BLOCKLOG
// Diagnostic build (make -C gelly-streaming_amd blocklog): every CC
// k_fold workgroup appends one record -- which XCD and CU ran it, its arguments, and
// what its edges found -- so a lost-work run can tell "never dispatched" from "ran
// with wrong arguments" from "ran, saw keys that should not be there".
struct BlockLog {
  unsigned long long t0, t1;   // wall clock at block start / end
  unsigned long long src, tab; // launch arguments as the block saw them
  uint32_t blk, nblk, n, xcc;  // blockIdx.x, gridDim.x, a.n, HW_REG_XCC_ID
  uint32_t hwid, valid, fresh, hooks;  // HW_REG_HW_ID; edges valid, inserted vertices, hook attempts
};
__device__ BlockLog* g_blog = nullptr;
__device__ unsigned long long g_blog_cap = 0;
__device__ unsigned long long g_blog_n = 0;
#endif

#ifdef GS_SERVER_TRACE
// Diagnostic build (make -C gelly-streaming_amd variant V=strace VFLAGS=-DGS_SERVER_TRACE;
// tools/server_trace.py): per window of the resident server, wall-clock stamps (100 MHz)
// of its phases, in record (seq mod cap):
//   [0] block 0 sees the window in the mailbox   [1] block 0 has broadcast it
//   [2] last block to start folding (max)        [3] last block done folding (max)
//   [4] publishing block enters take_tail        [5] completion word stored
//   [6] blocks that took part
// followed by 128 counters: histograms of every block's fold time in 0.5-us buckets (64..127: the
// session's first 64 windows).
__device__ unsigned long long* g_strace = nullptr;
__device__ unsigned long long g_strace_cap = 0;
#endif

// Tail of a fused window take (config 5's per-window fold + delta export + completion
// in ONE launch instead of fold, stage and completion kernels, each a kernel boundary of
// ~3 us). Each block reserves its rows in the output with one atomic and writes them
// from LDS with write-through (agent-scope) stores, so that they are in memory -- not
// in this XCD's L2 -- once the block's stores are acknowledged; the block then takes a
// ticket. The last block publishes the count, resets the take counters and stores the
// completion word (system scope) that the host spins on. The table writes need no
// fence: the next kernel of the stream starts after this one's end-of-kernel release,
// and only the rows and the count are read before that (by the host or other streams).
// A signed summary's count word carries the verdict (| kFailBit once it failed): the
// take's consumer replays the records AND the verdict (Candidates.merge :79-81).
// Returns true in the one thread that published the window (the last block's thread 0).
// Window-server CC windows carry their totals through the tickets: each block adds
// {1, its rows, its new vertices} packed in one 64-bit word (16 + 24 + 24 bits), so the
// last block knows the window's rows and inserts from the returned values, and the vertex
// count is the previous window's (CTR_SRV_NV, loaded at the start of the tail) plus this
// window's inserts: no round of counter loads after the ticket (config 5's latency).
#ifndef GS_TAKE_CARRY
#define GS_TAKE_CARRY 1  // 0: the publisher loads the counters after the ticket (experiment switch)
#endif
__device__ __forceinline__ unsigned long long tk_pack(unsigned long long n, unsigned long long rows,
                                                      unsigned long long newv) {
  return n | (rows << 16) | (newv << 40);
}
__device__ __forceinline__ unsigned long long tk_n(unsigned long long w) { return w & 0xFFFFull; }
__device__ __forceinline__ unsigned long long tk_rows(unsigned long long w) { return (w >> 16) & 0xFFFFFFull; }
__device__ __forceinline__ unsigned long long tk_newv(unsigned long long w) { return w >> 40; }

__device__ __forceinline__ bool take_tail(const Table& t, const FoldArgs& a, const int64_t* lrec, uint32_t lcnt,
                                          bool signed_kind, uint32_t blk, uint32_t nblocks, uint32_t newv = 0) {
  __shared__ unsigned long long base_sh;
  __shared__ uint32_t last_sh;
  const uint32_t nb = min(lcnt, kFoldBS);
  // a one-block window owns the whole output: no reservation and no ticket (two
  // dependent atomics of a small window's latency)
  const bool solo = nblocks == 1;
  unsigned long long* srv_nv = reinterpret_cast<unsigned long long*>(t.ctr + ctr_index(CTR_SRV_NV));
  // the ticket-carried form: window-server CC windows (the packed fields hold 2^16 blocks,
  // 2^24 rows and 2^24 new vertices: 4096 blocks of 256 edges stay far inside)
  const bool carried = GS_TAKE_CARRY && a.server && !signed_kind && nblocks <= 4096;
  // the vertex count before this window (server: exact, kept by every window's publisher
  // and set at the session's start; stable while the window runs)
  unsigned long long nv0 = 0;
  if (a.server && threadIdx.x == 0) nv0 = __hip_atomic_load(srv_nv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // a one-block window's vertex count is final once its own fold is (its inserts were
  // counted by returning atomics): the count loads go out now, beside the row stores.
  // (Not the verdict: the fold raises it with no-return atomics, ordered only by the
  // drain below.)
  unsigned long long nv = 0;
  if (solo && !carried && threadIdx.x < 64)
    nv = __hip_atomic_load(t.ctr + ctr_index(CTR_NV + threadIdx.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (solo && !signed_kind) {
    // A one-block CC window: the rows, the count word and the staged-rows tally go out
    // together and ONE drain covers them all (the multi-block path needs its rows in
    // memory before the ticket, and a signed window's verdict is read after the drain):
    // one dependent round trip less on the latency floor (the 64-edge window).
    for (uint32_t j = threadIdx.x; j < nb; j += kFoldBS) {
      if (j < a.take_cap) {
        int64_t* r = a.take_out + (size_t)j * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c)
          __hip_atomic_store(r + c, lrec[j * 3 + c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (threadIdx.x == 0) {
      __hip_atomic_store(a.take_count, (unsigned long long)lcnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicAdd(reinterpret_cast<unsigned long long*>(t.ctr + ctr_index(CTR_SENT)),
                (unsigned long long)(lcnt < a.take_cap ? lcnt : a.take_cap));
      if (carried) {
        nv = nv0 + newv;
        __hip_atomic_store(srv_nv, nv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x >= 64) return false;
    if (!carried) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) nv += __shfl_xor(nv, o, 64);
    }
    if (threadIdx.x != 0) return false;
    __hip_atomic_store(a.done + 1, done_value(a.seq, nv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(a.done + 2, done_value(a.seq, (unsigned long long)lcnt), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(a.done, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return true;
  }
  if (threadIdx.x == 0)
    base_sh = (nb && !solo) ? atomicAdd(reinterpret_cast<unsigned long long*>(t.ctr + ctr_index(CTR_TAKE)),
                                        (unsigned long long)nb)
                            : 0ull;
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < nb; j += kFoldBS) {
    const unsigned long long pos = base_sh + j;
    if (pos < a.take_cap) {
      int64_t* r = a.take_out + pos * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c)
        __hip_atomic_store(r + c, lrec[j * 3 + c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // every wave waits for its stores' acknowledgements before the barrier (the barrier
  // alone does not wait for global stores); no L2 writeback needed for write-through rows
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  // Two-level ticket: same-address atomics serialise at the memory side (11.4 ns each,
  // profiles/r01_calib_atomic.log), so 256 blocks on one counter cost ~2.9 us of the
  // window. Block b counts on shard b mod 16; the shard's last block counts on the top
  // word; the last of those is the window's last block. (Each count is a memory-side
  // atomic made after the counting block's rows were acknowledged: the chain of
  // returned values orders every block's rows before the last block's reads.)
  // (Up to 16 blocks count on the top word directly; one block needs no ticket.)
  constexpr uint32_t kTS = 16;
  if (carried) {
    if (threadIdx.x != 0) return false;
    unsigned long long* top = reinterpret_cast<unsigned long long*>(t.ctr + ctr_index(CTR_TAKE_DONE));
    unsigned long long mine = tk_pack(1, nb, newv);
    uint32_t expect = nblocks;
    if (nblocks > kTS) {
      const uint32_t shard = blk % kTS;
      const uint32_t in_shard = (nblocks - shard + kTS - 1) / kTS;
      unsigned long long* sw = reinterpret_cast<unsigned long long*>(t.ctr + ctr_index(CTR_TAKE_SHARD + shard));
      const unsigned long long o = atomicAdd(sw, mine);
      if (tk_n(o) != in_shard - 1) return false;
      mine = tk_pack(1, tk_rows(o) + nb, tk_newv(o) + newv);  // the shard's totals go up
      expect = kTS;
    }
    const unsigned long long o2 = atomicAdd(top, mine);
    if (tk_n(o2) != expect - 1) return false;
    const unsigned long long total = tk_rows(o2) + tk_rows(mine);
    const unsigned long long nvw = nv0 + tk_newv(o2) + tk_newv(mine);
    __hip_atomic_store(a.take_count, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    atomicAdd(reinterpret_cast<unsigned long long*>(t.ctr + ctr_index(CTR_SENT)),
              total < a.take_cap ? total : a.take_cap);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(t.ctr + ctr_index(CTR_TAKE)), 0ull, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(top, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (nblocks > kTS) {
#pragma unroll
      for (int k = 0; k < (int)kTS; ++k)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(t.ctr + ctr_index(CTR_TAKE_SHARD + k)), 0ull,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __hip_atomic_store(srv_nv, nvw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (as below)
    __hip_atomic_store(a.done + 1, done_value(a.seq, nvw), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(a.done + 2, done_value(a.seq, total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(a.done, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return true;
  }
  if (threadIdx.x == 0) {
    bool last = true;
    if (nblocks > kTS) {
      const uint32_t shard = blk % kTS;
      const uint32_t in_shard = (nblocks - shard + kTS - 1) / kTS;  // blocks b < nblocks with b mod 16 == shard
      last = atomicAdd(t.ctr + ctr_index(CTR_TAKE_SHARD + shard), 1u) == in_shard - 1;
      if (last) last = atomicAdd(t.ctr + ctr_index(CTR_TAKE_DONE), 1u) == kTS - 1;
    } else if (nblocks > 1) {
      last = atomicAdd(t.ctr + ctr_index(CTR_TAKE_DONE), 1u) == nblocks - 1;
    }
    last_sh = last;
  }
  __syncthreads();
  if (!last_sh || threadIdx.x >= 64) return false;
  // one round of loads, issued together (each is a dependent memory hop of the window's
  // latency): the 64 shard counts, the take total (lane 0) and, signed, the verdict
  // (lane 1; every block's verdict updates are memory-side atomics that preceded its
  // ticket, so the flag is read at the memory side too, never from a stale line)
  unsigned long long* take = reinterpret_cast<unsigned long long*>(t.ctr + ctr_index(CTR_TAKE));
  unsigned long long tot = lcnt;
  if (!solo) {
    nv = __hip_atomic_load(t.ctr + ctr_index(CTR_NV + threadIdx.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tot = threadIdx.x == 0 ? __hip_atomic_load(take, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
  }
  const uint32_t fl = (signed_kind && threadIdx.x == 1) ? atomicOr(&t.ctr[ctr_index(CTR_FAIL)], 0u) : 0u;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) nv += __shfl_xor(nv, o, 64);
  const bool failed = __shfl(fl, 1, 64) != 0u;
  if (threadIdx.x != 0) return false;
  const unsigned long long total = tot;
  const unsigned long long word = total | (failed ? kFailBit : 0ull);
  __hip_atomic_store(a.take_count, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // write-through
  atomicAdd(reinterpret_cast<unsigned long long*>(t.ctr + ctr_index(CTR_SENT)), total < a.take_cap ? total : a.take_cap);
  if (a.server) __hip_atomic_store(srv_nv, nv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // signed server windows
  if (!solo) {
    __hip_atomic_store(take, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(t.ctr + ctr_index(CTR_TAKE_DONE), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (nblocks > 16) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      __hip_atomic_store(t.ctr + ctr_index(CTR_TAKE_SHARD + k), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // Every store above is write-through (agent scope): draining them puts the count word
  // and the counter resets in memory before the host can see the window complete,
  // without an L2 write-back (a release fence costs ~1.7 us even on a clean L2,
  // MI355X_MICROARCH.md). The completion record then goes out undrained: its values
  // carry the sequence number as a tag, and the host takes them when the tags match
  // (gsi::done_value_read), whichever of the three host-memory stores lands first.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(a.done + 1, done_value(a.seq, nv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(a.done + 2, done_value(a.seq, word), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(a.done, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return true;
}

template <bool SIGNED, bool TRACK, bool TAKE, bool ROWS = false>
__device__ __forceinline__ void fold_block(const Table& t, const Delta& D, const FoldArgs& a, uint32_t blk,
                                           bool failed, unsigned long long n_word, uint32_t* dbg);

// ROWS: a group's gathered remote rows (exchange layout); they keep the insert re-read
// (profiles/r04_rank_replay.txt section 8: 47 M rows fold in 2.86 ms with it, 3.94 without)
template <bool SIGNED, bool TRACK, bool TAKE, bool ROWS = false>
__global__ __launch_bounds__(kFoldBS) void k_fold(Table t, Delta D, FoldArgs a) {
  __shared__ int64_t lrec[TAKE ? kFoldBS * 3 : 1];
  __shared__ uint32_t lcnt;
#ifdef GS_BLOCKLOG
  __shared__ uint32_t dbg[3];
  const unsigned long long dbg_t0 = wall_clock64();
  if (!SIGNED) {
    if (threadIdx.x < 3) dbg[threadIdx.x] = 0;
    __syncthreads();
  }
#endif
  if (TAKE) {
    D.lrec = lrec;
    D.lcnt = &lcnt;
    if (threadIdx.x == 0) lcnt = 0;
    __syncthreads();
  }
  // Counts and flags written on another stream (a copy, a collective, another summary's
  // export) are read with agent-scope loads: never from a line an XCD's L2 may hold.
  unsigned long long n_word = 0;
  if (a.n_dev) n_word = __hip_atomic_load(a.n_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (SIGNED && blockIdx.x == 0 && threadIdx.x == 0 &&
      ((a.fail_in && __hip_atomic_load(a.fail_in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ||
       (n_word & kFailBit)))
    atomicOr(&t.ctr[ctr_index(CTR_FAIL)], 1u);  // the verdict is the AND (Candidates.java:79-81)
  // the report of the earlier chunks of this stream (complete: stream order)
  if (a.rep_out && blockIdx.x == 0 && threadIdx.x < 64) report_wave(t.ctr, a.rep_claim, a.rep_out, a.rep_epoch);
  // a failed verdict is final: no more work (a TAKE block still reaches its ticket)
  const bool failed = SIGNED && __builtin_amdgcn_readfirstlane(t.ctr[ctr_index(CTR_FAIL)]) != 0;
  if (failed && !TAKE) return;
#ifdef GS_BLOCKLOG
  fold_block<SIGNED, TRACK, TAKE, ROWS>(t, D, a, blockIdx.x, failed, n_word, SIGNED ? nullptr : dbg);
#else
  fold_block<SIGNED, TRACK, TAKE, ROWS>(t, D, a, blockIdx.x, failed, n_word, nullptr);
#endif
#ifdef GS_BLOCKLOG
  if (!SIGNED) {
    __syncthreads();
    if (threadIdx.x == 0 && g_blog) {
      const unsigned long long k = atomicAdd(&g_blog_n, 1ull);
      if (k < g_blog_cap) {
        BlockLog r;
        r.t0 = dbg_t0;
        r.t1 = wall_clock64();
        r.src = (unsigned long long)a.src;
        r.tab = (unsigned long long)t.tab;
        r.blk = blockIdx.x;
        r.nblk = gridDim.x;
        r.n = a.n;
        r.xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID[3:0]
        r.hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID (CU, SE, ...)
        r.valid = dbg[0];
        r.fresh = dbg[1];
        r.hooks = dbg[2];
        g_blog[k] = r;
      }
    }
  }
#endif
  if (TAKE) {
    __syncthreads();
    take_tail(t, a, lrec, lcnt, SIGNED, blockIdx.x, gridDim.x);
  }
}

// The fold of one block's edges (edge i = blk * kFoldBS + threadIdx.x): relabel probes,
// shortcut, finds, wave-combined hooks. Shared by k_fold and the resident window server.
template <bool SIGNED, bool TRACK, bool TAKE, bool ROWS>
__device__ __forceinline__ void fold_block(const Table& t, const Delta& D, const FoldArgs& a, uint32_t blk,
                                           bool failed, unsigned long long n_word, uint32_t* dbg) {
  const int shard = (int)((blk + a.shard0) & (kShards - 1));
  const uint32_t i = blk * kFoldBS + threadIdx.x;
  bool valid = i < a.n && !failed;
  if (valid && a.n_dev) valid = (unsigned long long)(a.base + i) < (n_word & (kFailBit - 1));
  if (valid && a.rows) {  // exchange layout: the block's count word gives its live rows
    const uint32_t ig = a.base + i, r = ig / a.rows, j = ig - r * a.rows;
    const unsigned long long cw = __hip_atomic_load(a.counts + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (SIGNED && j == 0 && (cw & kFailBit) && (int)r != a.skip_rank) atomicOr(&t.ctr[ctr_index(CTR_FAIL)], 1u);
    valid = (int)r != a.skip_rank && (unsigned long long)j < (cw & (kFailBit - 1));
  }
  const uint32_t wi = (valid && a.w) ? a.w[(size_t)i * a.w_stride] : 1u;
  if (wi & 0x80u) valid = false;
  // the edge stream is read once: non-temporal loads leave the L2 to table lines
  // (RMAT-26: 40.37 -> 40.10 ms/step, 1.945 -> 1.941 fabric requests per edge)
  const int64_t ks = valid ? __builtin_nontemporal_load(a.src + (size_t)i * a.stride) : 0;
  const int64_t kd = valid ? __builtin_nontemporal_load(a.dst + (size_t)i * a.stride) : 0;
  uint32_t need = SIGNED ? (wi & 1u) : 0u;
  // both first relabel probes in flight together
  const uint32_t hu = hash_slot(ks, t.shift), hv = hash_slot(kd, t.shift);
  int64_t k0u = 0, k0v = 0;
  uint32_t l0u = 0, l0v = 0;
  if (valid) {
    load_slot(t.tab + hu, k0u, l0u);
    load_slot(t.tab + hv, k0v, l0v);
  }
  uint32_t ru = 0, rv = 0, lu = 0, lv = 0;
  int64_t kru = 0, krv = 0;
  bool act = false;
  NewVertices nvx;
  uint32_t fresh0 = kNoSlot, fresh1 = kNoSlot;  // slots this thread inserted
  bool has_rec = false;  // TRACK: this edge's record (a self-loop's new vertex, or its hook)
  int64_t rec[3] = {0, 0, 0};
  bool nu = false, nv = false;
  uint32_t su = kNoSlot, sv = kNoSlot;
  if (valid) {
    GS_DBG(CTR_DBG_EDGES);
    // (the re-read stays in the exchange's tracked own folds: one-rank RCCL step 42.6-43.2
    // with it vs 43.7-43.8 ms without, profiles/r04_insert_path_ab.txt section 7; rows: the
    // sides GS_ROWS_TTAS names, bit 0 the hooked root's, bit 1 its new parent's)
    constexpr bool kTu = !TAKE && (GS_INSERT_TTAS || TRACK || (ROWS && (GS_ROWS_TTAS & 1)));
    constexpr bool kTv = !TAKE && (GS_INSERT_TTAS || TRACK || (ROWS && (GS_ROWS_TTAS & 2)));
    if (GS_PAIR_INSERT && k0u == kEmpty && k0v == kEmpty && hu != hv && ks != kd && ks != kEmpty && kd != kEmpty) {
      insert_pair<kTu, kTv>(t, ks, hu, kd, hv, su, lu, nu, sv, lv, nv);
    } else {
      su = lookup_resolve<kTu>(t, ks, hu, k0u, l0u, lu, nu);
      sv = lookup_resolve<kTv>(t, kd, hv, k0v, l0v, lv, nv);
    }
  }
  nvx = reserve_new_vertices(t, shard, nu, su, nv, sv, TAKE ? D.lnv : nullptr);  // one atomic per wave
  if (valid) {
    if (nu) fresh0 = su;
    if (nv) fresh1 = sv;
    if (dbg) atomicAdd(&dbg[1], (nu ? 1u : 0u) + ((nv && sv != su) ? 1u : 0u));
    // Delta: a new vertex with an edge to another vertex is always named by a hook
    // record (as the hooked root or as the new parent: its singleton tree can only
    // change through a CAS on it or onto it), so only a new vertex seen through a
    // self-loop needs a record of its own.
    if (TRACK && nu && su == sv) {
      has_rec = true;
      rec[0] = ks;
      rec[1] = ks;
      rec[2] = 0;
    }
    ru = su;
    rv = sv;
    if (su != kNoSlot && sv != kNoSlot && su != sv) {  // a self-loop adds its vertex, never a conflict
      const uint32_t pu = lu >> 1, pv = lv >> 1;
      if (pu == pv || pu == sv || pv == su) {  // shared parent, or parent/child
        GS_DBG(CTR_DBG_SHORT);
        if (SIGNED) {
          const uint32_t par = (pu == pv) ? ((lu ^ lv) & 1u) : (pu == sv ? (lu & 1u) : (lv & 1u));
          if ((need ^ par) & 1u) atomicOr(&t.ctr[ctr_index(CTR_FAIL)], 1u);
        }
      } else {
        uint32_t pru = 0, prv = 0;
        kru = ks;
        krv = kd;
        find_root2<false>(t, ru, lu, kru, pru, rv, lv, krv, prv);
        need ^= pru ^ prv;
        if (ru == rv) {
          GS_DBG(CTR_DBG_SAME);
          if (SIGNED && (need & 1u)) atomicOr(&t.ctr[ctr_index(CTR_FAIL)], 1u);
        } else {
          act = true;
        }
      }
    }
  }
  if (__popcll(__ballot(act)) >= 2) combine_hooks(act, ru, kru, rv, krv, need, kCombineRounds);  // wave-uniform
  if (act) has_rec = hook<SIGNED, TRACK>(t, ru, ru << 1, kru, rv, rv << 1, krv, need, fresh0, fresh1, rec);
  if (TRACK) {  // a self-loop is never `act`: at most one record per edge
    if (!TAKE && GS_WAVE_APPEND)
      append_record_wave(t, D, shard, has_rec, rec[0], rec[1], rec[2]);
    else if (has_rec)
      append_record<TAKE>(t, D, shard, rec[0], rec[1], rec[2]);
  }
  write_new_vertices(t, shard, nvx);
  if (dbg) {
    if (valid) atomicAdd(&dbg[0], 1u);
    if (act) atomicAdd(&dbg[2], 1u);
  }
}

// Resident window server: one launch serves every window of a session (config 5's
// latency path without a kernel launch per window). Windows run one after another; in
// each, block b folds edges [256 b, 256 b + 256) exactly as k_fold<SIGNED, true, true>
// does and the window's last block publishes it (take_tail). The table needs no kernel
// boundary between windows: every access is already correct on stale lines (the
// concurrency model in gs_device.hpp), as between the blocks of one launch. Hand-offs:
//   host -> block 0: a 64-byte mailbox line in host-mapped memory, {seq, 7 descriptor
//     words}, each descriptor word tagged with seq mod 2^16 in its top 16 bits
//     (data-tagged granules, MI355X_MICROARCH.md handoff-1to1): 8 lanes of wave 0
//     poll the whole line with system-scope loads in ONE load round; a window is taken
//     when seq is new and every tag matches it (a torn read is polled again);
//   block 0 -> blocks: the same tagged line written to device memory with agent-scope
//     (write-through) stores and no wait; the other blocks poll it the same way with
//     agent-scope loads; the line reaches the block through LDS behind a barrier;
//   window -> host: take_tail's rows, count word and tagged completion record.
// (Round 3: descriptor loads after the poll and a drained broadcast cost 2.7 us of
// every window: tools/server_trace.py.)
// Exit conditions every wave reaches: a stop request, or no window for idle_ticks
// (block 0 then tells the others and the host), or -- for the other blocks -- 10 x
// idle_ticks without any word from block 0. Block 0 does not leave idle while the last
// window it handed out is incomplete (a workgroup that was not yet resident still has to
// fold its edges: leaving would cut the window in half), except after 8 x idle_ticks; it
// stores the seq of every window it takes in box->taken, so the host tells "left
// before the window" (post it again) from "left inside it" (an error). The other blocks'
// own limit lies beyond block 0's longest stay: a window block 0 takes while
// it waits for a late workgroup (its predecessor completes, the host posts the next one)
// finds every other block still polling. Block 0 always broadcasts its exit, so the
// others normally leave with it.
template <bool SIGNED>
__global__ __launch_bounds__(kFoldBS) void k_window_server(Table t, Delta D, ServerBox* box, ServerBcast* bc,
                                                           unsigned long long* done, unsigned long long seq0,
                                                           unsigned long long idle_ticks) {
  __shared__ int64_t lrec[kFoldBS * 3];
  __shared__ uint32_t lcnt, lnv;
  __shared__ unsigned long long w[8];
#ifdef GS_TEST_LATE_WORKGROUP
  // test build only (make testhooks -> lib_testhooks/): the last workgroup starts
  // GS_TEST_LATE_WORKGROUP us late, as one the dispatcher held back behind another
  // stream's kernels would (the exit paths' late-block test). The product kernel has no
  // such branch.
  if (blockIdx.x == gridDim.x - 1) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < 100ull * GS_TEST_LATE_WORKGROUP) __builtin_amdgcn_s_sleep(8);
  }
#endif
  D.lrec = lrec;
  D.lcnt = &lcnt;
  D.lnv = &lnv;
  // the session's vertex count (CTR_SRV_NV): every window's publisher adds its inserts
  // (take_tail); block 0 drains it before it hands out the first window
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    unsigned long long c =
        __hip_atomic_load(t.ctr + ctr_index(CTR_NV + threadIdx.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
    if (threadIdx.x == 0)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(t.ctr + ctr_index(CTR_SRV_NV)), c, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);
  }
  unsigned long long last = seq0;
  unsigned long long last_done = 0;  // block 0: completion number of the last window it took
#ifdef GS_SERVER_TRACE
  __shared__ unsigned long long tseen, tbc;
#endif
  for (;;) {
    if (threadIdx.x < 64) {  // wave 0: lanes 0..7 hold the line's words (wave-uniform loop)
      const uint32_t lane = threadIdx.x;
      const bool b0 = blockIdx.x == 0;
      const unsigned long long t0 = wall_clock64();
      const unsigned long long limit = b0 ? idle_ticks : 10 * idle_ticks;
      unsigned long long* line = b0 ? &box->seq : &bc->seq;
      unsigned long long v = 0, s = 0;
      for (;;) {
        if (lane < 8)
          v = b0 ? __hip_atomic_load(line + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                 : __hip_atomic_load(line + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s = __shfl(v, 0, 64);
        if (s != last) {
          if (s & kServerStop) break;
          const bool ok = lane == 0 || lane >= 8 || (v >> 48) == (s & 0xFFFFull);
          if (__ballot(!ok) == 0ull) break;  // every tag is this window's
          continue;                          // a torn line: poll again at once
        }
        if (wall_clock64() - t0 > limit) {
          if (b0 && last_done &&
              __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < last_done &&
              wall_clock64() - t0 < 8 * limit) {
            __builtin_amdgcn_s_sleep(2);
            continue;  // the last window is still being folded
          }
          s = kServerStop | last;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
#ifdef GS_SERVER_TRACE
      if (b0) tseen = wall_clock64();
#endif
      if (b0) {
        // broadcast the tagged line as it was read (no wait: the other blocks check tags)
        if (!(s & kServerStop)) {
          if (lane == 0) __hip_atomic_store(&box->taken, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if (lane < 8) __hip_atomic_store(&bc->seq + lane, lane == 0 ? s : v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          last_done = __shfl(v, 7, 64) & kServerTagMask;
        } else if (lane == 0) {
          __hip_atomic_store(&bc->seq, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&box->exited, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
#ifdef GS_SERVER_TRACE
        tbc = wall_clock64();
#endif
      }
      if (lane < 8) w[lane] = lane == 0 ? s : (v & kServerTagMask);
    }
    __syncthreads();
    const unsigned long long s = w[0];
    if (s & kServerStop) return;  // block-uniform
    last = s;
    FoldArgs a{};
    a.src = reinterpret_cast<const int64_t*>(w[1]);
    a.dst = reinterpret_cast<const int64_t*>(w[2]);
    a.n = (uint32_t)w[3];
    a.stride = 1;
    a.w_stride = 1;
    a.skip_rank = -1;
    a.shard0 = (uint32_t)(s * gridDim.x);
    a.take_out = reinterpret_cast<int64_t*>(w[4]);
    a.take_cap = w[5];
    a.take_count = reinterpret_cast<unsigned long long*>(w[6]);
    a.done = done;
    a.seq = w[7];
    a.server = true;
    // only the blocks that hold edges of this window take part (a small window is one
    // block's ticket, not the whole grid's)
    const uint32_t active = (a.n + kFoldBS - 1) / kFoldBS;
    if (blockIdx.x < active) {
      if (threadIdx.x == 0) lcnt = 0, lnv = 0;
      // a failed verdict is final (no kernel boundary here: read it at the memory side)
      const bool failed = SIGNED && __builtin_amdgcn_readfirstlane(
                                        __hip_atomic_load(&t.ctr[ctr_index(CTR_FAIL)], __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)) != 0;
      __syncthreads();
#ifdef GS_SERVER_TRACE
      const unsigned long long tgo = wall_clock64();
#endif
      fold_block<SIGNED, true, true>(t, D, a, blockIdx.x, failed, 0ull, nullptr);
      __syncthreads();
#ifdef GS_SERVER_TRACE
      const unsigned long long tfold = wall_clock64();
      unsigned long long* tr = g_strace ? g_strace + (size_t)(s & (g_strace_cap - 1)) * 8 : nullptr;
      if (tr && threadIdx.x == 0) {
        atomicMax(tr + 2, tgo);
        atomicMax(tr + 3, tfold);
        // histogram of per-block fold times (0.5 us buckets) after the cap records
        // (buckets 64..127: the session's first 64 windows, a young table)
        const unsigned long long bkt = min((tfold - tgo) / 50ull, 63ull) + (s - seq0 <= 64 ? 64ull : 0ull);
        atomicAdd(g_strace + g_strace_cap * 8 + bkt, 1ull);
        if (blockIdx.x == 0) {
          tr[0] = tseen;
          tr[1] = tbc;
          tr[6] = active;
        }
      }
      if (take_tail(t, a, lrec, lcnt, SIGNED, blockIdx.x, active, lnv) && tr) {
        tr[4] = tfold;
        tr[5] = wall_clock64();
      }
#else
      take_tail(t, a, lrec, lcnt, SIGNED, blockIdx.x, active, lnv);
#endif
    }
    __syncthreads();  // LDS (lrec, lcnt, w) is reused by the next window
  }
}

// Micro-batch dedup by hashing (north_star's staging stage, gs_set_batch_dedup): every
// edge of the batch is inserted as its unordered pair (min, max) into an open-addressing
// table of 16-B slots {a, b} (2 x batch slots, all bytes 0xFF = empty), and w[i] = 0x81
// (bit 7: skip) marks an edge whose pair another edge of the batch already stored;
// kept edges get w[i] = 1 (the stream edge's parity: different sides). The fold then
// skips the marked edges. Union is idempotent, so dropping an exact repeat is exact.
// The slot's a word is claimed by a 64-bit CAS and its b word stored by the claimer
// afterwards; a thread that finds a claimed slot whose b is not yet visible keeps its
// edge (never a wait on another thread): an edge is dropped only when its pair is
// fully stored by the edge that keeps it. Ids equal to the empty marker (-1) are
// never deduplicated.
__global__ __launch_bounds__(256) void k_dedup(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                               uint32_t n, unsigned long long* __restrict__ tab, uint32_t mask,
                                               uint8_t* __restrict__ w) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t u = __builtin_nontemporal_load(src + i), v = __builtin_nontemporal_load(dst + i);
  const int64_t a = u < v ? u : v, b = u < v ? v : u;
  uint8_t out = 1;
  if (a != -1 && b != -1) {
    uint32_t h = (uint32_t)(((uint64_t)a * 0x9E3779B97F4A7C15ull ^ (uint64_t)b * 0xC2B2AE3D27D4EB4Full) >> 32) & mask;
    for (uint32_t probes = 0; probes <= mask; ++probes) {
      unsigned long long* slot = tab + 2 * (size_t)h;
      unsigned long long ka = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ka == ~0ull) {
        ka = atomicCAS(slot, ~0ull, (unsigned long long)a);
        if (ka == ~0ull) {  // claimed: this edge keeps the pair
          __hip_atomic_store(slot + 1, (unsigned long long)b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      if (ka == (unsigned long long)a) {
        const unsigned long long kb = __hip_atomic_load(slot + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (kb == (unsigned long long)b) {
          out = 0x81;  // a repeat of a stored pair
          break;
        }
        if (kb == ~0ull) break;  // claimed, not yet stored: keep the edge
      }
      h = (h + 1) & mask;
    }
  }
  w[i] = out;
}

void launch_dedup(const int64_t* src, const int64_t* dst, uint32_t n, unsigned long long* tab, uint32_t mask,
                  uint8_t* w, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_dedup, dim3((n + 255) / 256), dim3(256), 0, st, src, dst, n, tab, mask, w);
}

// One listed vertex -> output row pos: its key, canonical label (root key) and parity.
__device__ __forceinline__ void export_one(const Table& t, uint32_t s, int64_t* ov, int64_t* ol, uint8_t* op,
                                           uint64_t pos, uint64_t cap_out) {
  int64_t k;
  uint32_t l, acc;
  load_slot(t.tab + s, k, l);
  const int64_t v = settle_key(t, s, k);
  int64_t kx = v;
  find_ro(t, s, l, kx, acc);
  if (pos < cap_out) {  // (non-temporal stores here measured no different: 0.82 ms either way)
    ov[pos] = v;
    ol[pos] = kx;
    if (op) op[pos] = (uint8_t)acc;
  }
}

// Export (vertex, label, parity) of every occupied slot of [s_begin, s_end). Each
// thread owns kExportPer slots of a kExportPer x kExportBS-slot tile (coalesced 16-B
// loads); the block reserves its output range with ONE atomic per tile.
constexpr uint32_t kExportBS = 1024;
#ifndef GS_EXPORT_LOCKSTEP
#define GS_EXPORT_LOCKSTEP 1  // 0: one find after another, 16 slots per thread (experiment switch)
#endif
constexpr int kExportPer = GS_EXPORT_LOCKSTEP ? 8 : 16;

// by_list: the whole table with a complete vertex list, whose fill the host only bounds (the
// bound charges 2 vertices to every fold whose capacity report has not landed: right after a
// pass of folds it overstates RMAT-20's 646 K vertices ~10x). The kernel reads the real count
// and walks the list when it is under 1/8 of the slots (use_vertex_list's rule), as
// k_export_list does; else it scans. RMAT-20's label pass: 90 us scanning 2^23 slots.
__global__ __launch_bounds__(kExportBS) void k_export(Table t, int64_t* __restrict__ ov, int64_t* __restrict__ ol,
                                                      uint8_t* __restrict__ op, uint64_t cap_out, uint64_t s_begin,
                                                      uint64_t s_end, int by_list) {
  constexpr int PER = kExportPer;
  __shared__ uint32_t wsum[kExportBS / 64];
  __shared__ uint32_t base_sh;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (by_list && !t.ctr[ctr_index(CTR_VOVF)]) {
    __shared__ uint32_t lcnt[kShards];
    __shared__ uint64_t lpre[kShards + 1];
    const uint64_t total = vlist_prefix(t, lcnt, lpre);
    if (total * 8 < s_end - s_begin) {  // block-uniform
      const uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
      if (g0 == 0) t.ctr[ctr_index(CTR_EXPORT)] = (uint32_t)total;
      for (uint64_t g = g0; g < total && g < cap_out; g += (uint64_t)gridDim.x * blockDim.x)
        export_one(t, vlist_at(t, lpre, g), ov, ol, op, g, cap_out);
      return;
    }
  }
  for (uint64_t tile = s_begin + (uint64_t)blockIdx.x * (kExportBS * PER); tile < s_end;
       tile += (uint64_t)gridDim.x * (kExportBS * PER)) {
    int64_t vk[PER], lk[PER];
    uint32_t pp[PER];
    uint32_t occ = 0, cnt = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {  // all of the thread's slots in flight together
      const uint64_t s = tile + (uint64_t)j * kExportBS + threadIdx.x;
      vk[j] = 0;
      pp[j] = 0;
      if (s < s_end) {
        load_slot(t.tab + s, vk[j], pp[j]);
        const bool present = (s == t.r0) ? ((t.tab[s].aux & kAuxPresent) != 0) : (vk[j] != kEmpty);
        if (present) {
          occ |= 1u << j;
          ++cnt;
        }
      }
    }
    // Read-only finds. Their first hops go out together (after the folds' path splitting
    // most vertices hang directly under their root), and only a vertex whose parent is
    // not a root walks on alone: 16 finds one after another made the final label pass
    // of RMAT-20 80 us, a chain of dependent loads per thread.
    int64_t kq[PER];
    uint32_t lq[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t sj = (uint32_t)(tile + (uint64_t)j * kExportBS + threadIdx.x);
      kq[j] = vk[j];
      lq[j] = pp[j];
      if (GS_EXPORT_LOCKSTEP && ((occ >> j) & 1u) && (pp[j] >> 1) != sj) load_slot(t.tab + (pp[j] >> 1), kq[j], lq[j]);
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      lk[j] = vk[j];
      if (!((occ >> j) & 1u)) continue;
      const uint32_t sj = (uint32_t)(tile + (uint64_t)j * kExportBS + threadIdx.x);
      const uint32_t p = pp[j] >> 1;
      if (p == sj) {  // a root
        pp[j] = 0;
        continue;
      }
      uint32_t acc;
      if (!GS_EXPORT_LOCKSTEP) load_slot(t.tab + p, kq[j], lq[j]);  // (the switch's form: the hop here)
      int64_t kx = kq[j];
      find_ro(t, p, lq[j], kx, acc);  // from the parent: zero more hops when it is the root
      lk[j] = kx;
      pp[j] = acc ^ (pp[j] & 1u);
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

// Export over the vertex list: entry g -> output row g (deterministic, no atomics).
// If the list overflowed (CTR_VOVF) every slot is scanned with appends instead.

__global__ __launch_bounds__(256) void k_export_list(Table t, int64_t* __restrict__ ov, int64_t* __restrict__ ol,
                                                     uint8_t* __restrict__ op, uint64_t cap_out) {
  __shared__ uint32_t cnt[kShards];
  __shared__ uint64_t pre[kShards + 1];
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t.ctr[ctr_index(CTR_VOVF)]) {  // rare: the list is incomplete (CTR_EXPORT was zeroed by the host)
    for (uint64_t s = g0; s <= t.r0; s += stride) {
      int64_t k;
      uint32_t l;
      load_slot(t.tab + s, k, l);
      const bool present = (s == t.r0) ? ((t.tab[s].aux & kAuxPresent) != 0) : (k != kEmpty);
      if (present) export_one(t, (uint32_t)s, ov, ol, op, atomicAdd(&t.ctr[ctr_index(CTR_EXPORT)], 1u), cap_out);
    }
    return;
  }
  const uint64_t total = vlist_prefix(t, cnt, pre);
  if (g0 == 0) t.ctr[ctr_index(CTR_EXPORT)] = (uint32_t)total;
  for (uint64_t g = g0; g < total && g < cap_out; g += stride) export_one(t, vlist_at(t, pre, g), ov, ol, op, g, cap_out);
}

// Order-independent 64-bit digest of the summary's (vertex, canonical label, parity)
// set (gs_digest): out += sum over vertices of mix64(v) * mix64(label + parity * K),
// mod 2^64. Replicas of one summary (a group's ranks, a replay) agree exactly when their
// partitions (and colourings) do, with no export to compare.
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ unsigned long long digest_term(const Table& t, uint32_t s) {
  int64_t k;
  uint32_t l, acc;
  load_slot(t.tab + s, k, l);
  const int64_t v = settle_key(t, s, k);
  int64_t kx = v;
  find_ro(t, s, l, kx, acc);
  return mix64((unsigned long long)v ^ 0x243F6A8885A308D3ull) *
         mix64((unsigned long long)kx + (acc ? 0x13198A2E03707344ull : 0ull));
}

__global__ __launch_bounds__(256) void k_digest(Table t, unsigned long long* out) {
  __shared__ uint32_t cnt[kShards];
  __shared__ uint64_t pre[kShards + 1];
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long sum = 0;
  if (t.ctr[ctr_index(CTR_VOVF)]) {  // rare: the list is incomplete -- scan the table
    for (uint64_t s = g0; s <= t.r0; s += stride) {
      int64_t k;
      uint32_t l;
      load_slot(t.tab + s, k, l);
      const bool present = (s == t.r0) ? ((t.tab[s].aux & kAuxPresent) != 0) : (k != kEmpty);
      if (present) sum += digest_term(t, (uint32_t)s);
    }
  } else {
    const uint64_t total = vlist_prefix(t, cnt, pre);
    for (uint64_t g = g0; g < total; g += stride) sum += digest_term(t, vlist_at(t, pre, g));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
  if ((threadIdx.x & 63u) == 0 && sum) atomicAdd(out, sum);
}

// Stage the sharded delta list as contiguous records. grid = kShards blocks: block s
// copies shard s to its prefix position (deterministic, no append atomics); rows past
// `cap` are dropped (the count says how many there were). Block 0 writes the count word
// (| kFailBit when with_fail and the verdict failed: the exchange carries the verdict,
// Candidates.merge :79-81); the last block (a ticket of kShards same-address atomics)
// resets the shard counters. Block size (profiles/r04_rank_replay.txt): alone, 1024
// threads copy an 8-rank shard's exchange in 13 us against 22 with 256; but in the
// exchange step the stage runs beside the folds, and 64 blocks of 1024 threads took
// slots the folds needed (one-rank RCCL step 46.9-47.5 ms vs 42.2-42.9 with 256).
#ifndef GS_STAGE_BS
#define GS_STAGE_BS 256  // threads per k_stage block (experiment switch)
#endif
constexpr uint32_t kStageBS = GS_STAGE_BS;
__global__ __launch_bounds__(kStageBS) void k_stage(Table t, Delta D, int64_t* __restrict__ out, uint64_t cap,
                                                    int width, unsigned long long* count_out, int with_fail) {
  __shared__ uint32_t cnt[kShards];
  __shared__ uint64_t off_sh, total_sh;
  __shared__ uint32_t last;
  const uint32_t s = blockIdx.x;
  if (threadIdx.x < kShards) cnt[threadIdx.x] = min(t.ctr[ctr_index(D.dctr + threadIdx.x)], D.shard_cap);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t off = 0, tot = 0;
    for (uint32_t q = 0; q < kShards; ++q) {
      if (q < s) off += cnt[q];
      tot += cnt[q];
    }
    off_sh = off;
    total_sh = tot;
  }
  __syncthreads();
  const int64_t* in = D.drec + (size_t)s * D.shard_cap * 3;
  const uint64_t off = off_sh;
  for (uint32_t j = threadIdx.x; j < cnt[s]; j += kStageBS) {
    const uint64_t pos = off + j;
    if (pos >= cap) break;
    int64_t* r = out + pos * width;
    r[0] = in[(size_t)j * 3];
    r[1] = in[(size_t)j * 3 + 1];
    if (width == 3) r[2] = in[(size_t)j * 3 + 2];
  }
  if (s == 0 && threadIdx.x == 0) {
    const uint64_t total = total_sh;
    const bool failed = with_fail && t.ctr[ctr_index(CTR_FAIL)] != 0;
    *count_out = total | (failed ? kFailBit : 0ull);
    atomicAdd((unsigned long long*)&t.ctr[ctr_index(CTR_SENT)], (unsigned long long)(total < cap ? total : cap));
  }
  __syncthreads();  // every block has read the counters before the last one resets them
  if (threadIdx.x == 0) last = atomicAdd(&t.ctr[ctr_index(CTR_STAGE_DONE)], 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  if (threadIdx.x < kShards) t.ctr[ctr_index(D.dctr + threadIdx.x)] = 0u;
  if (threadIdx.x == 0) atomicExch(&t.ctr[ctr_index(CTR_STAGE_DONE)], 0u);
}

// Capacity report, queued behind a fold on its stream: adds the fold's edge count
// to the completed-edges counter, then reads the new-vertex count and writes both,
// packed into one 64-bit word (count << 34 | epoch mod 8 << 31 | edges mod 2^31), to
// host-coherent memory. Every fold whose report preceded this one (by the atomic
// order of the adds) had completed before this read, so count + 2 x (edges
// launched - edges done) bounds the vertex count without a host synchronisation.
// The epoch tag (resets since create) lets the host ignore a late report of a
// summary that was reset without a synchronisation.
__global__ __launch_bounds__(64) void k_report(uint32_t* ctr, unsigned long long n, unsigned long long* out,
                                               unsigned epoch) {
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
    const unsigned long long w = ((unsigned long long)c << 34) | ((unsigned long long)(epoch & 7u) << 31) |
                                 (done_sh & ((1ull << 31) - 1));
    __hip_atomic_store(out, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Gathered exchange count words -> host-mapped memory, one thread per rank,
// system-scope stores; then out[nranks] = seq (release): the host polls that word
// instead of synchronising on an event.
__global__ __launch_bounds__(64) void k_headers(const unsigned long long* __restrict__ counts, int nranks,
                                                long long* out, long long seq) {
  for (int r = threadIdx.x; r < nranks; r += 64)
    __hip_atomic_store(out + r, (long long)counts[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(out + nranks, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Completion word of a host wait (gs_sync and every other host synchronisation of a
// handle). Queued last on the handle stream, it starts only after all earlier work of
// the stream has completed -- end-of-kernel releases included -- so its system-scope
// store tells the host that everything before it is done and visible. The host spins
// on host-mapped memory instead of waiting for the stream's completion signal: a
// one-wave kernel + hipStreamSynchronize costs 12.2 us, a kernel whose store the
// host polls 6.5 us (tools/calib_launch.hip). `vals` (optional): the sum of nvals
// device counters (stride apart, <= 64) handed to the host in the same round trip
// (row counts, the sharded vertex count) instead of a copy and a second wait.
__global__ __launch_bounds__(64) void k_signal(unsigned long long* out, unsigned long long seq, const uint32_t* vals,
                                               int nvals, int stride, int clear, const uint32_t* flag) {
  unsigned long long v = (vals && (int)threadIdx.x < nvals) ? vals[(size_t)threadIdx.x * stride] : 0ull;
  if (clear && vals && (int)threadIdx.x < nvals)  // (one wave: every lane has read before any lane stores)
    const_cast<uint32_t*>(vals)[(size_t)threadIdx.x * stride] = 0u;
  if (nvals < 0)  // one u64 word (a count word with its flag bits) instead of u32 counters
    v = (vals && threadIdx.x == 0) ? *reinterpret_cast<const unsigned long long*>(vals) : 0ull;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  if (threadIdx.x != 0) return;
  if (flag && *flag) v |= kSignalFlagBit;  // (a second value in the same round trip: the verdict)
  // (a system release: the host may read what earlier work of the stream wrote to host
  // memory once it sees the word; the value is tagged as take_tail's)
  if (vals) __hip_atomic_store(out + 1, done_value(seq, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(out, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Single-vertex lookup (gs_find): presence and label.
__global__ void k_find_one(Table t, int64_t key, int64_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  out[0] = 0;
  out[1] = 0;
  uint32_t l = 0;
  const uint32_t s = lookup_find(t, key, l);
  if (s == kNoSlot) return;
  uint32_t acc;
  int64_t kx = key;
  find_ro(t, s, l, kx, acc);
  out[0] = 1;
  out[1] = kx;
}

// Batched lookup (gs_find_labels_device): label[i] = canonical label of v[i] (min id
// of its component), found[i] = 0 for an id never seen (label then = v[i]).
__global__ __launch_bounds__(256) void k_find_batch(Table t, const int64_t* __restrict__ v, uint64_t n,
                                                    int64_t* __restrict__ label, uint8_t* __restrict__ found,
                                                    uint8_t* __restrict__ parity) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t key = v[i];
    uint32_t l = 0, acc = 0;
    const uint32_t s = lookup_find(t, key, l);
    int64_t kx = key;
    if (s != kNoSlot) find_ro(t, s, l, kx, acc);
    label[i] = kx;
    if (found) found[i] = s != kNoSlot;
    if (parity) parity[i] = (uint8_t)acc;
  }
}

// ---------------------------------------------------------------- launchers
#ifdef GS_BLOCKLOG
}  // namespace gs
extern "C" int gs_debug_blocklog(void* buf, unsigned long long cap) {  // diagnostic build only
  unsigned long long zero = 0;
  gs::BlockLog* p = static_cast<gs::BlockLog*>(buf);
  if (hipMemcpyToSymbol(HIP_SYMBOL(gs::g_blog), &p, sizeof p) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(gs::g_blog_cap), &cap, sizeof cap) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(gs::g_blog_n), &zero, sizeof zero) != hipSuccess)
    return -2;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
extern "C" unsigned long long gs_debug_blocklog_count() {
  unsigned long long n = 0;
  (void)hipDeviceSynchronize();
  (void)hipMemcpyFromSymbol(&n, HIP_SYMBOL(gs::g_blog_n), sizeof n);
  return n;
}
namespace gs {
#endif
#ifdef GS_SERVER_TRACE
}  // namespace gs
extern "C" int gs_debug_server_trace(void* buf, unsigned long long cap) {  // diagnostic build only (cap: power of 2)
  unsigned long long* p = static_cast<unsigned long long*>(buf);
  if (hipMemcpyToSymbol(HIP_SYMBOL(gs::g_strace), &p, sizeof p) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(gs::g_strace_cap), &cap, sizeof cap) != hipSuccess)
    return -2;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
namespace gs {
#endif
void launch_init(Slot* tab, uint64_t nslots, hipStream_t st, uint32_t* ctr) {
  // one slot per thread for large tables: 2 GiB in 0.30 ms vs 0.48 ms with 8192 grid-strided
  // blocks; at most 16 slots per thread below 2^26 slots, where the dispatch of one block per
  // 256 slots dominated (config 4's 2^22-slot reset: 41 us for 67 MB)
  const uint64_t blocks = (nslots + 255) / 256;
  const uint64_t want = nslots < (1ull << 26) ? (blocks + 15) / 16 : blocks;
  const unsigned g = (unsigned)(want < 1 ? 1 : (want < (1u << 22) ? want : (1u << 22)));
  hipLaunchKernelGGL(k_init, dim3(g), dim3(256), 0, st, tab, nslots, ctr);
}

static unsigned list_grid(uint64_t bound) {
  const uint64_t b = (bound + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}

void launch_reset_list(const Table& t, uint32_t* nxt, uint64_t bound, hipStream_t st) {
  hipLaunchKernelGGL(k_reset_list, dim3(list_grid(bound)), dim3(256), 0, st, t, nxt);
}

void launch_fold(bool sign, bool track, const Table& t, const Delta& D, const FoldLaunch& f, hipStream_t st) {
  FoldArgs a{f.src,       f.dst,    f.w,      f.n,       f.stride,   f.w_stride,  f.rows,
             f.skip_rank, f.counts, f.base,   f.n_dev,   f.fail_in,  f.shard0,    f.take_out,
             f.take_cap,  f.take_count, f.done, f.seq};
  a.rep_out = f.rep_out;
  a.rep_claim = f.rep_claim;
  a.rep_epoch = f.rep_epoch;
  const dim3 g((f.n + kFoldBS - 1) / kFoldBS), b(kFoldBS);
  if (f.take_out) {  // fused window take (always tracked)
    if (sign) hipLaunchKernelGGL((k_fold<true, true, true>), g, b, 0, st, t, D, a);
    else hipLaunchKernelGGL((k_fold<false, true, true>), g, b, 0, st, t, D, a);
    return;
  }
  if ((f.rows || f.stride == 3) && !track) {  // other replicas' rows (a group's exchange layout, or 24-B records)
    if (sign) hipLaunchKernelGGL((k_fold<true, false, false, true>), g, b, 0, st, t, D, a);
    else hipLaunchKernelGGL((k_fold<false, false, false, true>), g, b, 0, st, t, D, a);
    return;
  }
  if (!sign && !track) hipLaunchKernelGGL((k_fold<false, false, false>), g, b, 0, st, t, D, a);
  if (!sign && track) hipLaunchKernelGGL((k_fold<false, true, false>), g, b, 0, st, t, D, a);
  if (sign && !track) hipLaunchKernelGGL((k_fold<true, false, false>), g, b, 0, st, t, D, a);
  if (sign && track) hipLaunchKernelGGL((k_fold<true, true, false>), g, b, 0, st, t, D, a);
}

void launch_window_server(bool sign, const Table& t, const Delta& D, ServerBox* box, ServerBcast* bc,
                          unsigned long long* done, unsigned long long seq0, unsigned long long idle_ticks,
                          hipStream_t st) {
  if (sign)
    hipLaunchKernelGGL(k_window_server<true>, dim3(kServerBlocks), dim3(kFoldBS), 0, st, t, D, box, bc, done, seq0,
                       idle_ticks);
  else
    hipLaunchKernelGGL(k_window_server<false>, dim3(kServerBlocks), dim3(kFoldBS), 0, st, t, D, box, bc, done, seq0,
                       idle_ticks);
}

int window_server_resident_blocks(bool sign, int device) {
  int per_cu = 0, cus = 0;
  const hipError_t e = sign ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_window_server<true>, kFoldBS, 0)
                            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_window_server<false>, kFoldBS, 0);
  if (e != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return 0;
  return per_cu * cus;
}

void launch_export(const Table& t, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap_out, hipStream_t st, int part,
                   int nparts, bool by_list) {
  const uint64_t all = (uint64_t)t.r0 + 1;
  const uint64_t s0 = all * (uint64_t)part / (uint64_t)nparts, s1 = all * (uint64_t)(part + 1) / (uint64_t)nparts;
  const uint64_t tile = (uint64_t)kExportPer * kExportBS;
  const uint64_t tiles = (s1 - s0 + tile - 1) / tile;
  const uint64_t cap_blocks = 4096ull * 256 / kExportBS;
  const unsigned g = (unsigned)(tiles < cap_blocks ? (tiles ? tiles : 1) : cap_blocks);
  hipLaunchKernelGGL(k_export, dim3(g), dim3(kExportBS), 0, st, t, ov, ol, op, cap_out, s0, s1,
                     (by_list && nparts == 1) ? 1 : 0);
}

void launch_export_list(const Table& t, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap_out, uint64_t bound,
                        hipStream_t st) {
  hipLaunchKernelGGL(k_export_list, dim3(list_grid(bound)), dim3(256), 0, st, t, ov, ol, op, cap_out);
}

void launch_digest(const Table& t, unsigned long long* out, uint64_t bound, hipStream_t st) {
  hipLaunchKernelGGL(k_digest, dim3(list_grid(bound)), dim3(256), 0, st, t, out);
}

void launch_stage(const Table& t, const Delta& D, int64_t* out, uint64_t cap, int width,
                  unsigned long long* count_out, bool with_fail, hipStream_t st) {
  hipLaunchKernelGGL(k_stage, dim3(kShards), dim3(kStageBS), 0, st, t, D, out, cap, width, count_out, with_fail ? 1 : 0);
}

void launch_report(uint32_t* ctr, uint64_t n, unsigned long long* out, unsigned epoch, hipStream_t st) {
  hipLaunchKernelGGL(k_report, dim3(1), dim3(64), 0, st, ctr, (unsigned long long)n, out, epoch);
}

void launch_headers(const unsigned long long* counts, int nranks, long long* out, long long seq, hipStream_t st) {
  hipLaunchKernelGGL(k_headers, dim3(1), dim3(64), 0, st, counts, nranks, out, seq);
}

void launch_signal(unsigned long long* out, unsigned long long seq, const uint32_t* vals, int nvals, int stride,
                   hipStream_t st, bool clear, const uint32_t* flag) {
  hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, st, out, seq, vals, nvals, stride, clear ? 1 : 0, flag);
}

void launch_find_one(const Table& t, int64_t key, int64_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_find_one, dim3(1), dim3(64), 0, st, t, key, out);
}

void launch_find_batch(const Table& t, const int64_t* v, uint64_t n, int64_t* label, uint8_t* found, uint8_t* parity,
                       hipStream_t st) {
  const uint64_t b = (n + 255) / 256;
  const unsigned g = (unsigned)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
  hipLaunchKernelGGL(k_find_batch, dim3(g), dim3(256), 0, st, t, v, (unsigned long long)n, label, found, parity);
}

}  // namespace gs
