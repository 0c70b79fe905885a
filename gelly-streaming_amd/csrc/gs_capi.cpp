// gs_capi.cpp -- implementation of the summary C ABI (include/gs_summary.h).
//
// One handle = one GPU-resident summary: the slot table (relabel + forest), the
// vertex list, the sharded counters, the optional delta list, pinned staging for
// host-pointer folds, the combine export scratch and the handle's own HIP stream.
// All device work is enqueued on that stream (or on its pipelining lanes / the
// group's side stream); the host only synchronises when it must return data
// (counts, exports) or when the vertex table may need to grow.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <unordered_map>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "gs_ingest.h"
#include "gs_internal.hpp"

// Young-table head chunk (fold_device_impl): log2 of the edges of an empty table's first
// fold that go alone (0: off)
#ifndef GS_YOUNG_HEAD_LOG2
#define GS_YOUNG_HEAD_LOG2 14
#endif

namespace gsi {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// Device-memory accounting (gs_hbm_bytes): every allocation of summary / group state
// goes through dmalloc, which remembers its size and device.
std::atomic<uint64_t> g_hbm[kMaxDevices];
std::mutex g_alloc_mu;
std::unordered_map<void*, std::pair<int, size_t>> g_allocs;

hipError_t dmalloc(void** p, size_t bytes) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  const hipError_t e = hipMalloc(p, bytes);
  if (e == hipSuccess && *p) {
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    g_allocs[*p] = {dev, bytes};
    if (dev >= 0 && dev < kMaxDevices) g_hbm[dev] += bytes;
  }
  return e;
}

hipError_t dfree(void* p) {
  if (!p) return hipSuccess;
  {
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    auto it = g_allocs.find(p);
    if (it != g_allocs.end()) {
      if (it->second.first >= 0 && it->second.first < kMaxDevices) g_hbm[it->second.first] -= it->second.second;
      g_allocs.erase(it);
    }
  }
  return hipFree(p);
}

// include/gs_testing.h: process-wide test knobs, -1 = unset (the product value)
std::atomic<int64_t> g_testing[GS_TESTING_KNOBS] = {{-1}, {-1}, {-1}, {-1}, {-1}};

int64_t testing_value(int knob, int64_t product) {
  const int64_t v = g_testing[knob].load(std::memory_order_relaxed);
  return v < 0 ? product : v;
}

namespace {

uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

hipEvent_t take_event(gs_summary* h) {
  if (!h->ev_pool.empty()) {
    hipEvent_t e = h->ev_pool.back();
    h->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

// Bracket one launch with events on stream st when profiling.
struct Prof {
  gs_summary* h;
  int kid;
  hipStream_t st;
  hipEvent_t a = nullptr;
  Prof(gs_summary* h_, int k, hipStream_t s = nullptr) : h(h_), kid(k), st(s ? s : h_->stream) {
    if (h->profiling) {
      a = take_event(h);
      (void)hipEventRecord(a, st);
    }
  }
  ~Prof() {
    if (h->profiling) {
      hipEvent_t b = take_event(h);
      (void)hipEventRecord(b, st);
      h->prof_pending.push_back({kid, a, b});
    }
  }
};

void drain_profile(gs_summary* h) {
  for (auto& p : h->prof_pending) {
    float ms = 0.f;
    if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      h->launches[p.kid] += 1;
      h->total_ms[p.kid] += ms;
    }
    h->ev_pool.push_back(p.a);
    h->ev_pool.push_back(p.b);
  }
  h->prof_pending.clear();
}

// Order the handle's stream behind every fold still running on a lane (every lane
// that exists: pipelined folds use lanes 0..pipe_depth-1, a group's own folds lanes
// 0..2, whatever the handle's pipelining depth).
int join_pipe_lanes(gs_summary* h) {
  if (!h->lanes_dirty) return GS_OK;
  for (int i = 0; i < gs_summary::kLanes && h->lane[i]; ++i) {
    GS_HIP(hipEventRecord(h->lane_ev[i], h->lane[i]));
    GS_HIP(hipStreamWaitEvent(h->stream, h->lane_ev[i], 0));
  }
  h->xwait = true;
  h->lanes_dirty = false;
  return GS_OK;
}

// An export into the combine scratch must wait until the last consumer of the
// previous export (another summary's fold) has read it.
int wait_x_consumer(gs_summary* h) {
  if (!h->x_pending) return GS_OK;
  GS_HIP(hipStreamWaitEvent(h->stream, h->x_used, 0));
  h->xwait = true;
  h->x_pending = false;
  return GS_OK;
}

// Combine scratch of at least `rows` rows (v, label, parity), allocated on growth only.
int ensure_x(gs_summary* h, uint64_t rows) {
  if (!h->x_cnt) {
    GS_HIP(dmalloc(&h->x_cnt, 16));
    GS_HIP(hipEventCreateWithFlags(&h->x_ready, hipEventDisableTiming));
    GS_HIP(hipEventCreateWithFlags(&h->x_used, hipEventDisableTiming));
  }
  if (h->x_cap >= rows) return GS_OK;
  if (h->x_v) {
    if (int rc = wait_x_consumer(h)) return rc;
    GS_HIP(hipStreamSynchronize(h->stream));
    (void)dfree(h->x_v);
    (void)dfree(h->x_l);
    (void)dfree(h->x_p);
    h->x_v = h->x_l = nullptr;
    h->x_p = nullptr;
  }
  const uint64_t c = std::max<uint64_t>(rows, (uint64_t)(kMaxLoad * (double)h->cap) + 2);
  GS_HIP(dmalloc(&h->x_v, c * 8));
  GS_HIP(dmalloc(&h->x_l, c * 8));
  GS_HIP(dmalloc(&h->x_p, c));
  h->x_cap = c;
  return GS_OK;
}

// After a reset or rebuild: `nv` vertices exactly, no fold in flight of this epoch.
// Reports of earlier folds that land late carry an older epoch tag and are ignored.
void reset_capacity_tracking(gs_summary* h, uint64_t nv) {
  h->rep_epoch++;
  h->nv_ub = nv;
  h->nv_exact = nv;
  h->e_exact = 0;
  h->e_launched = 0;
  h->e_lost = 0;
  for (int i = 0; i < gs_summary::kRepStreams; ++i) h->rep_skip[i] = 0, h->rep_pending[i] = 0;
  h->rep_pending_edges = 0;
}

}  // namespace

// gs_create's table for a hint: kSlotsPerHintedVertex slots per expected vertex, a power of
// two, >= 1024
uint64_t create_capacity(uint64_t capacity_hint) {
  const uint64_t cap = next_pow2(std::max<uint64_t>(kSlotsPerHintedVertex * std::max<uint64_t>(capacity_hint, 1), 1024));
  return std::min(cap, kMaxCap);
}

// device bytes gs_create allocates for a table of cap slots (alloc_table + gs_create's own;
// the host-fold staging comes with the first host fold, sized for its chunks)
uint64_t create_bytes(uint64_t cap) {
  return (cap + 1) * sizeof(gs::Slot) + (uint64_t)gs::kShards * (cap / gs::kShards + 1024) * 4 +
         (uint64_t)gs::CTR_COUNT * gs::kCtrStride * 4 + 64;
}

namespace {

int alloc_vlist(gs_summary* h) {
  (void)dfree(h->vlist);
  h->vlist = nullptr;
  h->vshard_cap = (uint32_t)(h->cap / gs::kShards + 1024);
  GS_HIP(dmalloc(&h->vlist, (size_t)gs::kShards * h->vshard_cap * 4));
  return GS_OK;
}

// keep_delta: a rebuild (grow) keeps the pending delta counters.
int alloc_table(gs_summary* h, uint64_t cap, bool keep_delta = false) {
  h->cap = cap;
  h->logcap = 0;
  while ((1ull << h->logcap) < cap) ++h->logcap;
  GS_HIP(dmalloc(&h->tab, (cap + 1) * sizeof(gs::Slot)));
  if (int rc = alloc_vlist(h)) return rc;
  memset(h->h_flags, 0, 16);  // the device flags are cleared below (no kernel of the old table runs)
  if (keep_delta) {
    GS_HIP(hipMemsetAsync(h->ctr, 0, gs::ctr_index(gs::CTR_DELTA) * 4, h->stream));
    GS_HIP(hipMemsetAsync(h->ctr + gs::ctr_index(gs::CTR_FAIL), 0,
                          (gs::CTR_COUNT - gs::CTR_FAIL) * gs::kCtrStride * 4, h->stream));
  } else {
    GS_HIP(hipMemsetAsync(h->ctr, 0, gs::CTR_COUNT * gs::kCtrStride * 4, h->stream));
  }
  h->export_ctr_zero = true;  // (both forms clear CTR_EXPORT)
  {
    Prof p(h, KID_INIT);
    gs::launch_init(h->tab, cap + 1, h->stream);
  }
  GS_HIP(hipGetLastError());
  h->vlist_ok = true;
  reset_capacity_tracking(h, 0);
  return GS_OK;
}

// Rebuild into a table of capacity new_cap by re-folding (v, label, parity).
int grow(gs_summary* h, uint64_t new_cap) {
  if (new_cap > kMaxCap) return fail(GS_ERR_CAPACITY, "vertex table would exceed 2^30 slots");
  uint64_t nv = 0;
  int rc = read_nv(h, &nv);
  if (rc) return rc;
  int64_t *v = nullptr, *l = nullptr;
  uint8_t* p = nullptr;
  const size_t m = nv + 1;
  auto release = [&] {
    (void)dfree(v);
    (void)dfree(l);
    (void)dfree(p);
  };
  if (dmalloc(&v, m * 8) != hipSuccess || dmalloc(&l, m * 8) != hipSuccess || dmalloc(&p, m) != hipSuccess) {
    release();
    return fail(GS_ERR_HIP, "table rebuild: out of device memory");
  }
  size_t got = 0;
  uint32_t fail_flag = 0;
  rc = export_device_impl(h, v, l, p, m, &got);
  if (!rc && hipMemcpyAsync(&fail_flag, h->ctr + gs::ctr_index(gs::CTR_FAIL), 4, hipMemcpyDeviceToHost, h->stream) !=
                 hipSuccess)
    rc = fail(GS_ERR_HIP, "table rebuild: flag read failed");
  if (!rc && hipStreamSynchronize(h->stream) != hipSuccess) rc = fail(GS_ERR_HIP, "table rebuild: sync failed");
  if (rc) {
    release();
    return rc;
  }
  (void)dfree(h->tab);
  h->tab = nullptr;
  const bool track = h->track;
  h->track = false;  // the rebuild is not a delta
  rc = alloc_table(h, new_cap, /*keep_delta=*/true);
  if (!rc && fail_flag && hipMemsetAsync(h->ctr + gs::ctr_index(gs::CTR_FAIL), 1, 1, h->stream) != hipSuccess)
    rc = fail(GS_ERR_HIP, "table rebuild: flag write failed");
  if (!rc && h->changes) rc = change_tracking_reset(h, 2);
  if (!rc) {
    reset_capacity_tracking(h, got);
    rc = fold_device_impl(h, v, l, p, got, 1, 1, /*track=*/false, /*check_cap=*/false);
  }
  h->track = track;
  if (!rc && hipStreamSynchronize(h->stream) != hipSuccess) rc = fail(GS_ERR_HIP, "table rebuild: sync failed");
  release();
  return rc;
}

// Upper bound of the vertex count once `e_launched` edges have been folded: the
// last exact count, or any capacity report of this epoch, plus 2 new vertices per
// edge not covered. Also returns whether every issued report has landed.
uint64_t capacity_bound(gs_summary* h, bool* all_reported) {
  const uint64_t m31 = (1ull << 31) - 1;
  const uint64_t live = h->e_launched - h->e_lost;  // launched edges a report may still claim
  uint64_t best = h->nv_exact + 2 * (h->e_launched - h->e_exact);
  uint64_t max_done = h->e_exact;
  for (int i = 0; i < gs_summary::kRepRing; ++i) {
    const unsigned long long w = __atomic_load_n(&h->rep[i], __ATOMIC_ACQUIRE);
    if (!w || ((w >> 31) & 7u) != (h->rep_epoch & 7u)) continue;
    const uint64_t low = w & m31, c = w >> 34;
    const uint64_t behind = (live - low) & m31;  // claimable edges launched after that report
    if (behind > live) continue;
    best = std::min<uint64_t>(best, c + 2 * behind);
    max_done = std::max<uint64_t>(max_done, h->e_launched - behind);
  }
  // edges waiting on a stream for its next report will not be claimed by waiting
  if (all_reported) *all_reported = max_done + h->rep_pending_edges >= h->e_launched;
  return best;
}

// An exact vertex count read after every stream was joined and every queued fold
// (and report) completed.
void note_exact_count(gs_summary* h, uint64_t nv) {
  h->nv_exact = nv;
  h->e_exact = h->e_launched;
  // edges queued since their stream's last report are complete and counted in nv, but
  // no report will claim them: keep them out of later reports' "behind" 
  h->e_lost += h->rep_pending_edges;
  h->rep_pending_edges = 0;
  for (int i = 0; i < gs_summary::kRepStreams; ++i) h->rep_skip[i] = 0, h->rep_pending[i] = 0;
  memset(h->rep, 0, gs_summary::kRepRing * 8);  // every report of this epoch has landed
  h->nv_ub = nv;
}

int ensure_capacity(gs_summary* h, size_t n) {
  const double limit = kMaxLoad * (double)h->cap;
  bool all = false;
  uint64_t b = capacity_bound(h, nullptr);
  if ((double)(b + 2 * (uint64_t)n) <= limit) {
    h->nv_ub = b + 2 * (uint64_t)n;
    h->e_launched += n;
    return GS_OK;
  }
  // A table (below kSlackGrowMaxCap) too small to hold even the pipeline's slack --
  // pipe_depth + 1 folds of n edges in flight on top of the vertices known exactly --
  // goes straight to the synchronous path and is sized for that slack once. Waiting
  // for reports below is then only back-pressure with enough folds queued to keep the
  // GPU busy, instead of a drain before every fold (RMAT-20, config 2: 1.07 -> 0.72
  // ms/step).
  // (Not x 2 for the chunk per lane whose report rides on the lane's next launch: a wait
  // flushes those reports, and the larger table the doubled slack bought -- 2^25 instead of
  // 2^23 slots for config 2 -- cost more in the folds than the waits: 0.556 -> 0.62 ms/step.)
  const uint64_t slack = 2ull * n * (uint64_t)(std::max({1, h->pipe_depth, h->group_lanes}) + 1);
  const bool slack_grow = h->cap < kSlackGrowMaxCap && (double)(h->nv_exact + slack) > limit;
  if (!slack_grow) {
    // wait for reports of the folds in flight (the GPU keeps working: no drain). The reports
    // of queued chunks ride on the launches queued behind them and land as those start; only
    // when nothing more can land that way are the last chunks' reports launched on their own
    // (config 2 flushed before every wait: a standalone k_report beside most folds)
    h->cap_waits++;
    bool flushed = false;
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(200)) {
      b = capacity_bound(h, &all);
      if ((double)(b + 2 * (uint64_t)n) <= limit) {
        h->cap_wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        h->nv_ub = b + 2 * (uint64_t)n;
        h->e_launched += n;
        return GS_OK;
      }
      if (all) {
        if (flushed) break;
        if (int rc = flush_reports(h)) return rc;
        flushed = true;
        continue;
      }
      std::this_thread::yield();
    }
    h->cap_wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  uint64_t nv = 0;
  h->cap_syncs++;
  int rc = read_nv(h, &nv);  // exact (joins every stream: every issued report has landed)
  if (rc) return rc;
  note_exact_count(h, nv);
  h->nv_ub = nv + 2 * (uint64_t)n;
  uint64_t need = h->nv_ub;
  if (slack_grow) need = std::max<uint64_t>(need, nv + slack);
  if ((double)need > limit) {
    uint64_t nc = h->cap;
    while (kMaxLoad * (double)nc < (double)h->nv_ub) nc <<= 1;  // what this fold needs
    while (slack_grow && kMaxLoad * (double)nc < (double)need && nc < kSlackGrowMaxCap) nc <<= 1;  // + slack
    if (nc > h->cap) {
      rc = grow(h, nc);  // resets the tracking to the rebuilt table's exact count
      if (rc) return rc;
      h->nv_ub = h->nv_exact + 2 * (uint64_t)n;
    }
  }
  h->e_launched += n;
  return GS_OK;
}

int check(gs_handle h) {
  if (!h) return fail(GS_ERR_INVALID, "null handle");
  ++h->api_calls;  // (a group orders its own-fold lanes behind the handle stream after any call)
  return GS_OK;
}

}  // namespace

bool side_ok(const gs_summary* h) { return h->side && !h->profiling; }

// Pipelining lanes are created on first use, only as many as used: every stream of a
// process maps onto one of GPU_MAX_HW_QUEUES hardware queues (default 4), and two
// streams on one queue run in submission order -- a kernel waiting on another
// stream's event then blocks everything queued behind it on that queue.
int ensure_lanes(gs_summary* h, int n) {
  for (int i = 0; i < n && i < gs_summary::kLanes; ++i) {
    if (h->lane[i]) continue;
    GS_HIP(hipStreamCreateWithFlags(&h->lane[i], hipStreamNonBlocking));
    GS_HIP(hipEventCreateWithFlags(&h->lane_ev[i], hipEventDisableTiming));
  }
  return GS_OK;
}

// ---- resident window server (gs_set_window_server) -------------------------------
// Stop: the stop word, then the stream (the launch leaves within a poll interval).
int server_stop(gs_summary* h) {
  if (!h->srv_running) return GS_OK;
  __atomic_store_n(&h->srv_box->seq, gs::kServerStop | h->srv_seq, __ATOMIC_RELEASE);
  h->srv_running = false;
  GS_HIP(hipStreamSynchronize(h->stream));
  return GS_OK;
}

// Start a session whose first window is srv_seq + 1. The blocks' broadcast word starts
// at srv_seq (copied on the stream from the pinned mailbox, before the launch), so no
// block mistakes the previous session's stop word for this session's.
int server_start(gs_summary* h) {
  gs::ServerBox* b = h->srv_box;
  memset(b, 0, sizeof(gs::ServerBox));
  b->seq = h->srv_seq;
  b->bc_init = h->srv_seq;
  GS_HIP(hipMemcpyAsync(&h->srv_bc->seq, &b->bc_init, 8, hipMemcpyHostToDevice, h->stream));
  // ~2 ms without a window: the launch leaves on its own (wall clock 100 MHz). It holds
  // its stream's hardware queue while resident, so another stream that shares the queue
  // waits at most that long behind an idle server (the config-5 windows arrive
  // back to back; a restart costs one launch). Tests of the exit paths shorten it
  // (GS_TESTING_SERVER_IDLE_US, include/gs_testing.h).
  const int64_t idle_us = testing_value(GS_TESTING_SERVER_IDLE_US, 2000);
  const unsigned long long idle_ticks = (unsigned long long)std::max<int64_t>(idle_us, 1) * 100ull;
  gs::launch_window_server(h->kind == GS_KIND_SIGNED, h->table(), h->delta(), h->srv_box, h->srv_bc, h->done_dev,
                           h->srv_seq, idle_ticks, h->stream);
  GS_HIP(hipGetLastError());
  h->srv_running = true;
  h->srv_launches++;
  return GS_OK;
}

int join_lanes(gs_summary* h) {
  if (int rc = server_stop(h)) return rc;
  if (int rc = join_pipe_lanes(h)) return rc;
  if (h->side_dirty) {
    GS_HIP(hipEventRecord(h->side_ev, h->side));
    GS_HIP(hipStreamWaitEvent(h->stream, h->side_ev, 0));
    h->xwait = true;
    h->side_dirty = false;
  }
  return GS_OK;
}

// Whether every operation queued on st so far (cross-stream waits included) has completed: an
// event recorded now and queried. (hipStreamQuery reported a handle stream idle while it still
// waited on its lanes' events -- gs_sync returned with folds running in the multi-rank replay:
// 3.4 ms of "own folds" that a device-wide synchronisation put at 5.7-6.1 ms.)
bool stream_idle(gs_summary* h, hipStream_t st) {
  if (hipEventRecord(h->idle_ev, st) != hipSuccess) return false;
  return hipEventQuery(h->idle_ev) == hipSuccess;
}

// Host wait for h->stream: k_signal queued behind everything, then a spin on its
// host-mapped word (6.5 vs 12.2 us for hipStreamSynchronize after a short kernel,
// tools/calib_launch.hip). A wait that outlasts kSpinWait (a fold queue, not a small
// window) hands over to hipStreamSynchronize, which also surfaces asynchronous HIP
// errors and leaves the core to other threads (N emulated ranks in one process).
int wait_stream(gs_summary* h, const uint32_t* vals, uint64_t* value, int nvals, int stride, bool clear,
                hipStream_t st, const uint32_t* flag) {
  if (!st) st = h->stream;
  if (!vals && !(st == h->stream && h->xwait) && stream_idle(h, st)) return GS_OK;  // already idle (no launch)
  const unsigned long long seq = ++h->done_seq;
  gs::launch_signal(h->done_dev, seq, vals, nvals, stride, st, clear, flag);
  GS_HIP(hipGetLastError());
  if (int rc = wait_done(h, seq, st)) return rc;
  if (st == h->stream) h->xwait = false;
  if (value) return done_value_read(h, 1, seq, value);
  return GS_OK;
}

// Spin until the completion word reaches seq (its writer is queued on h->stream).
int wait_done(gs_summary* h, unsigned long long seq, hipStream_t st) {
  constexpr auto kSpinWait = std::chrono::microseconds(250);
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 1;; ++i) {
    if (__atomic_load_n(h->h_done, __ATOMIC_ACQUIRE) >= seq) return GS_OK;
    if ((i & 255u) == 0 && std::chrono::steady_clock::now() - t0 > kSpinWait) break;
    __builtin_ia32_pause();
  }
  GS_HIP(hipStreamSynchronize(st ? st : h->stream));
  if (__atomic_load_n(h->h_done, __ATOMIC_ACQUIRE) < seq) return fail(GS_ERR_HIP, "completion word not written");
  return GS_OK;
}

// Value i (1, 2) of the completion record written with sequence number seq: tagged
// with seq mod 2^16 (gs::done_value); once the sequence word is seen the value has
// landed too (its writer drains it first), the tag check makes that explicit.
int done_value_read(gs_summary* h, int i, unsigned long long seq, uint64_t* out) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t k = 1;; ++k) {
    const unsigned long long w = __atomic_load_n(h->h_done + i, __ATOMIC_ACQUIRE);
    if ((w >> 48) == (seq & 0xFFFFull)) {
      *out = gs::done_decode(w);
      return GS_OK;
    }
    if ((k & 1023u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1))
      return fail(GS_ERR_HIP, "completion record value not tagged with its sequence number");
    __builtin_ia32_pause();
  }
}

// Error flags, read with ONE host synchronisation. Also refreshes whether the
// vertex list is complete.
int check_device_flags(gs_summary* h) {
  // kernels mirror the rare flags into host-mapped memory (raise_flag): after the
  // stream wait they are read with no device-to-host copy (each copy is a launch and
  // a round trip of its own: the three per-flag copies cost ~10 us of a 2^16-edge
  // window, config 5)
  if (int rc = wait_stream(h)) return rc;
  return check_flags_now(h);
}

// The host-mapped flags as they stand (the caller has waited for the stream).
int check_flags_now(gs_summary* h) {
  const uint32_t err = __atomic_load_n(&h->h_flags[0], __ATOMIC_ACQUIRE);
  const uint32_t ovf = __atomic_load_n(&h->h_flags[1], __ATOMIC_ACQUIRE);
  const uint32_t vovf = __atomic_load_n(&h->h_flags[2], __ATOMIC_ACQUIRE);
  if (vovf) h->vlist_ok = false;
  if (err) return fail(GS_ERR_CAPACITY, "vertex table overflow (device probe limit)");
  if (ovf) return fail(GS_ERR_CAPACITY, "delta list overflow: stage or take the delta records after each fold");
  return GS_OK;
}

int read_nv(gs_summary* h, uint64_t* nv) {
  if (int rc = join_lanes(h)) return rc;
  // the 64 shard counts summed on the device and handed over with the wait
  if (int rc = wait_stream(h, h->ctr + gs::ctr_index(gs::CTR_NV), nv, gs::kShards, gs::kCtrStride)) return rc;
  if (__atomic_load_n(&h->h_flags[2], __ATOMIC_ACQUIRE)) h->vlist_ok = false;  // CTR_VOVF's mirror
  return GS_OK;
}

// Sparse tables export / reset over the vertex list; dense ones scan the table. A listed
// slot costs a random 16-B access (~50 G/s, the request ceiling), a scanned one a share
// of a streaming pass (~375 G slots/s at 6 TB/s): the list wins below ~1/8 load. The
// bound is tightened with the landed capacity reports (a reset right after a pass of
// folds would otherwise see 2 vertices per folded edge: config 4 re-initialised its
// whole 2^24-slot table, 41 us of every step, for 2^20 vertices).
bool use_vertex_list(gs_summary* h, uint64_t nv_bound) {
  nv_bound = std::min<uint64_t>(nv_bound, capacity_bound(h, nullptr));
  return h->vlist_ok && nv_bound * 8 < h->cap;
}

// report stream index of a stream: 0 the handle stream, 1.. the lanes, last the side stream
int report_stream(const gs_summary* h, hipStream_t st) {
  if (st == h->side && h->side) return gs_summary::kRepStreams - 1;
  for (int i = 0; i < gs_summary::kLanes; ++i)
    if (st == h->lane[i] && h->lane[i]) return 1 + i;
  return 0;
}

hipStream_t report_stream_of(const gs_summary* h, int rs) {
  if (rs == gs_summary::kRepStreams - 1) return h->side;
  if (rs >= 1) return h->lane[rs - 1];
  return h->stream;
}

// a standalone k_report claiming stream rs's pending chunks (queued on that stream)
int launch_report_now(gs_summary* h, int rs, hipStream_t st) {
  const uint64_t claim = h->rep_pending[rs];
  if (!claim) return GS_OK;
  gs::launch_report(h->ctr, claim, h->rep_dev + (h->rep_seq++ % gs_summary::kRepRing), (unsigned)(h->rep_epoch & 7u),
                    st);
  GS_HIP(hipGetLastError());
  h->rep_pending_edges -= claim;
  h->rep_pending[rs] = 0;
  return GS_OK;
}

// every stream's unclaimed chunks reported (before the host waits for reports)
int flush_reports(gs_summary* h) {
  for (int rs = 0; rs < gs_summary::kRepStreams; ++rs) {
    if (!h->rep_pending[rs]) continue;
    hipStream_t st = report_stream_of(h, rs);
    if (!st) continue;
    if (int rc = launch_report_now(h, rs, st)) return rc;
  }
  return GS_OK;
}

int fold_device_impl(gs_summary* h, const int64_t* src, const int64_t* dst, const uint8_t* w, size_t n,
                     size_t stride, size_t w_stride, bool track, bool check_cap, const FoldSource& fs) {
  if (n == 0) return GS_OK;
  // Capacity units (each may add 2 vertices): one per edge, or for a gathered
  // exchange buffer the caller's count of live rows it will fold. The valid rows may
  // sit in any chunk, so an exchange fold claims all its units with its last chunk.
  const uint64_t units = fs.rows ? fs.units : n;
  if (track && !fs.take_out) {  // refuse before any capacity accounting: edges charged there must be folded
    uint64_t fill = h->delta_fill_ub[h->dset];
    for (size_t off = 0; off < n; off += kMaxChunk) fill += per_shard_edges(std::min<size_t>(kMaxChunk, n - off));
    if (!h->drec || fill > h->delta_shard_cap)
      return fail(GS_ERR_CAPACITY, "delta list full: stage or take the delta records after at most " +
                                       std::to_string(h->delta_edges) + " folded edges");
  }
  // Young-table head: the first plain fold of an empty table folds its first 2^14 edges alone
  // on the handle stream, and every lane (this fold's rest and the next pipelined folds) waits
  // for it. On an empty table every occurrence of a hub reads EMPTY and CASes the hub's key,
  // and those same-address CASes serialise at the memory side (RMAT-20's first micro-batch:
  // 258 K of its 524 K key CASes lost, 611 K failed hook CASes, 150 us against ~30 us for a
  // later batch; tools/fold_stats.py). The head inserts the stream's hubs; the rest reads
  // their keys. Config 2: 0.597 -> 0.552-0.558 ms/step; config 4 (uniform endpoints, no hubs)
  // pays the head's latency: 0.852-0.857 -> 0.858-0.865 (profiles/r05_young_ab.txt).
  // A build with -DGS_YOUNG_HEAD_LOG2=k sets the size (0: off). The head runs on the handle
  // stream, so a fold the caller put on a lane or the side stream (and joins there) has none
  // (ADVICE r5).
  constexpr int young_head_log2 = GS_YOUNG_HEAD_LOG2;
  // (Gathered rows too: a partitioned group's label forest is empty at every pass and its
  // pairs name the giant component's few local labels over and over -- the head is then the
  // first 2^14 rows of the flat row range, whatever rank blocks they belong to.)
  const bool young_head = young_head_log2 > 0 && check_cap && !track && !fs.take_out && fs.lane < 0 && !fs.on_side &&
                          h->e_launched == 0 && h->nv_exact == 0 && n > ((size_t)2 << young_head_log2);
  if (check_cap && units) {
    if (int rc = ensure_capacity(h, units)) return rc;
  }
  // Pipelined: plain folds (no delta tracking, no exchange layout, not profiling) may
  // overlap the previous fold. Union is associative and commutative, so the forest
  // after both is the same; readers join the lanes.
  const bool pipe = fs.allow_pipe && h->pipe_depth > 1 && (!track || fs.pipe_tracked) && fs.rows == 0 &&
                    !h->profiling && !h->changes;
  const bool on_lane = fs.lane >= 0 && !h->profiling;
  // remote rows of a group exchange: on the side stream, overlapping own folds
  const bool side = fs.on_side && side_ok(h) && !track;
  if (!pipe && !side && !on_lane) {
    if (int rc = join_pipe_lanes(h)) return rc;  // the side stream is NOT joined: union commutes
  }
  const bool sign = h->kind == GS_KIND_SIGNED;
  for (size_t off = 0, c = 0; off < n; off += c) {
    const bool head = young_head && off == 0;
    c = head ? ((size_t)1 << young_head_log2) : std::min<size_t>(kMaxChunk, n - off);
    const uint32_t blocks = (uint32_t)((c + gs::kFoldBS - 1) / gs::kFoldBS);
    if (track && !fs.take_out) h->delta_fill_ub[h->dset] += per_shard_edges(c);  // (a fused take bypasses the set)
    hipStream_t st = side ? h->side : h->stream;
    if (side) h->side_dirty = true;
    if (head) {
      if (int rc = join_pipe_lanes(h)) return rc;  // (idle after a reset)
    } else if (pipe) {  // the lane waits for the caller's work on the handle stream, not for the other lane
      st = h->lane[h->lane_next];
      h->last_lane = h->lane_next;
      h->lane_next = (h->lane_next + 1) % h->pipe_depth;
      // An idle handle stream has nothing to order behind: no marker. (With 4 hardware
      // queues a lane can share one with the handle stream, and a marker recorded there
      // waits behind that lane's fold: every fold would then wait for the previous one.)
      GS_HIP(hipEventRecord(h->main_ev, h->stream));
      if (hipEventQuery(h->main_ev) != hipSuccess) GS_HIP(hipStreamWaitEvent(st, h->main_ev, 0));
      h->lanes_dirty = true;
    } else if (on_lane) {  // the caller ordered the lane (a group's own fold)
      st = h->lane[fs.lane];
      h->last_lane = fs.lane;
      h->lanes_dirty = true;
    }
    gs::FoldLaunch f;
    f.src = src + off * stride;
    f.dst = dst + off * stride;
    f.w = w ? w + off * w_stride : nullptr;
    f.n = c;
    f.stride = (uint32_t)stride;
    f.w_stride = (uint32_t)w_stride;
    if (h->dedup && !w && stride == 1 && fs.rows == 0 && !fs.n_dev) {
      // micro-batch dedup on the fold's own stream: exact repeats of a pair in this
      // chunk are marked skip (w bit 7) before the fold reads them
      int set = 0;
      if (st == h->side) set = gs_summary::kDedupSets - 1;
      for (int li = 0; li < gs_summary::kLanes; ++li)
        if (st == h->lane[li]) set = 1 + li;
      if (h->dd_edges[set] < c) {
        GS_HIP(hipStreamSynchronize(st));  // the set's previous user is done
        (void)dfree(h->dd_tab[set]);
        (void)dfree(h->dd_w[set]);
        h->dd_tab[set] = nullptr;
        h->dd_w[set] = nullptr;
        const uint64_t e = next_pow2(c);
        GS_HIP(dmalloc(&h->dd_tab[set], 2 * e * 16));
        GS_HIP(dmalloc(&h->dd_w[set], e));
        h->dd_edges[set] = e;
      }
      const uint64_t slots = 2 * next_pow2(c);  // load factor <= 1/2
      GS_HIP(hipMemsetAsync(h->dd_tab[set], 0xFF, slots * 16, st));
      gs::launch_dedup(f.src, f.dst, c, h->dd_tab[set], (uint32_t)(slots - 1), h->dd_w[set], st);
      GS_HIP(hipGetLastError());
      f.w = h->dd_w[set];
      f.w_stride = 1;
    }
    f.rows = fs.rows;
    f.skip_rank = fs.skip_rank;
    f.counts = fs.counts;
    f.base = (uint32_t)off;
    f.n_dev = fs.n_dev;
    f.fail_in = off == 0 ? fs.fail_in : nullptr;
    f.shard0 = h->shard0;
    if (fs.take_out) {
      f.take_out = fs.take_out;
      f.take_cap = fs.take_cap;
      f.take_count = fs.take_count;
      f.done = h->done_dev;
      // drawn here, after the capacity check: a table rebuild there waits on the same
      // completion word with sequence numbers of its own
      f.seq = *fs.take_seq = ++h->done_seq;
    }
    h->shard0 = (h->shard0 + blocks) & (gs::kShards - 1);
    // Capacity reports. A report may only claim chunks queued before it on ITS stream
    // (handle, lanes, side). Each launch carries the report of the earlier chunks of its
    // stream (report_wave in block 0: no launch of its own -- config 2's folds were each
    // followed by a 4-14 us k_report on their lane); the last chunks of a burst are claimed
    // by the next launch there, or by flush_reports before a capacity wait.
    const int rs = report_stream(h, st);
    const bool carry = check_cap && units && !fs.take_out && !fs.n_dev && h->rep_pending[rs];
    if (carry) {
      f.rep_out = h->rep_dev + (h->rep_seq++ % gs_summary::kRepRing);
      f.rep_claim = h->rep_pending[rs];
      f.rep_epoch = (unsigned)(h->rep_epoch & 7u);
    }
    {
      Prof p(h, KID_FOLD, st);
      gs::launch_fold(sign, track, h->table(), h->delta(), f, st);
    }
    GS_HIP(hipGetLastError());
    if (carry) {
      h->rep_pending_edges -= f.rep_claim;
      h->rep_pending[rs] = 0;
    }
    if (check_cap && units) {
      const uint64_t cu = fs.rows ? (off + c >= n ? units : 0) : c;
      h->rep_pending[rs] += cu;
      h->rep_pending_edges += cu;
      // A counted replay (the row count lives on the device) charges its full capacity: it
      // reports at once, so the bound drops to the real count as soon as it lands instead
      // of carrying phantom vertices. (A fused take is waited for: its caller
      // takes the exact count instead.)
      if (fs.n_dev && !fs.take_out)
        if (int rc = launch_report_now(h, rs, st)) return rc;
    }
  }
  return GS_OK;
}

// Export every (vertex, label, parity) into device arrays; returns the count.
// After a burst of pipelined folds the label pass runs on the lane of the LAST fold queued,
// behind events of the other lanes (and of the handle stream, if it holds work): the lanes
// that finished earlier are passed at once, and the pass follows its lane's last fold with
// no cross-queue wait. On the handle stream it waited for all lanes there (config 2: a
// 13-22 us gap per step before the label pass). Its host wait observes that lane's
// completion signal, so every stream the pass waited for is idle when it returns.
// A reader that ends in a host wait, after a burst of pipelined folds: it runs on the lane of
// the last fold queued, behind events of the other lanes and of the handle stream (*es; *on_lane
// true), else on the handle stream after join_lanes. The host wait then observes that lane's
// completion, so every stream it waited for is idle when it returns (clear lanes_dirty then).
int join_into_last_lane(gs_summary* h, hipStream_t* es, bool* on_lane) {
  if (int rc = server_stop(h)) return rc;
  *es = h->stream;
  *on_lane = h->lanes_dirty && !h->side_dirty && h->last_lane >= 0 && h->lane[h->last_lane] && !h->profiling;
  if (!*on_lane) return join_lanes(h);
  *es = h->lane[h->last_lane];
  for (int i = 0; i < gs_summary::kLanes && h->lane[i]; ++i) {
    if (i == h->last_lane) continue;
    GS_HIP(hipEventRecord(h->lane_ev[i], h->lane[i]));
    GS_HIP(hipStreamWaitEvent(*es, h->lane_ev[i], 0));
  }
  GS_HIP(hipEventRecord(h->main_ev, h->stream));
  if (h->xwait || hipEventQuery(h->main_ev) != hipSuccess) GS_HIP(hipStreamWaitEvent(*es, h->main_ev, 0));
  return GS_OK;
}

int export_device_impl(gs_summary* h, int64_t* v, int64_t* l, uint8_t* p, size_t cap, size_t* n, int part,
                       int nparts) {
  hipStream_t es = h->stream;
  bool on_lane = false;
  if (int rc = join_into_last_lane(h, &es, &on_lane)) return rc;
  if (!h->export_ctr_zero) GS_HIP(hipMemsetAsync(h->ctr + gs::ctr_index(gs::CTR_EXPORT), 0, 4, es));
  h->export_ctr_zero = false;
  {
    Prof pr(h, KID_EXPORT, es);
    if (nparts == 1 && use_vertex_list(h, h->nv_ub))
      gs::launch_export_list(h->table(), v, l, p, cap, h->nv_ub, es);
    else
      gs::launch_export(h->table(), v, l, p, cap, es, part, nparts, h->vlist_ok);
  }
  GS_HIP(hipGetLastError());
  uint64_t cnt = 0;
  const int rc = wait_stream(h, h->ctr + gs::ctr_index(gs::CTR_EXPORT), &cnt, 1, 0, true, es);
  if (rc) {
    if (on_lane) (void)join_lanes(h);  // (the handle stream still orders behind everything)
    return rc;
  }
  h->export_ctr_zero = true;  // cleared behind the read
  if (on_lane) h->lanes_dirty = false;  // every lane and the handle stream's work completed
  // a whole-table export after every queued fold completed counts the vertices exactly: the
  // capacity bound (and the next reset's choice of the listed reset over a table scan) starts
  // from it instead of 2 per edge of the chunks whose reports ride on launches not yet made
  if (nparts == 1) note_exact_count(h, cnt);
  *n = cnt;
  if (cnt > cap) return fail(GS_ERR_TRUNCATED, "output capacity " + std::to_string(cap) + " < " + std::to_string(cnt));
  return GS_OK;
}

int ensure_delta_list(gs_summary* h, uint64_t edges) {
  edges = std::max<uint64_t>(edges, kMaxChunk);
  if (h->drec && edges <= h->delta_edges) return GS_OK;
  uint64_t per = 256;  // slack
  for (uint64_t off = 0; off < edges; off += kMaxChunk) per += per_shard_edges(std::min<uint64_t>(kMaxChunk, edges - off));
  if (per > 0xFFFFFFFFull) return fail(GS_ERR_INVALID, "delta list too large");
  if (h->drec) {
    GS_HIP(hipStreamSynchronize(h->stream));
    (void)dfree(h->drec);
    h->drec = nullptr;
  }
  GS_HIP(dmalloc(&h->drec, (size_t)gs::kDeltaSets * gs::kShards * per * 24));
  h->delta_shard_cap = (uint32_t)per;
  h->delta_edges = edges;
  return GS_OK;
}

int stage_delta(gs_summary* h, int64_t* out, uint64_t cap, int width, unsigned long long* count_out, bool with_fail,
                hipStream_t st, int set) {
  if (!h->drec) return fail(GS_ERR_INVALID, "delta tracking was never enabled");
  st = st ? st : h->stream;
  if (set < 0) set = h->dset;
  {
    Prof p(h, KID_STAGE, st);
    gs::launch_stage(h->table(), h->delta(set), out, cap, width, count_out, with_fail, st);
  }
  GS_HIP(hipGetLastError());
  h->delta_fill_ub[set] = 0;
  return GS_OK;
}

}  // namespace gsi

using namespace gsi;

extern "C" {

const char* gs_last_error(void) { return g_err.c_str(); }

int gs_version(void) { return 20000; }

int gs_create(gs_handle* out, int device, int kind, uint64_t capacity_hint) {
  if (!out) return fail(GS_ERR_INVALID, "out is null");
  *out = nullptr;
  if (kind != GS_KIND_CC && kind != GS_KIND_SIGNED) return fail(GS_ERR_INVALID, "unknown kind");
  int ndev = 0;
  GS_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(GS_ERR_HIP, "no HIP device " + std::to_string(device));
  DeviceGuard g(device);
  gs_summary* h = new gs_summary();
  h->device = device;
  h->kind = kind;
  const uint64_t cap = create_capacity(capacity_hint);
  auto bail = [&](int code) {
    gs_destroy(h);
    return code;
  };
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
    return bail(fail(GS_ERR_HIP, "hipStreamCreate failed"));
  if (dmalloc(&h->ctr, gs::CTR_COUNT * gs::kCtrStride * 4) != hipSuccess)
    return bail(fail(GS_ERR_HIP, "hipMalloc(counters) failed"));
  if (dmalloc(&h->d_scratch, 64) != hipSuccess) return bail(fail(GS_ERR_HIP, "hipMalloc(scratch) failed"));
  if (hipHostMalloc(&h->h_flags, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hflags_dev), h->h_flags, 0) != hipSuccess)
    return bail(fail(GS_ERR_HIP, "hipHostMalloc(flags) failed"));
  memset(h->h_flags, 0, 64);
  h->h_done = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(h->h_flags) + 32);
  h->done_dev = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(h->hflags_dev) + 32);
  for (int i = 0; i < 2; ++i)
    if (hipEventCreateWithFlags(&h->stage_ev[i], hipEventDisableTiming) != hipSuccess)
      return bail(fail(GS_ERR_HIP, "hipEventCreate failed"));
  if (hipEventCreateWithFlags(&h->main_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ext_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->idle_ev, hipEventDisableTiming) != hipSuccess)
    return bail(fail(GS_ERR_HIP, "hipEventCreate failed"));
  memset(h->h_flags, 0, 16);
  if (hipHostMalloc(&h->rep, gs_summary::kRepRing * 8, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&h->rep_dev), h->rep, 0) != hipSuccess)
    return bail(fail(GS_ERR_HIP, "capacity report buffer allocation failed"));
  memset(h->rep, 0, gs_summary::kRepRing * 8);
  if (int rc = alloc_table(h, cap)) return bail(rc);
  if (hipStreamSynchronize(h->stream) != hipSuccess) return bail(fail(GS_ERR_HIP, "init failed"));
  *out = h;
  return GS_OK;
}

int gs_destroy(gs_handle h) {
  if (!h) return GS_OK;
  DeviceGuard g(h->device);
  (void)join_lanes(h);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  drain_profile(h);
  for (int i = 0; i < gs_summary::kLanes; ++i) {
    if (h->lane_ev[i]) (void)hipEventDestroy(h->lane_ev[i]);
    if (h->lane[i]) (void)hipStreamDestroy(h->lane[i]);
  }
  if (h->main_ev) (void)hipEventDestroy(h->main_ev);
  if (h->ext_ev) (void)hipEventDestroy(h->ext_ev);
  if (h->idle_ev) (void)hipEventDestroy(h->idle_ev);
  for (int i = 0; i < gs_summary::kDedupSets; ++i) {
    (void)dfree(h->dd_tab[i]);
    (void)dfree(h->dd_w[i]);
  }
  if (h->srv_box) (void)hipHostFree(h->srv_box);
  if (h->srv_bc) (void)dfree(h->srv_bc);
  for (auto e : h->ev_pool) (void)hipEventDestroy(e);
  for (int i = 0; i < 2; ++i) {
    if (h->stage_ev[i]) (void)hipEventDestroy(h->stage_ev[i]);
    if (h->text_ev[i]) (void)hipEventDestroy(h->text_ev[i]);
  }
  if (h->x_ready) (void)hipEventDestroy(h->x_ready);
  if (h->x_used) (void)hipEventDestroy(h->x_used);
  if (h->rep) (void)hipHostFree(h->rep);
  if (h->h_flags) (void)hipHostFree(h->h_flags);
  if (h->h_stage) (void)hipHostFree(h->h_stage);
  if (h->h_wstage) (void)hipHostFree(h->h_wstage);
  if (h->h_text) (void)hipHostFree(h->h_text);
  if (h->h_tres) (void)hipHostFree(h->h_tres);
  for (void* p : {(void*)h->d_text, (void*)h->d_tsrc, (void*)h->d_tdst, h->d_tscratch, (void*)h->tab, (void*)h->ctr,
                  (void*)h->vlist, (void*)h->drec, (void*)h->nxt, (void*)h->chg_scratch, (void*)h->chg_ov,
                  (void*)h->chg_ol, (void*)h->chg_op, (void*)h->d_stage,
                  (void*)h->d_wstage, (void*)h->d_scratch, (void*)h->x_v, (void*)h->x_l, (void*)h->x_p,
                  (void*)h->x_cnt})
    (void)dfree(p);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return GS_OK;
}

int gs_reset(gs_handle h) {
  if (int rc = check(h)) return rc;
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  const bool by_list = use_vertex_list(h, h->nv_ub);
  // the member lists are restored with the slots only while change tracking keeps them sized
  // for this table (they outlive tracking and a rebuild leaves them smaller than the table)
  const bool nxt_ok = h->changes && h->nxt && h->nxt_slots == h->cap + 1;
  {
    Prof p(h, KID_INIT);
    if (by_list) {  // O(vertices): only the touched slots (no host sync); its last block zeroes the counters
      gs::launch_reset_list(h->table(), nxt_ok ? h->nxt : nullptr, h->nv_ub, h->stream);
    } else {
      gs::launch_init(h->tab, h->cap + 1, h->stream, h->ctr);  // (its block 0 zeroes the counters)
    }
  }
  GS_HIP(hipGetLastError());
  if (int rc = change_tracking_reset(h, by_list && nxt_ok ? 0 : 1)) return rc;
  h->export_ctr_zero = true;
  // host mirror: a flag a fold queued before this reset raises later is an error of
  // that fold's epoch and surfaces at the next check
  memset(h->h_flags, 0, 16);
  h->vlist_ok = true;
  reset_capacity_tracking(h, 0);
  for (uint64_t& f : h->delta_fill_ub) f = 0;
  return GS_OK;
}

int gs_reset_config(gs_handle h) {
  if (int rc = check(h)) return rc;
  if (h->side) return fail(GS_ERR_INVALID, "the summary belongs to an exchange group: destroy the group first");
  DeviceGuard g(h->device);
  if (int rc = join_lanes(h)) return rc;
  if (h->changes)
    if (int rc = gs_set_change_tracking(h, 0)) return rc;
  if (h->track)
    if (int rc = gs_set_delta_tracking(h, 0)) return rc;
  h->changes_own_track = false;
  if (h->profiling)
    if (int rc = gs_set_profiling(h, 0)) return rc;
  h->srv_on = false;
  h->dedup = false;
  h->pipe_depth = 1;
  h->lane_next = 0;
  return gs_reset(h);
}

// Host edges, in chunks of up to 2^20 edges into a device staging buffer (two,
// alternating), then folded:
//  * a chunk of at most kDirectCopyEdges is copied by HIP straight from the caller's
//    buffer (no host-side memcpy): `--workload dropin` p = 8 (2^17-edge flushes)
//    59-62 (pinned staging) -> 78-81 M edges/s;
//  * a larger chunk is memcpy'd into pinned staging and copied by DMA. HIP's own
//    pageable path blocked the caller for 8-28 ms per 2^20-edge flush of the drop-in
//    operators (instrumented: all of it inside hipMemcpyAsync): p = 1 34-44 M edges/s
//    with direct copies of every size, 70-73 with this split (same box, tools/dropin_ab.sh).
//    Isolated 2^20-edge calls into an otherwise idle handle (tools/host_fold_rate.py) do
//    better with direct copies (2.63 vs 1.85-1.96 G edges/s); the operators' pattern wins.
// gs_fold's contract -- the caller may reuse its buffers when the call returns -- holds
// either way: the pinned path has copied them, and the direct path waits at the end for
// the last chunk's copies (pageable copies have consumed their source on return).
constexpr size_t kDirectCopyEdges = 1u << 18;

// Host memory HIP can DMA from as it is (hipHostMalloc'ed or hipHostRegister'ed): such a
// caller's chunks of every size are copied straight from its buffer, with no host memcpy
// into the staging buffer (the secondary, PCIe-inclusive figure of bench.py's headline
// line folds from pinned memory).
static bool host_pinned(const void* p) {
  if (!p) return true;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: not an error of this call
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

static int ensure_host_stage(gs_summary* h) {
  if (h->h_stage) return GS_OK;
  GS_HIP(hipHostMalloc(&h->h_stage, sizeof(int64_t) * 4 * kStageChunk, hipHostMallocDefault));
  GS_HIP(hipHostMalloc(&h->h_wstage, 2 * kStageChunk, hipHostMallocDefault));
  return GS_OK;
}

// The device staging buffers (two, alternating) come with the first host fold, sized for
// its chunks (a power of two, 4 K .. 2^20 edges), and grow with a larger one: a handle of
// the JNI pool whose flushes are small does not hold 34 MB of staging (gs_hbm_bytes).
static int ensure_dev_stage(gs_summary* h, size_t edges) {
  if (edges <= h->d_stage_chunk) return GS_OK;
  size_t c = 4096;
  while (c < edges) c <<= 1;
  c = std::min<size_t>(c, kStageChunk);
  if (h->d_stage) {  // folds queued on the stream or the lanes may still read the old buffers
    if (int rc = join_lanes(h)) return rc;
    GS_HIP(hipStreamSynchronize(h->stream));
    (void)dfree(h->d_stage);
    (void)dfree(h->d_wstage);
    h->d_stage = nullptr;
    h->d_wstage = nullptr;
    h->d_stage_chunk = 0;
  }
  GS_HIP(dmalloc(&h->d_stage, sizeof(int64_t) * 4 * c));
  GS_HIP(dmalloc(&h->d_wstage, 2 * c));
  h->d_stage_chunk = c;
  return GS_OK;
}

static int fold_host_impl(gs_handle h, const int64_t* src, const int64_t* dst, const uint8_t* w, size_t n) {
  bool direct_pending = false;
  const bool pinned = n > kDirectCopyEdges && host_pinned(src) && host_pinned(dst) && host_pinned(w);
  if (n) {
    if (int rc = ensure_dev_stage(h, std::min<size_t>(n, kStageChunk))) return rc;
  }
  const size_t sc = h->d_stage_chunk;
  for (size_t off = 0; off < n; off += kStageChunk) {
    const size_t c = std::min<size_t>(kStageChunk, n - off);
    const int b = h->stage_next;
    h->stage_next ^= 1;
    int64_t* ds = h->d_stage + (size_t)b * 2 * sc;
    uint8_t* dwp = w ? h->d_wstage + (size_t)b * sc : nullptr;
    if (c <= kDirectCopyEdges || pinned) {
      GS_HIP(hipMemcpyAsync(ds, src + off, c * 8, hipMemcpyHostToDevice, h->stream));
      GS_HIP(hipMemcpyAsync(ds + sc, dst + off, c * 8, hipMemcpyHostToDevice, h->stream));
      if (w) GS_HIP(hipMemcpyAsync(dwp, w + off, c, hipMemcpyHostToDevice, h->stream));
      direct_pending = true;
    } else {
      if (int rc = ensure_host_stage(h)) return rc;
      GS_HIP(hipEventSynchronize(h->stage_ev[b]));  // the pinned buffer's previous copy is done
      int64_t* hs = h->h_stage + (size_t)b * 2 * kStageChunk;
      memcpy(hs, src + off, c * 8);
      memcpy(hs + kStageChunk, dst + off, c * 8);
      GS_HIP(hipMemcpyAsync(ds, hs, c * 8, hipMemcpyHostToDevice, h->stream));
      GS_HIP(hipMemcpyAsync(ds + sc, hs + kStageChunk, c * 8, hipMemcpyHostToDevice, h->stream));
      if (w) {
        uint8_t* hw = h->h_wstage + (size_t)b * kStageChunk;
        memcpy(hw, w + off, c);
        GS_HIP(hipMemcpyAsync(dwp, hw, c, hipMemcpyHostToDevice, h->stream));
      }
      direct_pending = false;
    }
    GS_HIP(hipEventRecord(h->stage_ev[b], h->stream));  // this chunk's copies
    int rc = fold_device_impl(h, ds, ds + sc, dwp, c, 1, 1, h->track);
    if (rc) return rc;
  }
  // a direct chunk reads the caller's buffer until its copies are done: the last chunk's
  // event covers every earlier copy of the call (one stream). (Unpinned callers: only the
  // last chunk can be direct, every earlier one has kStageChunk > kDirectCopyEdges edges.)
  static_assert(kStageChunk > kDirectCopyEdges, "unpinned direct copies only for a call's last chunk");
  if (direct_pending) GS_HIP(hipEventSynchronize(h->stage_ev[h->stage_next ^ 1]));
  return GS_OK;
}

int gs_fold(gs_handle h, const int64_t* src, const int64_t* dst, size_t n) {
  if (int rc = check(h)) return rc;
  if (n && (!src || !dst)) return fail(GS_ERR_INVALID, "null edge arrays");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  return fold_host_impl(h, src, dst, nullptr, n);
}

int gs_fold_parity(gs_handle h, const int64_t* src, const int64_t* dst, const uint8_t* w, size_t n) {
  if (int rc = check(h)) return rc;
  if (n && (!src || !dst || !w)) return fail(GS_ERR_INVALID, "null edge arrays");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  return fold_host_impl(h, src, dst, w, n);
}

int gs_fold_device(gs_handle h, const int64_t* src, const int64_t* dst, const uint8_t* w, size_t n, size_t stride) {
  if (int rc = check(h)) return rc;
  if (n && (!src || !dst)) return fail(GS_ERR_INVALID, "null edge arrays");
  if (stride == 0) return fail(GS_ERR_INVALID, "stride must be >= 1");
  DeviceGuard g(h->device);
  FoldSource fs;
  fs.allow_pipe = true;
  return fold_device_impl(h, src, dst, w, n, stride, 1, h->track, true, fs);
}

// Cross-stream ordering for producers on other streams: every
// later fold of the handle starts behind the producer's work. Folds run on the handle
// stream, on pipelining lanes that wait for an event recorded on the handle stream at
// each fold, or on a group's own-fold lanes that do the same at each call -- so one
// wait on the handle stream orders all of them.
//
// A running window server folds every posted window at once, whatever is queued on the
// handle stream: a wait stops it first, so the next window starts a new
// server launch queued behind the wait.
int gs_wait_event(gs_handle h, void* event) {
  if (int rc = check(h)) return rc;
  if (!event) return fail(GS_ERR_INVALID, "null event");
  DeviceGuard g(h->device);
  if (int rc = server_stop(h)) return rc;
  GS_HIP(hipStreamWaitEvent(h->stream, static_cast<hipEvent_t>(event), 0));
  // the lanes wait for the producer themselves: a pipelined fold must not rely on a marker of
  // the handle stream to carry this wait (see xwait)
  for (int i = 0; i < gs_summary::kLanes && h->lane[i]; ++i)
    GS_HIP(hipStreamWaitEvent(h->lane[i], static_cast<hipEvent_t>(event), 0));
  h->xwait = true;
  return GS_OK;
}

int gs_wait_stream(gs_handle h, void* stream) {
  if (int rc = check(h)) return rc;
  DeviceGuard g(h->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (st == h->stream) return GS_OK;
  if (int rc = server_stop(h)) return rc;
  GS_HIP(hipEventRecord(h->ext_ev, st));  // (stream 0 = the device's null stream)
  GS_HIP(hipStreamWaitEvent(h->stream, h->ext_ev, 0));
  for (int i = 0; i < gs_summary::kLanes && h->lane[i]; ++i) GS_HIP(hipStreamWaitEvent(h->lane[i], h->ext_ev, 0));
  h->xwait = true;
  return GS_OK;
}

int gs_fold_device_after(gs_handle h, const int64_t* src, const int64_t* dst, const uint8_t* w, size_t n,
                         size_t stride, void* ready) {
  if (int rc = check(h)) return rc;
  if (ready)
    if (int rc = gs_wait_event(h, ready)) return rc;
  return gs_fold_device(h, src, dst, w, n, stride);
}

int gs_fold_records_device(gs_handle h, const int64_t* rec, size_t n, int track) {
  if (int rc = check(h)) return rc;
  // n may be a take's count word: bit 62 carries a failed signed verdict, which the
  // replay ANDs into this summary before folding the rows (Candidates.merge :79-81)
  const bool failed = (n & gs::kFailBit) != 0;
  n &= gs::kFailBit - 1;
  if (n && !rec) return fail(GS_ERR_INVALID, "null records");
  if (track && !h->drec) return fail(GS_ERR_INVALID, "delta tracking was never enabled");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  if (failed && h->kind == GS_KIND_SIGNED)
    GS_HIP(hipMemsetAsync(h->ctr + gs::ctr_index(gs::CTR_FAIL), 1, 1, h->stream));
  return fold_device_impl(h, rec, rec + 1, reinterpret_cast<const uint8_t*>(rec + 2), n, 3, 24, track != 0);
}

int gs_fold_records_counted_device(gs_handle h, const int64_t* rec, size_t cap, const uint64_t* count_dev, int track) {
  if (int rc = check(h)) return rc;
  if (!count_dev || (cap && !rec)) return fail(GS_ERR_INVALID, "null argument");
  if (track && !h->drec) return fail(GS_ERR_INVALID, "delta tracking was never enabled");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  FoldSource fs;
  fs.n_dev = reinterpret_cast<const unsigned long long*>(count_dev);  // rows (<= cap) and the verdict bit
  // at least one thread reads the verdict of a failed window with no rows
  const size_t n = std::max<size_t>(cap, h->kind == GS_KIND_SIGNED ? 1 : 0);
  return fold_device_impl(h, rec, rec + 1, reinterpret_cast<const uint8_t*>(rec + 2), n, 3, 24, track != 0, true, fs);
}

int gs_sync(gs_handle h) {
  if (int rc = check(h)) return rc;
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  return check_device_flags(h);  // its one stream sync completes all queued work
}

int gs_num_vertices(gs_handle h, uint64_t* n) {
  if (int rc = check(h)) return rc;
  if (!n) return fail(GS_ERR_INVALID, "n is null");
  DeviceGuard g(h->device);
  int rc = read_nv(h, n);
  if (rc) return rc;
  return check_flags_now(h);  // read_nv waited for the stream
}

int gs_find(gs_handle h, int64_t v, int64_t* label, int* found) {
  if (int rc = check(h)) return rc;
  if (!label || !found) return fail(GS_ERR_INVALID, "null output");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  gs::launch_find_one(h->table(), v, h->d_scratch, h->stream);
  GS_HIP(hipGetLastError());
  int64_t out[2];
  GS_HIP(hipMemcpyAsync(out, h->d_scratch, 16, hipMemcpyDeviceToHost, h->stream));
  GS_HIP(hipStreamSynchronize(h->stream));
  *found = (int)out[0];
  *label = out[1];
  return GS_OK;
}

int gs_find_labels_device(gs_handle h, const int64_t* v, size_t n, int64_t* label, uint8_t* found) {
  if (int rc = check(h)) return rc;
  if (n && (!v || !label)) return fail(GS_ERR_INVALID, "null arrays");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  if (!n) return GS_OK;
  gs::launch_find_batch(h->table(), v, n, label, found, nullptr, h->stream);
  GS_HIP(hipGetLastError());
  return GS_OK;
}

int gs_digest(gs_handle h, uint64_t* digest) {
  if (int rc = check(h)) return rc;
  if (!digest) return fail(GS_ERR_INVALID, "digest is null");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  unsigned long long* d = reinterpret_cast<unsigned long long*>(h->d_scratch);
  uint32_t failed = 0;
  GS_HIP(hipMemsetAsync(d, 0, 8, h->stream));
  gs::launch_digest(h->table(), d, std::min<uint64_t>(h->nv_ub, h->cap + 1), h->stream);
  GS_HIP(hipGetLastError());
  unsigned long long out = 0;
  GS_HIP(hipMemcpyAsync(&out, d, 8, hipMemcpyDeviceToHost, h->stream));
  GS_HIP(hipMemcpyAsync(&failed, h->ctr + gs::ctr_index(gs::CTR_FAIL), 4, hipMemcpyDeviceToHost, h->stream));
  GS_HIP(hipStreamSynchronize(h->stream));
  if (int rc = check_flags_now(h)) return rc;
  *digest = (h->kind == GS_KIND_SIGNED && failed) ? GS_DIGEST_FAILED : out;
  return GS_OK;
}

int gs_export_labels_device(gs_handle h, int64_t* v, int64_t* label, uint8_t* parity, size_t cap, size_t* n) {
  if (int rc = check(h)) return rc;
  if (!n) return fail(GS_ERR_INVALID, "n is null");
  DeviceGuard g(h->device);
  return export_device_impl(h, v, label, parity, cap, n);
}

int gs_export_labels_part_device(gs_handle h, int part, int nparts, int64_t* v, int64_t* label, uint8_t* parity,
                                 size_t cap, size_t* n) {
  if (int rc = check(h)) return rc;
  if (!n) return fail(GS_ERR_INVALID, "n is null");
  if (nparts < 1 || part < 0 || part >= nparts) return fail(GS_ERR_INVALID, "bad part");
  DeviceGuard g(h->device);
  return export_device_impl(h, v, label, parity, cap, n, part, nparts);
}

// Export to host arrays through the combine scratch (no allocation per call).
static int export_host(gs_handle h, int64_t* v, int64_t* l, uint8_t* p, size_t cap, size_t* n) {
  uint64_t nv = 0;
  int rc = read_nv(h, &nv);
  if (rc) return rc;
  *n = nv;
  if (cap < nv) return fail(GS_ERR_TRUNCATED, "output capacity " + std::to_string(cap) + " < " + std::to_string(nv));
  if (nv == 0) return GS_OK;
  if ((rc = ensure_x(h, nv + 1))) return rc;
  if ((rc = wait_x_consumer(h))) return rc;
  size_t got = 0;
  rc = export_device_impl(h, h->x_v, h->x_l, h->x_p, h->x_cap, &got);
  if (rc) return rc;
  if (v) GS_HIP(hipMemcpyAsync(v, h->x_v, got * 8, hipMemcpyDeviceToHost, h->stream));
  if (l) GS_HIP(hipMemcpyAsync(l, h->x_l, got * 8, hipMemcpyDeviceToHost, h->stream));
  if (p) GS_HIP(hipMemcpyAsync(p, h->x_p, got, hipMemcpyDeviceToHost, h->stream));
  GS_HIP(hipStreamSynchronize(h->stream));
  *n = got;
  return GS_OK;
}

int gs_export_labels(gs_handle h, int64_t* v, int64_t* label, size_t cap, size_t* n) {
  if (int rc = check(h)) return rc;
  if (!n) return fail(GS_ERR_INVALID, "n is null");
  DeviceGuard g(h->device);
  return export_host(h, v, label, nullptr, cap, n);
}

int gs_bip_status(gs_handle h, int* ok) {
  if (int rc = check(h)) return rc;
  if (!ok) return fail(GS_ERR_INVALID, "ok is null");
  DeviceGuard g(h->device);
  // the verdict handed to the host with the completion word (k_signal): no device-to-host
  // copy and no hipStreamSynchronize wake-up (config 4 reads it at the end of every step), on
  // the last fold's lane (no cross-queue join before it: 14-22 us of config 4's step)
  hipStream_t es = h->stream;
  bool on_lane = false;
  if (int rc = join_into_last_lane(h, &es, &on_lane)) return rc;
  // With it, the exact vertex count (every queued fold has completed when the host sees the
  // word): the next reset walks the vertex list instead of scanning a slack-sized table
  // (config 4: 2^24 slots, 42 us, for 2^20 vertices)
  uint64_t w = 0;
  const int rc = wait_stream(h, h->ctr + gs::ctr_index(gs::CTR_NV), &w, gs::kShards, gs::kCtrStride, false, es,
                             h->ctr + gs::ctr_index(gs::CTR_FAIL));
  if (rc) {
    if (on_lane) (void)join_lanes(h);
    return rc;
  }
  if (on_lane) h->lanes_dirty = false;  // every lane and the handle stream's work completed
  if (!h->side_dirty && !h->lanes_dirty) note_exact_count(h, w & ((1ull << 47) - 1));
  *ok = (w & gs::kSignalFlagBit) ? 0 : 1;
  return GS_OK;
}

int gs_export_colouring(gs_handle h, int64_t* comp, int64_t* v, uint8_t* sign, size_t cap, size_t* n) {
  if (int rc = check(h)) return rc;
  if (!n) return fail(GS_ERR_INVALID, "n is null");
  int ok = 1;
  int rc = gs_bip_status(h, &ok);
  if (rc) return rc;
  if (!ok) {
    *n = 0;
    return GS_OK;
  }
  DeviceGuard g(h->device);
  rc = export_host(h, v, comp, sign, cap, n);
  if (rc) return rc;
  if (sign)
    for (size_t i = 0; i < *n; ++i) sign[i] = sign[i] ? 0 : 1;  // parity 0 <=> same colour as the minimum
  return GS_OK;
}

// CombineCC.reduce / combineFunction.reduce: export `src` into its own scratch on
// its stream (O(vertices) over the vertex list of a sparse table), then fold those
// rows into `dst` on dst's stream behind an event. The fold reads the exported
// count and src's verdict on the device: no host synchronisation and no allocation
// once the scratch is sized.
int gs_combine(gs_handle dst, gs_handle src) {
  if (int rc = check(dst)) return rc;
  if (int rc = check(src)) return rc;
  if (dst == src) return GS_OK;
  if (dst->kind != src->kind) return fail(GS_ERR_INVALID, "summaries of different kinds");
  const bool sign = dst->kind == GS_KIND_SIGNED;
  uint64_t bound = 0;
  {
    DeviceGuard g(src->device);
    if (int rc = join_lanes(src)) return rc;
    bound = std::min<uint64_t>(src->nv_ub, src->cap + 1);
    if (int rc = ensure_x(src, bound + 1)) return rc;
    if (int rc = wait_x_consumer(src)) return rc;
    if (!src->export_ctr_zero) GS_HIP(hipMemsetAsync(src->ctr + gs::ctr_index(gs::CTR_EXPORT), 0, 4, src->stream));
    src->export_ctr_zero = false;  // (the count stays behind for the copy below)
    GS_HIP(hipMemsetAsync(src->x_cnt, 0, 16, src->stream));
    {
      Prof pr(src, KID_EXPORT);
      if (use_vertex_list(src, bound))
        gs::launch_export_list(src->table(), src->x_v, src->x_l, src->x_p, src->x_cap, bound, src->stream);
      else
        gs::launch_export(src->table(), src->x_v, src->x_l, src->x_p, src->x_cap, src->stream, 0, 1, src->vlist_ok);
    }
    GS_HIP(hipGetLastError());
    GS_HIP(hipMemcpyAsync(src->x_cnt, src->ctr + gs::ctr_index(gs::CTR_EXPORT), 4, hipMemcpyDeviceToDevice,
                          src->stream));
    GS_HIP(hipMemcpyAsync(src->x_cnt + 1, src->ctr + gs::ctr_index(gs::CTR_FAIL), 4, hipMemcpyDeviceToDevice,
                          src->stream));
    GS_HIP(hipEventRecord(src->x_ready, src->stream));
  }
  DeviceGuard g(dst->device);
  if (int rc = join_lanes(dst)) return rc;
  GS_HIP(hipStreamWaitEvent(dst->stream, src->x_ready, 0));
  gs_summary* rows = src;
  if (dst->device != src->device) {  // rows to dst's own scratch over xGMI
    if (int rc = ensure_x(dst, bound + 1)) return rc;
    if (int rc = wait_x_consumer(dst)) return rc;
    GS_HIP(hipMemcpyPeerAsync(dst->x_cnt, dst->device, src->x_cnt, src->device, 16, dst->stream));
    if (bound) {
      GS_HIP(hipMemcpyPeerAsync(dst->x_v, dst->device, src->x_v, src->device, bound * 8, dst->stream));
      GS_HIP(hipMemcpyPeerAsync(dst->x_l, dst->device, src->x_l, src->device, bound * 8, dst->stream));
      GS_HIP(hipMemcpyPeerAsync(dst->x_p, dst->device, src->x_p, src->device, bound, dst->stream));
    }
    GS_HIP(hipEventRecord(src->x_used, dst->stream));  // src's scratch is free again
    src->x_pending = true;
    rows = dst;
  }
  FoldSource fs;
  fs.n_dev = rows->x_cnt;
  fs.fail_in = sign ? reinterpret_cast<const uint32_t*>(rows->x_cnt + 1) : nullptr;
  // at least one thread reads the verdict of an empty failed summary (Candidates(false))
  const size_t n = std::max<uint64_t>(bound, sign ? 1 : 0);
  if (int rc = fold_device_impl(dst, rows->x_v, rows->x_l, rows->x_p, n, 1, 1, dst->track, true, fs)) return rc;
  GS_HIP(hipEventRecord(rows->x_used, dst->stream));
  rows->x_pending = true;
  return GS_OK;
}

int gs_combine_exported_device(gs_handle h, const int64_t* v, const int64_t* label, const uint8_t* parity, size_t n,
                               int failed) {
  if (int rc = check(h)) return rc;
  if (n && (!v || !label)) return fail(GS_ERR_INVALID, "null arrays");
  if (n && h->kind == GS_KIND_SIGNED && !parity) return fail(GS_ERR_INVALID, "a signed summary needs parity");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  if (failed) {  // the verdict is the AND (BipartitenessCheck.combineFunction -> Candidates.merge :79-81)
    GS_HIP(hipMemsetAsync(h->ctr + gs::ctr_index(gs::CTR_FAIL), 1, 1, h->stream));
    return GS_OK;
  }
  return fold_device_impl(h, v, label, parity, n, 1, 1, h->track);
}

// Serialized image: u32 magic 'GSS1', u32 kind, u32 ok, u32 0, u64 n, int64 v[n], int64 label[n], u8 parity[n]
int gs_serialize(gs_handle h, void* buf, size_t cap, size_t* len) {
  if (int rc = check(h)) return rc;
  if (!len) return fail(GS_ERR_INVALID, "len is null");
  DeviceGuard g(h->device);
  uint64_t nv = 0;
  int rc = read_nv(h, &nv);
  if (rc) return rc;
  const size_t need = 24 + nv * 17;
  *len = need;
  if (!buf) return GS_OK;
  if (cap < need) return fail(GS_ERR_TRUNCATED, "buffer too small");
  int ok = 1;
  rc = gs_bip_status(h, &ok);
  if (rc) return rc;
  uint8_t* b = static_cast<uint8_t*>(buf);
  std::vector<int64_t> v(nv), l(nv);
  std::vector<uint8_t> p(nv);
  size_t got = 0;
  if (nv) {
    rc = export_host(h, v.data(), l.data(), p.data(), nv, &got);
    if (rc) return rc;
  }
  const uint32_t hdr[4] = {0x31535347u, (uint32_t)h->kind, (uint32_t)ok, 0u};
  const uint64_t n64 = got;
  memcpy(b, hdr, 16);
  memcpy(b + 16, &n64, 8);
  memcpy(b + 24, v.data(), got * 8);
  memcpy(b + 24 + got * 8, l.data(), got * 8);
  memcpy(b + 24 + got * 16, p.data(), got);
  *len = 24 + got * 17;
  return GS_OK;
}

int gs_deserialize(gs_handle h, const void* buf, size_t len) {
  if (int rc = check(h)) return rc;
  if (!buf || len < 24) return fail(GS_ERR_INVALID, "truncated image");
  const uint8_t* b = static_cast<const uint8_t*>(buf);
  uint32_t hdr[4];
  uint64_t n = 0;
  memcpy(hdr, b, 16);
  memcpy(&n, b + 16, 8);
  if (hdr[0] != 0x31535347u) return fail(GS_ERR_INVALID, "bad magic");
  if ((int)hdr[1] != h->kind) return fail(GS_ERR_INVALID, "image of a different summary kind");
  if (len < 24 + n * 17) return fail(GS_ERR_INVALID, "truncated image");
  int rc = gs_reset(h);
  if (rc) return rc;
  DeviceGuard g(h->device);
  if (!hdr[2]) {
    GS_HIP(hipMemsetAsync(h->ctr + gs::ctr_index(gs::CTR_FAIL), 1, 1, h->stream));
    return gs_sync(h);
  }
  const int64_t* v = reinterpret_cast<const int64_t*>(b + 24);
  std::vector<int64_t> vv(v, v + n), ll(n);
  memcpy(ll.data(), b + 24 + n * 8, n * 8);
  rc = fold_host_impl(h, vv.data(), ll.data(), b + 24 + n * 16, n);
  if (rc) return rc;
  return gs_sync(h);
}

int gs_set_delta_tracking(gs_handle h, int on) {
  if (int rc = check(h)) return rc;
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  if (on)
    if (int rc = ensure_delta_list(h, kMaxChunk)) return rc;
  GS_HIP(hipMemsetAsync(h->ctr + gs::ctr_index(gs::CTR_DELTA), 0,
                        (size_t)gs::kDeltaSets * gs::kShards * gs::kCtrStride * 4, h->stream));
  for (uint64_t& f : h->delta_fill_ub) f = 0;
  h->dset = 0;
  h->track = on != 0;
  return GS_OK;
}

int gs_delta_capacity(gs_handle h, uint64_t* rows) {
  if (int rc = check(h)) return rc;
  if (!rows) return fail(GS_ERR_INVALID, "rows is null");
  *rows = (uint64_t)gs::kShards * h->delta_shard_cap;
  return GS_OK;
}

int gs_take_delta_records(gs_handle h, int64_t* rec, size_t cap, uint64_t* count) {
  if (int rc = check(h)) return rc;
  if (!count) return fail(GS_ERR_INVALID, "count is null");
  if (!h->track) return fail(GS_ERR_INVALID, "delta tracking is off");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  return stage_delta(h, rec, cap, 3, reinterpret_cast<unsigned long long*>(count), h->kind == GS_KIND_SIGNED);
}

// One window through the resident server: post it in the mailbox, spin on the
// completion word. A server that left on its own (idle) before it saw the window is
// started again and the window posted again.
static int server_take(gs_handle h, const int64_t* src, const int64_t* dst, size_t n, int64_t* rec, size_t cap,
                       unsigned long long* cd, uint64_t* count) {
  if (int rc = ensure_capacity(h, n)) return rc;  // (its slow path stops the server)
  const unsigned long long seq = h->srv_seq + 1, dseq = ++h->done_seq;
  for (int attempt = 0;; ++attempt) {
    if (!h->srv_running)
      if (int rc = server_start(h)) return rc;
    // the descriptor words tagged with seq (the server reads the whole line in one load
    // round and takes it when every tag matches), then seq itself
    gs::ServerBox* b = h->srv_box;
    b->src = gs::tag_word(seq, (unsigned long long)src);
    b->dst = gs::tag_word(seq, (unsigned long long)dst);
    b->n = gs::tag_word(seq, n);
    b->rec = gs::tag_word(seq, (unsigned long long)rec);
    b->cap = gs::tag_word(seq, std::min<unsigned long long>(cap, 1ull << 40));
    b->cnt = gs::tag_word(seq, (unsigned long long)cd);
    b->done_seq = gs::tag_word(seq, dseq);
    __atomic_store_n(&b->seq, seq, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    bool left = false;
    for (uint32_t i = 1;; ++i) {
      if (__atomic_load_n(h->h_done, __ATOMIC_ACQUIRE) >= dseq) break;
      if (__atomic_load_n(&b->exited, __ATOMIC_ACQUIRE)) {
        if (__atomic_load_n(h->h_done, __ATOMIC_ACQUIRE) >= dseq) break;
        left = true;
        break;
      }
      if ((i & 1023u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5))
        return fail(GS_ERR_HIP, "window server: no completion within 5 s");
      __builtin_ia32_pause();
    }
    if (!left) break;
    h->srv_running = false;
    GS_HIP(hipStreamSynchronize(h->stream));  // join the launch that left
    if (__atomic_load_n(&b->taken, __ATOMIC_ACQUIRE) == seq && __atomic_load_n(h->h_done, __ATOMIC_ACQUIRE) < dseq) {
      // It left INSIDE this window (a workgroup did not become resident within 8 x the
      // idle limit, ~16 ms): some
      // of the window's edges are folded and their rows written, the count word is not.
      // Replaying it would lose those hooks' records, so the window fails; the take
      // counters are cleared so that the handle's next take starts clean.
      GS_HIP(hipMemsetAsync(h->ctr + gs::ctr_index(gs::CTR_TAKE), 0,
                            (size_t)(gs::CTR_COUNT - gs::CTR_TAKE) * gs::kCtrStride * 4, h->stream));
      GS_HIP(hipStreamSynchronize(h->stream));
      return fail(GS_ERR_HIP, "window server left inside window " + std::to_string(seq) +
                                  " (workgroups not co-resident): the summary holds part of it; reset or restore it");
    }
    // it left before this window: start again and post it again
    if (attempt >= 3) return fail(GS_ERR_HIP, "window server: left before the window three times");
  }
  h->srv_seq = seq;
  h->srv_windows++;
  uint64_t nv = 0;
  if (int rc = done_value_read(h, 1, dseq, &nv)) return rc;
  if (int rc = done_value_read(h, 2, dseq, count)) return rc;
  note_exact_count(h, nv);
  return check_flags_now(h);
}

int gs_set_window_server(gs_handle h, int on) {
  if (int rc = check(h)) return rc;
  DeviceGuard g(h->device);
  if (int rc = join_lanes(h)) return rc;  // stops a running server
  if (on && !h->srv_box) {
    GS_HIP(hipHostMalloc(&h->srv_box, sizeof(gs::ServerBox), hipHostMallocMapped | hipHostMallocCoherent));
    GS_HIP(dmalloc(&h->srv_bc, sizeof(gs::ServerBcast)));
    memset(h->srv_box, 0, sizeof(gs::ServerBox));
  }
  h->srv_on = on != 0;
  return GS_OK;
}

int gs_set_batch_dedup(gs_handle h, int on) {
  if (int rc = check(h)) return rc;
  DeviceGuard g(h->device);
  if (int rc = join_lanes(h)) return rc;
  h->dedup = on != 0;
  return GS_OK;
}

int gs_window_server_stats(gs_handle h, uint64_t* launches, uint64_t* windows) {
  if (int rc = check(h)) return rc;
  if (launches) *launches = h->srv_launches;
  if (windows) *windows = h->srv_windows;
  return GS_OK;
}

int gs_fold_take_device(gs_handle h, const int64_t* src, const int64_t* dst, size_t n, int64_t* rec, size_t cap,
                        uint64_t* count_dev, uint64_t* count) {
  if (int rc = check(h)) return rc;
  if (n && (!src || !dst)) return fail(GS_ERR_INVALID, "null edge arrays");
  if (!count_dev || !count || (cap && !rec)) return fail(GS_ERR_INVALID, "null argument");
  if (!h->track) return fail(GS_ERR_INVALID, "delta tracking is off");
  if (h->side) return fail(GS_ERR_INVALID, "a group's summary exchanges its delta: no window take");
  DeviceGuard g(h->device);
  auto* cd = reinterpret_cast<unsigned long long*>(count_dev);
  // the resident server takes a window of at most one launch's worth of edges when
  // nothing else is pending on the handle, on a device where all its workgroups can be
  // resident at once (checked once per handle: a window completes only when every
  // workgroup runs; otherwise the fused launch below)
  if (h->srv_on && h->srv_fits < 0)
    h->srv_fits = gs::window_server_resident_blocks(h->kind == GS_KIND_SIGNED, h->device) >= (int)gs::kServerBlocks;
  if (h->srv_on && h->srv_fits > 0 && n > 0 && n <= gs::kServerMaxEdges && h->delta_fill_ub[h->dset] == 0 && !h->changes &&
      !h->profiling && !h->dedup && !h->lanes_dirty && !h->side_dirty)
    return server_take(h, src, dst, n, rec, cap, cd, count);
  if (int rc_ = join_lanes(h)) return rc_;
  // One launch when the window fits one k_fold launch and nothing else is pending in
  // the delta set (earlier tracked folds' records belong to this take too), and no
  // change emission consumes the records.
  const bool fused = n > 0 && n <= kMaxChunk && h->delta_fill_ub[h->dset] == 0 && !h->changes && !h->profiling;
  if (!fused) {
    if (int rc = fold_device_impl(h, src, dst, nullptr, n, 1, 1, true)) return rc;
    if (int rc = stage_delta(h, rec, cap, 3, cd, h->kind == GS_KIND_SIGNED)) return rc;
    // the whole count word (rows | kFailBit) handed over with the wait
    if (int rc = wait_stream(h, reinterpret_cast<const uint32_t*>(cd), count, -1)) return rc;
    return check_flags_now(h);
  }
  FoldSource fs;
  fs.take_out = rec;
  fs.take_cap = cap;
  fs.take_count = cd;
  unsigned long long seq = 0;
  fs.take_seq = &seq;
  if (int rc = fold_device_impl(h, src, dst, nullptr, n, 1, 1, true, true, fs)) return rc;
  if (int rc = wait_done(h, seq)) return rc;
  uint64_t nv = 0;
  if (int rc = done_value_read(h, 1, seq, &nv)) return rc;
  if (int rc = done_value_read(h, 2, seq, count)) return rc;
  note_exact_count(h, nv);
  return check_flags_now(h);
}

int gs_delta_stage(gs_handle h, int64_t* send, size_t cap, int width, uint64_t* count) {
  if (int rc = check(h)) return rc;
  if (!send || !count) return fail(GS_ERR_INVALID, "null argument");
  if (!h->track) return fail(GS_ERR_INVALID, "delta tracking is off");
  if (width != 2 && width != 3) return fail(GS_ERR_INVALID, "width must be 2 or 3");
  if (cap < (uint64_t)gs::kShards * h->delta_shard_cap)
    return fail(GS_ERR_INVALID, "cap below the delta capacity (gs_delta_capacity)");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  return stage_delta(h, send, cap, width, reinterpret_cast<unsigned long long*>(count),
                     h->kind == GS_KIND_SIGNED);
}

int gs_fold_exchange_device(gs_handle h, const int64_t* recv, const uint64_t* counts, size_t world, size_t rows,
                            int width, int skip_rank) {
  if (int rc = check(h)) return rc;
  if (!recv || !counts || rows == 0 || world == 0) return fail(GS_ERR_INVALID, "empty exchange buffer");
  if (width != 2 && width != 3) return fail(GS_ERR_INVALID, "width must be 2 or 3");
  if (world * rows > 0xFFFFFFFFull) return fail(GS_ERR_INVALID, "exchange buffer too large");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  FoldSource fs;
  fs.rows = (uint32_t)rows;
  fs.skip_rank = skip_rank;
  fs.counts = reinterpret_cast<const unsigned long long*>(counts);
  fs.units = world * rows;  // the counts live on the device: charge every row
  const uint8_t* w = width == 3 ? reinterpret_cast<const uint8_t*>(recv + 2) : nullptr;
  return fold_device_impl(h, recv, recv + 1, w, world * rows, width, 8 * width, /*track=*/false, true, fs);
}

int gs_get_stream(gs_handle h, void** stream) {
  if (int rc = check(h)) return rc;
  if (!stream) return fail(GS_ERR_INVALID, "stream is null");
  {
    DeviceGuard g(h->device);
    if (int rc_ = join_lanes(h)) return rc_;
  }
  *stream = (void*)h->stream;
  return GS_OK;
}

int gs_set_profiling(gs_handle h, int on) {
  if (int rc = check(h)) return rc;
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  (void)hipStreamSynchronize(h->stream);
  drain_profile(h);
  h->profiling = on != 0;
  for (int i = 0; i < KID_N; ++i) {
    h->launches[i] = 0;
    h->total_ms[i] = 0;
  }
  return GS_OK;
}

int gs_kernel_stats(gs_handle h, int id, uint64_t* launches, double* total_ms) {
  if (int rc = check(h)) return rc;
  if (id < 0 || id >= KID_N || !launches || !total_ms) return fail(GS_ERR_INVALID, "bad kernel id");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  drain_profile(h);
  *launches = h->launches[id];
  *total_ms = h->total_ms[id];
  return GS_OK;
}

int gs_counters(gs_handle h, uint64_t* out8) {
  if (int rc = check(h)) return rc;
  if (!out8) return fail(GS_ERR_INVALID, "out is null");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  std::vector<uint32_t> c(gs::CTR_COUNT * gs::kCtrStride);
  GS_HIP(hipMemcpyAsync(c.data(), h->ctr, c.size() * 4, hipMemcpyDeviceToHost, h->stream));
  GS_HIP(hipStreamSynchronize(h->stream));
  uint64_t nv = 0;
  for (int i = 0; i < gs::kShards; ++i) nv += c[gs::ctr_index(gs::CTR_NV + i)];
  auto u64 = [&](int idx) { return (uint64_t)c[gs::ctr_index(idx)] | ((uint64_t)c[gs::ctr_index(idx + 1)] << 32); };
  out8[0] = nv;
  out8[1] = c[gs::ctr_index(gs::CTR_FAIL)];
  out8[2] = c[gs::ctr_index(gs::CTR_ERR)];
  out8[3] = c[gs::ctr_index(gs::CTR_OVF)] | (c[gs::ctr_index(gs::CTR_VOVF)] ? 2u : 0u);
  out8[4] = u64(gs::CTR_SENT);
  out8[5] = c[gs::ctr_index(gs::CTR_DBG_HOOKS)];
  out8[6] = c[gs::ctr_index(gs::CTR_DBG_ITERS)];
  out8[7] = c[gs::ctr_index(gs::CTR_DBG_CASFAIL)];
  return GS_OK;
}

int gs_debug_counters(gs_handle h, uint64_t* out, int n) {
  if (int rc = check(h)) return rc;
  if (!out || n < 0) return fail(GS_ERR_INVALID, "out is null");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  std::vector<uint32_t> c(gs::CTR_COUNT * gs::kCtrStride);
  GS_HIP(hipMemcpyAsync(c.data(), h->ctr, c.size() * 4, hipMemcpyDeviceToHost, h->stream));
  GS_HIP(hipStreamSynchronize(h->stream));
  const int have = gs::CTR_DBG_LAST_ - gs::CTR_DBG_EDGES;
  for (int i = 0; i < n && i < 16; ++i) out[i] = i < have ? c[gs::ctr_index(gs::CTR_DBG_EDGES + i)] : 0;
  return GS_OK;
}

int gs_capacity_stats(gs_handle h, uint64_t* waits, uint64_t* syncs, double* wait_ms) {
  if (int rc = check(h)) return rc;
  if (waits) *waits = h->cap_waits;
  if (syncs) *syncs = h->cap_syncs;
  if (wait_ms) *wait_ms = h->cap_wait_s * 1e3;
  return GS_OK;
}

// ---- text ingest (include/gs_ingest.h) ----
namespace {
constexpr size_t kTextChunk = 16u << 20;  // bytes of text per parse + fold

// Copy into pinned staging with a few threads (one core's memcpy is far below PCIe).
void staged_copy(char* dst, const char* src, size_t n) {
  const int nt = n >= (4u << 20) ? 8 : 1;
  if (nt == 1) {
    memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) {
    const size_t a = n * t / nt, b = n * (t + 1) / nt;
    th.emplace_back([=] { memcpy(dst + a, src + a, b - a); });
  }
  for (auto& x : th) x.join();
}

// End of the chunk that starts at off: after the last '\n' within kTextChunk bytes
// (the whole rest when it fits); 0 = a single line longer than a chunk.
size_t chunk_end(const char* text, size_t len, size_t off) {
  if (len - off <= kTextChunk) return len;
  size_t end = off + kTextChunk;
  while (end > off && text[end - 1] != '\n') --end;
  return end == off ? 0 : end;
}
}  // namespace

int gs_fold_text(gs_handle h, const char* text, size_t len, int sep, uint64_t* n_edges, int64_t* bad_line) {
  if (int rc = check(h)) return rc;
  if (!n_edges || !bad_line || (len && !text)) return fail(GS_ERR_INVALID, "null argument");
  if (sep != GS_SEP_WHITESPACE && sep != GS_SEP_TAB) return fail(GS_ERR_INVALID, "unknown separator");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  *n_edges = 0;
  *bad_line = -1;
  const size_t max_lines = kTextChunk / 2 + 2;  // every line has >= 1 byte + '\n'
  if (!h->h_text) {
    size_t cub = 0;
    const size_t sb = gs::parse_scratch_bytes(kTextChunk, &cub);
    GS_HIP(hipHostMalloc(&h->h_text, 2 * kTextChunk, hipHostMallocDefault));
    GS_HIP(hipHostMalloc(&h->h_tres, 4 * sizeof(uint64_t), hipHostMallocDefault));
    GS_HIP(dmalloc(&h->d_text, 2 * kTextChunk));
    GS_HIP(dmalloc(&h->d_tsrc, max_lines * 8));
    GS_HIP(dmalloc(&h->d_tdst, max_lines * 8));
    GS_HIP(dmalloc(&h->d_tscratch, sb));
    for (int i = 0; i < 2; ++i) GS_HIP(hipEventCreateWithFlags(&h->text_ev[i], hipEventDisableTiming));
    gs::parse_scratch_init(h->tscratch, h->d_tscratch, kTextChunk);
  }
  // Double-buffered: while chunk k is copied to the device, parsed and folded, the
  // host copies chunk k+1 into the other pinned buffer.
  auto enqueue = [&](int b, size_t c) -> int {
    char* dt = h->d_text + (size_t)b * kTextChunk;
    GS_HIP(hipMemcpyAsync(dt, h->h_text + (size_t)b * kTextChunk, c, hipMemcpyHostToDevice, h->stream));
    if (gs::parse_text_enqueue(h->stream, dt, c, sep, h->d_tsrc, h->d_tdst, max_lines, h->tscratch))
      return fail(GS_ERR_HIP, "text parse launch failed");
    GS_HIP(hipMemcpyAsync(h->h_tres + 2 * b, h->tscratch.res, 16, hipMemcpyDeviceToHost, h->stream));
    GS_HIP(hipEventRecord(h->text_ev[b], h->stream));
    return GS_OK;
  };
  if (len == 0) return GS_OK;
  size_t end = chunk_end(text, len, 0);
  if (!end) return fail(GS_ERR_INVALID, "a line is longer than the 16 MiB ingest chunk");
  staged_copy(h->h_text, text, end);
  if (int rc = enqueue(0, end)) return rc;
  uint64_t line0 = 0;
  for (int b = 0;; b ^= 1) {
    // host: the next chunk into the other pinned buffer (its previous H2D is done:
    // that chunk's event was waited for in the previous iteration)
    const size_t noff = end, nend = noff < len ? chunk_end(text, len, noff) : noff;
    if (noff < len && !nend) return fail(GS_ERR_INVALID, "a line is longer than the 16 MiB ingest chunk");
    if (noff < len) staged_copy(h->h_text + (size_t)(b ^ 1) * kTextChunk, text + noff, nend - noff);
    GS_HIP(hipEventSynchronize(h->text_ev[b]));
    const uint64_t nl = h->h_tres[2 * b], bad = h->h_tres[2 * b + 1];
    if (bad != ~0ull) {
      *bad_line = (int64_t)(line0 + bad);
      return fail(GS_ERR_PARSE, "malformed edge line " + std::to_string(*bad_line));
    }
    if (int rc = fold_device_impl(h, h->d_tsrc, h->d_tdst, nullptr, nl, 1, 1, h->track)) return rc;
    *n_edges += nl;
    line0 += nl;
    if (noff >= len) break;
    if (int rc = enqueue(b ^ 1, nend - noff)) return rc;  // stream order: after this chunk's fold
    end = nend;
  }
  return GS_OK;
}

int gs_set_pipelining(gs_handle h, int depth) {
  if (int rc = check(h)) return rc;
  if (depth < 1 || depth > gs_summary::kLanes) return fail(GS_ERR_INVALID, "pipelining depth must be 1..4");
  DeviceGuard g(h->device);
  if (int rc_ = join_lanes(h)) return rc_;
  if (int rc_ = ensure_lanes(h, depth)) return rc_;
  h->pipe_depth = depth;
  h->lane_next = 0;
  return GS_OK;
}

int gs_table_capacity(gs_handle h, uint64_t* slots) {
  if (int rc = check(h)) return rc;
  if (!slots) return fail(GS_ERR_INVALID, "slots is null");
  *slots = h->cap;
  return GS_OK;
}

}  // extern "C"

extern "C" int gs_testing_set(int knob, int64_t value) {
  if (knob < 0 || knob >= GS_TESTING_KNOBS) return gsi::fail(GS_ERR_INVALID, "unknown test knob");
  gsi::g_testing[knob].store(value < 0 ? -1 : value, std::memory_order_relaxed);
  return GS_OK;
}

extern "C" int64_t gs_testing_get(int knob) {
  if (knob < 0 || knob >= GS_TESTING_KNOBS) return -1;
  static const int64_t product[GS_TESTING_KNOBS] = {2000, 1 << 16, 50000, 0, 2};
  return gsi::testing_value(knob, product[knob]);
}

extern "C" int gs_hbm_bytes(int device, uint64_t* bytes) {
  if (!bytes) return gsi::fail(GS_ERR_INVALID, "bytes is null");
  if (device < 0 || device >= gsi::kMaxDevices) return gsi::fail(GS_ERR_INVALID, "bad device");
  *bytes = gsi::g_hbm[device].load(std::memory_order_relaxed);
  return GS_OK;
}

extern "C" int gs_create_bytes(int kind, uint64_t capacity_hint, uint64_t* bytes) {
  if (!bytes) return gsi::fail(GS_ERR_INVALID, "bytes is null");
  if (kind != GS_KIND_CC && kind != GS_KIND_SIGNED) return gsi::fail(GS_ERR_INVALID, "unknown kind");
  *bytes = gsi::create_bytes(gsi::create_capacity(capacity_hint));
  return GS_OK;
}
