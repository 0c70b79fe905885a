// gs_group.cpp -- native multi-GPU group (include/gs_group.h).
//
// Each rank folds its own shard of every global micro-batch into a REPLICA of the
// global summary, and the replicas exchange their structural deltas over RCCL:
//
//   exchange b:  own fold b (tracked) -> stage b: records -> send[b%2], count word
//                -> count all-gather (communicator C, stream xc) -> k_headers: the
//                   gathered counts in host-mapped memory
//   then, still inside the call for exchange b, after fold b is queued, the DATA of
//                exchange b-2 (data lag 2; 1..3 through gs_testing_set(GS_TESTING_GROUP_DATA_LAG)):
//                host reads b-2's counts (landed while fold b-1 ran) -> data all-gather
//                of exactly max-count rows per rank (communicator D, stream xd) -> fold
//                of the other ranks' live rows on the apply (side) stream, beside this
//                rank's own folds.
//
// Only live rows move: the collective size is the largest record count of THIS
// exchange, known before the data collective is issued, so nothing is queued,
// padded to a capacity agreed in advance, or drained at the end. Two communicators
// keep each one's collectives in issue order on one stream. This replaces the
// reference's gather of per-partition summaries into one parallelism-1 reducer
// (SummaryBulkAggregation.java:77-83) and its Merger (SummaryAggregation.java:107-119).
#include <dlfcn.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "gs_group.h"
#include "gs_internal.hpp"
#include "gs_part.hpp"
#include "gs_testing.h"

using namespace gsi;

namespace {

constexpr int kIdBytes = 128;  // one ncclUniqueId
constexpr uint64_t kMaxGroupBatch = 1ull << 26;
// The data half of exchange b runs in the call for exchange b + kLag: by then its
// counts have long landed (a stage waits ~20 us for its fold's event on another
// queue, then the count collective and k_headers), so the host never blocks and its
// per-exchange launch work overlaps the folds. kLag buffer sets rotate.
#ifndef GS_GROUP_LAG
#define GS_GROUP_LAG 3
#endif
constexpr int kLag = GS_GROUP_LAG;
// Own folds are launched in micro-batches of 2^20 edges,
// alternating over two pipelining lanes of the summary so that each launch's tail
// overlaps the next one; every micro-batch of exchange b records into delta set b % 2.
constexpr uint64_t kMicro = 1ull << 20;
#ifndef GS_GROUP_LANES_N
#define GS_GROUP_LANES_N 3
#endif
constexpr int kGroupLanes = GS_GROUP_LANES_N;  // own-fold lanes (chunk c runs on lane c mod kGroupLanes)
#ifndef GS_GROUP_HOSTPROF
#define GS_GROUP_HOSTPROF 0
#endif
#ifndef GS_GROUP_NO_LANES
#define GS_GROUP_NO_LANES 0
#endif
#ifndef GS_GROUP_NO_SIDE
#define GS_GROUP_NO_SIDE 0
#endif
#ifndef GS_GROUP_HIPRIO
#define GS_GROUP_HIPRIO 0
#endif

// RCCL behind the gs_comm_api table (include/gs_group.h). ncclCommInitRank takes its
// ncclUniqueId (128 B) by value: the adapter copies the caller's bytes into one.
struct Id128 {
  char b[kIdBytes];
};
struct RcclSyms {
  void* lib = nullptr;
  int (*getUniqueId)(void*) = nullptr;
  int (*initRank)(void**, int, Id128, int) = nullptr;
  int (*commDestroy)(void*) = nullptr;
  int (*commCount)(void*, int*) = nullptr;
  int (*allGather)(const void*, void*, size_t, int, void*, hipStream_t) = nullptr;
  int (*allToAllv)(const void*, const size_t*, const size_t*, void*, const size_t*, const size_t*, int, void*,
                   hipStream_t) = nullptr;
  int (*send)(const void*, size_t, int, int, void*, hipStream_t) = nullptr;
  int (*recv)(void*, size_t, int, int, void*, hipStream_t) = nullptr;
  int (*groupStart)() = nullptr;
  int (*groupEnd)() = nullptr;
  const char* (*getErrorString)(int) = nullptr;
};
RcclSyms g_rs;

int rc_unique_id(void* id) { return g_rs.getUniqueId(id); }
int rc_init(void** comm, int n, const void* id, int rank) {
  Id128 u;
  memcpy(u.b, id, kIdBytes);
  return g_rs.initRank(comm, n, u, rank);
}
int rc_destroy(void* c) { return g_rs.commDestroy(c); }
int rc_count(void* c, int* n) { return g_rs.commCount ? g_rs.commCount(c, n) : 1; }
int rc_all_gather(const void* s, void* r, size_t n, int t, void* c, void* st) {
  return g_rs.allGather(s, r, n, t, c, (hipStream_t)st);
}
int rc_all_to_allv(const void* s, const size_t* sc, const size_t* sd, void* r, const size_t* rc, const size_t* rd,
                   int t, void* c, void* st) {
  return g_rs.allToAllv ? g_rs.allToAllv(s, sc, sd, r, rc, rd, t, c, (hipStream_t)st) : 1;
}
int rc_send(const void* b, size_t n, int t, int p, void* c, void* st) {
  return g_rs.send ? g_rs.send(b, n, t, p, c, (hipStream_t)st) : 1;
}
int rc_recv(void* b, size_t n, int t, int p, void* c, void* st) {
  return g_rs.recv ? g_rs.recv(b, n, t, p, c, (hipStream_t)st) : 1;
}
int rc_group_start() { return g_rs.groupStart ? g_rs.groupStart() : 1; }
int rc_group_end() { return g_rs.groupEnd ? g_rs.groupEnd() : 1; }
const char* rc_error(int r) { return g_rs.getErrorString ? g_rs.getErrorString(r) : "rccl error"; }

gs_comm_api g_rccl_api = {rc_unique_id, rc_init,  rc_destroy,     rc_count,     rc_all_gather, rc_all_to_allv,
                          rc_send,      rc_recv,  rc_group_start, rc_group_end, rc_error};

int rccl_load() {
  if (g_rs.lib) return GS_OK;
  void* l = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!l) l = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!l) return fail(GS_ERR_HIP, std::string("cannot load RCCL: ") + dlerror());
  RcclSyms s;
  s.getUniqueId = (int (*)(void*))dlsym(l, "ncclGetUniqueId");
  s.initRank = (int (*)(void**, int, Id128, int))dlsym(l, "ncclCommInitRank");
  s.allGather = (int (*)(const void*, void*, size_t, int, void*, hipStream_t))dlsym(l, "ncclAllGather");
  s.allToAllv = (int (*)(const void*, const size_t*, const size_t*, void*, const size_t*, const size_t*, int, void*,
                         hipStream_t))dlsym(l, "ncclAllToAllv");
  s.commDestroy = (int (*)(void*))dlsym(l, "ncclCommDestroy");
  s.getErrorString = (const char* (*)(int))dlsym(l, "ncclGetErrorString");
  s.send = (int (*)(const void*, size_t, int, int, void*, hipStream_t))dlsym(l, "ncclSend");
  s.recv = (int (*)(void*, size_t, int, int, void*, hipStream_t))dlsym(l, "ncclRecv");
  s.groupStart = (int (*)())dlsym(l, "ncclGroupStart");
  s.groupEnd = (int (*)())dlsym(l, "ncclGroupEnd");
  s.commCount = (int (*)(void*, int*))dlsym(l, "ncclCommCount");
  if (!s.getUniqueId || !s.initRank || !s.allGather || !s.commDestroy)
    return fail(GS_ERR_HIP, "RCCL is missing ncclGetUniqueId/ncclCommInitRank/ncclAllGather/ncclCommDestroy");
  s.lib = l;
  g_rs = s;
  return GS_OK;
}

int rccl_fail(const gs_comm_api* api, const char* what, int r) {
  return fail(GS_ERR_HIP, std::string(what) + ": " + (api && api->error_string ? api->error_string(r) : "comm error"));
}

constexpr int kNcclInt64 = 4;  // ncclInt64 (rccl.h)
constexpr int kNcclUint8 = 1;  // ncclUint8 (rccl.h)

// gs_group_set_comm_api: a caller's table (copied), or RCCL
std::mutex g_api_mu;
bool g_user_api_on = false;
gs_comm_api g_user_api;

// the communication API a new group (or id) uses; the returned table lives as long as
// the process (a group keeps a copy)
int comm_api(gs_comm_api* out) {
  {
    std::lock_guard<std::mutex> lk(g_api_mu);
    if (g_user_api_on) {
      *out = g_user_api;
      return GS_OK;
    }
  }
  if (int rc = rccl_load()) return rc;
  *out = g_rccl_api;
  return GS_OK;
}

}  // namespace

struct gs_group {
  gs_summary* h = nullptr;
  gs_comm_api api = {};          // RCCL, or the caller's backend (gs_group_set_comm_api)
  void* comm_c = nullptr;        // count collectives (stream xc)
  void* comm_d = nullptr;        // data collectives (stream xd) and the tree combine
  int nranks = 1, rank = 0;
  int width = 3;                 // int64 per exchange row: {a, b} for CC (16 B), {a, b, parity} signed
  bool exchange = false;         // false: tree-combine-only group
  bool prev_track = false;       // the summary's delta tracking before the group turned it on
  bool self_apply = false;       // test knob (GS_TESTING_GROUP_SELF_APPLY): also fold this rank's own rows back
  uint64_t batch = 0, rows_cap = 0;
  // exchange b uses buffer set b % kLag (send, counts, headers, receive) and delta set b % kDeltaSets
  int64_t* send[kLag] = {};                             // [rows_cap * width]
  int64_t* recv[kLag] = {};                             // [nranks * rows_cap * width]
  unsigned long long* cnt = nullptr;                    // device: [kLag] send counts, then [kLag][nranks] gathered
  long long* hdr_host = nullptr;                        // pinned host-mapped [kLag][nranks + 1]
  long long* hdr_dev = nullptr;
  hipStream_t xc = nullptr, xd = nullptr, as = nullptr;  // counts, data, apply (the summary's side stream)
  hipEvent_t as_ev = nullptr;
  hipEvent_t folded[gs::kDeltaSets][kGroupLanes] = {}, staged[gs::kDeltaSets] = {};  // per delta set (folded: per lane)
  uint64_t chunks = 0;                                  // own micro-batches launched (lane = chunks % 2)
  hipEvent_t counted[kLag] = {}, gathered[kLag] = {}, applied[kLag] = {};  // per buffer set
  uint64_t b = 0;       // exchanges since create / finish
  uint64_t own_edges = 0;  // own edges folded since create / finish (the ramp's position)
  uint64_t ramp_edges = 1ull << 22, ramp_batch = 1ull << 20;  // gs_group_set_ramp
  uint64_t done = 0;    // exchanges whose data half has been issued
  int data_lag = 2;     // exchanges between an exchange's own fold and its data half (GS_TESTING_GROUP_DATA_LAG: 1..kLag)
  uint64_t api_seen = 0;  // h->api_calls at the previous fold call (lane ordering)
  // statistics
  uint64_t exchanges = 0, rows_received = 0, live_received = 0;
  // diagnostic builds (make variant VFLAGS=-DGS_GROUP_HOSTPROF=1 ...): host seconds per
  // phase printed at destroy; own folds (GS_GROUP_NO_LANES) or remote folds
  // (GS_GROUP_NO_SIDE) on the handle stream
  bool hostprof = GS_GROUP_HOSTPROF != 0;
  bool no_lanes = GS_GROUP_NO_LANES != 0;
  bool no_side = GS_GROUP_NO_SIDE != 0;
  double hp[4] = {};      // own fold, stage + count collective, wait for counts, data collective + apply
  uint64_t hp_calls = 0;
  // per-phase timing (gs_group_set_phase_timing): HIP timing events around each phase's
  // device work; [0] own folds (lane time, summed over lanes), [1] remote-row folds,
  // [2] stage + count collective + headers, [3] data collective. Host wait for gathered
  // counts is always timed (wait_s).
  bool phases = false;
  struct PhaseEv {
    int ph;
    hipEvent_t a, b;
  };
  std::vector<PhaseEv> ph_pending;
  std::vector<hipEvent_t> ph_pool;
  double ph_ms[8] = {};
  uint64_t ph_exchanges = 0;
  double wait_s = 0;

  // ---- owner-partitioned mode (gs_group_create_partitioned)
  bool part = false;
  gs_summary* G = nullptr;       // the label forest: a replica of the labels that need a cross-rank union
  uint64_t window = 0;           // own edges between combines (0: one combine per pass, untracked folds)
  uint64_t win_edges = 0;        // own edges since the last combine
  gs::OwnerTable ot{};
  uint32_t* mark = nullptr;      // device [64]: vertex-list fill at the previous combine
  uint32_t* snap = nullptr;      // device [64]: the fill now
  uint32_t* pflags = nullptr;    // device: [0] owner-table overflow, [1] odd cycle found by an owner
  unsigned long long* pdev = nullptr;  // device: [0..2] snap out, [3] pairs, [4] count word, [5] label rows,
                                       // [8, 8 + N) send counts, then N x N all send counts, then N count words
  unsigned long long* phost = nullptr;  // pinned host mirror of pdev's words
  int64_t *stage = nullptr, *sendbuf = nullptr, *recvbuf = nullptr, *pairs = nullptr, *pairs_all = nullptr;
  uint64_t stage_cap = 0, send_cap = 0, recv_cap = 0, pairs_cap = 0, pairs_all_cap = 0;
  uint32_t* bcnt = nullptr;
  uint64_t bcnt_cap = 0;
  gs::PairSlot* pset = nullptr;  // the owner step's set of label pairs emitted this combine (N > 1)
  uint64_t pset_cap = 0;
  uint64_t cap_seen = 0;         // the local table's capacity at the previous combine (a rebuild re-exports all)
  hipEvent_t pev = nullptr;      // the combine's pair gather -> the label forest's fold
  uint64_t combines = 0, rows_exported = 0, rows_owned = 0, pairs_sent = 0, pairs_folded = 0;

  unsigned long long* cnt_send(int k) const { return cnt + k; }
  unsigned long long* cnt_recv(int k) const { return cnt + kLag + (size_t)k * nranks; }
  long long* hdr(int k) const { return hdr_host + (size_t)k * (nranks + 1); }
};

namespace {

struct HostTimer {
  double* acc;
  std::chrono::steady_clock::time_point t0;
  explicit HostTimer(double* a) : acc(a), t0(std::chrono::steady_clock::now()) {}
  void lap(double* next) {  // charge the time so far to acc, continue on next
    const auto t = std::chrono::steady_clock::now();
    if (acc) *acc += std::chrono::duration<double>(t - t0).count();
    t0 = t;
    acc = next;
  }
  ~HostTimer() { lap(nullptr); }
};

hipEvent_t ph_event(gs_group* g) {
  if (!g->ph_pool.empty()) {
    hipEvent_t e = g->ph_pool.back();
    g->ph_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}
// phase timing: an event on st now (the phase's start), or nullptr when timing is off
hipEvent_t ph_begin(gs_group* g, hipStream_t st) {
  if (!g->phases) return nullptr;
  hipEvent_t a = ph_event(g);
  (void)hipEventRecord(a, st);
  return a;
}
void ph_end(gs_group* g, int ph, hipEvent_t a, hipStream_t st) {
  if (!a) return;
  hipEvent_t b = ph_event(g);
  (void)hipEventRecord(b, st);
  g->ph_pending.push_back({ph, a, b});
}
void ph_drain(gs_group* g) {
  for (auto& p : g->ph_pending) {
    float ms = 0.f;
    if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess)
      g->ph_ms[p.ph] += ms;
    g->ph_pool.push_back(p.a);
    g->ph_pool.push_back(p.b);
  }
  g->ph_pending.clear();
}

// The data half of exchange e: wait for its gathered counts (host-mapped), gather
// exactly max-count rows per rank, fold the other ranks' live rows on the apply
// stream. No host synchronisation beyond the count poll.
int finish_data(gs_group* g, uint64_t e) {
  gs_summary* h = g->h;
  const int k = (int)(e % kLag);
  HostTimer ht(g->hostprof ? &g->hp[2] : nullptr);
  volatile long long* hd = g->hdr(k);
  const auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(&hd[g->nranks], __ATOMIC_ACQUIRE) != (long long)e) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) {  // long wait: block
      GS_HIP(hipEventSynchronize(g->counted[k]));
      if (__atomic_load_n(&hd[g->nranks], __ATOMIC_ACQUIRE) != (long long)e)
        return fail(GS_ERR_HIP, "exchange count sequence mismatch");
      break;
    }
  }
  g->wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t maxc = 0, live = 0;
  for (int r = 0; r < g->nranks; ++r) {
    const uint64_t c = (uint64_t)hd[r] & (gs::kFailBit - 1);
    if (c > g->rows_cap) return fail(GS_ERR_HIP, "exchange count above the delta capacity");
    maxc = std::max(maxc, c);
    if (r != g->rank || g->self_apply) live += c;
  }
  const uint64_t rows = std::max<uint64_t>(maxc, 1);  // >= 1 row: the fold reads every block's failure bit
  ht.lap(g->hostprof ? &g->hp[3] : nullptr);
  GS_HIP(hipStreamWaitEvent(g->xd, g->counted[k], 0));  // behind the stage (and the count collective)
  if (e >= (uint64_t)kLag) GS_HIP(hipStreamWaitEvent(g->xd, g->applied[k], 0));  // recv[k]: fold of e - kLag done
  hipEvent_t pa = ph_begin(g, g->xd);
  const int r = g->api.all_gather(g->send[k], g->recv[k], rows * g->width, kNcclInt64, g->comm_d, g->xd);
  if (r != 0) return rccl_fail(&g->api, "ncclAllGather(data)", r);
  ph_end(g, 3, pa, g->xd);
  GS_HIP(hipEventRecord(g->gathered[k], g->xd));
  const bool use_side = side_ok(h) && !g->no_side;
  hipStream_t s = use_side ? h->side : h->stream;
  if (g->nranks > 1 || g->self_apply) {
    GS_HIP(hipStreamWaitEvent(s, g->gathered[k], 0));
    FoldSource fs;
    fs.rows = (uint32_t)rows;
    fs.skip_rank = g->self_apply ? -1 : g->rank;
    fs.counts = g->cnt_recv(k);
    fs.units = live;
    fs.on_side = use_side;
    const uint8_t* w = g->width == 3 ? reinterpret_cast<const uint8_t*>(g->recv[k] + 2) : nullptr;
    hipEvent_t pf = ph_begin(g, s);
    if (int rc = fold_device_impl(h, g->recv[k], g->recv[k] + 1, w, (size_t)g->nranks * rows, g->width,
                                  8 * g->width, /*track=*/false, true, fs))
      return rc;
    ph_end(g, 1, pf, s);
  }
  GS_HIP(hipEventRecord(g->applied[k], s));
  g->rows_received += rows * (uint64_t)(g->nranks - 1);
  g->live_received += live;
  g->done = e + 1;
  return GS_OK;
}

// Communication streams at NORMAL priority. Highest-priority comm streams overlapped
// stages with folds slightly better (2^22-edge exchanges at one rank 47.9 -> 44.7
// ms/step), but under real multi-queue concurrency (GPU_MAX_HW_QUEUES=32, 5-8
// emulated ranks) they LOST work: in some own-fold launches every workgroup of one or
// more XCDs (blocks b = c mod 8) left no trace -- no key CAS, no vertex-count add --
// so every replica missed those edges' vertices (tools/emu_check.py; DESIGN.md
// section 5). Normal-priority streams, or the remote folds serialised on the handle
// stream, were exact in every run.
// A diagnostic build with -DGS_GROUP_HIPRIO=1 (tools/lostwork_probe.py) brings the highest
// priority back.
hipError_t create_comm_stream(hipStream_t* st) {
  if (GS_GROUP_HIPRIO) {
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess)
      return hipStreamCreateWithPriority(st, hipStreamNonBlocking, hi);
  }
  return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
}

}  // namespace

extern "C" {

int gs_group_set_comm_api(const gs_comm_api* api) {
  if (api && (!api->get_unique_id || !api->comm_init_rank || !api->comm_destroy || !api->all_gather))
    return fail(GS_ERR_INVALID, "comm api needs get_unique_id, comm_init_rank, comm_destroy and all_gather");
  std::lock_guard<std::mutex> lk(g_api_mu);
  g_user_api_on = api != nullptr;
  if (api) g_user_api = *api;
  return GS_OK;
}

int gs_group_unique_id(void* id) {
  if (!id) return fail(GS_ERR_INVALID, "id is null");
  gs_comm_api api;
  if (int rc = comm_api(&api)) return rc;
  for (int i = 0; i < 2; ++i) {  // two communicators: counts and data
    const int r = api.get_unique_id(static_cast<char*>(id) + i * kIdBytes);
    if (r) return rccl_fail(&api, "ncclGetUniqueId", r);
  }
  return GS_OK;
}

int gs_group_create(gs_group_t* out, gs_handle h, const void* id, int nranks, int rank, size_t batch_edges) {
  if (!out || !id) return fail(GS_ERR_INVALID, "null argument");
  *out = nullptr;
  if (!h) return fail(GS_ERR_INVALID, "null handle");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(GS_ERR_INVALID, "bad group shape");
  if (batch_edges > kMaxGroupBatch) return fail(GS_ERR_INVALID, "batch_edges above 2^26");
  gs_comm_api api;
  if (int rc = comm_api(&api)) return rc;
  DeviceGuard dg(h->device);
  gs_group* g = new gs_group();
  g->h = h;
  g->api = api;
  g->nranks = nranks;
  g->rank = rank;
  g->width = h->kind == GS_KIND_SIGNED ? 3 : 2;
  g->exchange = batch_edges != 0;
  g->batch = batch_edges;
  g->self_apply = testing_value(GS_TESTING_GROUP_SELF_APPLY, 0) != 0;
  g->data_lag = (int)std::min<int64_t>(kLag, std::max<int64_t>(1, testing_value(GS_TESTING_GROUP_DATA_LAG, 2)));
  auto bail = [&](int code) {
    gs_group_destroy(g);
    return code;
  };
  if (g->exchange) {
    if (h->side) return bail(fail(GS_ERR_INVALID, "the summary already belongs to an exchange group"));
    if (int rc = join_lanes(h)) return bail(rc);
    if (int rc = ensure_lanes(h, kGroupLanes)) return bail(rc);  // own folds rotate over the lanes
    if (int rc = ensure_delta_list(h, batch_edges)) return bail(rc);
    g->prev_track = h->track;
    if (int rc = gs_set_delta_tracking(h, 1)) return bail(rc);
    g->rows_cap = (uint64_t)gs::kShards * h->delta_shard_cap;
    bool ok = hipHostMalloc(&g->hdr_host, kLag * (size_t)(nranks + 1) * 8,
                            hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
              hipHostGetDevicePointer(reinterpret_cast<void**>(&g->hdr_dev), g->hdr_host, 0) == hipSuccess &&
              dmalloc(&g->cnt, (kLag + kLag * (size_t)nranks) * 8) == hipSuccess &&
              create_comm_stream(&g->xc) == hipSuccess && create_comm_stream(&g->xd) == hipSuccess &&
              hipStreamCreateWithFlags(&g->as, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&g->as_ev, hipEventDisableTiming) == hipSuccess;
    for (int k = 0; k < gs::kDeltaSets && ok; ++k) {
      for (int i = 0; i < kGroupLanes && ok; ++i)
        ok = hipEventCreateWithFlags(&g->folded[k][i], hipEventDisableTiming) == hipSuccess;
      ok = ok && hipEventCreateWithFlags(&g->staged[k], hipEventDisableTiming) == hipSuccess;
    }
    for (int k = 0; k < kLag && ok; ++k)
      ok = dmalloc(&g->send[k], g->rows_cap * g->width * 8) == hipSuccess &&
           dmalloc(&g->recv[k], (size_t)nranks * g->rows_cap * g->width * 8) == hipSuccess &&
           hipEventCreateWithFlags(&g->counted[k], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&g->gathered[k], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&g->applied[k], hipEventDisableTiming) == hipSuccess;
    if (!ok) return bail(fail(GS_ERR_HIP, "group buffer allocation failed"));
    for (int k = 0; k < kLag; ++k) g->hdr(k)[nranks] = -1;  // no exchange yet
    h->side = g->as;
    h->side_ev = g->as_ev;
    h->side_dirty = false;
    h->group_lanes = kGroupLanes;
  }
  if (g->exchange) {
    const int r = api.comm_init_rank(&g->comm_c, nranks, id, rank);
    if (r != 0) return bail(rccl_fail(&api, "ncclCommInitRank(counts)", r));
  }
  const int r = api.comm_init_rank(&g->comm_d, nranks, static_cast<const char*>(id) + kIdBytes, rank);
  if (r != 0) return bail(rccl_fail(&api, "ncclCommInitRank(data)", r));
  *out = g;
  return GS_OK;
}

int gs_group_fold_device(gs_group_t g, const int64_t* src, const int64_t* dst, size_t n) {
  if (!g) return fail(GS_ERR_INVALID, "null group");
  gs_summary* h = g->h;
  DeviceGuard dg(h->device);
  if (!g->exchange) return fail(GS_ERR_INVALID, "tree-combine-only group (created with batch_edges 0)");
  if (n && (!src || !dst)) return fail(GS_ERR_INVALID, "null edge arrays");
  if (n > g->batch) return fail(GS_ERR_INVALID, "n above the group's batch_edges");
  const uint64_t b = g->b;
  const int d = (int)(b % gs::kDeltaSets), k = (int)(b % kLag);  // delta set, buffer set
  g->hp_calls++;
  g->own_edges += n;
  // data lag kLag: the data half of exchange b - kLag (its counts landed long ago),
  // issued first, so buffer set k is released (events recorded) before this exchange
  // reuses it. A shorter lag issues it at the end of the call (below).
  if (g->data_lag == kLag && b >= (uint64_t)kLag)
    if (int rc = finish_data(g, b - kLag)) return rc;
  HostTimer ht(g->hostprof ? &g->hp[0] : nullptr);
  // The own fold records into delta set d. The summary stream only waits for the
  // stage of exchange b - kDeltaSets (which emptied set d): stages, collectives and the
  // remote folds all run on other streams, so own folds go back to back.
  const bool lanes = !h->profiling && !g->no_lanes;  // (profiling serialises folds on the handle stream)
  if (lanes) {
    // The lanes start behind the caller's work on the handle stream (a reset, edges
    // written there, a buffer reused after a sync through it), as gs_fold_device is
    // ordered after it: at the first exchange, and whenever any gs_* call was made on
    // the handle since the previous group call (a caller that queues its own
    // kernels on gs_get_stream(h) marks them with gs_wait_stream(h, that stream)).
    // Not at every call: with the box's 4 hardware queues the handle stream shares a
    // queue with a communication stream, so a marker recorded there waits behind the
    // collectives of earlier exchanges, and every lane with it (one-rank exchange step
    // 44.7 -> 74 ms, profiles/r03_exchange_lane_order.txt).
    if (b == 0 || h->api_calls != g->api_seen) {
      GS_HIP(hipEventRecord(h->main_ev, h->stream));
      for (int i = 0; i < kGroupLanes; ++i) GS_HIP(hipStreamWaitEvent(h->lane[i], h->main_ev, 0));
    }
    g->api_seen = h->api_calls;
    if (b >= (uint64_t)gs::kDeltaSets)
      for (int i = 0; i < kGroupLanes; ++i) GS_HIP(hipStreamWaitEvent(h->lane[i], g->staged[d], 0));
  } else if (b >= (uint64_t)gs::kDeltaSets) {
    GS_HIP(hipStreamWaitEvent(h->stream, g->staged[d], 0));
    h->xwait = true;
  }
  h->dset = d;
  int frc = GS_OK;
  bool used_lane[kGroupLanes] = {};
  hipEvent_t po[kGroupLanes] = {};
  if (g->phases)
    for (int i = 0; i < kGroupLanes; ++i) po[i] = ph_begin(g, lanes ? h->lane[i] : h->stream);
  for (size_t off = 0; off < n && !frc; off += kMicro) {
    FoldSource fs;
    if (lanes) {
      fs.lane = (int)(g->chunks++ % kGroupLanes);
      used_lane[fs.lane] = true;
    }
    frc = fold_device_impl(h, src + off, dst + off, nullptr, std::min<uint64_t>(kMicro, n - off), 1, 1,
                           /*track=*/true, true, fs);
  }
  h->dset = 0;
  if (frc) return frc;
  // the stage waits for every micro-batch of this exchange (one event per lane used)
  int nev = 0;
  hipEvent_t evs[kGroupLanes];
  for (int i = 0; i < kGroupLanes; ++i) {
    if (!po[i]) continue;
    if (lanes ? used_lane[i] : i == 0) ph_end(g, 0, po[i], lanes ? h->lane[i] : h->stream);
    else g->ph_pool.push_back(po[i]);  // (recorded, never timed)
  }
  if (!lanes) {
    GS_HIP(hipEventRecord(g->folded[d][0], h->stream));
    evs[nev++] = g->folded[d][0];
  } else {
    for (int i = 0; i < kGroupLanes; ++i)
      if (used_lane[i]) {
        GS_HIP(hipEventRecord(g->folded[d][i], h->lane[i]));
        evs[nev++] = g->folded[d][i];
      }
  }
  ht.lap(g->hostprof ? &g->hp[1] : nullptr);
  // communication stream C: stage set d behind the fold, once the remote fold of
  // exchange b - kLag has read cnt_recv[k] (it ran behind the data collective that
  // read send[k] / cnt_send[k])
  for (int i = 0; i < nev; ++i) GS_HIP(hipStreamWaitEvent(g->xc, evs[i], 0));
  if (b >= (uint64_t)kLag) GS_HIP(hipStreamWaitEvent(g->xc, g->applied[k], 0));
  hipEvent_t pc = ph_begin(g, g->xc);
  if (int rc = stage_delta(h, g->send[k], g->rows_cap, g->width, g->cnt_send(k), h->kind == GS_KIND_SIGNED, g->xc, d))
    return rc;
  GS_HIP(hipEventRecord(g->staged[d], g->xc));
  const int r = g->api.all_gather(g->cnt_send(k), g->cnt_recv(k), 1, kNcclInt64, g->comm_c, g->xc);
  if (r != 0) return rccl_fail(&g->api, "ncclAllGather(counts)", r);
  gs::launch_headers(g->cnt_recv(k), g->nranks, g->hdr_dev + (size_t)k * (g->nranks + 1), (long long)b, g->xc);
  GS_HIP(hipGetLastError());
  ph_end(g, 2, pc, g->xc);
  GS_HIP(hipEventRecord(g->counted[k], g->xc));
  ht.lap(nullptr);
  g->b++;
  g->exchanges++;
  if (g->phases) g->ph_exchanges++;
  // data lag L < kLag: the data half of exchange b - L, after this exchange's own folds
  // are queued -- the host waits for that exchange's counts (its folds done) while the
  // GPU already has this exchange's folds, and its remote rows are folded beside them:
  // every rank learns the others' hooks kLag - L exchanges sooner, so fewer of its own
  // hooks duplicate theirs. (The stage above reused buffer set k
  // after the data half of exchange b - kLag, issued in call b - kLag + L < b.)
  if (g->data_lag < kLag && b >= (uint64_t)g->data_lag)
    if (int rc = finish_data(g, b - g->data_lag)) return rc;
  return GS_OK;
}

int gs_group_fold_batches_device(gs_group_t g, const int64_t* src, const int64_t* dst, size_t n, size_t batch) {
  if (!g) return fail(GS_ERR_INVALID, "null group");
  if (batch == 0) return fail(GS_ERR_INVALID, "batch is 0");
  for (size_t off = 0; off < n;) {
    size_t m = batch;
    if (g->own_edges < g->ramp_edges && g->ramp_batch < m) m = g->ramp_batch;  // the ramp
    m = std::min(m, n - off);
    if (int rc = gs_group_fold_device(g, src + off, dst + off, m)) return rc;
    off += m;
  }
  return GS_OK;
}

int gs_group_set_ramp(gs_group_t g, size_t ramp_edges, size_t ramp_batch) {
  if (!g) return fail(GS_ERR_INVALID, "null group");
  if (ramp_edges && (ramp_batch == 0 || ramp_batch > g->batch))
    return fail(GS_ERR_INVALID, "ramp_batch must be in (0, batch_edges]");
  g->ramp_edges = ramp_edges;
  g->ramp_batch = ramp_edges ? ramp_batch : g->batch;
  return GS_OK;
}

int gs_group_finish(gs_group_t g) {
  if (!g) return fail(GS_ERR_INVALID, "null group");
  gs_summary* h = g->h;
  DeviceGuard dg(h->device);
  for (uint64_t e = g->done; e < g->b; ++e)
    if (int rc = finish_data(g, e)) return rc;
  if (int rc = gs_sync(h)) return rc;  // joins the apply stream
  if (g->xc) GS_HIP(hipStreamSynchronize(g->xc));
  if (g->xd) GS_HIP(hipStreamSynchronize(g->xd));
  g->b = g->done = 0;
  g->chunks = 0;
  g->own_edges = 0;
  if (g->hdr_host)
    for (int k = 0; k < kLag; ++k) __atomic_store_n(&g->hdr(k)[g->nranks], (long long)-1, __ATOMIC_RELEASE);
  return GS_OK;
}

}  // extern "C"

namespace {

// one tree edge, sending side: header {count, failed}, then the three arrays
int tree_send(gs_group* g, int peer, int64_t* hdr) {
  gs_summary* h = g->h;
  uint64_t nv = 0;
  if (int rc = read_nv(h, &nv)) return rc;
  int64_t *v = nullptr, *l = nullptr;
  uint8_t* p = nullptr;
  auto release = [&] {
    (void)dfree(v);
    (void)dfree(l);
    (void)dfree(p);
  };
  if (dmalloc(&v, (nv + 1) * 8) != hipSuccess || dmalloc(&l, (nv + 1) * 8) != hipSuccess ||
      dmalloc(&p, nv + 1) != hipSuccess) {
    release();
    return fail(GS_ERR_HIP, "tree combine: out of device memory");
  }
  size_t got = 0;
  uint32_t failed = 0;
  int rc = export_device_impl(h, v, l, p, nv + 1, &got);
  if (!rc && (hipMemcpyAsync(&failed, h->ctr + gs::ctr_index(gs::CTR_FAIL), 4, hipMemcpyDeviceToHost, h->stream) !=
                  hipSuccess ||
              hipStreamSynchronize(h->stream) != hipSuccess))
    rc = fail(GS_ERR_HIP, "tree combine: flag read failed");
  const int64_t hv[2] = {(int64_t)got, (int64_t)(failed != 0)};
  if (!rc && hipMemcpyAsync(hdr, hv, 16, hipMemcpyHostToDevice, h->stream) != hipSuccess)
    rc = fail(GS_ERR_HIP, "tree combine: header copy failed");
  if (!rc) {
    const int r = g->api.send(hdr, 2, kNcclInt64, peer, g->comm_d, h->stream);
    if (r) rc = rccl_fail(&g->api, "ncclSend", r);
  }
  if (!rc && got) {
    g->api.group_start();
    int r = g->api.send(v, got, kNcclInt64, peer, g->comm_d, h->stream);
    if (!r) r = g->api.send(l, got, kNcclInt64, peer, g->comm_d, h->stream);
    if (!r) r = g->api.send(p, got, kNcclUint8, peer, g->comm_d, h->stream);
    const int e = g->api.group_end();
    if (r || e) rc = rccl_fail(&g->api, "ncclSend", r ? r : e);
  }
  if (hipStreamSynchronize(h->stream) != hipSuccess && !rc) rc = fail(GS_ERR_HIP, "tree combine: sync failed");
  release();  // the sends have completed
  return rc;
}

// one tree edge, receiving side: fold the peer's exported summary into this one
int tree_recv(gs_group* g, int peer, int64_t* hdr) {
  gs_summary* h = g->h;
  int r = g->api.recv(hdr, 2, kNcclInt64, peer, g->comm_d, h->stream);
  if (r) return rccl_fail(&g->api, "ncclRecv", r);
  int64_t hv[2] = {0, 0};
  GS_HIP(hipMemcpyAsync(hv, hdr, 16, hipMemcpyDeviceToHost, h->stream));
  GS_HIP(hipStreamSynchronize(h->stream));
  const size_t got = (size_t)hv[0];
  int64_t *v = nullptr, *l = nullptr;
  uint8_t* p = nullptr;
  auto release = [&] {
    (void)dfree(v);
    (void)dfree(l);
    (void)dfree(p);
  };
  int rc = GS_OK;
  if (got && (dmalloc(&v, got * 8) != hipSuccess || dmalloc(&l, got * 8) != hipSuccess ||
              dmalloc(&p, got) != hipSuccess))
    rc = fail(GS_ERR_HIP, "tree combine: out of device memory");
  if (!rc && got) {
    g->api.group_start();
    r = g->api.recv(v, got, kNcclInt64, peer, g->comm_d, h->stream);
    if (!r) r = g->api.recv(l, got, kNcclInt64, peer, g->comm_d, h->stream);
    if (!r) r = g->api.recv(p, got, kNcclUint8, peer, g->comm_d, h->stream);
    const int e = g->api.group_end();
    if (r || e) rc = rccl_fail(&g->api, "ncclRecv", r ? r : e);
  }
  if (!rc) {
    const bool track = h->track;
    h->track = false;  // a bulk combine is not a structural delta of this rank's own fold
    rc = gs_combine_exported_device(h, v, l, p, got, (int)hv[1]);
    h->track = track;
  }
  if (hipStreamSynchronize(h->stream) != hipSuccess && !rc) rc = fail(GS_ERR_HIP, "tree combine: sync failed");
  release();
  return rc;
}

}  // namespace

extern "C" {

int gs_group_tree_combine(gs_group_t g) {
  if (!g) return fail(GS_ERR_INVALID, "null group");
  if (!g->api.send || !g->api.recv || !g->api.group_start || !g->api.group_end)
    return fail(GS_ERR_HIP, "RCCL is missing ncclSend/ncclRecv/ncclGroupStart/ncclGroupEnd");
  gs_summary* h = g->h;
  DeviceGuard dg(h->device);
  if (int rc = join_lanes(h)) return rc;
  int64_t* hdr = nullptr;  // device {count, failed}
  GS_HIP(dmalloc(&hdr, 16));
  int rc = GS_OK;
  // binomial tree (SummaryTreeReduce.enhance pairs partitions by f0/2, :107): at level l
  // rank r with r mod 2^(l+1) == 2^l sends to r - 2^l and leaves the tree
  for (int step = 1; step < g->nranks && rc == GS_OK; step <<= 1) {
    const int pos = g->rank % (2 * step);
    if (pos == step) {
      rc = tree_send(g, g->rank - step, hdr);
      break;
    }
    if (pos == 0 && g->rank + step < g->nranks) rc = tree_recv(g, g->rank + step, hdr);
  }
  (void)dfree(hdr);
  return rc;
}

int gs_group_stats(gs_group_t g, uint64_t* exchanges, uint64_t* records_sent, uint64_t* rows_received) {
  if (!g) return fail(GS_ERR_INVALID, "null group");
  gs_summary* h = g->h;
  DeviceGuard dg(h->device);
  uint64_t sent = 0;
  GS_HIP(hipMemcpyAsync(&sent, h->ctr + gs::ctr_index(gs::CTR_SENT), 8, hipMemcpyDeviceToHost, h->stream));
  GS_HIP(hipStreamSynchronize(h->stream));
  if (exchanges) *exchanges = g->exchanges;
  if (records_sent) *records_sent = sent;
  if (rows_received) *rows_received = g->rows_received;
  return GS_OK;
}

int gs_group_comm_ranks(gs_group_t g, int* count_comm, int* data_comm) {
  if (!g) return fail(GS_ERR_INVALID, "null group");
  if (!g->api.comm_count) return fail(GS_ERR_HIP, "the comm backend has no comm_count");
  int c = 0, d = 0;
  if (g->comm_c) {
    const int r = g->api.comm_count(g->comm_c, &c);
    if (r) return rccl_fail(&g->api, "ncclCommCount(counts)", r);
  }
  if (g->comm_d) {
    const int r = g->api.comm_count(g->comm_d, &d);
    if (r) return rccl_fail(&g->api, "ncclCommCount(data)", r);
  }
  if (count_comm) *count_comm = c;
  if (data_comm) *data_comm = d;
  return GS_OK;
}

int gs_group_set_phase_timing(gs_group_t g, int on) {
  if (!g) return fail(GS_ERR_INVALID, "null group");
  DeviceGuard dg(g->h->device);
  ph_drain(g);
  g->phases = on != 0;
  for (double& x : g->ph_ms) x = 0;
  g->ph_exchanges = 0;
  g->wait_s = 0;
  return GS_OK;
}

int gs_group_phase_stats(gs_group_t g, double* out6) {
  if (!g) return fail(GS_ERR_INVALID, "null group");
  if (!out6) return fail(GS_ERR_INVALID, "out is null");
  DeviceGuard dg(g->h->device);
  ph_drain(g);  // (synchronises the phases' end events)
  for (int i = 0; i < 4; ++i) out6[i] = g->ph_ms[i];
  out6[4] = g->wait_s * 1e3;
  out6[5] = (double)g->ph_exchanges;
  return GS_OK;
}

int gs_group_destroy(gs_group_t g) {
  if (!g) return GS_OK;
  if (g->hostprof && g->hp_calls) {
    const char* nm[4] = {"own fold", "stage+counts", "wait counts", "data+apply"};
    fprintf(stderr, "[gs_group rank %d] host us per exchange over %llu:", g->rank, (unsigned long long)g->hp_calls);
    for (int i = 0; i < 4; ++i) fprintf(stderr, " %s %.1f", nm[i], g->hp[i] * 1e6 / (double)g->hp_calls);
    fprintf(stderr, "; rows received %llu (live %llu); capacity waits %llu, syncs %llu\n",
            (unsigned long long)g->rows_received, (unsigned long long)g->live_received,
            (unsigned long long)g->h->cap_waits, (unsigned long long)g->h->cap_syncs);
  }
  DeviceGuard dg(g->h->device);
  (void)hipStreamSynchronize(g->h->stream);
  if (g->xc) (void)hipStreamSynchronize(g->xc);
  if (g->xd) (void)hipStreamSynchronize(g->xd);
  if (g->comm_c && g->api.comm_destroy) g->api.comm_destroy(g->comm_c);
  if (g->comm_d && g->api.comm_destroy) g->api.comm_destroy(g->comm_d);
  if (g->as) {
    (void)hipStreamSynchronize(g->as);
    if (g->h->side == g->as) {
      (void)join_lanes(g->h);  // (joins the side stream while it still exists)
      g->h->side = nullptr;
      g->h->side_ev = nullptr;
      g->h->side_dirty = false;
      g->h->group_lanes = 0;
      if (!g->prev_track) (void)gs_set_delta_tracking(g->h, 0);  // as before the group
    }
    (void)hipStreamDestroy(g->as);
  }
  if (g->as_ev) (void)hipEventDestroy(g->as_ev);
  for (int k = 0; k < gs::kDeltaSets; ++k) {
    for (hipEvent_t e : g->folded[k])
      if (e) (void)hipEventDestroy(e);
    if (g->staged[k]) (void)hipEventDestroy(g->staged[k]);
  }
  for (int k = 0; k < kLag; ++k) {
    for (hipEvent_t e : {g->counted[k], g->gathered[k], g->applied[k]})
      if (e) (void)hipEventDestroy(e);
    (void)dfree(g->send[k]);
    (void)dfree(g->recv[k]);
  }
  if (g->part) {
    if (g->G) (void)gs_destroy(g->G);
    for (void* q : {(void*)g->ot.tab, (void*)g->mark, (void*)g->snap, (void*)g->pflags, (void*)g->pdev, (void*)g->stage,
                    (void*)g->sendbuf, (void*)g->recvbuf, (void*)g->pairs, (void*)g->pairs_all, (void*)g->bcnt, (void*)g->pset})
      (void)dfree(q);
    if (g->phost) (void)hipHostFree(g->phost);
    if (g->pev) (void)hipEventDestroy(g->pev);
    if (g->window && !g->prev_track) (void)gs_set_delta_tracking(g->h, 0);
  }
  ph_drain(g);
  for (hipEvent_t e : g->ph_pool) (void)hipEventDestroy(e);
  (void)dfree(g->cnt);
  if (g->xc) (void)hipStreamDestroy(g->xc);
  if (g->xd) (void)hipStreamDestroy(g->xd);
  if (g->hdr_host) (void)hipHostFree(g->hdr_host);
  delete g;
  return GS_OK;
}


// ---------------------------------------------------------------------------
// Owner-partitioned mode (include/gs_group.h; kernels gs_part_k.hip)

}  // extern "C"

namespace {

int part_of(gs_group* g) {
  if (!g) return fail(GS_ERR_INVALID, "null group");
  if (!g->part) return fail(GS_ERR_INVALID, "not a partitioned group (gs_group_create_partitioned)");
  return GS_OK;
}

// grow-only device buffer of `need` elements of T; `keep` elements are carried over (stream st)
template <typename T>
int ensure_buf(T*& buf, uint64_t& cap, uint64_t need, hipStream_t st, uint64_t keep = 0) {
  if (need <= cap && buf) return GS_OK;
  const uint64_t c = std::max<uint64_t>(need + need / 4, 1024);
  T* nb = nullptr;
  GS_HIP(dmalloc(&nb, c * sizeof(T)));
  if (buf) {
    if (keep) GS_HIP(hipMemcpyAsync(nb, buf, keep * sizeof(T), hipMemcpyDeviceToDevice, st));
    GS_HIP(hipStreamSynchronize(st));
    (void)dfree(buf);
  }
  buf = nb;
  cap = c;
  return GS_OK;
}

// device words of pdev -> host (phost), one stream synchronisation
int part_read(gs_group* g, size_t first, size_t n) {
  hipStream_t st = g->h->stream;
  GS_HIP(hipMemcpyAsync(g->phost + first, g->pdev + first, n * 8, hipMemcpyDeviceToHost, st));
  GS_HIP(hipStreamSynchronize(st));
  return GS_OK;
}

int part_init_tables(gs_group* g) {
  hipStream_t st = g->h->stream;
  gs::launch_part_init(g->ot.tab, (uint64_t)g->ot.cap + 1, st);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemsetAsync(g->mark, 0, gs::kShards * 4, st));
  GS_HIP(hipMemsetAsync(g->pflags, 0, 16, st));
  g->win_edges = 0;
  g->cap_seen = g->h->cap;
  return GS_OK;
}

}  // namespace

extern "C" {

int gs_group_create_partitioned(gs_group_t* out, gs_handle h, const void* id, int nranks, int rank,
                                uint64_t vertices_hint, size_t window_edges) {
  if (!out || !id) return fail(GS_ERR_INVALID, "null argument");
  *out = nullptr;
  if (!h) return fail(GS_ERR_INVALID, "null handle");
  if (nranks < 1 || nranks > gs::kPartMaxRanks || rank < 0 || rank >= nranks)
    return fail(GS_ERR_INVALID, "bad group shape (1..64 ranks)");
  if (window_edges > kMaxGroupBatch) return fail(GS_ERR_INVALID, "window_edges above 2^26");
  if (h->side) return fail(GS_ERR_INVALID, "the summary already belongs to an exchange group");
  gs_comm_api api;
  if (int rc = comm_api(&api)) return rc;
  DeviceGuard dg(h->device);
  gs_group* g = new gs_group();
  g->h = h;
  g->api = api;
  g->nranks = nranks;
  g->rank = rank;
  g->width = h->kind == GS_KIND_SIGNED ? 3 : 2;
  g->part = true;
  g->window = window_edges;
  auto bail = [&](int code) {
    gs_group_destroy(g);
    return code;
  };
  if (int rc = join_lanes(h)) return bail(rc);
  g->prev_track = h->track;
  if (window_edges) {  // records of the window: roots hooked away since the previous combine
    if (int rc = ensure_delta_list(h, window_edges)) return bail(rc);
    if (int rc = gs_set_delta_tracking(h, 1)) return bail(rc);
  }
  // the label forest: grows on its own (capacity checks of its folds)
  if (int rc = gs_create(&g->G, h->device, h->kind, std::max<uint64_t>(vertices_hint / 64, 1u << 12)))
    return bail(rc);
  uint64_t ocap = 1024;
  while (ocap < 4 * (vertices_hint / (uint64_t)nranks)) ocap <<= 1;  // load <= 1/4 at the hinted count
  if (ocap > (1ull << 31)) return bail(fail(GS_ERR_INVALID, "vertices_hint too large for the owner table"));
  g->ot.cap = (uint32_t)ocap;
  g->ot.mask = (uint32_t)(ocap - 1);
  int lg = 0;
  while ((1ull << lg) < ocap) ++lg;
  g->ot.shift = 64 - lg;
  g->ot.r0 = (uint32_t)ocap;
  const size_t pwords = 8 + (size_t)nranks + (size_t)nranks * nranks + nranks;
  bool ok = dmalloc(&g->ot.tab, (ocap + 1) * sizeof(gs::OwnerSlot)) == hipSuccess &&
            dmalloc(&g->mark, gs::kShards * 4) == hipSuccess && dmalloc(&g->snap, gs::kShards * 4) == hipSuccess &&
            dmalloc(&g->pflags, 16) == hipSuccess && dmalloc(&g->pdev, pwords * 8) == hipSuccess &&
            hipHostMalloc(&g->phost, pwords * 8, hipHostMallocDefault) == hipSuccess &&
            hipEventCreateWithFlags(&g->pev, hipEventDisableTiming) == hipSuccess;
  if (!ok) return bail(fail(GS_ERR_HIP, "partitioned group allocation failed"));
  g->ot.err = g->pflags;
  if (int rc = part_init_tables(g)) return bail(rc);
  GS_HIP(hipStreamSynchronize(h->stream));
  int r = api.comm_init_rank(&g->comm_c, nranks, id, rank);
  if (r != 0) return bail(rccl_fail(&api, "ncclCommInitRank(counts)", r));
  r = api.comm_init_rank(&g->comm_d, nranks, static_cast<const char*>(id) + kIdBytes, rank);
  if (r != 0) return bail(rccl_fail(&api, "ncclCommInitRank(data)", r));
  *out = g;
  return GS_OK;
}

int gs_group_part_fold_device(gs_group_t g, const int64_t* src, const int64_t* dst, size_t n) {
  if (int rc = part_of(g)) return rc;
  if (n && (!src || !dst)) return fail(GS_ERR_INVALID, "null edge arrays");
  if (g->window && g->win_edges + n > g->window)
    return fail(GS_ERR_INVALID, "more than window_edges own edges since the last combine");
  gs_summary* h = g->h;
  DeviceGuard dg(h->device);
  FoldSource fs;
  // folds pipeline (gs_set_pipelining), tracked ones too: the combine joins the lanes before it
  // reads the window's records
  fs.allow_pipe = true;
  fs.pipe_tracked = g->window != 0;
  hipEvent_t pa = ph_begin(g, h->stream);
  if (int rc = fold_device_impl(h, src, dst, nullptr, n, 1, 1, /*track=*/g->window != 0, true, fs)) return rc;
  ph_end(g, 0, pa, h->stream);
  g->win_edges += n;
  return GS_OK;
}

int gs_group_part_combine(gs_group_t g) {
  if (int rc = part_of(g)) return rc;
  gs_summary* h = g->h;
  DeviceGuard dg(h->device);
  if (int rc = join_lanes(h)) return rc;
  hipStream_t st = h->stream;
  const int N = g->nranks, W = g->width;
  const bool sign = h->kind == GS_KIND_SIGNED;
  const bool full = h->cap != g->cap_seen;  // the table was rebuilt: every vertex again
  const gs::Delta D = h->delta(0);
  unsigned long long* sendcnt = g->pdev + 8;
  unsigned long long* allcnt = sendcnt + N;
  unsigned long long* words = allcnt + (size_t)N * N;
  // 1. what is new since the previous combine
  hipEvent_t p0 = ph_begin(g, st);
  gs::launch_part_snap(h->table(), g->mark, g->snap, full ? 1 : 0, D.dctr, h->drec ? D.shard_cap : 0u, g->pdev, st);
  GS_HIP(hipGetLastError());
  if (int rc = part_read(g, 0, 3)) return rc;
  if (g->phost[2]) return fail(GS_ERR_CAPACITY, "vertex list overflow: the partitioned combine needs the list");
  const uint64_t total = g->phost[0], nrec = (g->window && h->track) ? g->phost[1] : 0;
  const uint32_t nblocks = (uint32_t)((total + gs::kPartRowsPB - 1) / gs::kPartRowsPB);
  if (int rc = ensure_buf(g->stage, g->stage_cap, std::max<uint64_t>(total, 1) * W, st)) return rc;
  if (int rc = ensure_buf(g->bcnt, g->bcnt_cap, (uint64_t)std::max<uint32_t>(nblocks, 1) * N, st)) return rc;
  if (int rc = ensure_buf(g->pairs, g->pairs_cap, (nrec + 1) * W, st)) return rc;
  GS_HIP(hipMemsetAsync(g->pdev + 3, 0, 8, st));
  // 2. export the new vertices (marks their roots), then the marked roots hooked away
  gs::launch_part_export(sign, h->table(), g->mark, g->snap, full ? 1 : 0, total, g->stage, W, g->bcnt, N, st);
  GS_HIP(hipGetLastError());
  if (nrec) {
    gs::launch_part_records(sign, h->table(), D, g->pairs, W, g->pdev + 3, g->pairs_cap / W, st);
    GS_HIP(hipGetLastError());
  }
  if (h->track) {  // the window's records are consumed
    GS_HIP(hipMemsetAsync(h->ctr + gs::ctr_index(gs::CTR_DELTA), 0, (size_t)gs::kShards * gs::kCtrStride * 4, st));
    h->delta_fill_ub[0] = 0;
  }
  ph_end(g, 1, p0, st);
  // 3. bucket by owner
  hipEvent_t p1 = ph_begin(g, st);
  if (total) {
    gs::launch_part_scan(g->bcnt, nblocks, N, sendcnt, st);
  } else {
    GS_HIP(hipMemsetAsync(sendcnt, 0, (size_t)N * 8, st));
  }
  if (int rc = ensure_buf(g->sendbuf, g->send_cap, std::max<uint64_t>(total, 1) * W, st)) return rc;
  gs::launch_part_scatter(g->stage, total, W, g->bcnt, nblocks, sendcnt, N, g->sendbuf, st);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(g->mark, g->snap, gs::kShards * 4, hipMemcpyDeviceToDevice, st));
  g->cap_seen = h->cap;
  ph_end(g, 2, p1, st);
  // 4. counts, then the rows to their owners
  hipEvent_t p2 = ph_begin(g, st);
  int r = g->api.all_gather(sendcnt, allcnt, (size_t)N, kNcclInt64, g->comm_c, st);
  if (r) return rccl_fail(&g->api, "ncclAllGather(part counts)", r);
  if (int rc = part_read(g, 8 + N, (size_t)N * N)) return rc;
  std::vector<size_t> sc(N), sd(N), rcv(N), rd(N);
  uint64_t total_recv = 0, so = 0;
  for (int q = 0; q < N; ++q) {
    sc[q] = (size_t)g->phost[8 + N + (size_t)g->rank * N + q] * W;
    sd[q] = so;
    so += sc[q];
    rcv[q] = (size_t)g->phost[8 + N + (size_t)q * N + g->rank] * W;
    rd[q] = (size_t)total_recv * W;
    total_recv += rcv[q] / W;
  }
  if (int rc = ensure_buf(g->recvbuf, g->recv_cap, std::max<uint64_t>(total_recv, 1) * W, st)) return rc;
  if (!g->api.all_to_allv) return fail(GS_ERR_HIP, "the comm backend has no all_to_allv");
  r = g->api.all_to_allv(g->sendbuf, sc.data(), sd.data(), g->recvbuf, rcv.data(), rd.data(), kNcclInt64, g->comm_d,
                         st);
  if (r) return rccl_fail(&g->api, "ncclAllToAllv(part rows)", r);
  ph_end(g, 3, p2, st);
  // 5. the owner step: anchors and label pairs
  hipEvent_t p3 = ph_begin(g, st);
  if (int rc = ensure_buf(g->pairs, g->pairs_cap, (nrec + total_recv + 1) * W, st, nrec * W)) return rc;
  // the pair set: ~1 slot per 4 received rows (2^12 .. 2^20: its probe bound lets a full set
  // emit a repeat, never drop a pair), cleared per combine
  gs::PairSet ps{nullptr, 0};
  if (N > 1 && total_recv) {
    uint64_t slots = 1ull << 12;
    while (slots < total_recv / 4 && slots < (1ull << 20)) slots <<= 1;
    if (int rc = ensure_buf(g->pset, g->pset_cap, slots, st)) return rc;
    GS_HIP(hipMemsetAsync(g->pset, 0, slots * sizeof(gs::PairSlot), st));
    ps.tab = g->pset;
    ps.mask = (uint32_t)(slots - 1);
  }
  gs::launch_part_owner(sign, g->ot, ps, g->recvbuf, total_recv, W, g->pairs, g->pdev + 3, g->pairs_cap / W,
                        g->pflags + 1, st);
  GS_HIP(hipGetLastError());
  gs::launch_part_count_word(g->pdev + 3, sign ? h->ctr + gs::ctr_index(gs::CTR_FAIL) : nullptr,
                             sign ? g->pflags + 1 : nullptr, g->pdev + 4, st);
  GS_HIP(hipGetLastError());
  // 6. every rank's pairs into every rank's label forest
  ph_end(g, 4, p3, st);
  hipEvent_t p4 = ph_begin(g, st);
  r = g->api.all_gather(g->pdev + 4, words, 1, kNcclInt64, g->comm_c, st);
  if (r) return rccl_fail(&g->api, "ncclAllGather(pair counts)", r);
  GS_HIP(hipMemcpyAsync(g->phost, g->pflags, 4, hipMemcpyDeviceToHost, st));  // owner-table overflow
  if (int rc = part_read(g, 8 + N + (size_t)N * N, (size_t)N)) return rc;
  if ((uint32_t)g->phost[0]) return fail(GS_ERR_CAPACITY, "owner table overflow: raise vertices_hint");
  uint64_t maxp = 0, live = 0, own = 0;
  for (int q = 0; q < N; ++q) {
    const uint64_t c = g->phost[8 + N + (size_t)N * N + q] & (gs::kFailBit - 1);
    maxp = std::max(maxp, c);
    live += c;
    if (q == g->rank) own = c;
  }
  if (own > g->pairs_cap / W) return fail(GS_ERR_CAPACITY, "label pair buffer overflow");
  const uint64_t rows = std::max<uint64_t>(maxp, 1);
  if (int rc = ensure_buf(g->pairs, g->pairs_cap, rows * W, st, own * W)) return rc;
  if (int rc = ensure_buf(g->pairs_all, g->pairs_all_cap, (uint64_t)N * rows * W, st)) return rc;
  r = g->api.all_gather(g->pairs, g->pairs_all, rows * W, kNcclInt64, g->comm_d, st);
  if (r) return rccl_fail(&g->api, "ncclAllGather(label pairs)", r);
  GS_HIP(hipEventRecord(g->pev, st));
  ph_end(g, 5, p4, st);
  gs_summary* G = g->G;
  GS_HIP(hipStreamWaitEvent(G->stream, g->pev, 0));
  G->xwait = true;
  hipEvent_t p5 = ph_begin(g, G->stream);
  FoldSource fs;
  fs.rows = (uint32_t)rows;
  fs.skip_rank = -1;
  fs.counts = words;
  fs.units = live;
  const uint8_t* w = W == 3 ? reinterpret_cast<const uint8_t*>(g->pairs_all + 2) : nullptr;
  if (int rc = fold_device_impl(G, g->pairs_all, g->pairs_all + 1, w, (size_t)N * rows, W, 8 * W, false, true, fs))
    return rc;
  ph_end(g, 6, p5, G->stream);
  // the next combine reuses pairs_all and the words only after this fold
  GS_HIP(hipEventRecord(g->pev, G->stream));
  GS_HIP(hipStreamWaitEvent(st, g->pev, 0));
  h->xwait = true;
  g->combines++;
  g->rows_exported += total;
  g->rows_owned += total_recv;
  g->pairs_sent += own;
  g->pairs_folded += live;
  g->win_edges = 0;
  if (g->phases) g->ph_exchanges++;
  return GS_OK;
}

int gs_group_part_labels_device(gs_group_t g, int64_t* v, int64_t* label, uint8_t* parity, size_t cap, size_t* n) {
  if (int rc = part_of(g)) return rc;
  if (!n || (cap && (!v || !label))) return fail(GS_ERR_INVALID, "null output");
  gs_summary* h = g->h;
  DeviceGuard dg(h->device);
  hipStream_t st = h->stream;
  if (int rc = join_lanes(g->G)) return rc;
  GS_HIP(hipEventRecord(g->pev, g->G->stream));
  GS_HIP(hipStreamWaitEvent(st, g->pev, 0));
  h->xwait = true;
  GS_HIP(hipMemsetAsync(g->pdev + 5, 0, 8, st));
  gs::launch_part_labels(g->ot, g->G->table(), v, label, parity, cap, g->pdev + 5, st);
  GS_HIP(hipGetLastError());
  if (int rc = part_read(g, 5, 1)) return rc;
  *n = (size_t)g->phost[5];
  if (*n > cap) return fail(GS_ERR_TRUNCATED, "output too small for the owned vertices");
  return GS_OK;
}

int gs_group_part_status(gs_group_t g, int* ok) {
  if (int rc = part_of(g)) return rc;
  if (!ok) return fail(GS_ERR_INVALID, "ok is null");
  return gs_bip_status(g->G, ok);  // every rank's verdict travels in its pair count word
}

int gs_group_part_reset(gs_group_t g) {
  if (int rc = part_of(g)) return rc;
  gs_summary* h = g->h;
  DeviceGuard dg(h->device);
  if (int rc = gs_reset(h)) return rc;
  if (int rc = gs_reset(g->G)) return rc;
  if (int rc = part_init_tables(g)) return rc;
  g->cap_seen = h->cap;
  g->combines = g->rows_exported = g->rows_owned = g->pairs_sent = g->pairs_folded = 0;  // per pass
  return GS_OK;
}

int gs_group_part_stats(gs_group_t g, uint64_t* out8) {
  if (int rc = part_of(g)) return rc;
  if (!out8) return fail(GS_ERR_INVALID, "out is null");
  uint64_t gv = 0;
  if (int rc = gs_num_vertices(g->G, &gv)) return rc;
  out8[0] = g->combines;
  out8[1] = g->rows_exported;
  out8[2] = g->rows_owned;
  out8[3] = g->pairs_sent;
  out8[4] = g->pairs_folded;
  out8[5] = gv;
  out8[6] = (uint64_t)g->ot.cap;
  out8[7] = 0;
  return GS_OK;
}

int gs_testing_group_forest(void* gv, void** forest) {
  gs_group_t g = static_cast<gs_group_t>(gv);
  if (!g || !forest) return fail(GS_ERR_INVALID, "null argument");
  *forest = g->part ? g->G : nullptr;
  return GS_OK;
}

int gs_group_part_phase_stats(gs_group_t g, double* out8) {
  if (int rc = part_of(g)) return rc;
  if (!out8) return fail(GS_ERR_INVALID, "out is null");
  DeviceGuard dg(g->h->device);
  ph_drain(g);
  for (int i = 0; i < 7; ++i) out8[i] = g->ph_ms[i];
  out8[7] = (double)g->ph_exchanges;
  return GS_OK;
}

}  // extern "C"
