// gs_internal.hpp -- the summary handle and the internal entry points shared by
// gs_capi.cpp (include/gs_summary.h), gs_group.cpp (include/gs_group.h) and
// gs_changes.cpp (per-window change emission).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "gs_ingest.hpp"
#include "gs_kernels.hpp"
#include "gs_summary.h"
#include "gs_testing.h"

namespace gsi {

int fail(int code, const std::string& msg);
// gs_testing.h: a test knob's value, or `product` while the knob is unset
int64_t testing_value(int knob, int64_t product);

// Device memory of summaries and groups: hipMalloc / hipFree plus the per-device byte
// count gs_hbm_bytes reports (tables that grow inside a fold or combine included).
hipError_t dmalloc(void** p, size_t bytes);
template <typename T>
inline hipError_t dmalloc(T** p, size_t bytes) {
  return dmalloc(reinterpret_cast<void**>(p), bytes);
}
hipError_t dfree(void* p);
constexpr int kMaxDevices = 64;
uint64_t create_capacity(uint64_t capacity_hint);
uint64_t create_bytes(uint64_t cap);

#define GS_HIP(call)                                                                                  \
  do {                                                                                                \
    hipError_t e_ = (call);                                                                           \
    if (e_ != hipSuccess)                                                                             \
      return ::gsi::fail(GS_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));              \
  } while (0)

constexpr uint32_t kMaxChunk = 1u << 22;     // edges per k_fold launch
constexpr uint32_t kStageChunk = 1u << 20;   // edges per pinned staging buffer
constexpr double kMaxLoad = 0.70;            // grow the table past this load factor
// Slots per hinted vertex at create (load <= 1/4 at the hinted count). Linear-probe
// clusters set the tail of a small window: config 5 (ER, 2^16-edge windows) p50
// 20.5 -> 13.3 us going from load 1/2 to 1/4; a 2^28-slot table for RMAT-26's 32.8 M
// vertices (load 1/8) was 2 % slower than 2^27 (profiles/r03_capacity_ab.txt).
constexpr uint64_t kSlotsPerHintedVertex = 4;
constexpr uint64_t kMaxCap = 1ull << 30;     // link holds slot << 1 in 32 bits
// A table whose load limit is crossed by pipeline slack alone (the capacity bound
// charges 2 new vertices per in-flight edge) grows once instead of waiting for
// capacity reports on every fold -- up to this many slots (1 GiB); tables keep
// their capacity across resets.
constexpr uint64_t kSlackGrowMaxCap = 1ull << 26;

enum { KID_FOLD = 0, KID_STAGE = 1, KID_EXPORT = 2, KID_INIT = 3, KID_N = 4 };

// per-shard edges of one k_fold launch of c edges (blocks are dealt to the 64
// shards round-robin from a rotating first shard)
inline uint64_t per_shard_edges(uint64_t c) {
  const uint64_t blocks = (c + gs::kFoldBS - 1) / gs::kFoldBS;
  return ((blocks + gs::kShards - 1) / gs::kShards) * gs::kFoldBS;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace gsi

struct gs_summary {
  int device = 0;
  int kind = GS_KIND_CC;
  hipStream_t stream = nullptr;
  // table + vertex list
  gs::Slot* tab = nullptr;  // [cap + 1]: hashed slots + the reserved slot of INT64_MIN
  uint64_t cap = 0;
  int logcap = 0;
  uint32_t* ctr = nullptr;
  uint32_t* vlist = nullptr;  // [kShards][vshard_cap]
  uint32_t vshard_cap = 0;
  uint32_t shard0 = 0;        // first shard of the next fold launch (rotates)
  bool vlist_ok = true;       // false once a shard of the vertex list overflowed (until reset)
  uint32_t* h_flags = nullptr;     // host-mapped mirror of CTR_ERR / CTR_OVF / CTR_VOVF (raise_flag)
  uint32_t* hflags_dev = nullptr;  // its device address
  // host waits (wait_stream): completion word {seq, value} in the same host-mapped
  // allocation (bytes 32..47), written by k_signal
  unsigned long long* h_done = nullptr;
  unsigned long long* done_dev = nullptr;
  unsigned long long done_seq = 0;
  // capacity tracking: a host upper bound of the vertex count, refreshed without
  // host synchronisation from k_report words (ring in host-coherent memory)
  uint64_t nv_ub = 0;
  uint64_t cap_waits = 0, cap_syncs = 0;  // capacity checks that waited for reports / joined every stream
  double cap_wait_s = 0;                  // host seconds spent in those waits
  static constexpr int kRepRing = 16;
  unsigned long long* rep = nullptr;      // host pointer
  unsigned long long* rep_dev = nullptr;  // its device mapping
  uint64_t rep_seq = 0;
  uint64_t rep_epoch = 0;  // resets since create: tags reports (k_report) so late ones are ignored
  static constexpr int kRepEvery = 4;    // each stream reports every 4th capacity-checked chunk
  static constexpr int kRepStreams = 6;  // handle stream, 4 lanes, side stream
  int rep_skip[kRepStreams] = {};
  uint64_t rep_pending[kRepStreams] = {};  // per stream: edges of chunks queued since its last report
  uint64_t rep_pending_edges = 0;          // their sum
  uint64_t e_launched = 0;  // edges of capacity-checked folds since reset / rebuild
  uint64_t e_lost = 0;      // launched edges no report will ever claim (complete: dropped at a sync)
  uint64_t nv_exact = 0, e_exact = 0;  // an exact count and the edges complete when it was read
  // delta records (multi-GPU exchange, change emission)
  // Two delta sets: a group's own fold b records into set b % 2 while the stage of
  // exchange b - 1 reads the other set on the communication stream.
  bool track = false;
  int64_t* drec = nullptr;  // [kDeltaSets][kShards][delta_shard_cap][3]
  uint32_t delta_shard_cap = 0;
  uint64_t delta_edges = 0;  // fold edges one delta set holds between two stages
  int dset = 0;              // the set tracked folds record into
  uint64_t delta_fill_ub[gs::kDeltaSets] = {};  // worst-case per-shard fill of each set since its last stage
  // change tracking (gs_changes.cpp)
  bool changes = false;
  bool changes_own_track = false;  // change tracking turned delta tracking on (and turns it off)
  uint32_t* nxt = nullptr;  // [cap + 1] circular member lists
  uint64_t nxt_slots = 0;
  unsigned long long* chg_scratch = nullptr;  // emission scratch: count, marks, big roots, staged records
  uint64_t chg_scratch_rows = 0;
  int64_t* chg_ov = nullptr;  // gs_take_changes (host arrays): device rows before the copy
  int64_t* chg_ol = nullptr;
  uint8_t* chg_op = nullptr;
  uint64_t chg_ocap = 0;
  bool chg_scan_all = false;  // the next emission emits every vertex (after a rebuild)
  // staging for host folds
  int64_t* d_stage = nullptr;  // [2][2][d_stage_chunk] (allocated by the first host fold)
  uint8_t* d_wstage = nullptr; // [2][d_stage_chunk]
  uint64_t d_stage_chunk = 0;  // edges per staging buffer
  int64_t* h_stage = nullptr;  // pinned, same shape: large host folds (allocated on first use)
  uint8_t* h_wstage = nullptr;
  hipEvent_t stage_ev[2] = {nullptr, nullptr};  // after each buffer's copies
  int stage_next = 0;
  int64_t* d_scratch = nullptr;  // small scratch (find_one)
  // combine export scratch (gs_combine source side): reused across calls
  int64_t* x_v = nullptr;
  int64_t* x_l = nullptr;
  uint8_t* x_p = nullptr;
  uint64_t x_cap = 0;
  unsigned long long* x_cnt = nullptr;  // device: exported rows (u64) + failure flag (u32 at word 1)
  hipEvent_t x_ready = nullptr, x_used = nullptr;
  bool x_pending = false;  // x_used recorded by a consumer not yet waited for
  // text ingest (gs_fold_text): pinned + device text chunks, parsed edges, scratch
  char* h_text = nullptr;
  uint64_t* h_tres = nullptr;
  hipEvent_t text_ev[2] = {nullptr, nullptr};
  char* d_text = nullptr;
  int64_t* d_tsrc = nullptr;
  int64_t* d_tdst = nullptr;
  void* d_tscratch = nullptr;
  gs::ParseScratch tscratch;
  // pipelined folds (gs_set_pipelining): consecutive plain device folds alternate
  // over lane streams so that fold b+1 may start while fold b drains; every other
  // entry point joins the lanes onto `stream` first (join_lanes)
  int pipe_depth = 1;
  uint64_t api_calls = 0;  // gs_* calls made on the handle (gs_group_fold_device orders its lanes after any)
  int group_lanes = 0;  // own-fold lanes of an exchange group using this summary (0: none)
  static constexpr int kLanes = 4;
  hipStream_t lane[kLanes] = {};
  hipEvent_t lane_ev[kLanes] = {};
  hipEvent_t main_ev = nullptr;
  hipEvent_t ext_ev = nullptr;  // gs_wait_stream: recorded on a producer's stream
  hipEvent_t idle_ev = nullptr;  // stream_idle: recorded and queried
  // h->stream holds waits on other streams' events queued since its last completion-kernel wait:
  // only a kernel queued behind them observes them (an event recorded there completed at once
  // in the multi-rank replay), so an idle check must not be taken then
  bool xwait = false;
  int lane_next = 0;
  int last_lane = -1;  // lane of the most recently queued fold (the label pass runs there)
  bool lanes_dirty = false;
  bool export_ctr_zero = false;  // CTR_EXPORT is zero behind the queued work (no fill before an export)
  // side stream (a multi-GPU group's apply stream): folds of remote rows run there,
  // overlapping this rank's own folds; every reader joins it (join_lanes), the
  // handle's own folds do not (union commutes)
  hipStream_t side = nullptr;
  hipEvent_t side_ev = nullptr;
  bool side_dirty = false;
  // micro-batch dedup by hashing (gs_set_batch_dedup): one scratch set per stream a
  // fold may run on (handle stream, lanes, side stream): pair table + skip marks
  bool dedup = false;
  static constexpr int kDedupSets = kLanes + 2;
  unsigned long long* dd_tab[kDedupSets] = {};
  uint8_t* dd_w[kDedupSets] = {};
  uint64_t dd_edges[kDedupSets] = {};  // edges a set holds (its table has 2x that, a power of two)
  uint64_t dd_kept_hint = 0;
  // resident window server (gs_set_window_server): one persistent launch serves the
  // latency path's windows; every other entry point stops it first (join_lanes)
  bool srv_on = false, srv_running = false;
  int srv_fits = -1;                     // all kServerBlocks workgroups co-resident (-1: not yet checked)
  gs::ServerBox* srv_box = nullptr;      // host-mapped mailbox
  gs::ServerBcast* srv_bc = nullptr;     // device: block 0 -> other blocks
  unsigned long long srv_seq = 0;        // last window posted and completed
  uint64_t srv_launches = 0, srv_windows = 0;
  // profiling
  bool profiling = false;
  struct Pending {
    int kid;
    hipEvent_t a, b;
  };
  std::vector<Pending> prof_pending;
  std::vector<hipEvent_t> ev_pool;
  uint64_t launches[gsi::KID_N] = {0, 0, 0, 0};
  double total_ms[gsi::KID_N] = {0, 0, 0, 0};

  gs::Table table() const {
    gs::Table t;
    t.tab = tab;
    t.ctr = ctr;
    t.cap = (uint32_t)cap;
    t.mask = (uint32_t)(cap - 1);
    t.shift = 64 - logcap;
    t.r0 = (uint32_t)cap;
    t.vlist = vlist;
    t.vshard_cap = vshard_cap;
    t.mark_new = changes ? 1 : 0;
    t.hflags = hflags_dev;
    return t;
  }
  gs::Delta delta(int set = -1) const {
    if (set < 0) set = dset;
    gs::Delta D;
    D.drec = drec ? drec + (size_t)set * gs::kShards * delta_shard_cap * 3 : nullptr;
    D.shard_cap = delta_shard_cap;
    D.dctr = (uint32_t)(gs::CTR_DELTA + set * gs::kShards);
    return D;
  }
};

namespace gsi {

// Where a fold's rows come from (defaults: plain edge arrays on the handle stream).
struct FoldSource {
  uint32_t rows = 0;  // > 0: gathered exchange buffer, world blocks of `rows` rows
  int skip_rank = -1;
  const unsigned long long* counts = nullptr;  // device: live rows per block (| kFailBit)
  uint64_t units = 0;  // exchange layout: rows that may add vertices (capacity charge)
  const unsigned long long* n_dev = nullptr;   // device element count (<= n)
  const uint32_t* fail_in = nullptr;           // device failure flag of a combined summary
  bool on_side = false;  // launch on h->side (a group's apply stream) instead of h->stream
  bool allow_pipe = false;
  // a TRACKED fold may pipeline too: its caller takes the delta set only after joining the
  // lanes (the partitioned group's windows: records go to one set through sharded atomics)
  bool pipe_tracked = false;
  int lane = -1;         // >= 0: launch on this pipelining lane (a group's own tracked fold)
  // fused window take (gs_fold_take_device): one tracked launch that also writes the
  // rows, the count and the completion word {seq, vertices, rows}
  int64_t* take_out = nullptr;
  uint64_t take_cap = 0;
  unsigned long long* take_count = nullptr;
  unsigned long long* take_seq = nullptr;  // out: the completion sequence number, drawn at launch
};

int fold_device_impl(gs_summary* h, const int64_t* src, const int64_t* dst, const uint8_t* w, size_t n,
                     size_t stride, size_t w_stride, bool track, bool check_cap = true,
                     const FoldSource& fs = FoldSource());
int join_lanes(gs_summary* h);
bool side_ok(const gs_summary* h);
int flush_reports(gs_summary* h);  // standalone capacity reports of every stream's unclaimed chunks
int ensure_lanes(gs_summary* h, int n);  // create lane streams 0..n-1 on first use
int read_nv(gs_summary* h, uint64_t* nv);
// wait until every operation queued on h->stream (or `st`) so far has completed; *value
// (optional) = the sum of nvals device u32 counters vals[i * stride], read in the same
// round trip (and zeroed behind the read with `clear`)
int wait_stream(gs_summary* h, const uint32_t* vals = nullptr, uint64_t* value = nullptr, int nvals = 1,
                int stride = 0, bool clear = false, hipStream_t st = nullptr, const uint32_t* flag = nullptr);
int check_device_flags(gs_summary* h);
int check_flags_now(gs_summary* h);
int done_value_read(gs_summary* h, int i, unsigned long long seq, uint64_t* out);  // tagged completion value
int wait_done(gs_summary* h, unsigned long long seq, hipStream_t st = nullptr);  // spin on the completion word (h->stream / st)  // after a wait: the host-mapped flags only
int export_device_impl(gs_summary* h, int64_t* v, int64_t* l, uint8_t* p, size_t cap, size_t* n, int part = 0,
                       int nparts = 1);
// stage every pending delta record into out (first cap rows, `width` int64 each) and
// the count word into *count_out (device); the delta list is emptied
int stage_delta(gs_summary* h, int64_t* out, uint64_t cap, int width, unsigned long long* count_out, bool with_fail,
                hipStream_t st = nullptr, int set = -1);
int ensure_delta_list(gs_summary* h, uint64_t edges);
bool use_vertex_list(gs_summary* h, uint64_t nv_bound);
// gs_changes.cpp, after a reset (mode 0: vertex-list reset, 1: full table init) or a
// rebuild into a new table (mode 2)
int change_tracking_reset(gs_summary* h, int mode);

}  // namespace gsi
