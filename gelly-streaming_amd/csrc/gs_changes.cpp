// gs_changes.cpp -- per-window change emission (include/gs_summary.h,
// gs_set_change_tracking / gs_take_changes_device). Kernels and the member-list
// argument: gs_changes_k.hip.
//
// the reference's Merger emits the whole cumulative summary
// every window (SummaryAggregation.java:107-119) and its sinks flatten it
// (ConnectedComponentsExample.FlattenSet :143-156, DisjointSet.toString :134-150),
// O(V) per window. Here a window's emission is the rows whose canonical label
// changed -- members of every hooked old root, found by walking its member list --
// plus the vertices inserted since the previous emission: O(changes), not O(V).
// A relabelled component longer than the walk limit is emitted by one parallel
// scan instead (with its absorbing root's unchanged members: idempotent rows).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "gs_internal.hpp"

namespace gsi {

namespace {

constexpr uint32_t kWalkMax = 1u << 16;  // member-list walk limit per hooked root

uint32_t walk_max() {  // test knob GS_TESTING_CHANGES_WALK_MAX forces the scan path
  return (uint32_t)std::max<int64_t>(1, std::min<int64_t>(testing_value(GS_TESTING_CHANGES_WALK_MAX, kWalkMax), kWalkMax));
}

// scratch layout: [0] record count (u64), [1..8] vertex-list marks (64 x u32),
// then the big-root list (u32 x rows), then the staged records (3 x int64 x rows)
struct ChgScratch {
  unsigned long long* nrec;
  uint32_t* vmark;
  uint32_t* big;
  int64_t* rec;
};

ChgScratch scratch(gs_summary* h) {
  ChgScratch c;
  c.nrec = h->chg_scratch;
  c.vmark = reinterpret_cast<uint32_t*>(h->chg_scratch + 1);
  c.big = reinterpret_cast<uint32_t*>(h->chg_scratch + 1 + gs::kShards / 2);
  c.rec = reinterpret_cast<int64_t*>(h->chg_scratch + 1 + gs::kShards / 2 + (h->chg_scratch_rows + 1) / 2);
  return c;
}

int ensure_scratch(gs_summary* h) {
  const uint64_t rows = (uint64_t)gs::kShards * h->delta_shard_cap;
  if (h->chg_scratch && h->chg_scratch_rows >= rows) return GS_OK;
  if (h->chg_scratch) {
    GS_HIP(hipStreamSynchronize(h->stream));
    (void)dfree(h->chg_scratch);
    h->chg_scratch = nullptr;
  }
  const size_t words = 1 + gs::kShards / 2 + (rows + 1) / 2 + 3 * rows;
  GS_HIP(dmalloc(&h->chg_scratch, words * 8));
  GS_HIP(hipMemsetAsync(h->chg_scratch, 0, (1 + gs::kShards / 2) * 8, h->stream));
  h->chg_scratch_rows = rows;
  return GS_OK;
}

int ensure_nxt(gs_summary* h) {
  if (h->nxt && h->nxt_slots == h->cap + 1) return GS_OK;
  if (h->nxt) {
    GS_HIP(hipStreamSynchronize(h->stream));
    (void)dfree(h->nxt);
    h->nxt = nullptr;
  }
  GS_HIP(dmalloc(&h->nxt, (h->cap + 1) * 4));
  h->nxt_slots = h->cap + 1;
  return GS_OK;
}

}  // namespace

// mode 0: the vertex-list reset already restored nxt of the touched slots;
// 1: a full table init (reset of a dense table); 2: a rebuild into a new table
// (grow): the next emission emits every vertex and rebuilds the lists.
int change_tracking_reset(gs_summary* h, int mode) {
  if (!h->changes) return GS_OK;
  if (int rc = ensure_nxt(h)) return rc;
  if (int rc = ensure_scratch(h)) return rc;
  if (mode >= 1) gs::launch_iota(h->nxt, h->cap + 1, h->stream);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemsetAsync(scratch(h).vmark, 0, gs::kShards * 4, h->stream));
  h->chg_scan_all = mode == 2;
  return GS_OK;
}

}  // namespace gsi

using namespace gsi;

extern "C" {

int gs_set_change_tracking(gs_handle h, int on) {
  if (!h) return fail(GS_ERR_INVALID, "null handle");
  DeviceGuard g(h->device);
  if (int rc = join_lanes(h)) return rc;
  if (!on) {
    if (h->changes && h->changes_own_track) {  // the delta tracking it turned on goes with it
      h->changes = false;
      h->changes_own_track = false;
      return gs_set_delta_tracking(h, 0);
    }
    h->changes = false;
    return GS_OK;
  }
  if (h->changes) return GS_OK;
  if (h->side) return fail(GS_ERR_INVALID, "a group's summary exchanges its delta: no change tracking");
  h->changes_own_track = !h->track;
  if (!h->track)
    if (int rc = gs_set_delta_tracking(h, 1)) return rc;
  uint64_t nv = 0;
  if (int rc = read_nv(h, &nv)) return rc;
  h->changes = true;
  if (int rc = change_tracking_reset(h, 1)) return rc;
  if (nv) {  // existing vertices: lists of the current forest, first emission = everything
    gs::launch_relist(h->table(), h->nxt, h->stream);
    GS_HIP(hipGetLastError());
    h->chg_scan_all = true;
  }
  return GS_OK;
}

int gs_take_changes_device(gs_handle h, int64_t* v, int64_t* label, uint8_t* parity, size_t cap, uint64_t* n) {
  if (!h) return fail(GS_ERR_INVALID, "null handle");
  if (!n || (cap && (!v || !label))) return fail(GS_ERR_INVALID, "null argument");
  if (!h->changes) return fail(GS_ERR_INVALID, "change tracking is off");
  DeviceGuard g(h->device);
  uint64_t nv = 0;
  if (int rc = read_nv(h, &nv)) return rc;  // joins every stream
  *n = 0;
  if (cap < nv) return fail(GS_ERR_INVALID, "cap below the vertex count: " + std::to_string(nv));
  if (int rc = check_flags_now(h)) return rc;  // read_nv waited
  if (int rc = ensure_scratch(h)) return rc;
  const ChgScratch c = scratch(h);
  const gs::Table t = h->table();
  GS_HIP(hipMemsetAsync(h->ctr + gs::ctr_index(gs::CTR_EMIT), 0, 8, h->stream));
  GS_HIP(hipMemsetAsync(h->ctr + gs::ctr_index(gs::CTR_BIG), 0, 4, h->stream));
  // this window's hook records (every tracked fold since the previous emission)
  if (int rc = stage_delta(h, c.rec, h->chg_scratch_rows, 3, c.nrec, false)) return rc;
  const bool all = h->chg_scan_all || !h->vlist_ok;
  if (all) {  // after a rebuild (or a vertex-list overflow): every vertex, fresh lists
    gs::launch_emit_scan(t, v, label, parity, cap, true, h->stream);
    gs::launch_iota(h->nxt, h->cap + 1, h->stream);
    gs::launch_relist(t, h->nxt, h->stream);
    gs::launch_emit_new(t, c.vmark, v, label, parity, cap, h->vlist_ok ? nv : 0, false, h->stream);  // marks
    GS_HIP(hipGetLastError());
    h->chg_scan_all = false;
  } else {
    uint64_t nrec = 0;  // (< 2^32: at most the delta capacity)
    if (int rc = wait_stream(h, reinterpret_cast<const uint32_t*>(c.nrec), &nrec)) return rc;
    // phase 0 flags roots too large to walk, phase 1 walks the rest and splices
    if (nrec) gs::launch_emit_records(t, h->nxt, c.rec, c.nrec, nrec, walk_max(), v, label, parity, cap, c.big, h->stream);
    GS_HIP(hipGetLastError());
    uint64_t nbig = 0;
    if (int rc = wait_stream(h, h->ctr + gs::ctr_index(gs::CTR_BIG), &nbig)) return rc;
    if (nbig) {  // before k_emit_new clears the new bits the scan tests
      gs::launch_emit_scan(t, v, label, parity, cap, false, h->stream);
      gs::launch_clear_big(t, c.big, nbig, h->stream);
    }
    gs::launch_emit_new(t, c.vmark, v, label, parity, cap, nv, true, h->stream);
    GS_HIP(hipGetLastError());
  }
  uint64_t emitted = 0;  // (low word of the u64 counter: rows < 2^32)
  if (int rc = wait_stream(h, h->ctr + gs::ctr_index(gs::CTR_EMIT), &emitted)) return rc;
  *n = emitted;
  if (emitted > cap) {
    // the emission's side effects (spliced lists, cleared new bits, advanced marks)
    // happened: rows past cap cannot be emitted again by a retry, so the next take
    // emits every vertex
    h->chg_scan_all = true;
    return fail(GS_ERR_TRUNCATED, "emission rows above cap");
  }
  return GS_OK;
}

// Host-array variant for JVM sinks: the rows are emitted into
// grow-only device scratch of the handle, then copied out (synchronises).
int gs_take_changes(gs_handle h, int64_t* v, int64_t* label, uint8_t* parity, size_t cap, uint64_t* n) {
  if (!h) return fail(GS_ERR_INVALID, "null handle");
  if (!n || (cap && (!v || !label))) return fail(GS_ERR_INVALID, "null argument");
  if (!h->changes) return fail(GS_ERR_INVALID, "change tracking is off");
  DeviceGuard g(h->device);
  uint64_t nv = 0;
  if (int rc = read_nv(h, &nv)) return rc;
  *n = 0;
  if (cap < nv) return fail(GS_ERR_INVALID, "cap below the vertex count: " + std::to_string(nv));
  if (h->chg_ocap < nv + 1) {
    (void)dfree(h->chg_ov);
    (void)dfree(h->chg_ol);
    (void)dfree(h->chg_op);
    h->chg_ov = h->chg_ol = nullptr;
    h->chg_op = nullptr;
    h->chg_ocap = 0;
    const uint64_t rows = std::max<uint64_t>(nv + 1, 1024) * 5 / 4;  // headroom: fewer reallocations
    GS_HIP(dmalloc(&h->chg_ov, rows * 8));
    GS_HIP(dmalloc(&h->chg_ol, rows * 8));
    GS_HIP(dmalloc(&h->chg_op, rows));
    h->chg_ocap = rows;
  }
  uint64_t k = 0;
  if (int rc = gs_take_changes_device(h, h->chg_ov, h->chg_ol, parity ? h->chg_op : nullptr, h->chg_ocap, &k))
    return rc;
  if (k) {
    GS_HIP(hipMemcpyAsync(v, h->chg_ov, k * 8, hipMemcpyDeviceToHost, h->stream));
    GS_HIP(hipMemcpyAsync(label, h->chg_ol, k * 8, hipMemcpyDeviceToHost, h->stream));
    if (parity) GS_HIP(hipMemcpyAsync(parity, h->chg_op, k, hipMemcpyDeviceToHost, h->stream));
    GS_HIP(hipStreamSynchronize(h->stream));
  }
  *n = k;
  return GS_OK;
}

}  // extern "C"
