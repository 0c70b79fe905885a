/*
 * gs_summary.h -- C ABI of the MI355X-native summary-aggregation hot path.
 *
 * Drop-in boundary for gelly-streaming's SimpleEdgeStream.aggregate() ->
 * SummaryBulkAggregation path as used by ConnectedComponents (DisjointSet summary)
 * and BipartitenessCheck (Candidates summary). A GPU-resident union-find forest
 * (CC) or signed union-find forest (bipartiteness) lives behind an opaque handle;
 * the JVM-side summary objects buffer their per-edge callbacks and flush them here
 * (binding stubs: INTEGRATION.md). Reference paths are relative to
 * src/main/java/org/apache/flink/graph/streaming/ in jiexray/gelly-streaming.
 *
 * Conventions
 *   - Every function returns GS_OK (0) or a negative GS_ERR_* code; the message of
 *     the last failure on the calling thread is gs_last_error() (the reference's
 *     `throws Exception` on foldEdges/reduce, EdgesFold.java:47).
 *   - Plain pointers and sizes only. "host" buffers are caller-owned and copied
 *     before the call returns; "device" buffers must live on the handle's device.
 *   - A handle is thread-compatible (one thread at a time), the library is
 *     re-entrant across handles. Work is enqueued on the handle's own HIP stream;
 *     functions that return data to the host synchronise that stream.
 *   - Vertex ids are signed 64-bit (Edge<Long,...>; Integer ids widen losslessly).
 *     Canonical component label = minimum signed id in the component.
 */
#ifndef GS_SUMMARY_H
#define GS_SUMMARY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gs_summary* gs_handle;

enum gs_status {
  GS_OK = 0,
  GS_ERR_INVALID = -1,  /* bad argument / handle */
  GS_ERR_HIP = -2,      /* HIP runtime error (device missing, OOM, launch failure) */
  GS_ERR_CAPACITY = -3, /* vertex table cannot grow further */
  GS_ERR_TRUNCATED = -4 /* output buffer too small; *n holds the required count */
};

/* Count words (delta takes, exchange stages) carry a failed signed verdict in bit 62. */
#define GS_FAIL_BIT (1ull << 62)

enum gs_kind {
  GS_KIND_CC = 0,     /* DisjointSet (DisjointSet.java:25-151) via ConnectedComponents */
  GS_KIND_SIGNED = 1  /* Candidates (Candidates.java:27-196) via BipartitenessCheck  */
};

/* Last error message of the calling thread ("" if none). */
const char* gs_last_error(void);

/* Library/ABI version (major*10000 + minor*100 + patch). */
int gs_version(void);

/* Create an empty summary on HIP device `device`. `capacity_hint` = expected
 * number of distinct vertices: the table starts with >= 4 slots per hinted vertex
 * (load <= 1/4, short probe clusters) and grows past it automatically.
 * Replaces the summary's initial value: `new DisjointSet<>()`
 * (ConnectedComponents.java:52-54) / `new Candidates(true)` (BipartitenessCheck.java:50-52). */
int gs_create(gs_handle* out, int device, int kind, uint64_t capacity_hint);

/* Release the handle and its device memory. */
int gs_destroy(gs_handle h);

/* Reset to the initial value (empty forest, verdict true). Replaces
 * `summary = initialVal` of a transient Merger (SummaryAggregation.java:113-115)
 * and Flink's per-window copy of the initial value (a pooled handle is reset
 * instead of created). Asynchronous; O(vertices) on a sparse table
 * (only the touched slots are re-initialised). */
int gs_reset(gs_handle h);

/* gs_reset plus the handle's default configuration: delta and change tracking off,
 * pipelining depth 1, profiling off -- a pooled handle handed to the next summary
 * behaves as a fresh gs_create (the per-window initial-value copy, INTEGRATION.md
 * HandlePool). Not for a group's summary (destroy the group first). */
int gs_reset_config(gs_handle h);

/* Fold n edges from HOST memory: for each i, union(src[i], dst[i]).
 * Replaces UpdateCC.foldEdges -> DisjointSet.union (ConnectedComponents.java:83-86,
 * DisjointSet.java:92-118) and updateFunction.foldEdges ->
 * candidates.merge(edgeToCandidate(u, v)) (BipartitenessCheck.java:54-61,93-95),
 * called once per buffered micro-batch instead of once per edge.
 * New endpoints are added (DisjointSet.makeSet :53-56); a self-loop adds its vertex
 * and never fails the bipartiteness verdict (BipartitenessCheck.java:58-59).
 * src/dst may be pageable or pinned; the fold itself is asynchronous, but the edges
 * have been copied to the device when the call returns, so the caller may reuse them. */
int gs_fold(gs_handle h, const int64_t* src, const int64_t* dst, size_t n);

/* Same with a required colour parity per edge from HOST memory (GS_KIND_SIGNED; w[i]
 * bit 0: 1 = different sides, as every edge of the stream; 0 = same side). This is a
 * general Candidates merged in component by component (Candidates.merge :77-139 with
 * an input that is not a one-edge candidate: each vertex against its component's
 * anchor, parity = the two signs differ). A CC summary ignores w. */
int gs_fold_parity(gs_handle h, const int64_t* src, const int64_t* dst, const uint8_t* w, size_t n);

/* Same, from DEVICE memory already resident on the handle's device. Element i is
 * src[i*stride], dst[i*stride] (stride 1: two arrays; stride 2 with dst = src + 1:
 * interleaved pairs). `w` (device, optional, may be NULL) gives the required colour
 * parity per edge for GS_KIND_SIGNED (1 = different sides, the edge default;
 * 0 = same side, used when a serialized/exported summary is merged back). The
 * inputs must be complete before work on the handle's stream: written on that
 * stream (gs_get_stream), synchronised, or ordered with gs_wait_event /
 * gs_wait_stream / gs_fold_device_after below. */
int gs_fold_device(gs_handle h, const int64_t* src, const int64_t* dst, const uint8_t* w, size_t n, size_t stride);

/* Micro-batch dedup by hashing (north_star's staging stage). With it on, every fold of
 * edges without a parity array (gs_fold, gs_fold_device with stride 1, the window take)
 * first inserts each edge's unordered pair into a batch hash table and marks exact
 * repeats of a pair within the launch's chunk; the fold skips them (union is
 * idempotent: the result is identical). It pays one batch-table insert per edge, so it
 * is off by default: it wins on streams with many repeated edges (the reference's
 * bipartite example repeats every edge 10 times, BipartitenessCheckExample.java:109-118)
 * and loses on RMAT, whose repeats are rare. */
int gs_set_batch_dedup(gs_handle h, int on);

/* Cross-stream ordering for callers whose edges are produced on another stream (a
 * decoder, a copy engine, torch): gs_wait_event makes every later operation of the
 * handle wait for `event` (a hipEvent_t the producer recorded); gs_wait_stream for
 * all work queued on `stream` (a hipStream_t) so far. No host synchronisation.
 * gs_fold_device_after = gs_wait_event(ready) (skipped when ready is NULL) +
 * gs_fold_device. Pipelined folds and a group's own folds are ordered too. */
int gs_wait_event(gs_handle h, void* event);
int gs_wait_stream(gs_handle h, void* stream);
int gs_fold_device_after(gs_handle h, const int64_t* src, const int64_t* dst, const uint8_t* w, size_t n,
                         size_t stride, void* ready);

/* Pipelined windows: with depth d (1..4), up to d consecutive gs_fold_device calls
 * may run concurrently on the device (fold b+1 starts while fold b drains), the way Flink
 * runs the window fold of window w+1 while the Merger still handles window w
 * (SummaryBulkAggregation.java:77-90 is a pipelined dataflow). Union is associative
 * and commutative, so the forest after the folds is the same; every other call on
 * the handle (reads, exports, combine, serialize, sync, gs_get_stream) first orders
 * the handle's stream behind all pending folds. Device buffers passed to a
 * pipelined fold must stay valid until that next call. Applies to plain folds
 * (no delta or change tracking, profiling off); depth 1 (default) = in order.
 * Each lane is a HIP stream, and streams beyond GPU_MAX_HW_QUEUES share hardware
 * queues (run in submission order): depth 2 fits HIP's default of 4 queues beside the
 * handle's and the process's null stream in any creation order; depth 3 gains ~1 %
 * when its lanes land on distinct queues and loses ~15 % when two share one
 * (DESIGN.md section 7). */
int gs_set_pipelining(gs_handle h, int depth);

/* Merge summary `src` into `dst` (either may be on any device; `src` is unchanged).
 * Replaces CombineCC.reduce -> DisjointSet.merge (ConnectedComponents.java:116-126,
 * DisjointSet.java:127-131) and combineFunction.reduce -> Candidates.merge
 * (BipartitenessCheck.java:128-130, Candidates.java:77-139); the verdict is the AND.
 * Asynchronous: src is exported on its stream (over its vertex list when sparse:
 * O(vertices of src), not O(table)), dst folds the rows behind an event; the row
 * count and verdict are read on the device. No host synchronisation and, once the
 * reusable scratch is sized, no allocation. */
int gs_combine(gs_handle dst, gs_handle src);

/* Receiving half of a combine from EXPORTED arrays (gs_export_labels_device of
 * another summary, e.g. received from another rank): folds union(v[i], label[i])
 * with required parity parity[i] (NULL for GS_KIND_CC) -- DisjointSet.merge
 * (DisjointSet.java:127-131: union(k, parent(k)) for every entry) -- and ANDs the
 * verdict with !failed (BipartitenessCheck.java:128-130 -> Candidates.java:79-81).
 * DEVICE arrays on h's device; queued on h's stream. */
int gs_combine_exported_device(gs_handle h, const int64_t* v, const int64_t* label, const uint8_t* parity, size_t n,
                               int failed);

/* Block until all work queued on the handle has finished. */
int gs_sync(gs_handle h);

/* Number of distinct vertices seen (DisjointSet.getMatches().size(), :44-46). */
int gs_num_vertices(gs_handle h, uint64_t* n);

/* Canonical label of one vertex: *label = min id of its component; *found = 0 if
 * the vertex was never seen (DisjointSet.find returns null, :66-69). */
int gs_find(gs_handle h, int64_t v, int64_t* label, int* found);

/* Batched find over DEVICE arrays: label[i] = canonical label of v[i]; found[i]
 * (optional, may be NULL) = 0 for an id never seen (label[i] is then v[i]).
 * Asynchronous on the handle's stream (DisjointSet.find, :66-80, for many ids). */
int gs_find_labels_device(gs_handle h, const int64_t* v, size_t n, int64_t* label, uint8_t* found);

/* Order-independent 64-bit digest of the summary (synchronises): the sum, mod 2^64, over
 * every vertex v of mix64(v ^ C1) * mix64(label(v) + parity(v) * C2) (splitmix64
 * finaliser; parity = 0 for GS_KIND_CC). Two summaries with the same partition (and
 * colouring) have the same digest whatever their fold order, windows, devices or ranks,
 * so replicas are compared without an export -- what the reference's tests compare as
 * sorted strings (ConnectedComponentsTest.java:54-63, DisjointSet.toString :134-150).
 * A GS_KIND_SIGNED summary whose verdict failed digests to GS_DIGEST_FAILED, as its
 * output is (false,{}) (Candidates.java:194-196). Not part of the reference API. */
#define GS_DIGEST_FAILED (~0ull)
int gs_digest(gs_handle h, uint64_t* digest);

/* Export every (vertex, canonical label) pair to HOST arrays of capacity `cap`,
 * unordered. *n = number of vertices (GS_ERR_TRUNCATED if cap < *n; nothing
 * written). Replaces getMatches()/find()/toString() sinks (DisjointSet.java:44-46,
 * 134-150; ConnectedComponentsExample.FlattenSet :143-156). */
int gs_export_labels(gs_handle h, int64_t* v, int64_t* label, size_t cap, size_t* n);

/* Same into DEVICE arrays; *n is written on the host (synchronises). Used for
 * the final canonical label pass without a device->host copy. `parity` (device,
 * may be NULL) receives parity(v) xor parity(label) for GS_KIND_SIGNED. */
int gs_export_labels_device(gs_handle h, int64_t* v, int64_t* label, uint8_t* parity, size_t cap, size_t* n);

/* Part `part` of `nparts` of the same export: the vertices whose dense id (table
 * slot) lies in the part-th of nparts equal slot ranges. The parts are disjoint and
 * together are exactly gs_export_labels_device. Replicas kept equal by a group
 * (gs_group.h) emit the final label pass partitioned: rank r exports part r, like
 * a Flink sink at parallelism p consuming a keyed stream. DEVICE arrays; *n on the
 * host (synchronises). */
int gs_export_labels_part_device(gs_handle h, int part, int nparts, int64_t* v, int64_t* label, uint8_t* parity,
                                 size_t cap, size_t* n);

/* Bipartiteness verdict so far (Candidates.getSuccess, :44-46): 1 = bipartite. */
int gs_bip_status(gs_handle h, int* ok);

/* Canonical colouring to HOST arrays (Candidates.getMap, :48-50): comp = min id of
 * the component, sign = 1 when v has the colour of comp (SignedVertex sign,
 * SignedVertex.java:23-40). Unordered. When the verdict is false, *n = 0
 * (the reference's fail() state is (false,{}), Candidates.java:194-196). */
int gs_export_colouring(gs_handle h, int64_t* comp, int64_t* v, uint8_t* sign, size_t cap, size_t* n);

/* Checkpoint: compact (vertex, label, parity) image of the summary plus the
 * verdict, for Merger.snapshotState/restoreState (SummaryAggregation.java:127-135).
 * Call with buf = NULL to get *len. gs_deserialize replaces the summary. */
int gs_serialize(gs_handle h, void* buf, size_t cap, size_t* len);
int gs_deserialize(gs_handle h, const void* buf, size_t len);

/* ---- streaming delta (multi-GPU combine; see DESIGN.md "Multi-GPU") ----------
 * While tracking is on, every fold records the structural changes it made:
 * each successful hook as (root, new parent, parity) and each new vertex seen
 * only through a self-loop as (v, v, 0) (every other new vertex is named by a
 * hook record): at most one record per folded edge. Folding another replica's
 * delta into this summary reproduces that replica's changes (union is associative
 * and commutative), which replaces shipping whole summaries to one reducer
 * (SummaryBulkAggregation.java:77-83).
 *
 * The delta list holds the records of gs_delta_capacity() rows (the folds of at
 * least 2^22 edges, more after gs_group_create with a larger batch) between two
 * takes/stages; a tracked fold past that fails with GS_ERR_CAPACITY.
 *
 * gs_take_delta_records packs the delta accumulated since the previous take into
 * DEVICE records {a, b, w} (24 bytes; w bit 0 = parity, w bit 7 = skip), first
 * `cap` of them, and writes the COUNT WORD to the DEVICE word *count: the total
 * record count, | GS_FAIL_BIT (2^62) once a GS_KIND_SIGNED summary's verdict has
 * failed -- a failed verdict travels with the records even when no record names
 * the odd cycle (Candidates.merge :79-81). Both complete on the handle's stream (no
 * host synchronisation). gs_fold_records_device folds such records (track = 0:
 * apply another replica's delta without re-recording it); `n` may be a count word
 * (rows | GS_FAIL_BIT): the failure is ANDed into the verdict before the rows fold.
 * gs_fold_records_counted_device is the same replay with the count word read on the
 * DEVICE (*count_dev as a take wrote it; at most `cap` rows), so a consumer replays a
 * window with no host round trip.
 *
 * gs_fold_take_device is one small window of the latency path (BASELINE config 5:
 * per window fold + delta export + completion; PartialAgg.fold then CombineCC /
 * Merger, S/SummaryBulkAggregation.java:109-130, S/SummaryAggregation.java:107-119):
 * fold n device edges with tracking on, take the records since the previous take
 * as gs_take_delta_records does (rec, cap, DEVICE *count_dev), and return when the
 * window is complete with the same count word (rows | GS_FAIL_BIT) in the HOST word
 * *count. A window of at
 * most 2^22 edges with nothing else pending runs as ONE launch whose last workgroup
 * publishes the rows and signals the host through mapped memory. Tracking must be
 * on; change tracking (which consumes the records itself) takes the general path.
 *
 * gs_delta_stage is the exchange form: every pending record into `send` as rows of
 * `width` int64 ({a, b} for CC, {a, b, w} for the signed kind; cap must be at least
 * gs_delta_capacity), and the DEVICE count word *count = rows | 2^62 when the
 * signed verdict has failed (the exchange carries the verdict: Candidates.merge
 * :79-81). gs_fold_exchange_device folds a gathered buffer: `world` blocks of
 * `rows` rows of `width` int64, block r live for its first counts[r] rows (DEVICE
 * count words as staged, failure bits ORed into the verdict), skipping block
 * `skip_rank` (the caller's own). */
int gs_set_delta_tracking(gs_handle h, int on);
int gs_delta_capacity(gs_handle h, uint64_t* rows);
int gs_take_delta_records(gs_handle h, int64_t* rec, size_t cap, uint64_t* count);
int gs_fold_take_device(gs_handle h, const int64_t* src, const int64_t* dst, size_t n, int64_t* rec, size_t cap,
                        uint64_t* count_dev, uint64_t* count);
int gs_delta_stage(gs_handle h, int64_t* send, size_t cap, int width, uint64_t* count);

/* Resident window server for gs_fold_take_device (the latency path without a kernel
 * launch per window). With it on, a window of at most 2^16 edges with nothing else
 * pending is posted to ONE persistent launch through host-mapped memory: its block 0
 * polls the mailbox and hands the window to the other blocks, every block folds 256
 * edges, and the window's last block publishes rows, count word and completion word
 * exactly as the fused launch does. Results are identical; any other call on the
 * handle stops the server first (it restarts at the next window), and a server idle
 * for ~2 ms leaves on its own. While it runs, the server occupies the handle stream's
 * hardware queue: work of ANOTHER stream that HIP mapped onto the same queue
 * (GPU_MAX_HW_QUEUES, 4 by default, are shared round-robin by the process's streams)
 * starts only after the server leaves, i.e. within ~2 ms of the last window (a stop or a
 * call on this handle ends it at once). The edge buffers of a window must be complete before
 * the window is posted and must not be rewritten while the server runs (each window
 * reads its edges once; a stream pre-staged in HBM, as BASELINE config 5 has it).
 * gs_window_server_stats: server launches and windows served. */
int gs_set_window_server(gs_handle h, int on);
int gs_window_server_stats(gs_handle h, uint64_t* launches, uint64_t* windows);
int gs_fold_records_device(gs_handle h, const int64_t* rec, size_t n, int track);
int gs_fold_records_counted_device(gs_handle h, const int64_t* rec, size_t cap, const uint64_t* count_dev, int track);
int gs_fold_exchange_device(gs_handle h, const int64_t* recv, const uint64_t* counts, size_t world, size_t rows,
                            int width, int skip_rank);

/* ---- per-window change emission (sinks) ------------------------------------------
 * The reference's Merger emits the whole cumulative summary every window
 * (SummaryAggregation.java:107-119) and its sinks flatten it: FlattenSet emits
 * (v, find(v)) for every vertex (ConnectedComponentsExample.java:143-156), keyed
 * downstream; DisjointSet.toString groups every vertex (DisjointSet.java:134-150).
 * With change tracking on, gs_take_changes_device emits only the rows a keyed sink
 * needs to reach the same state: (v, canonical label[, parity]) for every vertex
 * inserted or relabelled since the previous take, into DEVICE arrays; *n on the host
 * (synchronises). Work is O(changes): members of each component whose old root was
 * hooked this window are enumerated by walking a member list, not by a table scan;
 * a relabelled component of more than 2^16 vertices is emitted by one parallel scan,
 * which also re-emits the absorbing component's unchanged members (idempotent
 * rows). The first take after a table rebuild emits every vertex. cap must be at
 * least gs_num_vertices (each vertex is emitted at most once). Turns delta
 * tracking on and consumes the delta records (not for a group's summary). */
int gs_set_change_tracking(gs_handle h, int on);
int gs_take_changes_device(gs_handle h, int64_t* v, int64_t* label, uint8_t* parity, size_t cap, uint64_t* n);
/* The same rows into HOST arrays (a JVM sink; parity may be
 * NULL); device scratch is kept in the handle. */
int gs_take_changes(gs_handle h, int64_t* v, int64_t* label, uint8_t* parity, size_t cap, uint64_t* n);

/* ---- introspection -----------------------------------------------------------
 * The HIP stream (hipStream_t) the handle enqueues on, and per-kernel timing:
 * when profiling is on, every launch is bracketed by HIP events on the stream it
 * runs on; gs_kernel_stats returns (launches, total milliseconds) for kernel `id`
 * (0 = fold, 1 = stage, 2 = export, 3 = init/reset). gs_capacity_stats: capacity
 * checks that had to wait for in-flight reports, those that synchronised, and the
 * host milliseconds spent waiting. */
int gs_get_stream(gs_handle h, void** stream);
int gs_set_profiling(gs_handle h, int on);
int gs_kernel_stats(gs_handle h, int id, uint64_t* launches, double* total_ms);
int gs_table_capacity(gs_handle h, uint64_t* slots);
int gs_capacity_stats(gs_handle h, uint64_t* waits, uint64_t* syncs, double* wait_ms);

/* HBM accounting for a handle pool's budget (the Java HandlePool,
 * S/SummaryAggregation.java:107-119 and S/SummaryBulkAggregation.java:79-83 drop partials
 * and copies without a release). gs_hbm_bytes: bytes of device memory held right now by
 * every live summary and group of this process on `device` -- tables, vertex lists, delta
 * lists, staging and scratch -- counted by the library's allocator, so a table that grew
 * inside a fold or combine while handed out is included at once. gs_create_bytes: the bytes
 * gs_create(kind, capacity_hint) allocates. Neither synchronises. */
int gs_hbm_bytes(int device, uint64_t* bytes);
int gs_create_bytes(int kind, uint64_t capacity_hint, uint64_t* bytes);

/* Device counters (synchronises): out[0] vertices, [1] bipartiteness failed,
 * [2] table-overflow error, [3] list overflow (bit 0 delta list, bit 1 vertex
 * list), [4] records staged,
 * [5] hook calls, [6] hook-loop iterations, [7] failed hook CASes -- [5..7] only
 * count in the debug build (make -C gelly-streaming_amd debug). */
int gs_counters(gs_handle h, uint64_t* out8);

/* Diagnostics of the fold's memory operations (synchronises), debug build only (all
 * zero otherwise): out[0] edges / rows folded, [1] key CASes issued, [2] key CASes that
 * found the slot taken, [3] agent-scope re-reads before a key CAS, [4] edges settled by
 * the shared-parent shortcut, [5] edges whose finds met one root, [6] parent loads of
 * the finds, [7] hooks that joined two trees, [8] extra linear-probe loads. n <= 16
 * entries are written. Not a reference interface: the tools behind DESIGN.md use it. */
int gs_debug_counters(gs_handle h, uint64_t* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* GS_SUMMARY_H */
