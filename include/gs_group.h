/*
 * gs_group.h -- native multi-GPU combine for the summary of include/gs_summary.h.
 *
 * One process (or thread) per GPU; each rank holds a REPLICA of the global summary
 * and folds its own shard of every global micro-batch. After its fold a rank
 * stages its structural delta (at most one record per folded edge), the ranks
 * all-gather the record COUNTS, then exactly max-count rows per rank over RCCL
 * (xGMI), and every rank folds the other ranks' live records on a side stream
 * that overlaps its next own fold -- no host synchronisation per batch beyond
 * reading the gathered counts from host-mapped memory. This replaces the
 * reference's gather of per-partition summaries into one parallelism-1 reducer
 * (SummaryBulkAggregation.java:77-83) and its Merger (SummaryAggregation.java:107-119):
 * after gs_group_finish every replica equals the union of all ranks' folds, and a
 * signed replica's verdict is the AND of every rank's (the count word carries it).
 * RCCL (librccl.so.1) is loaded on first use.
 */
#ifndef GS_GROUP_H
#define GS_GROUP_H

#include <stddef.h>
#include <stdint.h>

#include "gs_summary.h"

/* Collective order (round 6). Every collective the group issues -- count all-gathers on
 * communicator C, data all-gathers and the tree's send/recv on communicator D -- is
 * issued by the calling thread in a program order that depends only on the sequence of
 * gs_group_* calls (exchange numbers and the fixed data lag), never on timing (when a
 * count lands, which stream is idle). So every rank issues the same interleaving of
 * C and D operations, the condition RCCL places on several communicators of one
 * device. The test emulation (tests/cpp/gs_fake_comm.cpp) asserts it: each collective
 * carries the rank's running hash of the (communicator, call number) sequence so far,
 * and a collective whose ranks disagree fails instead of hanging. */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gs_group* gs_group_t;

#define GS_GROUP_ID_BYTES 256 /* two RCCL unique ids: count and data communicators */

/* Collectives backend. By default a group loads RCCL (librccl.so.1) on first use and
 * calls it through this table. A caller may install its own implementation of the
 * same calls before gs_group_unique_id / gs_group_create -- e.g. one over MPI, or the
 * in-process emulation the tests use (N ranks as N threads on one GPU,
 * tests/cpp/gs_fake_comm.cpp, which also checks that every rank issues its collectives
 * in one order). dtype values are rccl.h's (ncclUint8 = 1, ncclInt64 = 4); `stream`
 * is a hipStream_t; `id` is one 128-byte unique id; 0 = success. */
typedef struct gs_comm_api {
  int (*get_unique_id)(void* id);
  int (*comm_init_rank)(void** comm, int nranks, const void* id, int rank);
  int (*comm_destroy)(void* comm);
  int (*comm_count)(void* comm, int* nranks);
  int (*all_gather)(const void* send, void* recv, size_t count, int dtype, void* comm, void* stream);
  /* ncclAllToAllv: counts and displacements in elements, host arrays of nranks */
  int (*all_to_allv)(const void* send, const size_t* send_counts, const size_t* send_displs, void* recv,
                     const size_t* recv_counts, const size_t* recv_displs, int dtype, void* comm, void* stream);
  int (*send)(const void* buf, size_t count, int dtype, int peer, void* comm, void* stream);
  int (*recv)(void* buf, size_t count, int dtype, int peer, void* comm, void* stream);
  int (*group_start)(void);
  int (*group_end)(void);
  const char* (*error_string)(int code);
} gs_comm_api;

/* Process-wide: ids and groups created afterwards use `api` (the table is copied);
 * NULL restores RCCL. Groups already created keep the backend they were created with. */
int gs_group_set_comm_api(const gs_comm_api* api);

/* Create the communicator id on one rank and hand its GS_GROUP_ID_BYTES bytes to
 * every rank (any host channel: MPI, TCP, torch.distributed, a file). */
int gs_group_unique_id(void* id);

/* Join the group as `rank` of `nranks` and bind it to summary `h` (its device and
 * stream). `batch_edges` = maximum edges one gs_group_fold_device call folds (at
 * most 2^26; sizes the delta list and the exchange buffers). Turns delta tracking
 * on. batch_edges == 0 creates a tree-combine-only group (no exchange buffers,
 * tracking untouched: fold partials with gs_fold[_device], then
 * gs_group_tree_combine). Collective: every rank must call it. */
int gs_group_create(gs_group_t* g, gs_handle h, const void* id, int nranks, int rank, size_t batch_edges);

/* One global micro-batch on this rank: fold n DEVICE edges (as gs_fold_device,
 * stride 1; n <= batch_edges), stage the delta and all-gather its count, then
 * move and fold the PREVIOUS micro-batch's records (whose counts landed while this
 * fold was queued). Asynchronous. Collective: every rank calls it the same number
 * of times (n may differ, including 0). Ordering: the own folds run after the work
 * queued on the handle's stream at the first call and after any gs_* call on the
 * handle since the previous group call (a reset, gs_wait_event, gs_wait_stream, a
 * sync, ...). A caller that queues its own kernels on gs_get_stream(h) between group
 * calls (edges written there) marks them with gs_wait_stream(h, that stream). */
int gs_group_fold_device(gs_group_t g, const int64_t* src, const int64_t* dst, size_t n);

/* Consecutive gs_group_fold_device calls over src[0..n) in batch-edge micro-batches,
 * looped natively (no per-batch host-language hop) -- except that the first
 * `ramp_edges` this rank folds after create / finish go in exchanges of `ramp_batch`
 * edges (gs_group_set_ramp; default 2^22 edges in 2^20-edge exchanges). The start
 * of a stream is where the ranks discover the same vertices in parallel: exchanging
 * it sooner cuts the duplicate hook records every other rank folds (RMAT-26 at 8
 * ranks: 66.9 M -> 54.3 M records per pass). Collective: every
 * rank must issue the same number of micro-batches (equal n on every rank does). */
int gs_group_fold_batches_device(gs_group_t g, const int64_t* src, const int64_t* dst, size_t n, size_t batch);
/* ramp_edges 0 disables the ramp; 0 < ramp_batch <= batch_edges. Same on every rank. */
int gs_group_set_ramp(gs_group_t g, size_t ramp_edges, size_t ramp_batch);

/* Move and fold the last micro-batch's records and synchronise; then all replicas
 * are identical. Collective. */
int gs_group_finish(gs_group_t g);

/* Log-depth tree combine of PER-RANK PARTIAL summaries: the reference's
 * SummaryTreeReduce / ConnectedComponentsTree (SummaryTreeReduce.java:68-123:
 * `enhance` keys partition pairs by f0/2 and reduces them level by level until the
 * parallelism is <= 2, then the all-window reduce and Merger at parallelism 1).
 * Here a binomial tree over the group's ranks: at level l, rank r with
 * r mod 2^(l+1) == 2^l sends its summary -- (v, label, parity) arrays + verdict,
 * ncclSend on the summary's stream -- to r - 2^l, which folds it
 * (gs_combine_exported_device). After ceil(log2 n) levels rank 0 holds the
 * combination of every rank's partial; senders keep theirs unchanged. Collective
 * (every rank calls it), synchronous. Unlike gs_group_fold_device (replicas kept
 * equal by delta exchange) this is the bulk path: O(V) per level. */
int gs_group_tree_combine(gs_group_t g);

/* Exchange statistics: exchanges run, records this rank has staged, rows this rank
 * has received (max-count rows from each other rank per exchange; synchronises). */
int gs_group_stats(gs_group_t g, uint64_t* exchanges, uint64_t* records_sent, uint64_t* rows_received);

/* Ranks of the group's two communicators (ncclCommCount): the world that actually
 * formed, checked by bench.py's N > 1 line beside torch.distributed's world size. */
int gs_group_comm_ranks(gs_group_t g, int* count_comm, int* data_comm);

/* Per-phase timing of the exchange protocol (diagnostic; HIP timing events around each
 * phase's device work while on). gs_group_phase_stats (synchronises) returns, since the
 * last gs_group_set_phase_timing: out[0] own-fold lane milliseconds (summed over the
 * pipelining lanes), out[1] remote-row fold ms, out[2] stage + count collective + headers
 * ms, out[3] data collective ms, out[4] host ms spent waiting for gathered counts (timed
 * whether or not phase timing is on), out[5] exchanges timed. */
int gs_group_set_phase_timing(gs_group_t g, int on);
int gs_group_phase_stats(gs_group_t g, double* out6);

/* ---- Owner-partitioned mode (round 6) -----------------------------
 * The replica mode above makes every rank insert every vertex of the graph. Here each rank
 * keeps a LOCAL forest of its own edges only (the summary h: its min-key roots are local
 * labels), and the vertices are partitioned by owner (a hash of the id mod nranks). At
 * every combine (the window end of SummaryBulkAggregation.java:76-83; with window_edges 0,
 * once per pass: the bulk combine of SummaryTreeReduce.java:68-123):
 *   1. each rank exports (v, local root[, parity]) for the vertices new to it since the
 *      previous combine, bucketed by owner (and marks those roots), plus a label pair
 *      (a, root of a now) for every marked root a hooked away since then;
 *   2. the rows go to their owners (ncclAllToAllv on the data communicator, counts first
 *      on the count communicator);
 *   3. the owner of v keeps one anchor label per vertex (the first row's) and turns every
 *      other row (v, l) into the label pair (anchor, l) (deduplicated per block);
 *   4. every rank's pairs are all-gathered and folded into every rank's LABEL FOREST, a
 *      replica of only the labels that need a cross-rank union (a few % of V on RMAT).
 * The canonical label of an owned vertex v is the label forest's label of anchor(v);
 * gs_group_part_labels_device emits this rank's owned slice, and the slices of all ranks
 * are the Merger's output (bit-exact with a single summary: labels = min id, signed
 * colourings composed along anchor -> label). Collectives are issued on the handle's stream
 * in program order. vertices_hint sizes the owner table (4 slots per expected owned
 * vertex; overflow fails with GS_ERR_CAPACITY). window_edges > 0: at most that many own
 * edges between combines (delta tracking on, records of hooked roots); 0: untracked
 * (pipelinable) folds and one combine per pass -- gs_group_part_reset starts the next. */
int gs_group_create_partitioned(gs_group_t* g, gs_handle h, const void* id, int nranks, int rank,
                                uint64_t vertices_hint, size_t window_edges);
/* Fold n device edges of this rank into its local forest (as gs_fold_device, stride 1). */
int gs_group_part_fold_device(gs_group_t g, const int64_t* src, const int64_t* dst, size_t n);
/* The window end: steps 1-4 above. Collective; synchronises this rank's streams. */
int gs_group_part_combine(gs_group_t g);
/* This rank's owned vertices after the last combine: (v, canonical label[, parity]) into
 * DEVICE arrays of `cap` rows (parity may be NULL); *n = rows (GS_ERR_TRUNCATED if > cap). */
int gs_group_part_labels_device(gs_group_t g, int64_t* v, int64_t* label, uint8_t* parity, size_t cap, size_t* n);
/* The global bipartiteness verdict after the last combine (every rank's, AND-ed). */
int gs_group_part_status(gs_group_t g, int* ok);
/* Empty local forest, owner table and label forest, statistics zeroed (the next pass).
 * Not collective. */
int gs_group_part_reset(gs_group_t g);
/* out8 (since create or the last reset): combines, rows exported, rows owned (received), label
 * pairs sent, label pairs folded (all ranks), label-forest vertices, owner-table slots, 0. */
int gs_group_part_stats(gs_group_t g, uint64_t* out8);
/* With gs_group_set_phase_timing on, device ms per phase since: out8[0] own folds (handle
 * stream only), [1] export + records, [2] bucketing, [3] count + row all-to-all, [4] owner
 * step, [5] pair-count + pair all-gathers, [6] label-forest fold, [7] combines. The
 * collective phases [3], [5] include the wait for the other ranks. */
int gs_group_part_phase_stats(gs_group_t g, double* out8);

int gs_group_destroy(gs_group_t g);

#ifdef __cplusplus
}
#endif
#endif /* GS_GROUP_H */
