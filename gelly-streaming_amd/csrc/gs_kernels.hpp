// gs_kernels.hpp -- host-side launchers of the summary kernels (gs_kernels.hip,
// gs_changes.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_device.hpp"

namespace gs {

// One k_fold launch (see FoldArgs in gs_kernels.hip).
struct FoldLaunch {
  const int64_t* src = nullptr;
  const int64_t* dst = nullptr;
  const uint8_t* w = nullptr;
  uint32_t n = 0;
  uint32_t stride = 1;
  uint32_t w_stride = 1;
  uint32_t rows = 0;
  int skip_rank = -1;
  const unsigned long long* counts = nullptr;
  uint32_t base = 0;
  const unsigned long long* n_dev = nullptr;
  const uint32_t* fail_in = nullptr;
  uint32_t shard0 = 0;
  // fused window take (k_fold TAKE, one launch): rows, device count, completion word
  int64_t* take_out = nullptr;
  unsigned long long take_cap = 0;
  unsigned long long* take_count = nullptr;
  unsigned long long* done = nullptr;
  unsigned long long seq = 0;
  // the capacity report of the earlier chunks of this stream, carried by this launch
  unsigned long long* rep_out = nullptr;
  unsigned long long rep_claim = 0;
  unsigned rep_epoch = 0;
};

// Resident window server (latency path, gs_set_window_server): the host posts each
// window into a host-mapped mailbox; block 0 polls it and hands the window to the other
// blocks through device memory; every block folds its 256 edges, and the window's last
// block publishes rows, count word and the completion word as the fused take does.
constexpr uint32_t kServerBlocks = 256;                       // one per CU: a 2^16-edge window
constexpr uint64_t kServerMaxEdges = (uint64_t)kServerBlocks * kFoldBS;
constexpr unsigned long long kServerStop = 1ull << 63;        // mailbox seq bit: leave
// Mailbox / broadcast descriptor words and completion records carry a 16-bit tag (the
// sequence number mod 2^16) in bits 48..63 over a 48-bit value (data-tagged granules:
// a reader takes the line when every tag matches, with no fence on the writer's side).
constexpr unsigned long long kServerTagMask = (1ull << 48) - 1;
__host__ __device__ constexpr unsigned long long tag_word(unsigned long long seq, unsigned long long v) {
  return (seq & 0xFFFFull) << 48 | (v & kServerTagMask);
}
// Completion record values: a count word's failed-verdict bit (bit 62) travels as bit 47.
__host__ __device__ constexpr unsigned long long done_value(unsigned long long seq, unsigned long long v) {
  return (seq & 0xFFFFull) << 48 | ((v >> 62) & 1ull) << 47 | (v & ((1ull << 47) - 1));
}
__host__ __device__ constexpr unsigned long long done_decode(unsigned long long w) {
  return (w & ((1ull << 47) - 1)) | ((w >> 47) & 1ull) << 62;
}
struct alignas(64) ServerBox {      // host-mapped; written by the host, read by block 0 (one 64-B line + exited)
  unsigned long long seq;          // window number (stored last, release) | kServerStop
  unsigned long long src, dst, n, rec, cap, cnt, done_seq;  // each gs::tag_word(seq, value)
  unsigned long long exited;       // block 0 stores 1 when the server leaves (stop or idle)
  unsigned long long taken;        // block 0 stores the seq of every window it takes (before its broadcast)
  unsigned long long bc_init;      // host: the broadcast word's first value (copied to the device at start)
  unsigned long long pad[5];
};
struct alignas(64) ServerBcast {    // device memory: block 0 -> the other blocks (the tagged line)
  unsigned long long seq, src, dst, n, rec, cap, cnt, done_seq;
};
void launch_window_server(bool sign, const Table& t, const Delta& D, ServerBox* box, ServerBcast* bc,
                          unsigned long long* done, unsigned long long seq0, unsigned long long idle_ticks,
                          hipStream_t st);
// Workgroups of k_window_server that can be resident on the device at once (occupancy x
// CUs): a window completes only when all kServerBlocks of them run together.
int window_server_resident_blocks(bool sign, int device);

void launch_init(Slot* tab, uint64_t nslots, hipStream_t st, uint32_t* ctr = nullptr);
// micro-batch dedup: w[i] = 1 (keep) or 0x81 (skip: a repeat of an earlier pair of the batch)
void launch_dedup(const int64_t* src, const int64_t* dst, uint32_t n, unsigned long long* tab, uint32_t mask,
                  uint8_t* w, hipStream_t st);
void launch_reset_list(const Table& t, uint32_t* nxt, uint64_t bound, hipStream_t st);
void launch_fold(bool sign, bool track, const Table& t, const Delta& D, const FoldLaunch& f, hipStream_t st);
// by_list: the vertex list is complete as far as the host knows; the kernel walks it when the
// real vertex count (read on the device) is under 1/8 of the slots, else it scans
void launch_export(const Table& t, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap_out, hipStream_t st,
                   int part = 0, int nparts = 1, bool by_list = false);
void launch_export_list(const Table& t, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap_out, uint64_t bound,
                        hipStream_t st);
// order-independent digest of the (vertex, label, parity) set, added into *out
void launch_digest(const Table& t, unsigned long long* out, uint64_t bound, hipStream_t st);
void launch_stage(const Table& t, const Delta& D, int64_t* out, uint64_t cap, int width,
                  unsigned long long* count_out, bool with_fail, hipStream_t st);
void launch_report(uint32_t* ctr, uint64_t n, unsigned long long* out, unsigned epoch, hipStream_t st);
void launch_headers(const unsigned long long* counts, int nranks, long long* out, long long seq, hipStream_t st);
// completion word for host waits: out[1] = sum of nvals (<= 64) counters vals[i * stride]
// (if vals), then out[0] = seq (release, system scope); `clear`: the counters are zeroed
// behind the read (the export counter: no fill launch before the next export)
// `flag` (optional): bit 62 of the value is set when *flag != 0 (a count word's failed-verdict
// bit: the completion record carries it as bit 47, the sum stays below 2^47)
constexpr unsigned long long kSignalFlagBit = 1ull << 62;
void launch_signal(unsigned long long* out, unsigned long long seq, const uint32_t* vals, int nvals, int stride,
                   hipStream_t st, bool clear = false, const uint32_t* flag = nullptr);
void launch_find_one(const Table& t, int64_t key, int64_t* out, hipStream_t st);
void launch_find_batch(const Table& t, const int64_t* v, uint64_t n, int64_t* label, uint8_t* found, uint8_t* parity,
                       hipStream_t st);

// change emission (gs_changes_k.hip)
void launch_iota(uint32_t* nxt, uint64_t n, hipStream_t st);
void launch_relist(const Table& t, uint32_t* nxt, hipStream_t st);
void launch_emit_records(const Table& t, uint32_t* nxt, const int64_t* rec, const unsigned long long* nrec,
                         uint64_t nrec_bound, uint32_t walk_max, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap,
                         uint32_t* big, hipStream_t st);
void launch_emit_scan(const Table& t, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap, bool all, hipStream_t st);
void launch_clear_big(const Table& t, const uint32_t* big, uint64_t n, hipStream_t st);
void launch_emit_new(const Table& t, uint32_t* vmark, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap,
                     uint64_t bound, bool emit, hipStream_t st);

}  // namespace gs
