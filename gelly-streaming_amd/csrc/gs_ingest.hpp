// gs_ingest.hpp -- internal interface of the GPU text parser (gs_ingest.hip),
// used by gs_parse_edges_device and by gs_fold_text (gs_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_testing.h"

namespace gsi {
int64_t testing_value(int knob, int64_t product);  // include/gs_testing.h (gs_capi.cpp)
}

namespace gs {

struct ParseScratch {
  uint64_t* tile_cnt = nullptr;  // '\n' per 4 KiB tile
  uint64_t* tile_pre = nullptr;  // exclusive scan of tile_cnt
  unsigned long long* bad = nullptr;  // min malformed line index
  uint64_t* res = nullptr;            // [2] {line count, first malformed line or ~0}
  void* cub_tmp = nullptr;
  size_t cub_bytes = 0;
  uint64_t tiles_cap = 0;
  bool bad_ready = false;  // `bad` holds ~0 (k_parse_result resets it after every parse)
  bool st_zero = false;    // the one-pass status words are zero (the last one-pass parse's k_parse_finish cleared them)
  hipStream_t zero_stream = nullptr;  // the stream that k_parse_finish ran on (st_zero holds only there)
};

// Device bytes needed to parse up to max_len bytes of text.
size_t parse_scratch_bytes(size_t max_len, size_t* cub_bytes);
int parse_scratch_init(ParseScratch& s, void* mem, size_t max_len);
// Enqueue the parse of device text on st; the result {lines, bad or ~0} lands in s.res
// (device) and, with host_res (mapped), in host_res[1..2] behind host_res[0] = seq.
// fused: one pass (k_parse_fused, decoupled look-back) instead of count + scan + parse.
// Returns 0 or -1 (HIP failure).
int parse_text_enqueue(hipStream_t st, const char* text, size_t len, int sep, int64_t* src, int64_t* dst, size_t cap,
                       ParseScratch& s,
                       unsigned long long* host_res = nullptr, unsigned long long seq = 0, bool fused = true,
                       hipEvent_t kev0 = nullptr, hipEvent_t kev1 = nullptr);  // optional: bracket the parse kernel
// Parse device text; synchronises st. Returns 0 or -1 (HIP failure).
int parse_text(hipStream_t st, const char* text, size_t len, int sep, int64_t* src, int64_t* dst, size_t cap,
               ParseScratch& s, uint64_t* n_lines, int64_t* bad_line);

}  // namespace gs
