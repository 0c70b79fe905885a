// gs_kernels.hpp -- host-side launchers of the summary kernels (gs_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_device.hpp"

namespace gs {

void launch_init(Slot* tab, uint64_t nslots, hipStream_t st);
// inline_max: an edge whose roots differ is hooked inside k_fold when its wave has
// <= inline_max such edges (64: always), else appended to active set `cur`.
// drain: active set hooked by this launch too (-1: none); zero: set whose counters
// this launch resets (-1: none).
void launch_fold(bool sign, bool track, int ept, const Table& t, const Lists& L, const int64_t* src,
                 const int64_t* dst, const uint8_t* w, uint32_t n, uint32_t stride, uint32_t w_stride, int cur,
                 int drain, int zero, int inline_max, uint32_t rows, int skip_rank, const int64_t* hdr,
                 uint32_t base, hipStream_t st);
void launch_hook(bool sign, bool track, const Table& t, const Lists& L, int set, int blocks, hipStream_t st);
void launch_export(bool sign, const Table& t, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap_out,
                   hipStream_t st, int part = 0, int nparts = 1);
void launch_stage(const Table& t, const Lists& L, const int64_t* q_in, unsigned long long* qn_in, int64_t* q_out,
                  unsigned long long* qn_out, uint64_t qcap, int64_t* send, uint64_t cap, hipStream_t st,
                  unsigned long long* count_out = nullptr, int width = 3);
void launch_find_one(const Table& t, int64_t key, int64_t* out, hipStream_t st);
void launch_headers(const int64_t* recv, uint64_t rank_stride, int nranks, long long* out, long long seq,
                    hipStream_t st);
void launch_report(uint32_t* ctr, uint64_t n, unsigned long long* out, hipStream_t st);

}  // namespace gs
