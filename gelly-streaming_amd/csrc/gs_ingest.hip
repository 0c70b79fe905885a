// gs_ingest.hip -- text edge-file parsing on the GPU (include/gs_ingest.h).
//
// Replaces the reference's source map `s.split("\\s")` / `s.split("\\t")` +
// Long.parseLong(fields[0..1]) over env.readTextFile lines
// (ConnectedComponentsExample.java:109-118, BipartitenessCheckExample.java:97-106).
//
// Two launches + one scan, all HBM-streaming:
//   k_count_lines : per 16 KiB tile, the number of '\n' (coalesced 16-B loads)
//   k_tile_scan   : exclusive scan of the tile counts (one block) -> '\n' before each tile
//   k_parse       : per tile, the tile (+ 512 B of the next) is staged in LDS; every
//                   thread owns 64 bytes, finds the line starts in them (byte after a
//                   '\n') and their ends ('\n' masks of its and the next two segments
//                   in LDS), numbers the lines from the tile prefix + a block scan, and
//                   parses them with the Java split/parseLong rules: SWAR from LDS words
//                   (parse_line_swar), or one byte per step for long lines / fields;
//                   malformed lines -> atomicMin(bad).
// RMAT-26 text (684 MB, 2^24 lines): k_count_lines 120-133 us (5.4 TB/s); k_parse 771 us
// with a per-character parse of compacted line starts, 592 us with the SWAR parse, 370 us
// with lines parsed by the thread whose 32-byte segment they start in (no start list),
// 338-354 us with 16 KiB tiles (five 16-B loads in flight per thread instead of three).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gs_ingest.h"
#include "gs_ingest.hpp"

namespace gs {

#ifndef GS_PARSE_BRANCHLESS
#define GS_PARSE_BRANCHLESS 1
#endif

constexpr uint32_t kTile = 16384;  // bytes per parse block (64 per thread in the start scan)
constexpr uint32_t kOver = 512;    // bytes of the next tile staged for lines crossing the end

__device__ __forceinline__ bool is_sep(uint8_t c, int sep) {
  // Java regex \s = [ \t\n\x0B\f\r]; \t = tab only
  return sep == GS_SEP_TAB ? c == '\t' : (c == ' ' || (c >= '\t' && c <= '\r'));
}

__global__ __launch_bounds__(256) void k_count_lines(const uint8_t* __restrict__ text, uint64_t len,
                                                     uint64_t* __restrict__ tile_cnt, bool aligned, uint64_t tile0) {
  __shared__ uint32_t wsum[4];
  const uint64_t tile = tile0 + blockIdx.x;
  const uint64_t t0 = tile * kTile;
  uint32_t c = 0;
#pragma unroll
  for (uint32_t h = 0; h < kTile / 4096; ++h) {  // 16 B per thread per 4 KiB slice: coalesced
    const uint64_t p = t0 + h * 4096u + threadIdx.x * 16u;
    if (aligned && p + 16 <= len) {
      const uint4 v = *reinterpret_cast<const uint4*>(text + p);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int b = 0; b < 4; ++b) c += ((w[k] >> (8 * b)) & 0xFFu) == '\n';
    } else {
      for (uint64_t q = p; q < p + 16 && q < len; ++q) c += text[q] == '\n';
    }
  }
  // block sum
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tile_cnt[tile] = (uint64_t)wsum[0] + wsum[1] + wsum[2] + wsum[3];
}


constexpr uint32_t kLds0 = 32;  // LDS offset of byte t0 (byte t0 - 1 sits at kLds0 - 1; the SWAR
                                // windows of a line may read up to 27 bytes before it)

struct LineBuf {
  const uint8_t* lds;
  const uint8_t* text;
  uint64_t t0, len, staged_end;  // bytes [t0, staged_end) are staged in LDS
  // byte q, or '\n' past the end of the text (the last line needs no terminator)
  __device__ __forceinline__ uint8_t at(uint64_t q) const {
    if (q < staged_end) return lds[kLds0 + (q - t0)];
    return q < len ? text[q] : (uint8_t)'\n';
  }
};

enum { kFieldBad = 0, kFieldSep = 1, kFieldEol = 2 };

// Long.parseLong on the field starting at q: optional sign, >= 1 ASCII digit, int64
// range; the field must end at a separator or at the end of the line ('\n', end of
// text, or a '\r' right before either: Flink drops it). One byte read per step.
__device__ __forceinline__ int parse_long(const LineBuf& b, uint64_t& q, int sep, int64_t& out) {
  uint8_t c = b.at(q);
  const bool neg = c == '-';
  if (neg || c == '+') c = b.at(++q);
  // magnitude m <= 2^63 (negative) or 2^63 - 1: below kCut every next digit fits
  // without a check; at kCut only a last digit <= 8 / 7 fits (Long.parseLong range)
  constexpr uint64_t kCut = 922337203685477580ull;  // (2^63 - 1) / 10
  const uint32_t last_ok = neg ? 8u : 7u;
  uint64_t m = 0;
  int digits = 0;
  uint32_t d = (uint32_t)c - '0';
  while (d <= 9u) {
    if (m >= kCut && (m > kCut || d > last_ok)) return kFieldBad;
    m = (m << 3) + (m << 1) + d;
    ++digits;
    c = b.at(++q);
    d = (uint32_t)c - '0';
  }
  if (digits == 0) return kFieldBad;
  out = neg ? (int64_t)(0ull - m) : (int64_t)m;
  if (c == '\n') return kFieldEol;
  if (c == '\r' && b.at(q + 1) == '\n') return kFieldEol;
  return is_sep(c, sep) ? kFieldSep : kFieldBad;  // e.g. "12a"
}

// Fast path of one line whose '\n' position is known (the next line's start - 1): the
// two fields are delimited and converted four bytes per ALU op (SWAR) from LDS words,
// instead of one LDS round trip and ~15 ops per character (the per-character loop
// above ran k_parse at 0.9 TB/s of text). Same rules as parse_long. Returns 1
// (parsed), 0 (malformed) or -1 (a field of more than 23 bytes, e.g. leading zeros:
// the caller takes the per-character path). L = the tile's byte 0 in LDS (bytes from
// L - 32 are addressable); s, e: the line's start and its '\n' (tile-relative).

// bytes [o, o + 24) of LDS, any alignment: 7 aligned dword reads + v_alignbyte
__device__ __forceinline__ void lds_win24(const uint8_t* L, int o, uint32_t (&w)[6]) {
  const uint8_t* a = L + (o & ~3);
  const uint32_t sh = (uint32_t)o & 3u;
  uint32_t r[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) r[k] = *reinterpret_cast<const uint32_t*>(a + 4 * k);
#pragma unroll
  for (int k = 0; k < 6; ++k) w[k] = __builtin_amdgcn_alignbyte(r[k + 1], r[k], sh);
}

// index of the first byte of the window that is not an ASCII digit (24: none); with
// skip0, byte 0 (a sign) counts as a digit
__device__ __forceinline__ int first_nondigit(const uint32_t (&w)[6], bool skip0) {
  int p = 24;
#pragma unroll
  for (int k = 5; k >= 0; --k) {
    const uint32_t x = w[k] ^ 0x30303030u;  // digits -> 0..9
    uint32_t t = (((x & 0x7F7F7F7Fu) + 0x76767676u) | x) & 0x80808080u;  // bit 7 of a byte: x_b >= 10
    if (k == 0 && skip0) t &= ~0x80u;
    if (t) p = 4 * k + (__builtin_ctz(t) >> 3);
  }
  return p;
}

// Long.parseLong magnitude of the n (1..23) ASCII digits ending at L[end] (exclusive),
// four digits per word op; false when outside the int64 range
__device__ __forceinline__ bool digits_value(const uint8_t* L, int end, int n, bool neg, int64_t& out) {
  uint32_t w[6];
  lds_win24(L, end - 24, w);
  uint32_t g[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int v = 24 - n - 4 * k;  // first digit byte of word k
    const uint32_t keep = v <= 0 ? 0xFFFFFFFFu : (v >= 4 ? 0u : (0xFFFFFFFFu << (8 * v)));
    const uint32_t x = ((w[k] & keep) | (0x30303030u & ~keep)) - 0x30303030u;  // bytes 0..9, no borrows
    const uint32_t t = (x << 3) + (x << 1) + (x >> 8);  // byte 0 = 10 d0 + d1, byte 2 = 10 d2 + d3
    g[k] = (t & 0xFFu) * 100u + ((t >> 16) & 0xFFu);   // d0 d1 d2 d3 (byte 0 is the most significant)
  }
  const uint32_t hi = g[0] * 10000u + g[1];
  if (hi > 922u) return false;  // >= 9.23e18
  const uint64_t v = (uint64_t)hi * 10000000000000000ull + ((uint64_t)(g[2] * 10000u + g[3]) * 100000000ull +
                                                            (uint64_t)(g[4] * 10000u + g[5]));
  if (v > (neg ? (1ull << 63) : (1ull << 63) - 1)) return false;
  out = neg ? (int64_t)(0ull - v) : (int64_t)v;
  return true;
}

template <int SEP>
__device__ __forceinline__ bool sep_byte(uint32_t c) {
  return SEP == GS_SEP_TAB ? c == '\t' : (c == ' ' || (c - 9u) <= 4u);
}

// Branch-free form of digits_value and parse_line_swar (GS_PARSE_BRANCHLESS): every
// window and both values are computed and the verdict selected at the end, so a wave
// runs one straight path per line instead of exec-mask juggling around early returns
// (k_parse issued ~270 scalar instructions per wave; profiles/r04_ingest_stalls.txt).
// Out-of-range windows stay inside the staged LDS (fields clamped to 1..23 digits).
__device__ __forceinline__ bool digits_value_bf(const uint8_t* L, int end, int n, bool neg, int64_t& out) {
  uint32_t w[6];
  lds_win24(L, end - 24, w);
  uint32_t g[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int v = 24 - n - 4 * k;
    const uint32_t keep = v <= 0 ? 0xFFFFFFFFu : (v >= 4 ? 0u : (0xFFFFFFFFu << (8 * v)));
    const uint32_t x = ((w[k] & keep) | (0x30303030u & ~keep)) - 0x30303030u;
    const uint32_t t = (x << 3) + (x << 1) + (x >> 8);
    g[k] = (t & 0xFFu) * 100u + ((t >> 16) & 0xFFu);
  }
  const uint32_t hi = g[0] * 10000u + g[1];
  const uint64_t v = (uint64_t)hi * 10000000000000000ull + ((uint64_t)(g[2] * 10000u + g[3]) * 100000000ull +
                                                            (uint64_t)(g[4] * 10000u + g[5]));
  out = neg ? (int64_t)(0ull - v) : (int64_t)v;
  return hi <= 922u && v <= (neg ? (1ull << 63) : (1ull << 63) - 1);
}

template <int SEP>
__device__ __forceinline__ int parse_line_swar_bf(const uint8_t* L, int s, int e, int64_t& a, int64_t& b) {
  e = (e > s && L[e - 1] == '\r') ? e - 1 : e;  // a '\r' right before the line end is dropped
  uint32_t w[6];
  lds_win24(L, s, w);
  const uint32_t c0 = w[0] & 0xFFu;
  const bool sg0 = c0 == '+' || c0 == '-';
  const int f0 = first_nondigit(w, sg0);
  const int p1 = s + min(f0, 23), n0 = f0 - (sg0 ? 1 : 0);
  const bool ok0 = n0 > 0 && p1 < e && sep_byte<SEP>(L[p1]);
  const int q = p1 + 1;
  lds_win24(L, q, w);
  const uint32_t c1 = w[0] & 0xFFu;
  const bool sg1 = q < e && (c1 == '+' || c1 == '-');
  const int f1 = first_nondigit(w, sg1);
  const int p2 = max(q + 1, min(q + f1, e)), n1 = min(q + f1, e) - q - (sg1 ? 1 : 0);
  const bool ok1 = n1 > 0 && (q + f1 >= e || sep_byte<SEP>(L[q + min(f1, 23)]));
  const bool va = digits_value_bf(L, p1, min(max(n0, 1), 23), c0 == '-', a);
  const bool vb = digits_value_bf(L, p2, min(max(n1, 1), 23), sg1 && c1 == '-', b);
  return f0 >= 24 ? -1 : (!ok0 ? 0 : (f1 >= 24 ? -1 : ((ok1 && va && vb) ? 1 : 0)));
}

template <int SEP>
__device__ __forceinline__ int parse_line_swar(const uint8_t* L, int s, int e, int64_t& a, int64_t& b) {
  if (e > s && L[e - 1] == '\r') --e;  // a '\r' right before the line end is dropped
  uint32_t w[6];
  lds_win24(L, s, w);
  const uint32_t c0 = w[0] & 0xFFu;
  const bool sg0 = c0 == '+' || c0 == '-';
  const int f0 = first_nondigit(w, sg0);
  if (f0 >= 24) return -1;
  const int p1 = s + f0, n0 = f0 - (sg0 ? 1 : 0);
  // field 0 needs >= 1 digit and must end at a separator inside the line
  if (n0 <= 0 || p1 >= e || !sep_byte<SEP>(L[p1])) return 0;
  const int q = p1 + 1;
  lds_win24(L, q, w);
  const uint32_t c1 = w[0] & 0xFFu;
  const bool sg1 = q < e && (c1 == '+' || c1 == '-');
  const int f1 = first_nondigit(w, sg1);
  if (f1 >= 24) return -1;
  const int p2 = min(q + f1, e), n1 = p2 - q - (sg1 ? 1 : 0);
  // field 1 needs >= 1 digit and ends at the line end or a separator (fields past it ignored)
  if (n1 <= 0 || (p2 < e && !sep_byte<SEP>(L[p2]))) return 0;
  if (!digits_value(L, p1, n0, c0 == '-', a)) return 0;
  if (!digits_value(L, p2, n1, sg1 && c1 == '-', b)) return 0;
  return 1;
}

// '\n' mask (bit j: byte 32 q + j) of the 32-byte LDS segment q of the tile, with every
// byte at or past the text's end `vend` (tile-relative, when the tile holds it) counted
// as the end of the last line: bit vend set, bits above it cleared
__device__ __forceinline__ uint32_t seg_nl_mask(const uint8_t* L, uint32_t q, uint64_t vend) {
  const uint4 w0 = *reinterpret_cast<const uint4*>(L + 32 * q);
  const uint4 w1 = *reinterpret_cast<const uint4*>(L + 32 * q + 16);
  const uint32_t ww[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
  uint32_t nl = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) nl |= (((ww[k] >> (8 * bb)) & 0xFFu) == '\n' ? 1u : 0u) << (4 * k + bb);
  const uint64_t b0 = 32ull * q;
  if (vend < b0 + 32) nl = vend <= b0 ? (vend == b0 ? 1u : 0u) : ((nl & ((1u << (vend - b0)) - 1u)) | (1u << (vend - b0)));
  return nl;
}

// '\n' mask (bit j: byte 16 c + j) of the 16-byte LDS chunk c of the tile, with the
// same end-of-text rule as seg_nl_mask. Chunks are read block-contiguously (lane i of a
// wave reads bytes 16 i ..): conflict-free 16-B LDS reads, where a thread reading its own
// 64-byte segment put the lanes of a wave 64 B apart (16-way bank conflicts).
__device__ __forceinline__ uint32_t chunk_nl_mask(const uint8_t* L, uint32_t c, uint64_t vend) {
  const uint4 w = *reinterpret_cast<const uint4*>(L + 16 * c);
  const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
  uint32_t nl = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) nl |= (((ww[k] >> (8 * bb)) & 0xFFu) == '\n' ? 1u : 0u) << (4 * k + bb);
  const uint64_t b0 = 16ull * c;
  if (vend < b0 + 16) nl = vend <= b0 ? (vend == b0 ? 1u : 0u) : ((nl & ((1u << (vend - b0)) - 1u)) | (1u << (vend - b0)));
  return nl;
}

template <bool FUSED>
__device__ __forceinline__ void parse_tile(const uint8_t* __restrict__ text, uint64_t len, int sep,
                                           const uint64_t* __restrict__ tile_pre, int64_t* __restrict__ src,
                                           int64_t* __restrict__ dst, uint64_t cap,
                                           unsigned long long* __restrict__ bad, bool aligned, uint64_t tile,
                                           unsigned long long* __restrict__ status, unsigned long long* __restrict__ pstat,
                                           unsigned long long lb_timeout);

// Single pass (GS_PARSE_FUSED, default): no k_count_lines pass and no scan. Every block
// counts its tile's '\n' from the masks it builds anyway and finds the count before its
// tile by a decoupled look-back over per-tile status words (status[t]: bit 63 = the
// inclusive count through tile t is final, bit 62 = tile t's own count is, value in bits
// 0..61): wave 0 reads the 64 nearest predecessors' words in one round, sums own counts
// back to the nearest final prefix, publishes its own. A block only waits for lower
// tiles, which are dispatched before it on their XCD; should a wait ever outlast ~50 ms,
// the block counts the '\n' before its tile itself (no deadlock either way). The text
// is read once instead of twice (the count pass was 126 us of a 684 MB parse).

constexpr unsigned long long kStP = 1ull << 63, kStA = 1ull << 62, kStVal = (1ull << 62) - 1;
#ifndef GS_LB_SLEEP0
#define GS_LB_SLEEP0 8  // look-back back-off: s_sleep of the first three unsuccessful rounds (experiment switch)
#endif
#ifndef GS_LB_SLEEP1
#define GS_LB_SLEEP1 64  // ... and of the later ones
#endif
// Early aggregates: a tile that lies wholly inside the text publishes its '\n' count as
// soon as its staging loads arrive, before the LDS staging, masks and scan: each wave adds
// (1 << kStWaveShift) | (its count) to the tile's status word, and the aggregate is
// complete once all four waves have added. (The look-back's waits are for predecessors'
// aggregates; this moves them a staging-and-scan earlier.)
#ifndef GS_PARSE_REGMASK
#define GS_PARSE_REGMASK 1  // '\n' masks from the staging registers (0: from LDS after staging; experiment switch)
#endif
#ifndef GS_PARSE_EARLY
#define GS_PARSE_EARLY 1  // 0: aggregates published after the scan (experiment switch)
#endif
constexpr int kStWaveShift = 56;
constexpr unsigned long long kStWaves = 7ull << kStWaveShift, kStCnt = (1ull << kStWaveShift) - 1;
// The inclusive prefixes (kStP | value) live in a second array, pstat: the aggregate word
// takes atomic adds that may still be in flight when the tile's prefix is known.
__device__ __forceinline__ bool st_has_agg(unsigned long long w) {
  return (w & kStA) != 0 || (w & kStWaves) == (4ull << kStWaveShift);
}
__device__ __forceinline__ unsigned long long st_agg(unsigned long long w) {
  return (w & kStA) ? (w & kStVal) : (w & kStCnt);
}
// '\n' bytes in 16 staged bytes (exact zero-byte count of x ^ 0x0A0A0A0A per word)
__device__ __forceinline__ uint32_t nl_count16(const uint4& v) {
  uint32_t c = 0;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = w[i] ^ 0x0A0A0A0Au;
    const uint32_t t = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
    c += __popc(t);
  }
  return c;
}

// '\n' mask of 16 bytes held in registers (bit j: byte j), exact: the zero-byte test of
// w ^ 0x0A0A0A0A leaves bit 8 b + 7 of a word for a '\n' in its byte b, and one multiply by
// 2^0 + 2^7 + 2^14 + 2^21 gathers the four bits into bits 21..24 (no two partial products
// share a bit, so nothing carries)
__device__ __forceinline__ uint32_t nl_mask16(const uint4& v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t x = w[k] ^ 0x0A0A0A0Au;
    const uint32_t t = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
    m |= ((((t >> 7) * 0x00204081u) >> 21) & 0xFu) << (4 * k);
  }
  return m;
}

// Inclusive prefix sum over the 64 lanes of a wave with DPP (no LDS round trips: __shfl_up is
// a ds_bpermute per step): row_shr 1, 2, 4, 8 within each row of 16 lanes, then row_bcast 15
// and 31 carry the rows' totals upward
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// Wave 0 of tile `tile`: '\n' before the tile (decoupled look-back over 64 predecessors
// per round); publishes the tile's inclusive count. agg = the tile's own '\n' count.
// Between unsuccessful rounds the wave backs off (s_sleep 8 -> 64): every waiting wave
// re-reading 64 status words at once slowed the other blocks' staging loads.
// The look-back's fallback: every '\n' before the tile, counted by the waiting wave with 4 B per
// lane and load (one byte per lane and load made a late tile of a large text millions
// of loads). 4 B, not 16: the 16-B loop took the parse kernel from 58 to 69 VGPRs (73 out of
// line, the call's ABI), 8 -> 7 waves per SIMD, and the whole parse 3-7 % slower
// (profiles/r05_ingest_ab.txt); one word per lane keeps it at 64 VGPRs, 8 waves.
__device__ __forceinline__ unsigned long long count_nl_before(const uint8_t* __restrict__ text, uint64_t end) {
  const uint32_t lane = threadIdx.x & 63;
  unsigned long long c = 0;
  const uint64_t head = min(end, (uint64_t)((4u - ((uintptr_t)text & 3u)) & 3u));
  for (uint64_t q = lane; q < head; q += 64) c += text[q] == '\n';
  const uint32_t* v4 = reinterpret_cast<const uint32_t*>(text + head);
  const uint64_t n4 = (end - head) / 4;
  for (uint64_t q = lane; q < n4; q += 64) {
    const uint32_t x = v4[q] ^ 0x0A0A0A0Au;  // as nl_count16, on one word
    c += __popc(~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu));
  }
  for (uint64_t q = head + 4 * n4 + lane; q < end; q += 64) c += text[q] == '\n';
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
  return c;
}

#ifdef GS_LB_STATS  // experiment: per-tile look-back statistics {ticks before, ticks waited, sleeps, windows}
constexpr uint32_t kLbsTiles = 65536;
__device__ uint32_t g_lbt[kLbsTiles][8];  // + [4] staged, [5] masks, [6] scanned, [7] loads landed (wave 0)
#endif
__device__ __forceinline__ unsigned long long look_back(const uint8_t* __restrict__ text, unsigned long long* status,
                                                        unsigned long long* pstat, uint64_t tile, unsigned long long agg,
                                                        bool published, unsigned long long lb_timeout) {
  const int lane = threadIdx.x & 63;
  if (tile == 0) {
    if (lane == 0) __hip_atomic_store(pstat, kStP | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  // (published: the waves' early adds already carry the aggregate; a store here could
  // overtake one of them)
  if (lane == 0 && !published)
    __hip_atomic_store(status + tile, kStA | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long excl = 0;
  int64_t base = (int64_t)tile - 1;
  const unsigned long long t_start = wall_clock64();
  int backoff = 0;
  unsigned wins = 0;
  for (;;) {
    const int64_t ti = base - lane;  // lane 0: the nearest predecessor
    const unsigned long long wp =
        ti >= 0 ? __hip_atomic_load(pstat + ti, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kStP;
    const unsigned long long wa =
        ti >= 0 ? __hip_atomic_load(status + ti, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    const bool has_p = (wp & kStP) != 0;
    const unsigned long long w = has_p ? wp : wa;
    const unsigned long long pm = __ballot(has_p), am = __ballot(has_p || st_has_agg(wa));
    const int j = pm ? __ffsll((long long)pm) - 1 : 64;  // nearest final prefix in this window
    const unsigned long long need = j >= 64 ? ~0ull : ((2ull << j) - 1ull);  // lanes 0..j
    if ((am & need) == need) {
      unsigned long long v = lane <= j ? (has_p ? (w & kStVal) : st_agg(w)) : 0ull;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
      excl += v;
      if (j < 64) break;
      base -= 64;  // the whole window was own counts: continue further back
      ++wins;
      continue;
    }
    if (wall_clock64() - t_start > lb_timeout) {  // ~50 ms (100 MHz clock) by default: count it directly
      excl = count_nl_before(text, tile * kTile);
      break;
    }
    if (backoff < 3) {
      __builtin_amdgcn_s_sleep(GS_LB_SLEEP0);
    } else {
      __builtin_amdgcn_s_sleep(GS_LB_SLEEP1);
    }
    ++backoff;
  }
  if (lane == 0) __hip_atomic_store(pstat + tile, kStP | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef GS_LB_STATS
  if (lane == 0 && tile < kLbsTiles) {
    g_lbt[tile][1] = (uint32_t)(wall_clock64() - t_start);
    g_lbt[tile][2] = (uint32_t)backoff;
    g_lbt[tile][3] = wins;
  }
#endif
  (void)wins;
  return excl;
}

__global__ __launch_bounds__(256) void k_parse_fused(const uint8_t* __restrict__ text, uint64_t len, int sep,
                                                     int64_t* __restrict__ src, int64_t* __restrict__ dst, uint64_t cap,
                                                     unsigned long long* __restrict__ bad, bool aligned,
                                                     unsigned long long* __restrict__ status, unsigned long long* __restrict__ pstat,
                                                     unsigned long long lb_timeout) {
  parse_tile<true>(text, len, sep, nullptr, src, dst, cap, bad, aligned, blockIdx.x, status, pstat, lb_timeout);
}

// One tile per block (44 VGPRs, 8 blocks per CU).
__global__ __launch_bounds__(256) void k_parse(const uint8_t* __restrict__ text, uint64_t len, int sep,
                                               const uint64_t* __restrict__ tile_pre, int64_t* __restrict__ src,
                                               int64_t* __restrict__ dst, uint64_t cap,
                                               unsigned long long* __restrict__ bad, bool aligned, uint64_t tile0) {
  parse_tile<false>(text, len, sep, tile_pre, src, dst, cap, bad, aligned, tile0 + blockIdx.x, nullptr, nullptr, 0ull);
}

template <bool FUSED>
__device__ __forceinline__ void parse_tile(const uint8_t* __restrict__ text, uint64_t len, int sep,
                                           const uint64_t* __restrict__ tile_pre, int64_t* __restrict__ src,
                                           int64_t* __restrict__ dst, uint64_t cap,
                                           unsigned long long* __restrict__ bad, bool aligned, uint64_t tile,
                                           unsigned long long* __restrict__ status, unsigned long long* __restrict__ pstat,
                                           unsigned long long lb_timeout) {
  constexpr uint32_t kSeg = kTile / 256;  // bytes per thread in the line-start scan
  constexpr uint32_t kExtra = 2;          // '\n' masks past the tile: lines that cross its end
  constexpr uint32_t kSlots = (kTile + kOver + 4095) / 4096;
  static_assert(kSeg == 64 && kSlots == 5, "one 64-bit mask and five staging slots per thread");
  static_assert(kExtra * kSeg <= kOver, "the extra masks lie in the staged bytes");
  __shared__ __align__(16) uint8_t lds[kLds0 + kTile + kOver];
  __shared__ uint64_t nlm[256 + kExtra];
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t wnl[4];
  const uint64_t t0 = tile * kTile;
  const uint64_t staged_end = min(len, t0 + kTile + kOver);
#ifdef GS_LB_STATS
  const unsigned long long blk_start = wall_clock64();
#endif
  // stage [t0, staged_end) at lds[kLds0..] with 16-B stores; lds[kLds0 - 1] = byte t0 - 1.
  // Every thread's global loads (five 16-B slots, 4 KiB apart) are issued before any is
  // waited for; named registers, not an array (an indexed array of them went to scratch).
  if (threadIdx.x == 0) lds[kLds0 - 1] = t0 == 0 ? (uint8_t)'\n' : text[t0 - 1];
  const uint32_t i0 = threadIdx.x * 16u;
  auto full = [&](uint32_t i) { return aligned && i < kTile + kOver && t0 + i + 16 <= staged_end; };
  const bool f0 = full(i0), f1 = full(i0 + 4096u), f2 = full(i0 + 8192u), f3 = full(i0 + 12288u),
             f4 = full(i0 + 16384u);
  uint4 v0 = {}, v1 = {}, v2 = {}, v3 = {}, v4 = {};
  if (f0) v0 = *reinterpret_cast<const uint4*>(text + t0 + i0);
  if (f1) v1 = *reinterpret_cast<const uint4*>(text + t0 + i0 + 4096u);
  if (f2) v2 = *reinterpret_cast<const uint4*>(text + t0 + i0 + 8192u);
  if (f3) v3 = *reinterpret_cast<const uint4*>(text + t0 + i0 + 12288u);
  if (f4) v4 = *reinterpret_cast<const uint4*>(text + t0 + i0 + 16384u);
  // one-pass: a tile wholly inside the (aligned) text publishes its '\n' count from the
  // staged registers (slots 0-3 are exactly its 16 KiB), wave by wave, right away
  const bool early = GS_PARSE_EARLY && FUSED && tile != 0 && aligned && t0 + kTile <= len;
  // a tile whose staged bytes all lie inside the (aligned) text: every thread's '\n' masks
  // of its five slots straight from the registers (no LDS read-back and one barrier less);
  // the count the early aggregate publishes is theirs
  const bool regmask = GS_PARSE_REGMASK && aligned && staged_end == t0 + kTile + kOver;
  uint16_t* m16 = reinterpret_cast<uint16_t*>(nlm);
  uint32_t mk0 = 0, mk1 = 0, mk2 = 0, mk3 = 0;
  if (regmask) {
    mk0 = nl_mask16(v0);
    mk1 = nl_mask16(v1);
    mk2 = nl_mask16(v2);
    mk3 = nl_mask16(v3);
    m16[threadIdx.x] = (uint16_t)mk0;
    m16[256 + threadIdx.x] = (uint16_t)mk1;
    m16[512 + threadIdx.x] = (uint16_t)mk2;
    m16[768 + threadIdx.x] = (uint16_t)mk3;
    if (threadIdx.x < 4 * kExtra) m16[1024 + threadIdx.x] = (uint16_t)nl_mask16(v4);
  }
  if (early) {
    uint32_t c = regmask ? __popc(mk0) + __popc(mk1) + __popc(mk2) + __popc(mk3)
                         : nl_count16(v0) + nl_count16(v1) + nl_count16(v2) + nl_count16(v3);
    c = __builtin_amdgcn_readlane(wave_incl_sum(c), 63);
    if ((threadIdx.x & 63u) == 0) {
      __hip_atomic_fetch_add(status + tile, (1ull << kStWaveShift) | (unsigned long long)c, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      wnl[threadIdx.x >> 6] = c;  // (the look-back's aggregate: this wave's quarter of the tile)
    }
  }
  auto put = [&](bool f, uint32_t i, const uint4& v) {
    if (f) {
      *reinterpret_cast<uint4*>(lds + kLds0 + i) = v;
    } else if (i < kTile + kOver) {  // the text's end (or an unaligned text): byte by byte
      for (uint64_t q = t0 + i; q < t0 + i + 16 && q < staged_end; ++q) lds[kLds0 + (q - t0)] = text[q];
    }
  };
#ifdef GS_LB_STATS
  if (threadIdx.x == 0 && tile < kLbsTiles) {
    const uint32_t x = v0.x ^ v1.x ^ v2.x ^ v3.x ^ v4.x;  // the loads have landed (for this wave)
    g_lbt[tile][7] = (uint32_t)(wall_clock64() - blk_start) | (x & 0u);
  }
#endif
  put(f0, i0, v0);
  put(f1, i0 + 4096u, v1);
  put(f2, i0 + 8192u, v2);
  put(f3, i0 + 12288u, v3);
  put(f4, i0 + 16384u, v4);
  __syncthreads();
#ifdef GS_LB_STATS
  if (threadIdx.x == 0 && tile < kLbsTiles) g_lbt[tile][4] = (uint32_t)(wall_clock64() - blk_start);
#endif
  // (1) each thread's 64-byte segment: its '\n' mask (to LDS: a line's end may lie in a
  //     later segment) and its line starts (byte p - 1 is '\n', or p == 0); a block
  //     scan of the start counts numbers the lines.
  const uint8_t* L = lds + kLds0;
  const uint32_t seg = threadIdx.x * kSeg;
  const uint64_t tile_end = min(len, t0 + kTile);
  const uint64_t vend = staged_end == len ? len - t0 : ~0ull;  // the text ends inside the staged bytes
  // 16-bit chunk masks written as the u16 quarters of nlm (little endian: nlm[q] is
  // then segment q's 64-bit mask); 4 chunks per thread + the kExtra segments' chunks
  if (!regmask) {  // (block-uniform) the text's last tiles, unaligned texts: from LDS, with the end rule
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) m16[r * 256 + threadIdx.x] = (uint16_t)chunk_nl_mask(L, r * 256 + threadIdx.x, vend);
    if (threadIdx.x < 4 * kExtra) m16[1024 + threadIdx.x] = (uint16_t)chunk_nl_mask(L, 1024 + threadIdx.x, vend);
    __syncthreads();
  }
#ifdef GS_LB_STATS
  if (threadIdx.x == 0 && tile < kLbsTiles) g_lbt[tile][5] = (uint32_t)(wall_clock64() - blk_start);
#endif
  const uint64_t nl = nlm[threadIdx.x];
  // bit j: a line starts at seg + j (byte seg + j - 1 is '\n': the previous segment's top bit)
  const bool prev_nl = threadIdx.x == 0 ? L[-1] == '\n' : (nlm[threadIdx.x - 1] >> 63) != 0;
  uint64_t mine = (nl << 1) | (prev_nl ? 1ull : 0ull);
  const uint64_t valid = t0 + seg >= tile_end ? 0 : min<uint64_t>(kSeg, tile_end - (t0 + seg));
  if (valid < 64) mine &= (1ull << valid) - 1ull;
  const uint32_t c = __popcll(mine);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t x = wave_incl_sum(c);
  if (lane == 63) wsum[wid] = x;
  if (FUSED && !early) {  // the tile's own '\n' (its bytes only): the look-back's aggregate (early: counted above)
    const uint32_t cn = __popcll(valid >= 64 ? nl : (nl & ((1ull << valid) - 1ull)));
    const uint32_t tot = __builtin_amdgcn_readlane(wave_incl_sum(cn), 63);
    if (lane == 0) wnl[wid] = tot;
  }
  __syncthreads();
#ifdef GS_LB_STATS
  if (threadIdx.x == 0 && tile < kLbsTiles) g_lbt[tile][6] = (uint32_t)(wall_clock64() - blk_start);
#endif
  uint32_t wbase = 0;
  for (int q = 0; q < 4; ++q)
    if (q < wid) wbase += wsum[q];
  // (2) each thread parses the lines that start in its segment; the k-th start of the
  //     tile follows k '\n' of the tile if a line starts at t0, else k + 1
  const uint64_t line_off = (L[-1] == '\n' ? 0u : 1u) + wbase + (x - c);  // within the text after the tile's prefix
  const LineBuf b{lds, text, t0, len, staged_end};
#if GS_PARSE_BRANCHLESS
  const uint64_t nx1 = nlm[threadIdx.x + 1], nx2 = nlm[threadIdx.x + 2];  // the next two segments' '\n' masks
#endif
  // one line starting at segment byte j: (a, d) and whether it is well formed
  auto parse_at = [&](uint32_t j, int64_t& a, int64_t& d) -> bool {
    const int so = (int)(seg + j);
    // the line's '\n': the first one at or after its start, within this segment or
    // the next two (longer lines take the per-character path)
    int e = -1;
    const uint64_t own = nl & (~0ull << j);
#if GS_PARSE_BRANCHLESS
    e = own ? (int)seg + __builtin_ctzll(own)
            : (nx1 ? (int)seg + 64 + __builtin_ctzll(nx1) : (nx2 ? (int)seg + 128 + __builtin_ctzll(nx2) : -1));
#else
    if (own) {
      e = (int)seg + __builtin_ctzll(own);
    } else {
      const uint64_t n1 = nlm[threadIdx.x + 1];
      if (n1) {
        e = (int)seg + 64 + __builtin_ctzll(n1);
      } else {
        const uint64_t n2 = nlm[threadIdx.x + 2];
        if (n2) e = (int)seg + 128 + __builtin_ctzll(n2);
      }
    }
#endif
#ifdef GS_PARSE_FLOOR  // experiment: no field parse (the kernel's floor without the SWAR work)
    a = so;
    d = e;
    return e >= 0;
#endif
    uint64_t q = t0 + (uint64_t)so;
    a = 0;
    d = 0;
    int r = -1;
#if GS_PARSE_BRANCHLESS
    const int ee = e >= 0 ? e : so + 1;  // (no '\n' in reach: the result is discarded, r = -1)
    r = sep == GS_SEP_TAB ? parse_line_swar_bf<GS_SEP_TAB>(L, so, ee, a, d)
                          : parse_line_swar_bf<GS_SEP_WHITESPACE>(L, so, ee, a, d);
    if (e < 0) r = -1;
#else
    if (e >= 0)
      r = sep == GS_SEP_TAB ? parse_line_swar<GS_SEP_TAB>(L, so, e, a, d)
                            : parse_line_swar<GS_SEP_WHITESPACE>(L, so, e, a, d);
#endif
    bool ok = r == 1;
    if (r < 0) {  // a long line or field: one byte per step
      // two fields: the first must end at a separator (else fields[1] does not exist)
      ok = parse_long(b, q, sep, a) == kFieldSep;
      if (ok) {
        ++q;
        ok = parse_long(b, q, sep, d) != kFieldBad;
      }
    }
    return ok;
  };
  auto emit = [&](uint64_t line, bool ok, int64_t a, int64_t d) {
    if (!ok) {
      atomicMin(bad, (unsigned long long)line);
    } else if (line < cap) {
      src[line] = a;
      dst[line] = d;
    }
  };
  uint64_t line;
  if (FUSED) {
    // a thread's first two lines (nearly always all of them) are parsed into registers
    // BEFORE the look-back, so that the predecessors' counts are published by the time
    // wave 0 reads them, and only the stores wait for the tile's line numbers
    int64_t a0 = 0, d0 = 0, a1 = 0, d1 = 0;
    bool ok0 = true, ok1 = true;
    uint32_t k = 0;
    if (mine) {
      const uint32_t j = __ffsll((unsigned long long)mine) - 1;
      mine &= mine - 1;
      ok0 = parse_at(j, a0, d0);
      k = 1;
    }
    if (mine) {
      const uint32_t j = __ffsll((unsigned long long)mine) - 1;
      mine &= mine - 1;
      ok1 = parse_at(j, a1, d1);
      k = 2;
    }
    __shared__ unsigned long long pre_sh;
#ifdef GS_PARSE_NOLB  // experiment: no look-back (wrong line numbers; the kernel's cost without it)
    if (threadIdx.x == 0) pre_sh = 0;
    if (false) {
#else
    if (wid == 0) {
#endif
#ifdef GS_LB_STATS
      if (lane == 0 && tile < kLbsTiles) g_lbt[tile][0] = (uint32_t)(wall_clock64() - blk_start);
#endif
      const unsigned long long e =
          look_back(text, status, pstat, tile, (unsigned long long)wnl[0] + wnl[1] + wnl[2] + wnl[3], early,
                    lb_timeout);
      if (lane == 0) pre_sh = e;
    }
    __syncthreads();
    line = pre_sh + line_off;
    if (k >= 1) emit(line, ok0, a0, d0);
    if (k >= 2) emit(line + 1, ok1, a1, d1);
    line += k;
  } else {
    line = tile_pre[tile] + line_off;
  }
  while (mine) {
    const uint32_t j = __ffsll((unsigned long long)mine) - 1;
    mine &= mine - 1;
    int64_t a, d;
    const bool ok = parse_at(j, a, d);
    emit(line, ok, a, d);
    ++line;
  }
}

// Exclusive scan of the tiles' '\n' counts (the two-pass path): one block walks the tiles in
// rounds of 1024 with a wave scan + the wave totals, carrying the sum.
__global__ __launch_bounds__(1024) void k_tile_scan(const uint64_t* __restrict__ cnt, uint64_t* __restrict__ pre,
                                                    uint64_t n) {
  __shared__ unsigned long long wsum[16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned long long carry = 0;
  for (uint64_t c0 = 0; c0 < n; c0 += 1024) {
    const uint64_t i = c0 + threadIdx.x;
    const unsigned long long v = i < n ? cnt[i] : 0ull;
    unsigned long long x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    unsigned long long wb = 0, tot = 0;
    for (int q = 0; q < 16; ++q) {
      if (q < wid) wb += wsum[q];
      tot += wsum[q];
    }
    if (i < n) pre[i] = carry + wb + (x - v);
    carry += tot;
    __syncthreads();
  }
}

// {line count, first malformed line (~0: none)} of a parsed text; with `host` (mapped
// memory) also host[1..2] = the same two words and then host[0] = seq (system-scope
// release): the caller spins on that word instead of a copy and a stream synchronisation
__global__ void k_parse_result(const uint64_t* tile_pre, const uint64_t* tile_cnt, uint64_t tiles,
                               const uint8_t* text, uint64_t len, unsigned long long* bad, uint64_t* res,
                               unsigned long long* host, unsigned long long seq, const unsigned long long* status) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  // '\n' through the last tile (fused: its prefix word), + 1: a last line may lack '\n'
  const uint64_t nl = status ? (status[tiles - 1] & kStVal) : tile_pre[tiles - 1] + tile_cnt[tiles - 1];
  const uint64_t lines = nl + (text[len - 1] != '\n' ? 1u : 0u);
  const uint64_t b = *bad;
  *bad = ~0ull;  // ready for the next parse (the one-pass path does not memset it)
  res[0] = lines;
  res[1] = b;
  if (host) {
    __hip_atomic_store(host + 1, (unsigned long long)lines, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host + 2, (unsigned long long)b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The one-pass parse's result (as k_parse_result, from the last tile's prefix word) and the
// reset of the status words it used, for the next parse: the aggregate and prefix words of
// its tiles. One launch instead of a fill before the parse and a result
// kernel after it. Block 0 reads the last prefix before it clears it; nothing else reads
// the words once k_parse_fused has finished (stream order).
__global__ __launch_bounds__(256) void k_parse_finish(unsigned long long* agg, unsigned long long* pre,
                                                      uint64_t tiles, uint64_t tiles_cap, const uint8_t* text,
                                                      uint64_t len, unsigned long long* bad, uint64_t* res,
                                                      unsigned long long* host, unsigned long long seq) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const uint64_t nl = pre[tiles - 1] & kStVal;
    const uint64_t lines = nl + (text[len - 1] != '\n' ? 1u : 0u);
    const uint64_t b = *bad;
    *bad = ~0ull;
    res[0] = lines;
    res[1] = b;
    pre[tiles - 1] = 0;
    if (host) {
      __hip_atomic_store(host + 1, (unsigned long long)lines, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(host + 2, (unsigned long long)b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(host, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tiles; i += stride) {
    agg[i] = 0;
    if (i + 1 < tiles) pre[i] = 0;
  }
}

int parse_text_enqueue(hipStream_t st, const char* text, size_t len, int sep, int64_t* src, int64_t* dst, size_t cap,
                       ParseScratch& s, unsigned long long* host_res, unsigned long long seq, bool fused,
                       hipEvent_t kev0, hipEvent_t kev1) {
  if (len == 0) return hipMemsetAsync(s.res, 0xFF, 16, st) == hipSuccess &&
                        hipMemsetAsync(s.res, 0, 8, st) == hipSuccess ? 0 : -1;
  const uint64_t tiles = (len + kTile - 1) / kTile;
  if (tiles > s.tiles_cap) return -1;
  const bool aligned = ((uintptr_t)text & 15u) == 0;
  const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
  // Block 0 of k_parse_finish publishes the result before the other blocks have cleared
  // every status word; on the same stream the next parse starts after that whole kernel,
  // on another one it could overlap the late clears: fill again there.
  const bool st_zero = s.st_zero && s.zero_stream == st;
  s.st_zero = false;  // until this call has queued a k_parse_finish
  if (fused) {  // aggregate words (s.tile_cnt) and prefix words (s.tile_pre) zero, then one pass
    // the previous one-pass parse's k_parse_finish left them zero; else one fill (the
    // aggregate words and the prefix words are adjacent: tile_pre = tile_cnt + tiles_cap);
    // `bad` is reset by the previous parse's k_parse_result / k_parse_finish
    if (!st_zero && hipMemsetAsync(s.tile_cnt, 0, (s.tiles_cap + s.tiles_cap) * 8, st) != hipSuccess) return -1;
    if (!s.bad_ready && hipMemsetAsync(s.bad, 0xFF, 8, st) != hipSuccess) return -1;
    s.bad_ready = true;
    unsigned long long* agg = reinterpret_cast<unsigned long long*>(s.tile_cnt);
    unsigned long long* pre = reinterpret_cast<unsigned long long*>(s.tile_pre);
    if (kev0 && hipEventRecord(kev0, st) != hipSuccess) return -1;
    // how long a look-back waits before it counts the '\n' before its tile itself (~50 ms;
    // tests shorten it with GS_TESTING_PARSE_LB_TIMEOUT_US, 0: at once)
    const unsigned long long lb_timeout = 100ull * (unsigned long long)gsi::testing_value(GS_TESTING_PARSE_LB_TIMEOUT_US, 50000);
    hipLaunchKernelGGL(k_parse_fused, dim3((unsigned)tiles), dim3(256), 0, st, t, (uint64_t)len, sep, src, dst,
                       (uint64_t)cap, s.bad, aligned, agg, pre, lb_timeout);
    if (kev1 && hipEventRecord(kev1, st) != hipSuccess) return -1;
#ifdef GS_LB_STATS
    if (tiles > 4096 && tiles <= kLbsTiles) {  // the large parses only: per-tile figures, summarised
      static uint32_t v[kLbsTiles][8];
      if (hipStreamSynchronize(st) == hipSuccess &&
          hipMemcpyFromSymbol(v, HIP_SYMBOL(g_lbt), tiles * 32) == hipSuccess) {
        double sum[8] = {};
        uint32_t slept = 0;
        std::vector<uint32_t> w(tiles), b(tiles);
        for (uint64_t q = 0; q < tiles; ++q) {
          for (int c = 0; c < 8; ++c) sum[c] += v[q][c];
          slept += v[q][2] > 0;
          b[q] = v[q][0];
          w[q] = v[q][1];
        }
        std::sort(w.begin(), w.end());
        std::sort(b.begin(), b.end());
        const double n = (double)tiles;
        fprintf(stderr, "LBSTATS tiles %llu before_us avg %.2f p50 %.2f p90 %.2f | wait_us avg %.2f p50 %.2f p90 %.2f "
                "p99 %.2f | sleeps/blk %.2f slept %.3f windows/blk %.3f\n", (unsigned long long)tiles,
                sum[0] / n / 100, b[tiles / 2] / 100.0, b[tiles * 9 / 10] / 100.0, sum[1] / n / 100,
                w[tiles / 2] / 100.0, w[tiles * 9 / 10] / 100.0, w[tiles * 99 / 100] / 100.0, sum[2] / n, slept / n,
                sum[3] / n);
        fprintf(stderr, "LBPHASES landed %.2f staged %.2f masks %.2f scanned %.2f parsed %.2f (us after block start)\n",
                sum[7] / n / 100, sum[4] / n / 100, sum[5] / n / 100, sum[6] / n / 100, sum[0] / n / 100);
      }
    }
#endif
    hipLaunchKernelGGL(k_parse_finish, dim3((unsigned)std::min<uint64_t>(64, (tiles + 255) / 256)), dim3(256), 0, st,
                       agg, pre, tiles, s.tiles_cap, t, (uint64_t)len, s.bad, s.res, host_res, seq);
    if (hipGetLastError() != hipSuccess) return -1;
    s.st_zero = true;
    s.zero_stream = st;
    return 0;
  }
  hipLaunchKernelGGL(k_count_lines, dim3((unsigned)tiles), dim3(256), 0, st, t, (uint64_t)len, s.tile_cnt, aligned,
                     (uint64_t)0);
  hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(1024), 0, st, s.tile_cnt, s.tile_pre, tiles);
  if (hipMemsetAsync(s.bad, 0xFF, 8, st) != hipSuccess) return -1;
  hipLaunchKernelGGL(k_parse, dim3((unsigned)tiles), dim3(256), 0, st, t, (uint64_t)len, sep, s.tile_pre, src, dst,
                     (uint64_t)cap, s.bad, aligned, (uint64_t)0);
  hipLaunchKernelGGL(k_parse_result, dim3(1), dim3(64), 0, st, s.tile_pre, s.tile_cnt, tiles, t, (uint64_t)len,
                     s.bad, s.res, host_res, seq, nullptr);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int parse_text(hipStream_t st, const char* text, size_t len, int sep, int64_t* src, int64_t* dst, size_t cap,
               ParseScratch& s, uint64_t* n_lines, int64_t* bad_line) {
  *n_lines = 0;
  *bad_line = -1;
  if (parse_text_enqueue(st, text, len, sep, src, dst, cap, s, nullptr, 0)) return -1;
  uint64_t res[2];
  if (hipMemcpyAsync(res, s.res, 16, hipMemcpyDeviceToHost, st) != hipSuccess) return -1;
  if (hipStreamSynchronize(st) != hipSuccess) return -1;
  *n_lines = res[0];
  *bad_line = res[1] == ~0ull ? -1 : (int64_t)res[1];
  return 0;
}

size_t parse_scratch_bytes(size_t max_len, size_t* cub_bytes) {
  const uint64_t tiles = (max_len + kTile - 1) / kTile + 1;
  const size_t tmp = 0;  // (no library scan scratch: k_tile_scan)
  *cub_bytes = tmp;
  return tiles * 16 + 48 + tmp + 256;
}

int parse_scratch_init(ParseScratch& s, void* mem, size_t max_len) {
  size_t cub = 0;
  parse_scratch_bytes(max_len, &cub);
  const uint64_t tiles = (max_len + kTile - 1) / kTile + 1;
  uint8_t* p = static_cast<uint8_t*>(mem);
  s.tile_cnt = reinterpret_cast<uint64_t*>(p);
  s.tile_pre = s.tile_cnt + tiles;
  s.bad = reinterpret_cast<unsigned long long*>(s.tile_pre + tiles);
  s.res = reinterpret_cast<uint64_t*>(s.bad + 2);
  s.cub_tmp = reinterpret_cast<void*>(((uintptr_t)(s.res + 4) + 255) & ~(uintptr_t)255);
  s.cub_bytes = cub;
  s.tiles_cap = tiles;
  s.bad_ready = false;
  s.st_zero = false;
  return 0;
}

}  // namespace gs

namespace {
// Scratch of gs_parse_edges_device kept per thread and device (grown, never shrunk), and
// a host-mapped result record: a call costs the parse's launches and one spin on host
// memory, not an allocation, a device-to-host copy and two stream synchronisations
// (~40 us of a 2^24-line parse; profiles/r04_ingest_ab.txt).
struct ParseCache {
  int device = -1;
  size_t len_cap = 0;
  void* mem = nullptr;
  gs::ParseScratch s;
  unsigned long long* host = nullptr;  // mapped {seq, lines, bad}
  unsigned long long* host_dev = nullptr;
  unsigned long long seq = 0;
  // gs_parse_set_profiling: the parse kernel between two events, summed
  bool prof = false;
  hipEvent_t kev[2] = {nullptr, nullptr};
  double prof_us = 0.0;
  uint64_t prof_n = 0;
};
thread_local ParseCache t_parse;

// Free the cache's device scratch, mapped result record and timing events (on the device
// they belong to). gs_parse_edges_device returns once the parse's result is published,
// but the other blocks of k_parse_finish may still be clearing status words:
// the device is synchronised before the scratch goes.
int parse_cache_free(ParseCache& c) {
  if (c.device < 0) return 0;
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) return -1;
  if (cur != c.device && hipSetDevice(c.device) != hipSuccess) return -1;
  int rc = hipDeviceSynchronize() == hipSuccess ? 0 : -1;
  if (c.mem && hipFree(c.mem) != hipSuccess) rc = -1;
  if (c.host && hipHostFree(c.host) != hipSuccess) rc = -1;
  for (hipEvent_t e : c.kev)
    if (e && hipEventDestroy(e) != hipSuccess) rc = -1;
  if (cur != c.device && hipSetDevice(cur) != hipSuccess) rc = -1;
  c = ParseCache();
  return rc;
}

int parse_cache_ready(hipStream_t st, size_t len) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  ParseCache& c = t_parse;
  if (c.device != dev) {  // first use, or the thread moved to another device: free the old device's cache
    const bool prof = c.prof;
    if (parse_cache_free(c)) return -1;
    if (prof && gs_parse_set_profiling(1) != GS_OK) return -1;  // the timing events live on the new device
    c.device = dev;
    if (hipHostMalloc(&c.host, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&c.host_dev), c.host, 0) != hipSuccess)
      return -1;
    memset(c.host, 0, 64);
  }
  if (c.len_cap < len || !c.mem) {
    if (c.mem) {
      // the old scratch's last user (k_parse_finish of the previous parse, on any stream)
      if (hipDeviceSynchronize() != hipSuccess) return -1;
      (void)hipFree(c.mem);
      c.mem = nullptr;
    }
    const size_t want = std::max<size_t>(len + len / 4, 1u << 20);
    size_t cub = 0;
    if (hipMalloc(&c.mem, gs::parse_scratch_bytes(want, &cub)) != hipSuccess) return -1;
    gs::parse_scratch_init(c.s, c.mem, want);
    c.len_cap = want;
  }
  return 0;
}
}  // namespace

extern "C" int gs_parse_edges_device(void* stream, const char* text, size_t len, int sep, int64_t* src, int64_t* dst,
                                     size_t cap, uint64_t* n_lines, int64_t* bad_line) {
  if (!n_lines || !bad_line || (len && !text)) return GS_ERR_INVALID;
  if (sep != GS_SEP_WHITESPACE && sep != GS_SEP_TAB) return GS_ERR_INVALID;
  hipStream_t st = static_cast<hipStream_t>(stream);
  *n_lines = 0;
  *bad_line = -1;
  if (len == 0) return GS_OK;
  if (parse_cache_ready(st, len)) return GS_ERR_HIP;
  ParseCache& c = t_parse;
  const unsigned long long seq = ++c.seq;
  constexpr bool one_pass = true;  // (the count pass + scan + parse pass serves gs_fold_text's chunks)
  const bool prof = c.prof && one_pass;
  const int rc = gs::parse_text_enqueue(st, text, len, sep, src, dst, cap, c.s, c.host_dev, seq, one_pass,
                                        prof ? c.kev[0] : nullptr, prof ? c.kev[1] : nullptr);
  if (rc) return GS_ERR_HIP;
  // spin on the mapped record; a long parse hands over to the stream synchronisation
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 1; __atomic_load_n(c.host, __ATOMIC_ACQUIRE) != seq; ++i) {
    if ((i & 255u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(2000)) {
      if (hipStreamSynchronize(st) != hipSuccess) return GS_ERR_HIP;
      if (__atomic_load_n(c.host, __ATOMIC_ACQUIRE) != seq) return GS_ERR_HIP;
      break;
    }
    __builtin_ia32_pause();
  }
  if (hipGetLastError() != hipSuccess) return GS_ERR_HIP;
  *n_lines = __atomic_load_n(c.host + 1, __ATOMIC_ACQUIRE);
  const unsigned long long b = __atomic_load_n(c.host + 2, __ATOMIC_ACQUIRE);
  *bad_line = b == ~0ull ? -1 : (int64_t)b;
  if (prof) {
    float ms = 0.f;
    if (hipEventSynchronize(c.kev[1]) != hipSuccess || hipEventElapsedTime(&ms, c.kev[0], c.kev[1]) != hipSuccess)
      return GS_ERR_HIP;
    c.prof_us += 1e3 * (double)ms;
    ++c.prof_n;
  }
  if (*bad_line >= 0) return GS_ERR_PARSE;
  if (*n_lines > cap) return GS_ERR_TRUNCATED;
  return GS_OK;
}

extern "C" int gs_parse_set_profiling(int on) {
  ParseCache& c = t_parse;
  if (on && !c.kev[0]) {
    for (hipEvent_t& e : c.kev)
      if (hipEventCreate(&e) != hipSuccess) return GS_ERR_HIP;  // timing events
  }
  c.prof = on != 0;
  c.prof_us = 0.0;
  c.prof_n = 0;
  return GS_OK;
}

extern "C" int gs_parse_release(void) {
  return parse_cache_free(t_parse) ? GS_ERR_HIP : GS_OK;
}

extern "C" int gs_parse_profile(double* kernel_us, uint64_t* parses) {
  if (!kernel_us || !parses) return GS_ERR_INVALID;
  *kernel_us = t_parse.prof_us;
  *parses = t_parse.prof_n;
  return GS_OK;
}
