/*
 * gs_gen.h -- device-side synthetic edge-stream generators (bench/test workloads).
 *
 * Not part of the reference interface: the reference reads edge streams from
 * Flink sources (ConnectedComponentsExample.java:106-140). These generators let
 * every GPU produce its own shard of the BASELINE.json streams directly in HBM,
 * following the counter-based spec in DESIGN.md "Workloads" (the CPU oracle holds
 * an independent implementation of the same spec). All pointers are DEVICE
 * pointers on the current HIP device; `stream` is a hipStream_t (NULL = default).
 */
#ifndef GS_GEN_H
#define GS_GEN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Graph500 RMAT (a,b,c,d) = (0.57,0.19,0.19,0.05), 2^scale vertices; edges
 * [start, start+count) of the stream keyed by `seed`. scramble != 0 maps raw
 * vertex numbers through a 64-bit bijection (sparse signed ids). */
int gs_gen_rmat(void* stream, int64_t* src, int64_t* dst, uint64_t start, uint64_t count, int scale, uint64_t seed,
                int scramble);

/* Erdos-Renyi G(2^logn, m): uniform endpoints. */
int gs_gen_er(void* stream, int64_t* src, int64_t* dst, uint64_t start, uint64_t count, int logn, uint64_t seed,
              int scramble);

/* Random bipartite stream over 2 x 2^logside vertices (left l -> id 2l, right r ->
 * id 2r+1). `inject` (HOST array of ascending absolute positions, may be NULL)
 * replaces those edges with same-side (left-left) edges. */
int gs_gen_bip(void* stream, int64_t* src, int64_t* dst, uint64_t start, uint64_t count, int logside, uint64_t seed,
               const uint64_t* inject, size_t ninject);

#ifdef __cplusplus
}
#endif
#endif /* GS_GEN_H */
