// Drop-in operator benchmark: the reference's SummaryBulkAggregation dataflow with
// the unchanged ConnectedComponents operators (S/library/ConnectedComponents.java:
// UpdateCC per edge, CombineCC per window, Merger per window), over GPU-backed
// DisjointSet summaries -- the call sequence Flink would issue through the JNI glue
// of INTEGRATION.md: per edge foldEdges -> DisjointSet.union (buffered), per
// (partition, window) a fresh initial value (pooled handle), per window CombineCC of
// the p partials and Merger(s, summary) into the running summary.
//
// Workload: BASELINE config 2 (RMAT scale 20, 2^24 edges, sparse scrambled ids) in
// host memory, one window per 2^20 edges, edges dealt to p partitions round-robin
// (PartitionMapper, SummaryBulkAggregation.java:93-107).
// Usage: dropin_bench <scale> <seed> <log2 edges> <log2 window> <p> <labels out path>
// Prints one JSON line; writes the final (vertex, label) pairs (int64 LE) for the
// caller's oracle check.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "gelly_streaming.hpp"
#include "gs_gen.h"

using namespace gelly;

int main(int argc, char** argv) {
  if (argc != 7) {
    std::fprintf(stderr, "usage: dropin_bench <scale> <seed> <log2 edges> <log2 window> <p> <labels out>\n");
    return 2;
  }
  const int scale = atoi(argv[1]);
  const uint64_t seed = strtoull(argv[2], nullptr, 0);
  const uint64_t E = 1ull << atoi(argv[3]), W = 1ull << atoi(argv[4]);
  const int p = atoi(argv[5]);
  // the stream: generated on the GPU (same generator as bench.py), then host-resident
  int64_t *ds = nullptr, *dd = nullptr;
  if (hipMalloc(&ds, E * 8) != hipSuccess || hipMalloc(&dd, E * 8) != hipSuccess) return 3;
  if (gs_gen_rmat(nullptr, ds, dd, 0, E, scale, seed, 1) != GS_OK) return 3;
  std::vector<int64_t> hs(E), hd(E);
  if (hipMemcpy(hs.data(), ds, E * 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(hd.data(), dd, E * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return 3;
  (void)hipFree(ds);
  (void)hipFree(dd);
  EdgeStream<int64_t, NullValue> s;
  s.parallelism = p;
  s.edges.resize(E);
  s.timestamps.resize(E);
  for (uint64_t i = 0; i < E; ++i) {
    s.edges[i] = {hs[i], hd[i], NullValue{}};
    s.timestamps[i] = (int64_t)i;  // event time = position: window w = edges [w W, (w+1) W)
  }
  SimpleEdgeStream<int64_t, NullValue> stream(s);
  // capacity hint of one partition's window partial; the running summary grows
  ConnectedComponents<NullValue> cc((int64_t)W, 0, 2 * W / (uint64_t)p);
  DisjointSetRef last;
  size_t windows = 0;
  const auto t0 = std::chrono::steady_clock::now();
  stream.aggregate(cc, [&](const DisjointSetRef& ds) {
    last = ds;  // the Merger emission (a sink would read it here)
    ++windows;
  });
  uint64_t nv = last ? last->size() : 0;  // joins the last window's work
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const auto rows = last ? last->rows() : std::vector<GpuSummary::Row>{};
  if (FILE* f = std::fopen(argv[6], "wb")) {
    for (const auto& r : rows) {
      std::fwrite(&r.v, 8, 1, f);
      std::fwrite(&r.label, 8, 1, f);
    }
    std::fclose(f);
  }
  std::printf("{\"edges\": %llu, \"seconds\": %.6f, \"edges_per_s\": %.1f, \"windows\": %zu, \"partitions\": %d, "
              "\"vertices\": %llu, \"handles_created\": %zu, \"handles_reused\": %zu, \"flush_seconds\": %.6f, \"fold_loop_seconds\": %.6f, \"combine_merger_seconds\": %.6f}\n",
              (unsigned long long)E, secs, (double)E / secs, windows, p, (unsigned long long)nv,
              HandlePool::instance().created(), HandlePool::instance().reused(), GpuSummary::flush_seconds(), cc.run_seconds()[0], cc.run_seconds()[1]);
  return 0;
}
