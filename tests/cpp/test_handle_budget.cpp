// The GPU summaries' HBM lifetime under Flink's default object handling,
// modelled on the C++ host mirror. With object reuse off Flink
//   * copies the initial value for every (partition, window) fold state
//     (TypeSerializer.copy, S/SummaryBulkAggregation.java:79-80) -- a GPU copy is a pooled
//     handle plus gs_combine, sized from its source's vertex count;
//   * clears a window's fold state after the window fires: the partial is dropped, never
//     released (S/SummaryAggregation.java:107-119);
//   * copies the Merger's output for every chained collect before the sink reads it; the
//     copy is dropped once the sink is done.
// The dropped summaries' handles come back only when the JVM finalizes them. Here they go
// to a finalizer queue that is emptied only when the pool's byte budget asks for it (the
// Java pool's System.gc() + System.runFinalization()). The run must keep the HBM the pool
// accounts (handles handed out + pooled) within the budget (plus one table) and end with the
// oracle's summary.
// Round 6: the budget is checked against the library's count of device
// memory (gs_hbm_bytes), so the Merger's running summary, which grows while handed out,
// counts at once. With a small default hint (the "grow" case) that summary grows 16x and
// more during the run. The window partial is a copy of the (empty) initial value
// (ADVICE r5): the pool must keep reusing grown pooled tables for it instead of creating.
// Usage: test_handle_budget <edges.bin: int64 src,dst pairs> <window edges> <budget bytes> <out.bin> [default hint]
// out.bin: int64 n, then n rows of int64 {v, label}. Prints one JSON line of pool statistics.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gelly_streaming.hpp"

using namespace gelly;

static void die(const std::string& m) {
  std::fprintf(stderr, "FAIL %s\n", m.c_str());
  std::exit(1);
}

// GpuSummarySerializer.copy: a fresh summary sized from the source's vertex count (x 2: the
// combine's capacity check charges each exported row as an edge), combined into
static DisjointSetRef copy_of(DisjointSet& src, uint64_t default_hint) {
  auto c = std::make_shared<DisjointSet>(0, default_hint);
  c->size_for(2 * src.size());
  c->merge(src);
  return c;
}

static uint64_t slots_of(DisjointSet& s) {
  uint64_t n = 0;
  gs_check(gs_table_capacity(s.handle(), &n));
  return n;
}

int main(int argc, char** argv) {
  if (argc != 5 && argc != 6) die("usage: test_handle_budget <edges.bin> <window> <budget bytes> <out.bin> [hint]");
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) die("cannot open edges");
  std::vector<int64_t> e;
  int64_t buf[4096];
  size_t got;
  while ((got = std::fread(buf, 8, 4096, f)) > 0) e.insert(e.end(), buf, buf + got);
  std::fclose(f);
  const size_t n = e.size() / 2, window = std::strtoull(argv[2], nullptr, 0);
  const uint64_t budget = std::strtoull(argv[3], nullptr, 0);
  const uint64_t default_hint = argc == 6 ? std::strtoull(argv[5], nullptr, 0) : 1 << 16;  // the pool's default hint
  std::vector<std::shared_ptr<GpuSummary>> finalizer_queue;  // dropped, not yet finalized
  size_t finalized = 0, max_queue = 0;
  HandlePool& pool = HandlePool::instance();
  pool.set_budget(budget, [&] {  // System.gc() + System.runFinalization()
    finalized += finalizer_queue.size();
    finalizer_queue.clear();
  });
  uint64_t worst = 0;     // gs_hbm_bytes after each window's emission
  uint64_t worst_over = 0;  // max over windows of (gs_hbm_bytes - budget - the largest table created in it)
  uint64_t summary_slots0 = 0, summary_slots1 = 0;
  try {
    ConnectedComponents<NullValue>::CombineCC combine;
    const auto initialVal = std::make_shared<DisjointSet>(0, default_hint);  // never used itself
    DisjointSetRef summary = std::make_shared<DisjointSet>(0, default_hint);  // Merger.summary
    summary_slots0 = slots_of(*summary);
    size_t windows = 0;
    for (size_t i = 0; i < n; i += window, ++windows) {
      // the window's fold state: Flink's copy of the initial value (empty: sized 2 x 0)
      DisjointSetRef partial = copy_of(*initialVal, default_hint);
      const size_t j = std::min(n, i + window);
      for (size_t k = i; k < j; ++k) partial->union_(e[2 * k], e[2 * k + 1]);  // UpdateCC.foldEdges
      // Merger.flatMap: summary = reduce(partial, summary); the input the combine dropped is
      // NOT released -- Flink clears the window state and the object waits for finalization
      DisjointSetRef kept = combine.reduce(partial, summary);
      DisjointSetRef dropped = kept == partial ? summary : partial;
      summary = kept;
      finalizer_queue.push_back(dropped);
      // the emission: copied for the chained collect, read by the sink, dropped
      DisjointSetRef out = copy_of(*summary, default_hint);
      if (out->size() != summary->size()) die("the emitted copy differs from the summary");
      finalizer_queue.push_back(out);
      max_queue = std::max(max_queue, finalizer_queue.size());
      const uint64_t now = HandlePool::device_bytes(0);
      worst = std::max(worst, now);
      // one table over the budget at most: the largest table of the run so far -- a copy sized
      // from the summary (or the default) -- which covers what a window may add after its last
      // acquire (a table growing in place, the running summary's combine scratch: ~12 B/slot
      // against a table's 20)
      uint64_t a = 0, b = 0;
      gs_check(gs_create_bytes(GS_KIND_CC, 2 * summary->size(), &a));
      gs_check(gs_create_bytes(GS_KIND_CC, default_hint, &b));
      const uint64_t table = std::max(a, b);
      if (now > budget + table) worst_over = std::max(worst_over, now - budget - table);
    }
    summary_slots1 = slots_of(*summary);
    const auto rows = summary->rows();
    std::vector<int64_t> o = {(int64_t)rows.size()};
    for (const auto& r : rows) {
      o.push_back(r.v);
      o.push_back(r.label);
    }
    FILE* g = std::fopen(argv[4], "wb");
    if (!g || std::fwrite(o.data(), 8, o.size(), g) != o.size()) die("cannot write output");
    std::fclose(g);
    std::printf(
        "{\"windows\": %zu, \"budget\": %llu, \"peak_total\": %llu, \"worst_after_window\": %llu, "
        "\"worst_over_budget_plus_table\": %llu, \"summary_slots_start\": %llu, \"summary_slots_end\": %llu, "
        "\"created\": %zu, \"reused\": %zu, \"reused_larger\": %zu, \"collections\": %zu, \"finalized\": %zu, "
        "\"max_queue\": %zu, \"live_handles\": %zu}\n",
        windows, (unsigned long long)budget, (unsigned long long)pool.peak_total_bytes(), (unsigned long long)worst,
        (unsigned long long)worst_over, (unsigned long long)summary_slots0, (unsigned long long)summary_slots1,
        pool.created(), pool.reused(), pool.reused_larger(), pool.collections(), finalized, max_queue,
        pool.live_handles());
    finalizer_queue.clear();
    summary.reset();
  } catch (const std::exception& x) {
    die(x.what());
  }
  return 0;
}
