// The Java-serialization path of the GPU summaries, modelled on the
// C++ host mirror: Flink ships SummaryAggregation's Merger to the TaskManagers by Java
// serialization with its `initialVal` and `summary` fields (SummaryAggregation.java:
// 95-103), and a restore after a failure reads the running summary back into a NEW
// object (snapshotState / restoreState, :127-135). The GPU summary must survive both:
//   * the job client builds the operator's initial value (ConnectedComponents.java:52-54,
//     BipartitenessCheck.java:50-52) without touching a GPU: no handle is taken, and the
//     value serialises as a "never used" marker;
//   * every window's partial starts from a copy of that shipped value (FoldingState,
//     SummaryBulkAggregation.java:79-80);
//   * the Merger combines (CombineCC.reduce :116-126 / combineFunction.reduce :128-130)
//     and the glue releases the input the combine dropped back to the handle pool;
//   * at window `ckpt` the Merger's `summary` and `initialVal` are written and read back
//     into new objects, which take handles on first use and apply the image, and the
//     stream continues through them; the restored summary first buffers three extra
//     edges (ids from 2^50) and goes through writeObject / readObject once more.
// Usage: test_java_serialization <cc|signed> <edges.bin: int64 src,dst pairs> <window edges>
//                                <ckpt window> <out.bin>
// out.bin: int64 ok, int64 n, then n rows of int64 {v, label or component, parity or sign}.
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

template <typename S>
static std::shared_ptr<S> fresh_initial();
template <>
std::shared_ptr<DisjointSet> fresh_initial<DisjointSet>() {
  return std::make_shared<DisjointSet>();
}
template <>
std::shared_ptr<Candidates> fresh_initial<Candidates>() {
  return std::make_shared<Candidates>(true);
}

static void fold_edge(DisjointSet& s, int64_t u, int64_t v) { s.union_(u, v); }  // UpdateCC.foldEdges
static void fold_edge(Candidates& s, int64_t u, int64_t v) {                     // updateFunction.foldEdges
  s.merge(BipartitenessCheck<>::edgeToCandidate(u, v));
}

// the GPU-aware combine: the reference's reduce, then the dropped input released
static std::shared_ptr<DisjointSet> combine(std::shared_ptr<DisjointSet> s1, std::shared_ptr<DisjointSet> s2) {
  if (s1->size() <= s2->size()) {  // CombineCC.reduce (ConnectedComponents.java:116-126)
    s2->merge(*s1);
    if (s1 != s2) s1->release();
    return s2;
  }
  s1->merge(*s2);
  s2->release();
  return s1;
}
static std::shared_ptr<Candidates> combine(std::shared_ptr<Candidates> c1, std::shared_ptr<Candidates> c2) {
  c1->merge(*c2);  // combineFunction.reduce (BipartitenessCheck.java:128-130)
  if (c1 != c2) c2->release();
  return c1;
}

template <typename S>
static int run(const std::vector<int64_t>& e, size_t window, size_t ckpt, const char* out_path) {
  const size_t n = e.size() / 2;
  // job client: the initial value is built and serialised with the job graph, no GPU used
  auto client_init = fresh_initial<S>();
  if (client_init->acquired()) die("the job client's initial value took a GPU handle");
  const std::vector<uint8_t> shipped = client_init->writeObject();
  if (shipped.size() != 2 || shipped[0] != 0) die("an unused initial value must serialise as a marker");
  // TaskManager: the Merger's fields as deserialised (one object: summary == initialVal)
  std::shared_ptr<S> initialVal = S::readObject(shipped);
  std::shared_ptr<S> summary = initialVal;
  if (initialVal->acquired()) die("a deserialised summary took a handle before its first use");
  size_t w = 0;
  for (size_t i = 0; i < n; i += window, ++w) {
    // the window's partial: a copy of the shipped initial value (FoldingState)
    std::shared_ptr<S> partial = S::readObject(shipped);
    const size_t j = std::min(n, i + window);
    for (size_t k = i; k < j; ++k) fold_edge(*partial, e[2 * k], e[2 * k + 1]);
    summary = combine(partial, summary);  // Merger.flatMap: summary = reduce(s, summary)
    if (w == ckpt) {
      // snapshotState + restoreState into new objects (Java serialization keeps the
      // identity of one object referenced by both fields)
      const bool same = summary == initialVal;
      const std::vector<uint8_t> img_s = summary->writeObject();
      const std::vector<uint8_t> img_i = initialVal->writeObject();
      if (img_s.size() < 2 || img_s[0] != 1) die("a used summary must serialise its image");
      summary->release();
      initialVal->release();
      summary = S::readObject(img_s);
      initialVal = same ? summary : S::readObject(img_i);
      if (summary->acquired()) die("restored summary took a handle before its first use");
      // edges buffered on a deserialised copy that has no handle yet (its image
      // still pending) must travel in its next image. Three edges outside the stream (ids
      // from 2^50; the driver adds them to the oracle's input) are folded into the restored
      // summary, which is serialised and read back once more before the stream continues.
      const int64_t X = (int64_t)1 << 50;
      fold_edge(*summary, X + 1, e[0]);
      fold_edge(*summary, X + 2, X + 1);
      if constexpr (std::is_same<S, DisjointSet>::value) fold_edge(*summary, X + 3, X + 3);
      const std::vector<uint8_t> img_b = summary->writeObject();
      summary->release();
      summary = S::readObject(img_b);
      if (same) initialVal = summary;
    }
  }
  // final emission
  std::vector<int64_t> out = {1, 0};
  for (const auto& r : summary->rows()) {
    out.push_back(r.v);
    out.push_back(r.label);
    out.push_back(r.parity);
  }
  if constexpr (std::is_same<S, Candidates>::value) out[0] = summary->getSuccess() ? 1 : 0;
  out[1] = (int64_t)((out.size() - 2) / 3);
  FILE* f = std::fopen(out_path, "wb");
  if (!f || std::fwrite(out.data(), 8, out.size(), f) != out.size()) die("cannot write output");
  std::fclose(f);
  std::printf("PASS java-serialization %s: %zu edges, %zu windows, checkpoint at window %zu, %lld rows, handles "
              "created %zu reused %zu\n",
              std::is_same<S, Candidates>::value ? "signed" : "cc", n, w, ckpt, (long long)out[1],
              HandlePool::instance().created(), HandlePool::instance().reused());
  return 0;
}

int main(int argc, char** argv) {
  if (argc != 6) die("usage: test_java_serialization <cc|signed> <edges.bin> <window> <ckpt> <out.bin>");
  FILE* f = std::fopen(argv[2], "rb");
  if (!f) die("cannot open edges");
  std::vector<int64_t> e;
  int64_t buf[4096];
  size_t got;
  while ((got = std::fread(buf, 8, 4096, f)) > 0) e.insert(e.end(), buf, buf + got);
  std::fclose(f);
  const size_t window = std::strtoull(argv[3], nullptr, 0), ckpt = std::strtoull(argv[4], nullptr, 0);
  try {
    if (std::string(argv[1]) == "cc") return run<DisjointSet>(e, window, ckpt, argv[5]);
    return run<Candidates>(e, window, ckpt, argv[5]);
  } catch (const std::exception& x) {
    die(x.what());
  }
  return 1;
}
