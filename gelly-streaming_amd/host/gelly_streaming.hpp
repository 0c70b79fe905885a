// gelly_streaming.hpp -- C++ host mirror of gelly-streaming's summary-aggregation API,
// backed by the MI355X C ABI (include/gs_summary.h).
//
// The reference is Java 8 / Flink 1.8 (pom.xml:15-17) and no JVM exists in this
// image, so the host side above the C ABI is C++ with the reference's names,
// argument meanings and error behaviour (exceptions where Java throws):
//
//   EdgesFold<K,EV,T>           EdgesFold.java:33-47
//   SummaryAggregation          SummaryAggregation.java:36-136 (fold/combine/transform/
//                               initial value/transient contract + Merger)
//   SummaryBulkAggregation      SummaryBulkAggregation.java:44-131 (run(): partition tag ->
//                               keyed window fold -> all-window reduce -> Merger)
//   SimpleEdgeStream::aggregate SimpleEdgeStream.java:100-102
//   DisjointSet                 summaries/DisjointSet.java:25-151  (GPU-resident forest)
//   Candidates                  summaries/Candidates.java:27-196   (GPU-resident signed forest)
//   ConnectedComponents         library/ConnectedComponents.java:41-134
//   BipartitenessCheck          library/BipartitenessCheck.java:37-133
//
// Summaries are held by std::shared_ptr (Java object references). A GPU-backed
// summary buffers its per-edge callbacks (union / merge of a one-edge candidate)
// and flushes them to the device as one micro-batch on any read, combine or
// serialization -- the drop-in design of INTEGRATION.md.
#pragma once

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <set>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "gs_summary.h"

namespace gelly {

struct NullValue {};

class GsException : public std::runtime_error {
 public:
  GsException(int code, const std::string& what) : std::runtime_error(what), code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

inline void gs_check(int rc) {
  if (rc != GS_OK) throw GsException(rc, std::string("gs: ") + gs_last_error());
}

// Edge<K, EV> is a Tuple3 (f0 = source, f1 = target, f2 = value).
template <typename K, typename EV>
struct Edge {
  K f0;
  K f1;
  EV f2;
  K getSource() const { return f0; }
  K getTarget() const { return f1; }
  EV getValue() const { return f2; }
};

// EdgesFold.java:47 -- T foldEdges(T accum, K vertexID, K neighborID, EV edgeValue)
template <typename K, typename EV, typename T>
struct EdgesFold {
  virtual ~EdgesFold() = default;
  virtual T foldEdges(T accum, K vertexID, K neighborID, EV edgeValue) = 0;
};

// Flink ReduceFunction<S> / MapFunction<S, T>
template <typename S>
struct ReduceFunction {
  virtual ~ReduceFunction() = default;
  virtual S reduce(S value1, S value2) = 0;
};
template <typename S, typename T>
struct MapFunction {
  virtual ~MapFunction() = default;
  virtual T map(S value) = 0;
};

// --------------------------------------------------------------------------
// Handle pool. Flink copies the summary's initial value for every (partition,
// window) fold (SummaryBulkAggregation.java:80, FoldingState) and drops the partial
// after the all-window reduce; creating a GPU summary each time would cost a table
// allocation and initialisation per window. Released handles are reset (O(touched
// vertices) on the device, asynchronous) and handed to the next summary of the same
// kind and device: one whose table size class fits (up to kClassSlack classes larger),
// else any larger pooled one -- reusing HBM that is already held costs nothing against
// the budget, a create does (the per-window copy of the EMPTY initial value
// asks for the smallest class, and grown pooled tables must still serve it).
//
// HBM budget (the Java HandlePool's model). The budget is
// checked against the library's own count of the device memory every live summary holds
// (gs_hbm_bytes: tables, vertex lists, staging, scratch), so a table that grew inside a
// fold or combine while handed out -- the Merger's running summary -- counts at once, not
// at its release. A create of gs_create_bytes(hint) that would pass the budget first runs
// set_budget's `collect` hook (System.gc() + System.runFinalization(): summaries a Flink
// job dropped without release() come back through their finalizers), then destroys pooled
// handles until it fits. Tables also grow in place (a reused pooled table inside the window's
// fold), so any acquire that finds the device past the budget collects first, too, and trims
// the pool back to it. The total then stays within the budget plus the table being created,
// unless live summaries alone need more.
// --------------------------------------------------------------------------
class HandlePool {
 public:
  static constexpr int kClassSlack = 2;
  static constexpr size_t kMaxFree = 64;
  static HandlePool& instance() {
    static HandlePool p;
    return p;
  }
  // gs_create's table for a capacity hint: 4 slots per expected vertex, a power of two, >= 1024
  static uint64_t slots_for(uint64_t hint) {
    const uint64_t want = std::max<uint64_t>(4 * std::max<uint64_t>(hint, 1), 1024);
    uint64_t s = 1;
    while (s < want) s <<= 1;
    return s;
  }
  static int size_class(uint64_t slots) {
    int c = 0;
    while ((2ull << c) <= slots) ++c;
    return c;
  }
  // the library's count of device memory held by live summaries on `device`
  static uint64_t device_bytes(int device) {
    uint64_t b = 0;
    gs_check(gs_hbm_bytes(device, &b));
    return b;
  }
  // budget of the device's summary HBM (0: none) and the finalization hook it runs
  void set_budget(uint64_t bytes, std::function<void()> collect) {
    budget_ = bytes;
    collect_ = std::move(collect);
  }
  gs_handle acquire(int kind, int device, uint64_t capacity_hint) {
    const int cls = size_class(slots_for(capacity_hint));
    // tables grow in place inside folds and combines, pooled or handed out: a device already
    // past the budget finalizes the dropped summaries first even when a pooled handle would
    // serve this request, takes any larger pooled table, and gives up pooled ones beyond it
    const bool over = budget_ && device_bytes(device) > budget_;
    if (over) collect();
    if (gs_handle h = take(kind, device, cls, over)) {
      if (over) evict_for(device, 0);
      return h;
    }
    uint64_t need = 0;
    gs_check(gs_create_bytes(kind, capacity_hint, &need));
    if (budget_ && device_bytes(device) + need > budget_) {
      if (!over) {
        collect();  // the dropped summaries' destructors release into this pool
        if (gs_handle h = take(kind, device, cls, true)) return h;
      }
      evict_for(device, need);  // still over: pooled handles (largest first) make room
    }
    gs_handle h = nullptr;
    gs_check(gs_create(&h, device, kind, capacity_hint));
    ++created_;
    live_.insert(h);
    note(device);
    return h;
  }
  void release(gs_handle h, int kind, int device) {
    uint64_t slots = 0;
    // the value AND the configuration (tracking, pipelining, profiling) of a fresh handle;
    // a table keeps a grown capacity across resets: pool it by its real size
    if (gs_reset_config(h) != GS_OK || gs_table_capacity(h, &slots) != GS_OK) {  // a broken handle is not pooled
      live_.erase(h);
      gs_destroy(h);
      return;
    }
    note(device);
    if (nfree_ < kMaxFree) {
      free_[{kind, device, size_class(slots)}].push_back(h);
      ++nfree_;
    } else {
      live_.erase(h);
      gs_destroy(h);
    }
  }
  size_t created() const { return created_; }
  size_t reused() const { return reused_; }
  size_t reused_larger() const { return reused_larger_; }
  size_t collections() const { return collections_; }
  uint64_t peak_total_bytes() const { return peak_total_; }  // gs_hbm_bytes seen at acquires / releases
  size_t live_handles() const { return live_.size(); }       // handed out + pooled
  ~HandlePool() {
    for (auto& kv : free_)
      for (gs_handle h : kv.second) gs_destroy(h);
  }

 private:
  // a pooled handle of class cls .. cls + kClassSlack, or (any_larger) of any larger class
  gs_handle take(int kind, int device, int cls, bool any_larger) {
    for (auto it = free_.lower_bound({kind, device, cls}); it != free_.end(); ++it) {
      const auto& k = it->first;
      if (std::get<0>(k) != kind || std::get<1>(k) != device) break;
      const bool near = std::get<2>(k) <= cls + kClassSlack;
      if (!near && !any_larger) break;
      if (it->second.empty()) continue;
      gs_handle h = it->second.back();
      it->second.pop_back();
      --nfree_;
      ++reused_;
      if (!near) ++reused_larger_;
      return h;
    }
    return nullptr;
  }
  void note(int device) { peak_total_ = std::max(peak_total_, device_bytes(device)); }
  void collect() {
    if (!collect_) return;
    ++collections_;
    collect_();
  }
  // destroy pooled handles, largest first, until a create of `need` bytes fits the budget
  void evict_for(int device, uint64_t need) {
    for (auto it = free_.rbegin(); it != free_.rend() && device_bytes(device) + need > budget_; ++it)
      while (!it->second.empty() && device_bytes(device) + need > budget_) {
        gs_handle f = it->second.back();
        it->second.pop_back();
        --nfree_;
        live_.erase(f);
        gs_destroy(f);
      }
  }
  std::map<std::tuple<int, int, int>, std::vector<gs_handle>> free_;
  std::set<gs_handle> live_;
  size_t nfree_ = 0, created_ = 0, reused_ = 0, reused_larger_ = 0, collections_ = 0;
  uint64_t budget_ = 0, peak_total_ = 0;
  std::function<void()> collect_;
};

// --------------------------------------------------------------------------
// GPU-resident summaries
// --------------------------------------------------------------------------
//
// The handle is taken from the pool at first use, not at construction: a summary built
// where no GPU work happens (the Flink job client builds the operator's initial value,
// ConnectedComponents.java:52-54, then ships it to the TaskManagers by Java
// serialization) holds no device state. writeObject / readObject model that Java
// serialization (GpuDisjointSet / GpuCandidates writeObject + readObject): a summary that
// was never used travels as a one-byte marker, any other as its gs_serialize image, which
// the copy applies on its own first use (SummaryAggregation.Merger's initialVal and
// summary fields, SummaryAggregation.java:95-103).
class GpuSummary {
 public:
  GpuSummary(int kind, int device, uint64_t capacity_hint, size_t flush_edges)
      : kind_(kind), device_(device), hint_(capacity_hint), flush_edges_(flush_edges) {}
  virtual ~GpuSummary() { release(); }
  GpuSummary(const GpuSummary&) = delete;
  GpuSummary& operator=(const GpuSummary&) = delete;

  // push one buffered edge (flushes a full micro-batch); the buffers are sized for
  // a whole micro-batch on first use, so the per-edge path is two stores and a compare
  void push(int64_t u, int64_t v) {
    if (!src_) {
      src_.reset(new int64_t[flush_edges_]);
      dst_.reset(new int64_t[flush_edges_]);
    }
    src_[n_] = u;
    dst_[n_] = v;
    if (++n_ == flush_edges_) flush();
  }
  void flush() {
    if (n_ == 0) return;
    gs_handle h = ensure();
    const auto t0 = std::chrono::steady_clock::now();
    gs_check(gs_fold(h, src_.get(), dst_.get(), n_));
    flush_seconds() += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    n_ = 0;
  }
  // the device handle, taken at first use; a pending image (readObject) or an initial
  // failed verdict (Candidates(false)) is applied to it then
  gs_handle ensure() {
    if (h_) return h_;
    // the table for the size asked for (size_for), else the pending image's vertex count
    // (its header: u32 magic, kind, ok, 0, u64 n), else the constructor's hint
    uint64_t hint = sized_ ? sized_ : hint_;
    if (!sized_ && image_.size() >= 24) {
      uint64_t n = 0;
      std::memcpy(&n, image_.data() + 16, 8);
      if (n) hint = n;
    }
    h_ = HandlePool::instance().acquire(kind_, device_, hint);
    if (!image_.empty()) {
      std::vector<uint8_t> img;
      img.swap(image_);
      gs_check(gs_deserialize(h_, img.data(), img.size()));
    } else if (failed_initially_) {
      // :194-196 fail() == new Candidates(false): the image of a failed, empty summary
      // (header only: magic 'GSS1', kind, ok = 0, n = 0)
      std::vector<uint8_t> img(24, 0);
      const uint32_t hdr[4] = {0x31535347u, (uint32_t)kind_, 0u, 0u};
      std::memcpy(img.data(), hdr, 16);
      gs_check(gs_deserialize(h_, img.data(), img.size()));
    }
    return h_;
  }
  bool acquired() const { return h_ != nullptr; }
  // size the handle taken at first use for about `vertices` vertices (GpuSummary.sizeFor: a
  // copy asks for its source's count); no effect once a handle is held
  void size_for(uint64_t vertices) {
    if (!h_) sized_ = std::max<uint64_t>(vertices, 1);
  }
  // back to the pool (the glue's explicit release of a summary the combine dropped); the
  // object reads as a fresh initial value afterwards
  void release() {
    n_ = 0;
    sized_ = 0;
    image_.clear();
    if (h_) HandlePool::instance().release(h_, kind_, device_);
    h_ = nullptr;
  }
  // Java serialization of the summary object: [0] 1 = an image follows, [1] failed
  // initially (Candidates(false)), then the gs_serialize image
  std::vector<uint8_t> writeObject() {
    std::vector<uint8_t> out = {0, (uint8_t)(failed_initially_ ? 1 : 0)};
    if (!h_ && image_.empty() && n_ == 0) return out;  // never used: no device state to ship
    const std::vector<uint8_t> img = h_ || n_ ? serialize() : image_;
    out[0] = 1;
    out.insert(out.end(), img.begin(), img.end());
    return out;
  }
  void readObjectInto(const std::vector<uint8_t>& bytes) {  // (on a fresh object)
    if (bytes.size() < 2) throw GsException(GS_ERR_INVALID, "readObject: truncated stream");
    release();
    failed_initially_ = bytes[1] != 0;
    if (bytes[0]) image_.assign(bytes.begin() + 2, bytes.end());
  }
  // host seconds spent in gs_fold (micro-batch flushes), process-wide (dropin_bench)
  static double& flush_seconds() {
    static double s = 0;
    return s;
  }
  gs_handle handle() {
    flush();
    return ensure();
  }
  size_t size() {
    uint64_t n = 0;
    gs_check(gs_num_vertices(handle(), &n));
    return (size_t)n;
  }
  void reset() {
    n_ = 0;
    image_.clear();
    gs_check(gs_reset(ensure()));
  }
  // all (vertex, canonical label, parity) rows, sorted by vertex
  struct Row {
    int64_t v, label;
    uint8_t parity;
  };
  std::vector<Row> rows() {
    gs_handle h = handle();
    uint64_t n = 0;
    gs_check(gs_num_vertices(h, &n));
    std::vector<int64_t> v(n), l(n);
    std::vector<uint8_t> s(n);
    size_t got = 0;
    if (kind_ == GS_KIND_SIGNED) {
      int ok = 1;
      gs_check(gs_bip_status(h, &ok));
      if (!ok) return {};
      gs_check(gs_export_colouring(h, l.data(), v.data(), s.data(), n, &got));
    } else {
      gs_check(gs_export_labels(h, v.data(), l.data(), n, &got));
    }
    std::vector<Row> r(got);
    for (size_t i = 0; i < got; ++i) r[i] = {v[i], l[i], (uint8_t)(kind_ == GS_KIND_SIGNED ? s[i] : 0)};
    std::sort(r.begin(), r.end(), [](const Row& a, const Row& b) { return a.v < b.v; });
    return r;
  }
  std::vector<uint8_t> serialize() {
    size_t len = 0;
    gs_check(gs_serialize(handle(), nullptr, 0, &len));
    std::vector<uint8_t> buf(len);
    gs_check(gs_serialize(h_, buf.data(), len, &len));
    buf.resize(len);
    return buf;
  }
  void deserialize(const std::vector<uint8_t>& buf) {
    n_ = 0;
    image_.clear();
    gs_check(gs_deserialize(ensure(), buf.data(), buf.size()));
  }
  int device() const { return device_; }

 protected:
  int kind_;
  int device_;
  uint64_t hint_;
  uint64_t sized_ = 0;  // size_for(): vertices of the first handle (0: hint_ / the image's count)
  size_t flush_edges_;
  gs_handle h_ = nullptr;
  std::unique_ptr<int64_t[]> src_, dst_;  // [flush_edges_] each, allocated on first push
  size_t n_ = 0;                          // buffered edges
  std::vector<uint8_t> image_;            // readObject: applied at first use
  bool failed_initially_ = false;         // Candidates(false), applied at first use
};

// DisjointSet<Long> (DisjointSet.java:25-151) over the GPU forest. find() returns
// the canonical representative (minimum id of the component): the reference
// returns an arbitrary member as root (:66-80); every caller only compares roots
// for equality or prints components, which the canonical choice preserves.
class DisjointSet : public GpuSummary {
 public:
  explicit DisjointSet(int device = 0, uint64_t capacity_hint = 1 << 16, size_t flush_edges = 1 << 20)
      : GpuSummary(GS_KIND_CC, device, capacity_hint, flush_edges) {}

  void makeSet(int64_t e) { push(e, e); }               // :53-56
  void union_(int64_t e1, int64_t e2) { push(e1, e2); }  // :92-118 ("union" is a C++ keyword)
  std::optional<int64_t> find(int64_t e) {               // :66-80 (null -> nullopt)
    int64_t label = 0;
    int found = 0;
    gs_check(gs_find(handle(), e, &label, &found));
    if (!found) return std::nullopt;
    return label;
  }
  void merge(DisjointSet& other) {  // :127-131
    if (&other == this) return;
    gs_check(gs_combine(handle(), other.handle()));
  }
  static std::shared_ptr<DisjointSet> readObject(const std::vector<uint8_t>& bytes, int device = 0,
                                                 uint64_t capacity_hint = 1 << 16) {
    auto d = std::make_shared<DisjointSet>(device, capacity_hint);
    d->readObjectInto(bytes);
    return d;
  }
  // getMatches() (:44-46) as (vertex, representative) pairs
  std::vector<std::pair<int64_t, int64_t>> getMatches() {
    std::vector<std::pair<int64_t, int64_t>> m;
    for (const Row& r : rows()) m.push_back({r.v, r.label});
    return m;
  }
  // toString() (:134-150): "{root=[members], ...}", components keyed by their
  // minimum id, members ascending (the reference prints HashMap order).
  std::string toString() {
    std::map<int64_t, std::vector<int64_t>> comps;
    for (const Row& r : rows()) comps[r.label].push_back(r.v);
    std::string s = "{";
    bool first = true;
    for (auto& kv : comps) {
      if (!first) s += ", ";
      first = false;
      s += std::to_string(kv.first) + "=[";
      for (size_t i = 0; i < kv.second.size(); ++i) s += (i ? ", " : "") + std::to_string(kv.second[i]);
      s += "]";
    }
    return s + "}";
  }
};

// Candidates (Candidates.java:27-196) over the GPU signed forest. A one-edge
// candidate (BipartitenessCheck.edgeToCandidate, :54-61) is a host-only value
// that merge() buffers; merging two GPU summaries runs gs_combine.
class Candidates : public GpuSummary {
 public:
  struct EdgeCandidate {  // {min(u,v): {min: +, max: -}}
    int64_t u, v;
  };
  explicit Candidates(bool success = true, int device = 0, uint64_t capacity_hint = 1 << 16,
                      size_t flush_edges = 1 << 20)
      : GpuSummary(GS_KIND_SIGNED, device, capacity_hint, flush_edges) {
    failed_initially_ = !success;  // applied when the handle is taken
  }
  static std::shared_ptr<Candidates> readObject(const std::vector<uint8_t>& bytes, int device = 0,
                                                uint64_t capacity_hint = 1 << 16) {
    auto c = std::make_shared<Candidates>(true, device, capacity_hint);
    c->readObjectInto(bytes);
    return c;
  }
  bool getSuccess() {  // :44-46
    int ok = 1;
    gs_check(gs_bip_status(handle(), &ok));
    return ok != 0;
  }
  // :77-139: merge(input) with input = one edge (the fold) ...
  Candidates& merge(const EdgeCandidate& e) {
    push(e.u, e.v);
    return *this;
  }
  // ... or another summary (the combine); the verdict is the AND.
  Candidates& merge(Candidates& input) {
    if (&input != this) gs_check(gs_combine(handle(), input.handle()));
    return *this;
  }
  // getMap() (:48-50): component (min id) -> {vertex -> sign}
  std::map<int64_t, std::map<int64_t, bool>> getMap() {
    std::map<int64_t, std::map<int64_t, bool>> m;
    for (const Row& r : rows()) m[r.label][r.v] = r.parity != 0;
    return m;
  }
  // Tuple2.toString(): "(true,{1={1=(1,true), 2=(2,false)}, ...})" / "(false,{})"
  std::string toString() {
    const bool ok = getSuccess();
    std::string s = std::string("(") + (ok ? "true" : "false") + ",{";
    if (ok) {
      bool first = true;
      for (auto& c : getMap()) {
        if (!first) s += ", ";
        first = false;
        s += std::to_string(c.first) + "={";
        bool f2 = true;
        for (auto& v : c.second) {
          if (!f2) s += ", ";
          f2 = false;
          s += std::to_string(v.first) + "=(" + std::to_string(v.first) + "," + (v.second ? "true" : "false") + ")";
        }
        s += "}";
      }
    }
    return s + "})";
  }
};

// --------------------------------------------------------------------------
// Operators
// --------------------------------------------------------------------------
// SummaryAggregation<K, EV, S, T> (SummaryAggregation.java:36-91)
template <typename K, typename EV, typename S, typename T>
class SummaryAggregation {
 public:
  using Fold = EdgesFold<K, EV, S>;
  using Combine = ReduceFunction<S>;
  using Transform = MapFunction<S, T>;
  using Factory = std::function<S()>;  // the initial value (Flink copies it per window)

  SummaryAggregation(std::shared_ptr<Fold> updateFun, std::shared_ptr<Combine> combineFun,
                     std::shared_ptr<Transform> transform, Factory initialValue, bool transientState)
      : updateFun_(std::move(updateFun)),
        combineFun_(std::move(combineFun)),
        transform_(std::move(transform)),
        initialValue_(std::move(initialValue)),
        transientState_(transientState) {}
  virtual ~SummaryAggregation() = default;

  std::shared_ptr<Combine> getCombineFun() const { return combineFun_; }
  std::shared_ptr<Fold> getUpdateFun() const { return updateFun_; }
  std::shared_ptr<Transform> getTransform() const { return transform_; }
  bool isTransientState() const { return transientState_; }
  S getInitialValue() const { return initialValue_(); }

  // Merger (SummaryAggregation.java:93-136): running combine at parallelism 1.
  class Merger {
   public:
    Merger(Factory initialVal, std::shared_ptr<Combine> combiner, bool transientState)
        : initialVal_(std::move(initialVal)), combiner_(std::move(combiner)), transientState_(transientState) {
      summary_ = initialVal_();
    }
    // flatMap (:107-119): summary = combine.reduce(s, summary); emit; reset if transient
    S flatMap(S s) {
      if (!combiner_) return s;
      summary_ = combiner_->reduce(s, summary_);
      S out = summary_;
      if (transientState_) summary_ = initialVal_();
      return out;
    }
    // snapshotState / restoreState (:127-135) through the summary's serializer
    S snapshotState() { return summary_; }
    void restoreState(S s) { summary_ = std::move(s); }

   private:
    Factory initialVal_;
    std::shared_ptr<Combine> combiner_;
    bool transientState_;
    S summary_;
  };

 protected:
  std::shared_ptr<Fold> updateFun_;
  std::shared_ptr<Combine> combineFun_;
  std::shared_ptr<Transform> transform_;
  Factory initialValue_;
  bool transientState_;
};

// A bounded, timestamped edge stream with a source parallelism: the stand-in for
// DataStream<Edge<K, EV>> (SimpleEdgeStream.java:69-90). Edges are dealt to the p
// fold subtasks round-robin (a rebalanced parallelism-1 source).
template <typename K, typename EV>
struct EdgeStream {
  std::vector<Edge<K, EV>> edges;
  std::vector<int64_t> timestamps;  // event/ingestion time in ms (empty: all 0)
  int parallelism = 1;
};

// SummaryBulkAggregation (SummaryBulkAggregation.java:44-131)
template <typename K, typename EV, typename S, typename T>
class SummaryBulkAggregation : public SummaryAggregation<K, EV, S, T> {
  using Base = SummaryAggregation<K, EV, S, T>;

 public:
  SummaryBulkAggregation(std::shared_ptr<typename Base::Fold> updateFun,
                         std::shared_ptr<typename Base::Combine> combineFun,
                         std::shared_ptr<typename Base::Transform> transformFun, typename Base::Factory initialVal,
                         int64_t timeMillis, bool transientState)
      : Base(std::move(updateFun), std::move(combineFun), std::move(transformFun), std::move(initialVal),
             transientState),
        timeMillis_(timeMillis) {}
  SummaryBulkAggregation(std::shared_ptr<typename Base::Fold> updateFun,
                         std::shared_ptr<typename Base::Combine> combineFun, typename Base::Factory initialVal,
                         int64_t timeMillis, bool transientState)
      : SummaryBulkAggregation(std::move(updateFun), std::move(combineFun), nullptr, std::move(initialVal),
                               timeMillis, transientState) {}

  // run (:68-90): PartitionMapper -> keyBy(partition).timeWindow(t).fold(initial,
  // PartialAgg) -> timeWindowAll(t).reduce(combine) -> Merger -> (transform).
  // Every emission (one per window that holds edges) is handed to `sink` at
  // emission time (the addSink(...) of the reference tests); the running summary
  // object is reused across windows exactly like the Merger's.
  using Sink = std::function<void(const T&)>;
  void run(const EdgeStream<K, EV>& stream, const Sink& sink) {
    const size_t n = stream.edges.size();
    const int p = std::max(1, stream.parallelism);
    typename Base::Merger merger(this->initialValue_, this->combineFun_, this->transientState_);
    size_t i = 0;
    while (i < n) {
      const int64_t w = window_of(stream, i);
      size_t j = i;
      if (stream.timestamps.empty() || timeMillis_ <= 0) {
        j = n;  // one window
      } else {  // the edges with ts / timeMillis_ == w: compared against the window's
                // bounds, not divided one by one (a 64-bit division per edge was ~5 ns)
        int64_t lo, hi;
        window_bounds(w, &lo, &hi);
        const int64_t* ts = stream.timestamps.data();
        while (j < n && ts[j] >= lo && ts[j] <= hi) ++j;
      }
      std::vector<S> partial(p);  // per-(partition, window) fold state
      const auto tf = std::chrono::steady_clock::now();
      int part = (int)(i % (size_t)p);  // PartitionMapper.map (:103-105): edge k -> k mod p
      for (size_t k = i; k < j; ++k, part = (part + 1 == p) ? 0 : part + 1) {
        if (!partial[part]) partial[part] = this->getInitialValue();
        const Edge<K, EV>& e = stream.edges[k];
        // the accumulator is handed over and returned (Java passes the reference):
        // moved, so no reference-count traffic per edge
        partial[part] =
            this->updateFun_->foldEdges(std::move(partial[part]), e.getSource(), e.getTarget(), e.getValue());
      }
      const auto tc = std::chrono::steady_clock::now();
      S acc{};
      for (int q = 0; q < p; ++q) {  // timeWindowAll reduce, arrival order = partition order
        if (!partial[q]) continue;
        acc = acc ? this->combineFun_->reduce(acc, partial[q]) : partial[q];
      }
      S emitted = merger.flatMap(acc);
      sink(emit(emitted));
      run_seconds()[0] += std::chrono::duration<double>(tc - tf).count();
      run_seconds()[1] += std::chrono::duration<double>(std::chrono::steady_clock::now() - tc).count();
      i = j;
    }
  }
  // host seconds in run(): [0] per-edge folds (incl. flushes), [1] reduce + Merger + sink
  static double* run_seconds() {
    static double t[2] = {0, 0};
    return t;
  }
  // Convenience: collect the emissions (references to live summaries; read them
  // before the next window mutates the running summary, or use the sink form).
  std::vector<T> run(const EdgeStream<K, EV>& stream) {
    std::vector<T> out;
    run(stream, [&out](const T& x) { out.push_back(x); });
    return out;
  }

 private:
  int64_t window_of(const EdgeStream<K, EV>& s, size_t i) const {
    const int64_t ts = s.timestamps.empty() ? 0 : s.timestamps[i];
    return timeMillis_ > 0 ? ts / timeMillis_ : 0;
  }
  // [lo, hi]: every ts with ts / timeMillis_ == w (C++ truncating division), saturated
  void window_bounds(int64_t w, int64_t* lo, int64_t* hi) const {
    const int64_t tm = timeMillis_;
    const int64_t base = w * tm;  // |base| <= |ts| of an existing edge: no overflow
    const int64_t kMax = std::numeric_limits<int64_t>::max(), kMin = std::numeric_limits<int64_t>::min();
    if (w > 0) {
      *lo = base;
      *hi = base > kMax - (tm - 1) ? kMax : base + (tm - 1);
    } else if (w < 0) {
      *lo = base < kMin + (tm - 1) ? kMin : base - (tm - 1);
      *hi = base;
    } else {
      *lo = -(tm - 1);
      *hi = tm - 1;
    }
  }
  T emit(S s) {
    if constexpr (std::is_same<S, T>::value) {
      if (!this->transform_) return s;
    }
    return this->transform_->map(s);
  }
  int64_t timeMillis_;
};

// SimpleEdgeStream.aggregate (SimpleEdgeStream.java:100-102)
template <typename K, typename EV>
class SimpleEdgeStream {
 public:
  explicit SimpleEdgeStream(EdgeStream<K, EV> edges) : edges_(std::move(edges)) {}
  template <typename S, typename T>
  void aggregate(SummaryBulkAggregation<K, EV, S, T>& summaryAggregation,
                 const typename SummaryBulkAggregation<K, EV, S, T>::Sink& sink) {
    summaryAggregation.run(edges_, sink);
  }
  template <typename S, typename T>
  std::vector<T> aggregate(SummaryBulkAggregation<K, EV, S, T>& summaryAggregation) {
    return summaryAggregation.run(edges_);
  }

 private:
  EdgeStream<K, EV> edges_;
};

// --------------------------------------------------------------------------
// Library algorithms
// --------------------------------------------------------------------------
using DisjointSetRef = std::shared_ptr<DisjointSet>;
using CandidatesRef = std::shared_ptr<Candidates>;

// ConnectedComponents<K, EV> (ConnectedComponents.java:41-134)
template <typename EV = NullValue>
class ConnectedComponents : public SummaryBulkAggregation<int64_t, EV, DisjointSetRef, DisjointSetRef> {
  using Base = SummaryBulkAggregation<int64_t, EV, DisjointSetRef, DisjointSetRef>;

 public:
  // UpdateCC.foldEdges (:83-86): ds.union(vertex, vertex2); return ds
  struct UpdateCC : EdgesFold<int64_t, EV, DisjointSetRef> {
    DisjointSetRef foldEdges(DisjointSetRef ds, int64_t vertex, int64_t vertex2, EV) override {
      ds->union_(vertex, vertex2);
      return ds;
    }
  };
  // CombineCC.reduce (:116-126): merge the smaller into the larger
  struct CombineCC : ReduceFunction<DisjointSetRef> {
    DisjointSetRef reduce(DisjointSetRef s1, DisjointSetRef s2) override {
      if (s1->size() <= s2->size()) {
        s2->merge(*s1);
        return s2;
      }
      s1->merge(*s2);
      return s1;
    }
  };
  // ConnectedComponents(long mergeWindowTime) (:52-54); device/capacity are the GPU knobs
  explicit ConnectedComponents(int64_t mergeWindowTime, int device = 0, uint64_t capacity_hint = 1 << 16)
      : Base(std::make_shared<UpdateCC>(), std::make_shared<CombineCC>(),
             [device, capacity_hint] { return std::make_shared<DisjointSet>(device, capacity_hint); },
             mergeWindowTime, false) {}
};

// BipartitenessCheck<K, EV> (BipartitenessCheck.java:37-133)
template <typename EV = NullValue>
class BipartitenessCheck : public SummaryBulkAggregation<int64_t, EV, CandidatesRef, CandidatesRef> {
  using Base = SummaryBulkAggregation<int64_t, EV, CandidatesRef, CandidatesRef>;

 public:
  // edgeToCandidate (:54-61)
  static Candidates::EdgeCandidate edgeToCandidate(int64_t v1, int64_t v2) {
    return {std::min(v1, v2), std::max(v1, v2)};
  }
  // updateFunction.foldEdges (:93-95): candidates.merge(edgeToCandidate(v1, v2))
  struct updateFunction : EdgesFold<int64_t, EV, CandidatesRef> {
    CandidatesRef foldEdges(CandidatesRef candidates, int64_t v1, int64_t v2, EV) override {
      candidates->merge(edgeToCandidate(v1, v2));
      return candidates;
    }
  };
  // combineFunction.reduce (:128-130): c1.merge(c2)
  struct combineFunction : ReduceFunction<CandidatesRef> {
    CandidatesRef reduce(CandidatesRef c1, CandidatesRef c2) override {
      c1->merge(*c2);
      return c1;
    }
  };
  explicit BipartitenessCheck(int64_t mergeWindowTime, int device = 0, uint64_t capacity_hint = 1 << 16)
      : Base(std::make_shared<updateFunction>(), std::make_shared<combineFunction>(),
             [device, capacity_hint] { return std::make_shared<Candidates>(true, device, capacity_hint); },
             mergeWindowTime, false) {}
};

}  // namespace gelly
