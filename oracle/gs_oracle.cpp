// =============================================================================
// gs_oracle.cpp -- TEST INFRASTRUCTURE ONLY (the parity checker, never shipped).
//
// CPU restatement of the gelly-streaming hot path this repo accelerates:
//   * DisjointSet            -> src/main/java/org/apache/flink/graph/streaming/summaries/DisjointSet.java
//   * ConnectedComponents    -> .../library/ConnectedComponents.java (UpdateCC, CombineCC)
//   * Candidates/SignedVertex-> .../summaries/Candidates.java, .../util/SignedVertex.java
//   * BipartitenessCheck     -> .../library/BipartitenessCheck.java (edgeToCandidate, fold, combine)
//   * SummaryBulkAggregation -> .../SummaryBulkAggregation.java:68-90 dataflow (partition -> window
//                               fold -> all-window reduce -> Merger), Merger at SummaryAggregation.java:107-119
// plus the canonicaliser (component label = min signed int64 id) and the synthetic
// stream generators (a second, independent implementation of the spec the GPU
// generator in gelly-streaming_amd/csrc/gs_gen.hip follows).
//
// Pinning: the reference is Java/Flink and cannot run in this image (no JVM; see
// DESIGN.md "Oracle"). This restatement is pinned by the reference's own test
// strings (ConnectedComponentsTest.java:41, BipartitenessCheckTest.java:40-42,63-65,
// DisjointSetTest.java:37-77), checked in tests/test_oracle.py.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
// =============================================================================
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace oracle {

// ----------------------------------------------------------------------------
// Synthetic stream spec (DESIGN.md "Workloads"). splitmix64 finaliser.
// ----------------------------------------------------------------------------
static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static const uint32_t RMAT_TA = 37356, RMAT_TB = 12452, RMAT_TC = 12452;  // (0.57,0.19,0.19,0.05) * 2^16
static inline int64_t scramble_id(uint64_t raw, uint64_t seed) {
  return (int64_t)mix64(raw ^ mix64(seed ^ 0x5CA3B1E5D00DFEEDULL));
}

void rmat_edge(uint64_t seed, int scale, uint64_t i, int scramble, int64_t* s, int64_t* d) {
  uint64_t base = mix64(seed), src = 0, dst = 0, r = 0;
  for (int l = 0; l < scale; ++l) {
    if ((l & 3) == 0) r = mix64(base ^ (i * 8 + (uint64_t)(l >> 2)));
    uint32_t u = (uint32_t)(r >> (16 * (l & 3))) & 0xFFFFu;
    uint64_t sb = u >= RMAT_TA + RMAT_TB;
    uint64_t db = (u >= RMAT_TA && u < RMAT_TA + RMAT_TB) || (u >= RMAT_TA + RMAT_TB + RMAT_TC);
    src = (src << 1) | sb;
    dst = (dst << 1) | db;
  }
  *s = scramble ? scramble_id(src, seed) : (int64_t)src;
  *d = scramble ? scramble_id(dst, seed) : (int64_t)dst;
}

void er_edge(uint64_t seed, int logn, uint64_t i, int scramble, int64_t* s, int64_t* d) {
  uint64_t base = mix64(seed);
  uint64_t a = mix64(base ^ (2 * i)) >> (64 - logn);
  uint64_t b = mix64(base ^ (2 * i + 1)) >> (64 - logn);
  *s = scramble ? scramble_id(a, seed) : (int64_t)a;
  *d = scramble ? scramble_id(b, seed) : (int64_t)b;
}

// Random bipartite stream: left vertex l -> id 2l, right vertex r -> id 2r+1.
// An injected position gets a same-side (left-left) edge instead.
void bip_edge(uint64_t seed, int logside, uint64_t i, int inject, int64_t* s, int64_t* d) {
  uint64_t base = mix64(seed);
  uint64_t a = mix64(base ^ (2 * i)) >> (64 - logside);
  uint64_t b = mix64(base ^ (2 * i + 1)) >> (64 - logside);
  *s = (int64_t)(2 * a);
  *d = inject ? (int64_t)(2 * b) : (int64_t)(2 * b + 1);
}

// ----------------------------------------------------------------------------
// DisjointSet restatement (DisjointSet.java:25-151).
// ----------------------------------------------------------------------------
struct DisjointSet {
  std::unordered_map<int64_t, int64_t> matches;  // :28
  std::unordered_map<int64_t, int> ranks;        // :29

  void makeSet(int64_t e) {  // :53-56
    matches[e] = e;
    ranks[e] = 0;
  }
  // :66-80 recursive find with path compression; false == Java null
  bool find(int64_t e, int64_t* out) {
    auto it = matches.find(e);
    if (it == matches.end()) return false;
    int64_t parent = it->second;
    if (parent != e) {
      int64_t tmp = parent;
      find(parent, &tmp);
      if (parent != tmp) {
        parent = tmp;
        matches[e] = parent;
      }
    }
    *out = parent;
    return true;
  }
  // :92-118 union by rank; tie -> root2 under root1, rank(root1)++
  void unite(int64_t e1, int64_t e2) {
    if (!matches.count(e1)) makeSet(e1);
    if (!matches.count(e2)) makeSet(e2);
    int64_t r1 = 0, r2 = 0;
    find(e1, &r1);
    find(e2, &r2);
    if (r1 == r2) return;
    int d1 = ranks[r1], d2 = ranks[r2];
    if (d1 > d2) {
      matches[r2] = r1;
    } else if (d1 < d2) {
      matches[r1] = r2;
    } else {
      matches[r2] = r1;
      ranks[r1] = d1 + 1;
    }
  }
  // :127-131 union(k, parent(k)) for every entry of other
  void merge(const DisjointSet& other) {
    if (&other == this) return;
    for (const auto& kv : other.matches) unite(kv.first, kv.second);
  }
  size_t size() const { return matches.size(); }
};

// ConnectedComponents.CombineCC.reduce (ConnectedComponents.java:116-126):
// merge the smaller into the larger, return the larger (moved into *out).
static void combine_cc(DisjointSet& s1, DisjointSet& s2, DisjointSet* out) {
  if (s1.size() <= s2.size()) {
    s2.merge(s1);
    *out = std::move(s2);
  } else {
    s1.merge(s2);
    *out = std::move(s1);
  }
}

// Canonical labels: label(v) = min signed int64 id of v's component. Sorted by v.
static void cc_canonical(DisjointSet& ds, std::vector<int64_t>* vs, std::vector<int64_t>* ls) {
  std::unordered_map<int64_t, int64_t> rootmin;
  rootmin.reserve(ds.size() * 2);
  std::vector<std::pair<int64_t, int64_t>> vr;
  vr.reserve(ds.size());
  std::vector<int64_t> keys;
  keys.reserve(ds.size());
  for (const auto& kv : ds.matches) keys.push_back(kv.first);
  for (int64_t v : keys) {
    int64_t r = 0;
    ds.find(v, &r);
    vr.push_back({v, r});
    auto it = rootmin.find(r);
    if (it == rootmin.end())
      rootmin[r] = v;
    else if (v < it->second)
      it->second = v;
  }
  std::sort(vr.begin(), vr.end());
  vs->resize(vr.size());
  ls->resize(vr.size());
  for (size_t i = 0; i < vr.size(); ++i) {
    (*vs)[i] = vr[i].first;
    (*ls)[i] = rootmin[vr[i].second];
  }
}

// Canonical DisjointSet string: HashMap<root, List<v>>.toString() shape
// ("{k=[a, b], ...}", DisjointSet.java:134-150) with components keyed by their min
// and members ascending (Java's own key order is HashMap order).
static std::string cc_canonical_string(DisjointSet& ds) {
  std::vector<int64_t> vs, ls;
  cc_canonical(ds, &vs, &ls);
  std::map<int64_t, std::vector<int64_t>> comps;
  for (size_t i = 0; i < vs.size(); ++i) comps[ls[i]].push_back(vs[i]);
  std::string s = "{";
  bool first = true;
  for (auto& kv : comps) {
    if (!first) s += ", ";
    first = false;
    s += std::to_string(kv.first) + "=[";
    for (size_t j = 0; j < kv.second.size(); ++j) {
      if (j) s += ", ";
      s += std::to_string(kv.second[j]);
    }
    s += "]";
  }
  return s + "}";
}

// ----------------------------------------------------------------------------
// Candidates restatement, quirk for quirk (Candidates.java:27-196).
// Tuple2<Boolean, TreeMap<Long, TreeMap<Long, SignedVertex>>>; SignedVertex = (v, sign).
// ----------------------------------------------------------------------------
struct Candidates {
  bool f0 = true;                                      // :31-34
  std::map<int64_t, std::map<int64_t, bool>> f1;       // TreeMap<comp, TreeMap<v, sign>>

  // :61-74
  bool add(int64_t component, int64_t v, bool sign) {
    auto& comp = f1[component];  // put(component, new TreeMap) if absent
    auto it = comp.find(v);
    if (it != comp.end() && it->second != sign) return false;
    comp[v] = sign;
    return true;
  }
  // :52-59 (stops at the first conflicting vertex; earlier ones stay added)
  bool add(int64_t component, const std::map<int64_t, bool>& vertices) {
    for (const auto& kv : vertices)
      if (!add(component, kv.first, kv.second)) return false;
    return true;
  }
  void fail() {  // :194-196 -> new Candidates(false)
    f0 = false;
    f1.clear();
  }

  // :142-192 private merge(input, candidates, inputKey, selfKey) with candidates == this
  bool merge_component(const Candidates& input, int64_t inputKey, int64_t selfKey) {
    const std::map<int64_t, bool>& inputComponent = input.f1.at(inputKey);
    const std::map<int64_t, bool>& selfComponent = f1.at(selfKey);
    std::vector<int64_t> mergeBy;  // :147-153
    for (const auto& kv : inputComponent)
      if (selfComponent.count(kv.first)) mergeBy.push_back(kv.first);
    if (mergeBy.empty()) throw std::runtime_error("IndexOutOfBounds: mergeBy.get(0)");
    bool reversed = inputComponent.at(mergeBy[0]) != selfComponent.at(mergeBy[0]);  // :156-158
    for (int64_t mv : mergeBy) {  // :161-173
      bool is = inputComponent.at(mv), ss = selfComponent.at(mv);
      bool ok = reversed ? (is != ss) : (is == ss);
      if (!ok) return false;
    }
    int64_t commonKey = std::min(inputKey, selfKey);  // :176
    // :179-189. inputComponent may alias a component of *this (the i-loop call at
    // :128); std::map nodes are stable under insertion of other keys, and
    // commonKey != inputKey there, so iterating a snapshot is equivalent.
    std::vector<std::pair<int64_t, bool>> snap(inputComponent.begin(), inputComponent.end());
    for (const auto& kv : snap) {
      bool sign = reversed ? !kv.second : kv.second;
      if (!add(commonKey, kv.first, sign)) return false;
    }
    return true;
  }

  // :77-139 public merge(input); result replaces *this (fail() => (false,{})).
  void merge(const Candidates& input_ref) {
    Candidates input_copy;
    const Candidates* inp = &input_ref;
    if (inp == this) {
      input_copy = input_ref;
      inp = &input_copy;
    }
    const Candidates& input = *inp;
    if (!input.f0 || !f0) {  // :79-81
      fail();
      return;
    }
    for (const auto& inEntry : input.f1) {  // :84
      std::vector<int64_t> mergeWith;
      for (const auto& selfEntry : f1) {  // :88
        int64_t selfKey = selfEntry.first;
        // :92-95 identical key sets are skipped
        if (inEntry.second.size() == selfEntry.second.size()) {
          bool same = true;
          auto a = inEntry.second.begin();
          auto b = selfEntry.second.begin();
          for (; a != inEntry.second.end(); ++a, ++b)
            if (a->first != b->first) {
              same = false;
              break;
            }
          if (same) continue;
        }
        for (const auto& iv : inEntry.second) {  // :98-105
          if (selfEntry.second.count(iv.first)) {
            if (std::find(mergeWith.begin(), mergeWith.end(), selfKey) == mergeWith.end()) {
              mergeWith.push_back(selfKey);
              break;
            }
          }
        }
      }
      if (mergeWith.empty()) {
        add(inEntry.first, inEntry.second);  // :111, result ignored
      } else {
        std::sort(mergeWith.begin(), mergeWith.end());  // :114
        int64_t firstKey = mergeWith[0];
        if (!merge_component(input, inEntry.first, firstKey)) {  // :118-121
          fail();
          return;
        }
        firstKey = std::min(inEntry.first, firstKey);  // :123
        for (size_t i = 1; i < mergeWith.size(); ++i) {  // :126-134
          merge_component(*this, mergeWith[i], firstKey);  // failure ignored (:129-131)
          f1.erase(mergeWith[i]);
        }
      }
    }
  }

  // Tuple2.toString of (Boolean, TreeMap<Long, TreeMap<Long, SignedVertex>>)
  std::string toString() const {
    std::string s = std::string("(") + (f0 ? "true" : "false") + ",{";
    bool first = true;
    for (const auto& c : f1) {
      if (!first) s += ", ";
      first = false;
      s += std::to_string(c.first) + "={";
      bool f2 = true;
      for (const auto& v : c.second) {
        if (!f2) s += ", ";
        f2 = false;
        s += std::to_string(v.first) + "=(" + std::to_string(v.first) + "," + (v.second ? "true" : "false") + ")";
      }
      s += "}";
    }
    return s + "})";
  }
};

// BipartitenessCheck.edgeToCandidate (BipartitenessCheck.java:54-61)
static Candidates edgeToCandidate(int64_t v1, int64_t v2) {
  int64_t src = std::min(v1, v2), trg = std::max(v1, v2);
  Candidates c;
  c.add(src, src, true);
  c.add(src, trg, false);  // result ignored: a self-loop stays {u={u=(u,true)}}
  return c;
}

// ----------------------------------------------------------------------------
// Ground truth for bipartiteness: parity union-find (independent of Candidates).
// ----------------------------------------------------------------------------
struct ParityDSU {
  std::unordered_map<int64_t, std::pair<int64_t, int>> p;  // v -> (parent, parity to parent)
  bool ok = true;
  void touch(int64_t v) {
    if (!p.count(v)) p[v] = {v, 0};
  }
  std::pair<int64_t, int> find(int64_t v) {
    int par = 0;
    int64_t x = v;
    std::vector<int64_t> path;
    while (p[x].first != x) {
      path.push_back(x);
      par ^= p[x].second;
      x = p[x].first;
    }
    // compress
    int acc = par;
    for (int64_t y : path) {
      int own = p[y].second;
      p[y] = {x, acc};
      acc ^= own;
    }
    return {x, par};
  }
  void edge(int64_t u, int64_t v) {
    touch(u);
    touch(v);
    if (u == v) return;  // self-loop: vertex added, never a failure (BipartitenessCheck.java:54-61)
    auto a = find(u), b = find(v);
    if (a.first == b.first) {
      if (a.second == b.second) ok = false;
      return;
    }
    // hook the larger root under the smaller so roots are component minima
    if (a.first < b.first)
      p[b.first] = {a.first, a.second ^ b.second ^ 1};
    else
      p[a.first] = {b.first, a.second ^ b.second ^ 1};
  }
};

}  // namespace oracle

// =============================================================================
// C ABI for ctypes (tests/oracle_binding.py). All buffers caller-owned.
// =============================================================================
using namespace oracle;

static std::string g_err;
static int put_string(const std::string& s, char* out, size_t cap, size_t* len) {
  *len = s.size();
  if (out && cap) {
    size_t n = std::min(cap - 1, s.size());
    memcpy(out, s.data(), n);
    out[n] = 0;
  }
  return s.size() + 1 <= cap ? 0 : 1;
}

extern "C" {

const char* or_last_error() { return g_err.c_str(); }

void or_rmat_edges(uint64_t seed, int scale, uint64_t start, uint64_t count, int scramble, int64_t* src,
                   int64_t* dst) {
  for (uint64_t k = 0; k < count; ++k) rmat_edge(seed, scale, start + k, scramble, src + k, dst + k);
}
void or_er_edges(uint64_t seed, int logn, uint64_t start, uint64_t count, int scramble, int64_t* src, int64_t* dst) {
  for (uint64_t k = 0; k < count; ++k) er_edge(seed, logn, start + k, scramble, src + k, dst + k);
}
// inject: sorted list of absolute stream positions that carry a same-side edge
void or_bip_edges(uint64_t seed, int logside, uint64_t start, uint64_t count, const uint64_t* inject, size_t ninject,
                  int64_t* src, int64_t* dst) {
  for (uint64_t k = 0; k < count; ++k) {
    uint64_t i = start + k;
    int inj = std::binary_search(inject, inject + ninject, i) ? 1 : 0;
    bip_edge(seed, logside, i, inj, src + k, dst + k);
  }
}
int64_t or_scramble_id(uint64_t raw, uint64_t seed) { return scramble_id(raw, seed); }

// Fold all edges into one DisjointSet (one window, p = 1) and return canonical
// labels sorted by vertex. Returns the number of vertices (call with cap=0 to size).
size_t or_cc_labels(const int64_t* src, const int64_t* dst, size_t n, int64_t* out_v, int64_t* out_l, size_t cap) {
  DisjointSet ds;
  for (size_t i = 0; i < n; ++i) ds.unite(src[i], dst[i]);
  std::vector<int64_t> vs, ls;
  cc_canonical(ds, &vs, &ls);
  for (size_t i = 0; i < vs.size() && i < cap; ++i) {
    out_v[i] = vs[i];
    out_l[i] = ls[i];
  }
  return vs.size();
}

// SummaryBulkAggregation dataflow emulation for ConnectedComponents.
// win[i] = window index of edge i (non-decreasing), part[i] = partition (subtask)
// index. For every window with edges: each partition folds its edges into a fresh
// initial value (PartialAgg.fold :121-123), the partials are reduced with CombineCC
// in ascending partition order (timeWindowAll().reduce, :81-82; arrival order is
// Flink-internal -- parity unpinned for p>1, irrelevant for CC), then
// Merger: summary = combine(s, summary) (SummaryAggregation.java:110), emit.
// Emissions are canonical strings separated by '\n'. Returns 0 or 1 (truncated).
int or_cc_dataflow(const int64_t* src, const int64_t* dst, const int64_t* win, const int32_t* part, size_t n,
                   int transient_state, char* out, size_t cap, size_t* len) {
  DisjointSet summary;  // Merger.summary = initialVal
  std::string emitted;
  size_t i = 0;
  while (i < n) {
    size_t j = i;
    int maxp = 0;
    while (j < n && win[j] == win[i]) maxp = std::max(maxp, part[j++]);
    std::vector<DisjointSet> partial(maxp + 1);
    std::vector<int> used(maxp + 1, 0);
    for (size_t k = i; k < j; ++k) {
      partial[part[k]].unite(src[k], dst[k]);  // UpdateCC.foldEdges :83-86
      used[part[k]] = 1;
    }
    DisjointSet acc;
    bool have = false;
    for (int p = 0; p <= maxp; ++p) {
      if (!used[p]) continue;
      if (!have) {
        acc = std::move(partial[p]);
        have = true;
      } else {
        DisjointSet r;
        combine_cc(acc, partial[p], &r);
        acc = std::move(r);
      }
    }
    DisjointSet r;
    combine_cc(acc, summary, &r);  // reduce(s, summary)
    summary = std::move(r);
    if (!emitted.empty()) emitted += "\n";
    emitted += cc_canonical_string(summary);
    if (transient_state) summary = DisjointSet();
    i = j;
  }
  return put_string(emitted, out, cap, len);
}

// The same dataflow for BipartitenessCheck over the quirk-exact Candidates.
int or_bip_dataflow(const int64_t* src, const int64_t* dst, const int64_t* win, const int32_t* part, size_t n,
                    int transient_state, char* out, size_t cap, size_t* len) {
  try {
    Candidates summary;  // initial value new Candidates(true) (BipartitenessCheck.java:50-52)
    std::string emitted;
    size_t i = 0;
    while (i < n) {
      size_t j = i;
      int maxp = 0;
      while (j < n && win[j] == win[i]) maxp = std::max(maxp, part[j++]);
      std::vector<Candidates> partial(maxp + 1);
      std::vector<int> used(maxp + 1, 0);
      for (size_t k = i; k < j; ++k) {
        partial[part[k]].merge(edgeToCandidate(src[k], dst[k]));  // updateFunction.foldEdges :93-95
        used[part[k]] = 1;
      }
      Candidates acc;
      bool have = false;
      for (int p = 0; p <= maxp; ++p) {
        if (!used[p]) continue;
        if (!have) {
          acc = partial[p];
          have = true;
        } else {
          acc.merge(partial[p]);  // combineFunction.reduce(c1, c2) = c1.merge(c2) :128-130
        }
      }
      acc.merge(summary);  // Merger: reduce(s, summary) = s.merge(summary)
      summary = acc;
      if (!emitted.empty()) emitted += "\n";
      emitted += summary.toString();
      if (transient_state) summary = Candidates();
      i = j;
    }
    return put_string(emitted, out, cap, len);
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// Truth: verdict + canonical colouring. out arrays sorted by (comp, v): comp = min
// vertex of the component, sign = (parity(v) == parity(comp)). Returns vertex count
// (0 arrays written when not bipartite). *ok receives the verdict.
size_t or_bip_truth(const int64_t* src, const int64_t* dst, size_t n, int* ok, int64_t* out_comp, int64_t* out_v,
                    uint8_t* out_sign, size_t cap) {
  ParityDSU d;
  for (size_t i = 0; i < n; ++i) {
    if (!d.ok) break;
    d.edge(src[i], dst[i]);
  }
  *ok = d.ok ? 1 : 0;
  if (!d.ok) return 0;
  std::vector<std::tuple<int64_t, int64_t, uint8_t>> rows;
  std::vector<int64_t> keys;
  for (auto& kv : d.p) keys.push_back(kv.first);
  for (int64_t v : keys) {
    auto r = d.find(v);
    rows.emplace_back(r.first, v, (uint8_t)(r.second == 0));
  }
  std::sort(rows.begin(), rows.end());
  for (size_t i = 0; i < rows.size() && i < cap; ++i) {
    out_comp[i] = std::get<0>(rows[i]);
    out_v[i] = std::get<1>(rows[i]);
    out_sign[i] = std::get<2>(rows[i]);
  }
  return rows.size();
}

// Position (0-based edge index) at which the truth verdict first becomes false, or -1.
int64_t or_bip_first_failure(const int64_t* src, const int64_t* dst, size_t n) {
  ParityDSU d;
  for (size_t i = 0; i < n; ++i) {
    d.edge(src[i], dst[i]);
    if (!d.ok) return (int64_t)i;
  }
  return -1;
}

// ---------------- DisjointSetTest helpers (DisjointSetTest.java:37-77) ----------------
// Runs the reference unit test body on the restatement; returns 0 when every
// assertion of the reference test holds, else the failing assertion number.
int or_disjointset_unit_test() {
  DisjointSet ds;
  for (int i = 0; i < 8; ++i) ds.unite(i, i + 2);
  if (ds.size() != 10) return 1;  // testGetMatches
  int64_t r1 = 0, r2 = 0;
  ds.find(0, &r1);
  ds.find(1, &r2);
  if (r1 == r2) return 2;  // testFind
  for (int i = 0; i < 10; ++i) {
    int64_t r = 0;
    ds.find(i, &r);
    if (r != ((i % 2) == 0 ? r1 : r2)) return 3;
  }
  DisjointSet ds2;  // testMerge
  for (int i = 0; i < 8; ++i) ds2.unite(i, i + 100);
  ds2.merge(ds);
  if (ds2.size() != 18) return 4;
  std::vector<int64_t> keys;
  for (auto& kv : ds2.matches) keys.push_back(kv.first);
  std::vector<int64_t> roots;
  for (int64_t k : keys) {
    int64_t r = 0;
    ds2.find(k, &r);
    roots.push_back(r);
  }
  std::sort(roots.begin(), roots.end());
  roots.erase(std::unique(roots.begin(), roots.end()), roots.end());
  if (roots.size() != 2) return 5;
  return 0;
}

// ---------------- CPU baseline (bench.py cpu_baseline leg) ----------------
// Single thread: Flink p=1 fold without Flink overhead (an upper bound on the
// reference's speed): every edge is DisjointSet.union on hash maps, then the
// Merger's CombineCC against the running summary once per batch-window.
// Returns wall seconds.
double or_cpu_baseline_cc(const int64_t* src, const int64_t* dst, size_t n, size_t window) {
  auto t0 = std::chrono::steady_clock::now();
  DisjointSet summary;
  for (size_t i = 0; i < n; i += window) {
    size_t j = std::min(n, i + window);
    DisjointSet part;
    for (size_t k = i; k < j; ++k) part.unite(src[k], dst[k]);
    DisjointSet r;
    combine_cc(part, summary, &r);
    summary = std::move(r);
  }
  auto t1 = std::chrono::steady_clock::now();
  volatile size_t sink = summary.size();
  (void)sink;
  return std::chrono::duration<double>(t1 - t0).count();
}

// p threads: each folds a contiguous 1/p slice of every window (PartitionMapper +
// keyed fold, SummaryBulkAggregation.java:77-80), then the partials are combined
// (CombineCC) and merged into the running summary (Merger) on the caller thread.
double or_cpu_baseline_cc_threads(const int64_t* src, const int64_t* dst, size_t n, size_t window, int p) {
  auto t0 = std::chrono::steady_clock::now();
  DisjointSet summary;
  for (size_t i = 0; i < n; i += window) {
    size_t j = std::min(n, i + window);
    std::vector<DisjointSet> parts(p);
    std::vector<std::thread> th;
    size_t len = j - i;
    for (int t = 0; t < p; ++t) {
      th.emplace_back([&, t] {
        size_t a = i + len * t / p, b = i + len * (t + 1) / p;
        for (size_t k = a; k < b; ++k) parts[t].unite(src[k], dst[k]);
      });
    }
    for (auto& x : th) x.join();
    DisjointSet acc = std::move(parts[0]);
    for (int t = 1; t < p; ++t) {
      DisjointSet r;
      combine_cc(acc, parts[t], &r);
      acc = std::move(r);
    }
    DisjointSet r;
    combine_cc(acc, summary, &r);
    summary = std::move(r);
  }
  auto t1 = std::chrono::steady_clock::now();
  volatile size_t sink = summary.size();
  (void)sink;
  return std::chrono::duration<double>(t1 - t0).count();
}

// Per-window latency of the 1-thread restatement (config 5 CPU leg): window fold +
// CombineCC into the running summary (the Merger), seconds per window into out[].
void or_cpu_window_latency_cc(const int64_t* src, const int64_t* dst, size_t n, size_t window, double* out) {
  DisjointSet summary;
  size_t w = 0;
  for (size_t i = 0; i < n; i += window, ++w) {
    auto t0 = std::chrono::steady_clock::now();
    size_t j = std::min(n, i + window);
    DisjointSet part;
    for (size_t k = i; k < j; ++k) part.unite(src[k], dst[k]);
    DisjointSet r;
    combine_cc(part, summary, &r);
    summary = std::move(r);
    out[w] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
}

// ---------------- text edge ingest (include/gs_ingest.h) ----------------
// Restatement of the reference's source map, per line of env.readTextFile:
//   String[] fields = s.split("\\s" or "\\t"); Long.parseLong(fields[0]); Long.parseLong(fields[1])
// (ConnectedComponentsExample.java:109-118, BipartitenessCheckExample.java:97-106), with
// Java 8 String.split semantics (a leading empty field is kept, trailing empty fields are
// removed, no match -> the whole line) and Long.parseLong semantics (optional sign,
// >= 1 digit, int64 range), and Flink TextInputFormat line handling ('\n' delimiter, a
// trailing '\r' dropped, no record after a final '\n').
static bool java_is_sep(char c, int sep) {
  if (sep == 1) return c == '\t';
  return c == ' ' || c == '\t' || c == '\n' || c == '\x0B' || c == '\f' || c == '\r';
}
static std::vector<std::string> java_split(const std::string& s, int sep) {
  std::vector<std::string> out;
  size_t start = 0;
  bool matched = false;
  for (size_t i = 0; i < s.size(); ++i) {
    if (java_is_sep(s[i], sep)) {
      out.push_back(s.substr(start, i - start));
      start = i + 1;
      matched = true;
    }
  }
  if (!matched) return {s};
  out.push_back(s.substr(start));
  while (!out.empty() && out.back().empty()) out.pop_back();  // limit 0: trailing empties removed
  return out;
}
static bool java_parse_long(const std::string& f, int64_t* v) {
  if (f.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (f[0] == '-' || f[0] == '+') {
    neg = f[0] == '-';
    if (f.size() == 1) return false;
    i = 1;
  }
  // magnitude in unsigned arithmetic, range-checked against 2^63 (neg) / 2^63 - 1
  const unsigned long long lim = neg ? (1ull << 63) : (1ull << 63) - 1;
  unsigned long long m = 0;
  for (; i < f.size(); ++i) {
    if (f[i] < '0' || f[i] > '9') return false;
    const unsigned d = (unsigned)(f[i] - '0');
    if (m > (lim - d) / 10) return false;
    m = m * 10 + d;
  }
  *v = neg ? (int64_t)(0ull - m) : (int64_t)m;
  return true;
}

// Test/bench input generator: "src<sep>dst\n" lines (sep 0 = ' ', 1 = '\t'); returns bytes
// written (0 if cap is too small).
size_t or_format_edges(const int64_t* src, const int64_t* dst, size_t n, int sep, char* out, size_t cap) {
  size_t w = 0;
  char tmp[48];
  for (size_t i = 0; i < n; ++i) {
    int k = snprintf(tmp, sizeof tmp, "%lld%c%lld\n", (long long)src[i], sep == 1 ? '\t' : ' ', (long long)dst[i]);
    if (w + (size_t)k > cap) return 0;
    memcpy(out + w, tmp, (size_t)k);
    w += (size_t)k;
  }
  return w;
}

int or_parse_edges(const char* text, size_t len, int sep, int64_t* src, int64_t* dst, size_t cap, uint64_t* n_lines,
                   int64_t* bad_line) {
  *n_lines = 0;
  *bad_line = -1;
  size_t pos = 0;
  uint64_t line = 0;
  while (pos < len) {
    size_t e = pos;
    while (e < len && text[e] != '\n') ++e;
    std::string s(text + pos, e - pos);
    if (!s.empty() && s.back() == '\r') s.pop_back();
    std::vector<std::string> f = java_split(s, sep);
    int64_t a = 0, b = 0;
    const bool ok = f.size() >= 2 && java_parse_long(f[0], &a) && java_parse_long(f[1], &b);
    if (!ok && *bad_line < 0) *bad_line = (int64_t)line;
    if (ok && line < cap) {
      src[line] = a;
      dst[line] = b;
    }
    ++line;
    pos = e + 1;  // past the '\n' (a final '\n' yields no further record)
  }
  *n_lines = line;
  return *bad_line >= 0 ? -5 : 0;
}

// Quirk-exact Candidates fold of a prefix, one window, p = 1; returns wall seconds.
double or_cpu_baseline_bip(const int64_t* src, const int64_t* dst, size_t n) {
  auto t0 = std::chrono::steady_clock::now();
  Candidates c;
  for (size_t k = 0; k < n; ++k) c.merge(edgeToCandidate(src[k], dst[k]));
  auto t1 = std::chrono::steady_clock::now();
  volatile size_t sink = c.f1.size();
  (void)sink;
  return std::chrono::duration<double>(t1 - t0).count();
}

}  // extern "C"
