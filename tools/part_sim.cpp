// part_sim.cpp -- CPU model of the owner-partitioned combine (DESIGN.md section 5,
// "Partitioned forest"): N ranks each fold their contiguous shard of the RMAT stream
// into a LOCAL forest (min-key hooking), and at every window end
//   * each rank exports (v, root) for the vertices new to it, to v's owner, and
//     (a, root) for every exported root a that was hooked away in the window;
//   * each owner keeps one anchor per owned vertex: old = atomicMin(anchor[v], l),
//     and a pair (old, l) when old != l;
//   * the pairs (deduplicated per window) fold into a label forest G.
// The final label of v is G.find(anchor[v]). Counts every term of the per-rank cost
// and, with --check, compares every label with a single global union-find.
//
// build: g++ -O2 -std=c++17 -pthread tools/part_sim.cpp -o tools/bin/part_sim
// run:   tools/bin/part_sim <scale> <log2 edges> <ranks> <log2 window per rank> [--check]
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <unordered_set>
#include <vector>

static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static const uint32_t TA = 37356, TB = 12452, TC = 12452;
static void rmat_raw(uint64_t seed, int scale, uint64_t i, uint32_t* s, uint32_t* d) {
  uint64_t base = mix64(seed), src = 0, dst = 0, r = 0;
  for (int l = 0; l < scale; ++l) {
    if ((l & 3) == 0) r = mix64(base ^ (i * 8 + (uint64_t)(l >> 2)));
    uint32_t u = (uint32_t)(r >> (16 * (l & 3))) & 0xFFFFu;
    uint64_t sb = u >= TA + TB;
    uint64_t db = (u >= TA && u < TA + TB) || (u >= TA + TB + TC);
    src = (src << 1) | sb;
    dst = (dst << 1) | db;
  }
  *s = (uint32_t)src;
  *d = (uint32_t)dst;
}

static std::vector<int64_t> g_key;  // raw id -> scrambled signed key (the order of labels)

struct UF {  // min-key union-find over raw ids; parent -1 = absent
  std::vector<int32_t> p;
  explicit UF(size_t n) : p(n, -1) {}
  bool has(uint32_t v) const { return p[v] >= 0; }
  uint32_t find(uint32_t v) {
    while ((uint32_t)p[v] != v) {
      p[v] = p[p[v]];
      v = p[v];
    }
    return v;
  }
  // returns the root hooked away (or -1)
  int64_t unite(uint32_t a, uint32_t b) {
    a = find(a);
    b = find(b);
    if (a == b) return -1;
    if (g_key[a] < g_key[b]) std::swap(a, b);  // a: larger key -> under b
    p[a] = (int32_t)b;
    return a;
  }
};

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: part_sim scale log2_edges ranks log2_window [--check]\n");
    return 2;
  }
  const int scale = atoi(argv[1]);
  const uint64_t E = 1ull << atoi(argv[2]);
  const int N = atoi(argv[3]);
  const uint64_t W = 1ull << atoi(argv[4]);
  const bool check = argc > 5 && !strcmp(argv[5], "--check");
  const uint64_t seed = scale == 20 ? 0x5EED0020ull : 0x5EED0026ull;
  const size_t V = 1ull << scale;
  g_key.resize(V);
  for (size_t v = 0; v < V; ++v) g_key[v] = (int64_t)mix64(v ^ mix64(seed ^ 0x5CA3B1E5D00DFEEDULL));
  auto owner = [&](uint32_t v) { return (int)(mix64((uint64_t)g_key[v] ^ 0x0123456789ABCDEFull) % (uint64_t)N); };

  const uint64_t per = E / N;
  std::vector<UF> loc;
  loc.reserve(N);
  for (int r = 0; r < N; ++r) loc.emplace_back(V);
  std::vector<std::vector<uint8_t>> exported(N, std::vector<uint8_t>(V, 0));
  std::vector<std::vector<uint32_t>> fresh(N), hooked(N);
  std::vector<int32_t> anchor(V, -1);
  UF G(V);
  uint64_t n_export = 0, n_hookpairs = 0, n_rows = 0, n_rawpairs = 0, n_uniqpairs = 0, n_windows = 0,
           n_records = 0;
  std::vector<uint64_t> rows_per_owner(N, 0);
  for (uint64_t w0 = 0; w0 < per; w0 += W) {
    const uint64_t w1 = std::min(per, w0 + W);
    std::vector<std::thread> th;
    for (int r = 0; r < N; ++r)
      th.emplace_back([&, r] {
        UF& u = loc[r];
        fresh[r].clear();
        hooked[r].clear();
        for (uint64_t i = w0; i < w1; ++i) {
          uint32_t s, d;
          rmat_raw(seed, scale, (uint64_t)r * per + i, &s, &d);
          for (uint32_t x : {s, d})
            if (!u.has(x)) {
              u.p[x] = (int32_t)x;
              fresh[r].push_back(x);
            }
          const int64_t a = u.unite(s, d);
          if (a >= 0) hooked[r].push_back((uint32_t)a);
        }
      });
    for (auto& t : th) t.join();
    // combine
    std::vector<std::pair<uint32_t, uint32_t>> rows;  // (v, label) to owners
    std::vector<std::pair<uint32_t, uint32_t>> pairs;
    for (int r = 0; r < N; ++r) {
      UF& u = loc[r];
      n_records += hooked[r].size();
      for (uint32_t a : hooked[r])
        if (exported[r][a]) {
          const uint32_t R = u.find(a);
          pairs.push_back({a, R});
          exported[r][R] = 1;
          n_hookpairs++;
        }
      for (uint32_t v : fresh[r]) {
        const uint32_t R = u.find(v);
        exported[r][R] = 1;
        rows.push_back({v, R});
        rows_per_owner[owner(v)]++;
        n_export++;
      }
    }
    n_rows += rows.size();
    for (auto& [v, l] : rows) {
      const int32_t old = anchor[v];
      if (old < 0) {
        anchor[v] = (int32_t)l;
      } else if ((uint32_t)old != l) {
        pairs.push_back({(uint32_t)old, l});
        n_rawpairs++;
        if (g_key[l] < g_key[old]) anchor[v] = (int32_t)l;
      }
    }
    std::unordered_set<uint64_t> uq;
    for (auto& [a, b] : pairs) {
      const uint64_t k = a < b ? ((uint64_t)a << 32 | b) : ((uint64_t)b << 32 | a);
      if (!uq.insert(k).second) continue;
      for (uint32_t x : {a, b})
        if (!G.has(x)) G.p[x] = (int32_t)x;
      G.unite(a, b);
    }
    n_uniqpairs += uq.size();
    n_windows++;
  }
  uint64_t Vt = 0, sumVr = 0, Gn = 0;
  std::vector<uint64_t> Vr(N, 0);
  for (size_t v = 0; v < V; ++v) {
    Vt += anchor[v] >= 0;
    Gn += G.has(v);
    for (int r = 0; r < N; ++r) Vr[r] += loc[r].has(v);
  }
  for (int r = 0; r < N; ++r) sumVr += Vr[r];
  printf("scale %d E 2^%d ranks %d window 2^%d per rank (%llu windows)\n", scale, atoi(argv[2]), N, atoi(argv[4]),
         (unsigned long long)n_windows);
  printf("V %llu  sum V_r %llu (%.3f V)  max V_r %llu (%.3f V)\n", (unsigned long long)Vt, (unsigned long long)sumVr,
         (double)sumVr / Vt, (unsigned long long)*std::max_element(Vr.begin(), Vr.end()),
         (double)*std::max_element(Vr.begin(), Vr.end()) / Vt);
  printf("local hook records (all ranks) %llu (%.3f V)\n", (unsigned long long)n_records, (double)n_records / Vt);
  printf("new-vertex exports (all ranks) %llu (%.3f V); rows per owner max %llu (%.3f V)\n",
         (unsigned long long)n_export, (double)n_export / Vt,
         (unsigned long long)*std::max_element(rows_per_owner.begin(), rows_per_owner.end()),
         (double)*std::max_element(rows_per_owner.begin(), rows_per_owner.end()) / Vt);
  printf("hook pairs (exported roots hooked away) %llu (%.4f V)\n", (unsigned long long)n_hookpairs,
         (double)n_hookpairs / Vt);
  printf("owner pairs raw %llu (%.4f V); unique pairs per window, summed %llu (%.4f V); G nodes %llu (%.4f V)\n",
         (unsigned long long)n_rawpairs, (double)n_rawpairs / Vt, (unsigned long long)n_uniqpairs,
         (double)n_uniqpairs / Vt, (unsigned long long)Gn, (double)Gn / Vt);
  if (check) {
    UF all(V);
    for (uint64_t i = 0; i < per * N; ++i) {
      uint32_t s, d;
      rmat_raw(seed, scale, i, &s, &d);
      for (uint32_t x : {s, d})
        if (!all.has(x)) all.p[x] = (int32_t)x;
      all.unite(s, d);
    }
    uint64_t bad = 0;
    for (size_t v = 0; v < V; ++v) {
      if (!all.has(v)) {
        bad += anchor[v] >= 0;
        continue;
      }
      const uint32_t want = all.find(v);
      const uint32_t a = (uint32_t)anchor[v];
      const uint32_t got = G.has(a) ? G.find(a) : a;
      bad += got != want;
    }
    printf("check: %llu labels differ from the global union-find\n", (unsigned long long)bad);
    return bad != 0;
  }
  return 0;
}
