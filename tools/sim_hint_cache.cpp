// sim_hint_cache.cpp -- host simulation: hit rate of a per-XCD direct-mapped
// (key -> slot, link) hint cache under the RMAT-26 endpoint stream, for sizing the
// k_fold L2 hint cache. XCD 0 sees every 8th 256-edge block (round-robin dispatch).
// Build: g++ -O2 tools/sim_hint_cache.cpp -Loracle -lgs_oracle -Wl,-rpath,$PWD/oracle -o /tmp/sim
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

extern "C" void or_rmat_edges(uint64_t seed, int scale, uint64_t start, uint64_t count, int scramble, int64_t* src,
                              int64_t* dst);

static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

struct Cache {
  int log2, policy;  // 0 always replace, 1 fill empty only, 2 replace w.p. 1/4, 3 replace w.p. 1/16
  std::vector<int64_t> k;
  uint64_t hit = 0, acc = 0, hit_ss = 0, acc_ss = 0;
  Cache(int l, int p) : log2(l), policy(p), k(1ull << l, INT64_MIN) {}
  void access(int64_t key, bool ss, uint64_t t) {
    const uint64_t h = ((uint64_t)key * 0xD6E8FEB86659FD93ull) >> (64 - log2);
    const bool ht = k[h] == key;
    hit += ht;
    ++acc;
    if (ss) {
      hit_ss += ht;
      ++acc_ss;
    }
    if (ht) return;
    bool rep = false;
    if (policy == 0) rep = true;
    if (policy == 1) rep = k[h] == INT64_MIN;
    if (policy == 2) rep = k[h] == INT64_MIN || (mix64(t) & 3) == 0;
    if (policy == 3) rep = k[h] == INT64_MIN || (mix64(t) & 15) == 0;
    if (rep) k[h] = key;
  }
};

int main(int argc, char** argv) {
  const int scale = 26;
  const uint64_t E = (1ull << scale) * 16;
  const int xcds = argc > 1 ? atoi(argv[1]) : 8;
  std::vector<Cache> cs;
  for (int l : {15, 16, 17, 18, 19})
    for (int p : {0, 1, 2, 3}) cs.emplace_back(l, p);
  const uint64_t chunk = 1ull << 20;
  std::vector<int64_t> s(chunk), d(chunk);
  uint64_t t = 0;
  for (uint64_t b = 0; b < E / chunk; ++b) {
    or_rmat_edges(0x5EED0026, scale, b * chunk, chunk, 1, s.data(), d.data());
    const bool ss = b >= 64;
    for (uint64_t blk = 0; blk < chunk / 256; blk += xcds)
      for (uint64_t i = blk * 256; i < blk * 256 + 256; ++i) {
        ++t;
        for (auto& c : cs) {
          c.access(s[i], ss, 2 * t);
          c.access(d[i], ss, 2 * t + 1);
        }
      }
    if ((b & 127) == 127) fprintf(stderr, "batch %llu\n", (unsigned long long)b);
  }
  for (auto& c : cs)
    printf("log2=%d (%5.1f MiB) policy=%d: hit %.3f overall, %.3f steady (batches >= 64)\n", c.log2,
           (16.0 * (1ull << c.log2)) / 1048576.0, c.policy, (double)c.hit / c.acc, (double)c.hit_ss / c.acc_ss);
  return 0;
}
