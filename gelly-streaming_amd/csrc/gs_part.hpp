// gs_part.hpp -- owner-partitioned combine of a gs_group (include/gs_group.h,
// gs_group_create_partitioned): the device layout of the owner
// table and the launchers of gs_part_k.hip.
//
// Each rank folds its own edges into a LOCAL forest (its summary's table; min-key roots
// are the local labels). At every combine:
//   export  -- every vertex new to the local forest since the previous combine becomes a
//              row (v, local root, parity) bucketed by owner(v); each root handed out this
//              way is marked kAuxExported;
//   records -- every marked root that was hooked away since the previous combine becomes
//              a label pair (a, its root now, parity): its label changed;
//   owner   -- after the all-to-all, the owner of v keeps ONE anchor label per vertex (the
//              first row's) and turns every other row (v, l) into a label pair (anchor, l);
//   label forest G -- every rank folds every rank's label pairs: a replica of only the
//              labels that need a cross-rank union.
// The canonical label of v is G's label of anchor(v) (parity composed).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_device.hpp"

namespace gs {

constexpr uint32_t kAuxExported = 8u;  // local table aux bit: a root handed out as a label
constexpr int kPartMaxRanks = 64;
constexpr uint32_t kPartRowsPB = 2048;  // export / scatter rows per block (256 threads x 8)

// owner table slot (32 B: one probe is one request): key, the vertex's anchor label, the
// anchor word (kAnc* bits)
struct alignas(32) OwnerSlot {
  int64_t key;
  int64_t anchor;
  uint32_t aw;
  uint32_t pad0;
  int64_t pad1;
};
constexpr uint32_t kAncPublished = 2u;  // anchor written (the row whose key CAS inserted v sets it)
constexpr uint32_t kAncParity = 4u;     // parity of the vertex relative to its anchor
constexpr uint32_t kAncPresent = 8u;    // reserved slot only: INT64_MIN is an owned vertex

struct OwnerTable {
  OwnerSlot* tab;
  uint32_t cap, mask;
  int shift;
  uint32_t r0;        // reserved slot of INT64_MIN (== cap)
  uint32_t* err;      // device flag: probe limit hit (the table is too small)
};

// Label pairs already emitted in this combine (exact): open addressing on a 64-bit fingerprint
// of (a, b, w); the inserting row writes the pair, then marks the slot ready; a row that meets
// its fingerprint compares the pair itself once the slot is ready. The giant component's pairs
// (its local roots, a few per rank) recur in every block of the owner step: without the set
// they reached the label forest ~460 K times per rank and pass at RMAT-26, N = 8.
struct alignas(32) PairSlot {
  unsigned long long fp;  // 0: empty
  int64_t a, b;
  uint32_t state;         // bit 0 ready, bit 1 parity w
  uint32_t pad;
};
struct PairSet {
  PairSlot* tab;  // nullptr: no set (every pair is emitted)
  uint32_t mask;
};

// owner rank of a vertex id: the same function on every rank
__host__ __device__ __forceinline__ int part_owner(int64_t v, int nranks) {
  unsigned long long z = (unsigned long long)v ^ 0x5851F42D4C957F2Dull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (int)((z >> 32) % (unsigned long long)nranks);
}

void launch_part_init(OwnerSlot* tab, uint64_t nslots, hipStream_t st);
// new vertices of the local forest since the previous combine: snap[s] = the shard counts
// now; out[0] = new vertices (sum of snap - mark, or of snap with full), out[1] = records
// of delta set `dset`, out[2] = vertex-list overflow flag
void launch_part_snap(const Table& t, const uint32_t* mark, uint32_t* snap, int full, uint32_t dctr,
                      uint32_t shard_cap, unsigned long long* out, hipStream_t st);
void launch_part_export(bool sign, const Table& t, const uint32_t* mark, const uint32_t* snap, int full,
                        uint64_t total, int64_t* stage, int width, uint32_t* bcnt, int nranks, hipStream_t st);
void launch_part_records(bool sign, const Table& t, const Delta& D, int64_t* pairs, int width,
                         unsigned long long* npairs, uint64_t pair_cap, hipStream_t st);
// per-owner exclusive offsets of the export blocks (bcnt[o * nblocks + b], in place) and the
// per-owner row counts (send_counts[o], u64)
void launch_part_scan(uint32_t* bcnt, uint32_t nblocks, int nranks, unsigned long long* send_counts, hipStream_t st);
void launch_part_scatter(const int64_t* stage, uint64_t total, int width, const uint32_t* bcnt, uint32_t nblocks,
                         const unsigned long long* send_counts, int nranks, int64_t* sendbuf, hipStream_t st);
void launch_part_owner(bool sign, const OwnerTable& ot, const PairSet& ps, const int64_t* rows, uint64_t nrows,
                       int width, int64_t* pairs, unsigned long long* npairs, uint64_t pair_cap, uint32_t* fail,
                       hipStream_t st);
// the pair count word: npairs | kFailBit when the local summary, the owner step or the
// previous combines failed (signed)
void launch_part_count_word(const unsigned long long* npairs, const uint32_t* local_fail, const uint32_t* part_fail,
                            unsigned long long* word, hipStream_t st);
// owned vertices -> (v, label, parity): anchor's label in the label forest G
void launch_part_labels(const OwnerTable& ot, const Table& G, int64_t* ov, int64_t* ol, uint8_t* op, uint64_t cap_out,
                        unsigned long long* count, hipStream_t st);

}  // namespace gs
