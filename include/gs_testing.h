/*
 * gs_testing.h -- PRIVATE test controls of libgs_summary.so. Not part of the drop-in
 * boundary (include/gs_summary.h, gs_group.h, gs_ingest.h): the product path never
 * calls these, and the library reads no environment variable. Tests (tests/test_*.py, the
 * C++ harnesses) use them to reach paths that are otherwise timing-dependent: the
 * window server's idle exit, the change emission's scan fallback, the parse
 * look-back's self-count, and a group folding its own rows back.
 *
 * Every knob is process-wide and starts at its product value; a value < 0 restores
 * the product value. Set them before the operation they affect (a server start, an
 * emission, a parse, a group create).
 */
#ifndef GS_TESTING_H
#define GS_TESTING_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum gs_testing_knob {
  /* resident window server: leave after this many microseconds without a window
   * (product: 2000) */
  GS_TESTING_SERVER_IDLE_US = 0,
  /* change emission: member-list walk limit per hooked root before the scan path
   * (product: 65536) */
  GS_TESTING_CHANGES_WALK_MAX = 1,
  /* text parse: microseconds a look-back waits for its predecessors before it counts
   * the lines before its tile itself (product: ~50000; 0 = at once) */
  GS_TESTING_PARSE_LB_TIMEOUT_US = 2,
  /* exchange group (created afterwards): also fold this rank's own rows back (1) */
  GS_TESTING_GROUP_SELF_APPLY = 3,
  /* exchange group (created afterwards): exchanges between an own fold and its data
   * half, 1..3 (product: 2) */
  GS_TESTING_GROUP_DATA_LAG = 4,
  GS_TESTING_KNOBS = 5
};

/* Set knob `knob` to `value` (< 0: the product value). Returns GS_OK or GS_ERR_INVALID. */
int gs_testing_set(int knob, int64_t value);

/* The current value of a knob (the product value when unset). */
int64_t gs_testing_get(int knob);

/* Diagnostics: the label forest of a partitioned group (gs_group_create_partitioned), as a
 * summary handle the caller may read (gs_counters, gs_debug_counters, gs_num_vertices) but
 * not destroy; *forest = NULL for a replica group. `g` is a gs_group_t. */
int gs_testing_group_forest(void* g, void** forest);

#ifdef __cplusplus
}
#endif
#endif /* GS_TESTING_H */
