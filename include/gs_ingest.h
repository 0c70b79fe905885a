/*
 * gs_ingest.h -- text edge-file ingest on the GPU.
 *
 * Replaces the reference's per-record source map
 *     String[] fields = s.split("\\s");          (or "\\t")
 *     long src = Long.parseLong(fields[0]);
 *     long trg = Long.parseLong(fields[1]);
 * of ConnectedComponentsExample.java:109-118 (whitespace; also SpannerExample,
 * DegreeDistribution, WindowTriangles) and BipartitenessCheckExample.java:97-106
 * (tab), applied to the lines of env.readTextFile: '\n'-delimited, a trailing
 * '\r' dropped, no record after a final '\n'.
 *
 * A line is MALFORMED exactly when that map would throw: fewer than two fields,
 * an empty field 0 or 1 (leading or doubled separator), a field that is not an
 * optionally signed run of decimal digits, or a value outside the int64 range.
 * Fields after the second are ignored (as the reference ignores fields[2..]).
 * Deviation: Java's Long.parseLong also accepts non-ASCII Unicode decimal digits;
 * the byte parser accepts ASCII '0'-'9' only.
 */
#ifndef GS_INGEST_H
#define GS_INGEST_H

#include <stddef.h>
#include <stdint.h>

#include "gs_summary.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
  GS_SEP_WHITESPACE = 0, /* split("\\s"): any of ' ' '\t' '\n' '\x0B' '\f' '\r' */
  GS_SEP_TAB = 1         /* split("\\t") */
};

#define GS_ERR_PARSE (-5)

/* Parse `len` bytes of DEVICE text (on the current HIP device) into DEVICE arrays:
 * line i -> src[i], dst[i] for i < cap. *n_lines (HOST) = number of lines; *bad_line
 * (HOST) = 0-based index of the first malformed line, or -1. Returns GS_OK,
 * GS_ERR_PARSE (a malformed line; the other lines are still written) or
 * GS_ERR_TRUNCATED (more lines than cap). Work is queued on `stream`
 * (hipStream_t, NULL = default) and the call synchronises it. */
int gs_parse_edges_device(void* stream, const char* text, size_t len, int sep, int64_t* src, int64_t* dst,
                          size_t cap, uint64_t* n_lines, int64_t* bad_line);

/* HOST text (e.g. a memory-mapped edge file) -> fold: copied through pinned staging
 * in chunks that end at line boundaries, parsed on the device and folded into h
 * (gs_fold semantics, one fold per chunk). *n_edges = edges folded. On a malformed
 * line returns GS_ERR_PARSE with *bad_line = its 0-based line index; the chunks
 * before it have been folded (the reference's job would have processed those
 * records before its map threw). */
int gs_fold_text(gs_handle h, const char* text, size_t len, int sep, uint64_t* n_edges, int64_t* bad_line);

/* Kernel timing of gs_parse_edges_device (measurement; per calling thread): with it on,
 * each parse brackets its parse kernel with HIP events, and gs_parse_profile returns
 * the summed kernel time (microseconds) and the number of parses since it was turned
 * on. Off by default (the events cost a synchronisation per parse). */
int gs_parse_set_profiling(int on);
int gs_parse_profile(double* kernel_us, uint64_t* parses);

/* gs_parse_edges_device keeps a per-thread cache (device scratch of ~1.25 x the longest
 * text parsed, a mapped result record, timing events) across calls. gs_parse_release frees
 * the calling thread's cache; a thread that parses calls it before it ends (a pool thread of
 * a JNI host: when its task finishes). A thread that moves to another device frees the old
 * device's cache at its next parse. */
int gs_parse_release(void);

#ifdef __cplusplus
}
#endif
#endif /* GS_INGEST_H */
