/*
 * gs_jni.c -- JNI glue between the GPU-backed summaries
 * (java/src/main/java/org/apache/flink/graph/streaming/summaries/, class GsNative) and
 * the C ABI of libgs_summary.so (include/gs_summary.h, include/gs_group.h).
 *
 * Build (needs a JDK for jni.h; none exists in this repository's image):
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *      native/gs_jni.c -Lgelly-streaming_amd/lib -lgs_summary -Wl,-rpath,'$ORIGIN' -o libgs_jni.so
 *
 * Every ABI failure is rethrown as java.lang.RuntimeException(gs_last_error()), the
 * reference's `throws Exception` on EdgesFold.foldEdges / ReduceFunction.reduce
 * (S/EdgesFold.java:47). Edge arrays are copied with Get<T>ArrayRegion into a
 * per-thread native buffer before gs_fold / gs_fold_parity run: a fold of more than 2^18
 * edges does host copies, HIP copies and an event wait, which JNI forbids inside a
 * Get*ArrayCritical region (and which would stall the JVM's garbage collector for the
 * whole fold). Output arrays use Get/Release*ArrayElements so that the rows are written
 * back.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "gs_group.h"
#include "gs_summary.h"

#define FN(name) Java_org_apache_flink_graph_streaming_summaries_GsNative_##name
#define H(x) ((gs_handle)(intptr_t)(x))
#define G(x) ((gs_group_t)(intptr_t)(x))

static void throw_gs(JNIEnv* env) {
  jclass ex = (*env)->FindClass(env, "java/lang/RuntimeException");
  if (ex) (*env)->ThrowNew(env, ex, gs_last_error());
}

static void throw_msg(JNIEnv* env, const char* msg) {
  jclass ex = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
  if (ex) (*env)->ThrowNew(env, ex, msg);
}

#define CHECK(call)                \
  do {                             \
    if ((call) != GS_OK) {         \
      throw_gs(env);               \
      return;                      \
    }                              \
  } while (0)

/* ---- lifecycle ------------------------------------------------------------ */

JNIEXPORT jlong JNICALL FN(create)(JNIEnv* env, jclass c, jint device, jint kind, jlong hint) {
  (void)c;
  gs_handle h = NULL;
  if (gs_create(&h, device, kind, (uint64_t)hint) != GS_OK) {
    throw_gs(env);
    return 0;
  }
  return (jlong)(intptr_t)h;
}

JNIEXPORT void JNICALL FN(destroy)(JNIEnv* env, jclass c, jlong h) {
  (void)env;
  (void)c;
  gs_destroy(H(h));
}

JNIEXPORT void JNICALL FN(reset)(JNIEnv* env, jclass c, jlong h) {
  (void)c;
  CHECK(gs_reset(H(h)));
}

JNIEXPORT void JNICALL FN(resetConfig)(JNIEnv* env, jclass c, jlong h) {
  (void)c;
  CHECK(gs_reset_config(H(h)));
}

/* ---- fold / combine ------------------------------------------------------- */

/* Per-thread native copy of a flush (one Flink subtask thread per summary): grown once
 * to the summaries' flush size, reused by every later flush of the thread. */
typedef struct {
  int64_t *s, *d;
  uint8_t* w;
  size_t cap;
} EdgeStage;
static _Thread_local EdgeStage t_stage;

static int stage_reserve(JNIEnv* env, size_t n) {
  if (n <= t_stage.cap) return 1;
  int64_t* s = realloc(t_stage.s, n * 8);
  if (s) t_stage.s = s;
  int64_t* d = s ? realloc(t_stage.d, n * 8) : NULL;
  if (d) t_stage.d = d;
  uint8_t* w = d ? realloc(t_stage.w, n) : NULL;
  if (w) t_stage.w = w;
  if (!w) {
    jclass ex = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
    if (ex) (*env)->ThrowNew(env, ex, "gs_jni: edge staging buffer");
    return 0;
  }
  t_stage.cap = n;
  return 1;
}

JNIEXPORT void JNICALL FN(fold)(JNIEnv* env, jclass c, jlong h, jlongArray src, jlongArray dst, jint n) {
  (void)c;
  if (n < 0 || (*env)->GetArrayLength(env, src) < n || (*env)->GetArrayLength(env, dst) < n) {
    throw_msg(env, "fold: n outside the arrays");
    return;
  }
  if (!stage_reserve(env, (size_t)n)) return;
  (*env)->GetLongArrayRegion(env, src, 0, n, (jlong*)t_stage.s);
  (*env)->GetLongArrayRegion(env, dst, 0, n, (jlong*)t_stage.d);
  if ((*env)->ExceptionCheck(env)) return;
  /* outside any critical region: gs_fold may copy, launch and wait */
  if (gs_fold(H(h), t_stage.s, t_stage.d, (size_t)n) != GS_OK) throw_gs(env);
}

JNIEXPORT void JNICALL FN(foldParity)(JNIEnv* env, jclass c, jlong h, jlongArray src, jlongArray dst,
                                      jbyteArray par, jint n) {
  (void)c;
  if (n < 0 || (*env)->GetArrayLength(env, src) < n || (*env)->GetArrayLength(env, dst) < n ||
      (*env)->GetArrayLength(env, par) < n) {
    throw_msg(env, "foldParity: n outside the arrays");
    return;
  }
  if (!stage_reserve(env, (size_t)n)) return;
  (*env)->GetLongArrayRegion(env, src, 0, n, (jlong*)t_stage.s);
  (*env)->GetLongArrayRegion(env, dst, 0, n, (jlong*)t_stage.d);
  (*env)->GetByteArrayRegion(env, par, 0, n, (jbyte*)t_stage.w);
  if ((*env)->ExceptionCheck(env)) return;
  if (gs_fold_parity(H(h), t_stage.s, t_stage.d, t_stage.w, (size_t)n) != GS_OK) throw_gs(env);
}

JNIEXPORT void JNICALL FN(combine)(JNIEnv* env, jclass c, jlong dst, jlong src) {
  (void)c;
  CHECK(gs_combine(H(dst), H(src)));
}

/* Candidates.fail() / a failed input (Candidates.java:79-81,194-196): the sticky verdict */
JNIEXPORT void JNICALL FN(markFailed)(JNIEnv* env, jclass c, jlong h) {
  (void)c;
  CHECK(gs_combine_exported_device(H(h), NULL, NULL, NULL, 0, 1));
}

/* ---- queries -------------------------------------------------------------- */

JNIEXPORT jobject JNICALL FN(find)(JNIEnv* env, jclass c, jlong h, jlong v) {
  (void)c;
  int64_t label = 0;
  int found = 0;
  if (gs_find(H(h), (int64_t)v, &label, &found) != GS_OK) {
    throw_gs(env);
    return NULL;
  }
  if (!found) return NULL; /* DisjointSet.find -> null (:67-69) */
  jclass L = (*env)->FindClass(env, "java/lang/Long");
  jmethodID valueOf = (*env)->GetStaticMethodID(env, L, "valueOf", "(J)Ljava/lang/Long;");
  return (*env)->CallStaticObjectMethod(env, L, valueOf, (jlong)label);
}

JNIEXPORT jlong JNICALL FN(numVertices)(JNIEnv* env, jclass c, jlong h) {
  (void)c;
  uint64_t n = 0;
  if (gs_num_vertices(H(h), &n) != GS_OK) {
    throw_gs(env);
    return 0;
  }
  return (jlong)n;
}

JNIEXPORT jlong JNICALL FN(hbmBytes)(JNIEnv* env, jclass c, jint device) {
  (void)c;
  uint64_t b = 0;
  if (gs_hbm_bytes(device, &b) != GS_OK) {
    throw_gs(env);
    return 0;
  }
  return (jlong)b;
}

JNIEXPORT jlong JNICALL FN(createBytes)(JNIEnv* env, jclass c, jint kind, jlong hint) {
  (void)c;
  uint64_t b = 0;
  if (gs_create_bytes(kind, (uint64_t)hint, &b) != GS_OK) {
    throw_gs(env);
    return 0;
  }
  return (jlong)b;
}

JNIEXPORT jlong JNICALL FN(tableCapacity)(JNIEnv* env, jclass c, jlong h) {
  (void)c;
  uint64_t slots = 0;
  if (gs_table_capacity(H(h), &slots) != GS_OK) {
    throw_gs(env);
    return 0;
  }
  return (jlong)slots;
}

JNIEXPORT jint JNICALL FN(exportLabels)(JNIEnv* env, jclass c, jlong h, jlongArray v, jlongArray l) {
  (void)c;
  const jsize cap = (*env)->GetArrayLength(env, v);
  if ((*env)->GetArrayLength(env, l) < cap) {
    throw_msg(env, "exportLabels: label array shorter than vertex array");
    return 0;
  }
  size_t n = 0;
  jlong* pv = (*env)->GetLongArrayElements(env, v, NULL);
  jlong* pl = (*env)->GetLongArrayElements(env, l, NULL);
  const int rc = (pv && pl) ? gs_export_labels(H(h), (int64_t*)pv, (int64_t*)pl, (size_t)cap, &n) : GS_ERR_INVALID;
  if (pl) (*env)->ReleaseLongArrayElements(env, l, pl, rc == GS_OK ? 0 : JNI_ABORT);
  if (pv) (*env)->ReleaseLongArrayElements(env, v, pv, rc == GS_OK ? 0 : JNI_ABORT);
  if (rc != GS_OK) {
    throw_gs(env);
    return 0;
  }
  return (jint)n;
}

JNIEXPORT jboolean JNICALL FN(bipStatus)(JNIEnv* env, jclass c, jlong h) {
  (void)c;
  int ok = 1;
  if (gs_bip_status(H(h), &ok) != GS_OK) {
    throw_gs(env);
    return JNI_FALSE;
  }
  return ok ? JNI_TRUE : JNI_FALSE;
}

JNIEXPORT jint JNICALL FN(exportColouring)(JNIEnv* env, jclass c, jlong h, jlongArray comp, jlongArray v,
                                           jbyteArray sign) {
  (void)c;
  const jsize cap = (*env)->GetArrayLength(env, v);
  if ((*env)->GetArrayLength(env, comp) < cap || (*env)->GetArrayLength(env, sign) < cap) {
    throw_msg(env, "exportColouring: arrays of different lengths");
    return 0;
  }
  size_t n = 0;
  jlong* pc = (*env)->GetLongArrayElements(env, comp, NULL);
  jlong* pv = (*env)->GetLongArrayElements(env, v, NULL);
  jbyte* ps = (*env)->GetByteArrayElements(env, sign, NULL);
  const int rc = (pc && pv && ps) ? gs_export_colouring(H(h), (int64_t*)pc, (int64_t*)pv, (uint8_t*)ps, (size_t)cap, &n)
                                  : GS_ERR_INVALID;
  const jint mode = rc == GS_OK ? 0 : JNI_ABORT;
  if (ps) (*env)->ReleaseByteArrayElements(env, sign, ps, mode);
  if (pv) (*env)->ReleaseLongArrayElements(env, v, pv, mode);
  if (pc) (*env)->ReleaseLongArrayElements(env, comp, pc, mode);
  if (rc != GS_OK) {
    throw_gs(env);
    return 0;
  }
  return (jint)n;
}

/* ---- checkpoint ----------------------------------------------------------- */

JNIEXPORT jbyteArray JNICALL FN(serialize)(JNIEnv* env, jclass c, jlong h) {
  (void)c;
  size_t len = 0;
  if (gs_serialize(H(h), NULL, 0, &len) != GS_OK) {
    throw_gs(env);
    return NULL;
  }
  jbyteArray out = (*env)->NewByteArray(env, (jsize)len);
  if (!out) return NULL; /* OutOfMemoryError pending */
  jbyte* b = (*env)->GetByteArrayElements(env, out, NULL);
  size_t got = len;
  const int rc = b ? gs_serialize(H(h), b, len, &got) : GS_ERR_INVALID;
  if (b) (*env)->ReleaseByteArrayElements(env, out, b, rc == GS_OK ? 0 : JNI_ABORT);
  if (rc != GS_OK) {
    throw_gs(env);
    return NULL;
  }
  return out;
}

JNIEXPORT void JNICALL FN(deserialize)(JNIEnv* env, jclass c, jlong h, jbyteArray img) {
  (void)c;
  const jsize len = (*env)->GetArrayLength(env, img);
  jbyte* b = (*env)->GetByteArrayElements(env, img, NULL);
  const int rc = b ? gs_deserialize(H(h), b, (size_t)len) : GS_ERR_INVALID;
  if (b) (*env)->ReleaseByteArrayElements(env, img, b, JNI_ABORT);
  if (rc != GS_OK) throw_gs(env);
}

/* ---- per-window change emission ------------------------------------------ */

JNIEXPORT void JNICALL FN(setChangeTracking)(JNIEnv* env, jclass c, jlong h, jboolean on) {
  (void)c;
  CHECK(gs_set_change_tracking(H(h), on ? 1 : 0));
}

JNIEXPORT jint JNICALL FN(takeChanges)(JNIEnv* env, jclass c, jlong h, jlongArray v, jlongArray l, jbyteArray par) {
  (void)c;
  const jsize cap = (*env)->GetArrayLength(env, v); /* >= numVertices */
  if ((*env)->GetArrayLength(env, l) < cap || (par && (*env)->GetArrayLength(env, par) < cap)) {
    throw_msg(env, "takeChanges: arrays of different lengths");
    return 0;
  }
  uint64_t n = 0;
  jlong* pv = (*env)->GetLongArrayElements(env, v, NULL);
  jlong* pl = (*env)->GetLongArrayElements(env, l, NULL);
  jbyte* pp = par ? (*env)->GetByteArrayElements(env, par, NULL) : NULL;
  const int rc = (pv && pl) ? gs_take_changes(H(h), (int64_t*)pv, (int64_t*)pl, (uint8_t*)pp, (size_t)cap, &n)
                            : GS_ERR_INVALID;
  const jint mode = rc == GS_OK ? 0 : JNI_ABORT;
  if (pp) (*env)->ReleaseByteArrayElements(env, par, pp, mode);
  if (pl) (*env)->ReleaseLongArrayElements(env, l, pl, mode);
  if (pv) (*env)->ReleaseLongArrayElements(env, v, pv, mode);
  if (rc != GS_OK) {
    throw_gs(env);
    return 0;
  }
  return (jint)n;
}

/* ---- latency path (device addresses, e.g. from the ingest path) ----------- */

JNIEXPORT void JNICALL FN(setDeltaTracking)(JNIEnv* env, jclass c, jlong h, jboolean on) {
  (void)c;
  CHECK(gs_set_delta_tracking(H(h), on ? 1 : 0));
}

/* one window: fold + delta take + completion in one launch; returns the count word
 * (rows | GsNative.FAIL_BIT once a signed verdict failed) */
JNIEXPORT jlong JNICALL FN(foldTake)(JNIEnv* env, jclass c, jlong h, jlong s, jlong d, jlong n, jlong rec, jlong cap,
                                     jlong cnt) {
  (void)c;
  uint64_t k = 0;
  if (gs_fold_take_device(H(h), (const int64_t*)(intptr_t)s, (const int64_t*)(intptr_t)d, (size_t)n,
                          (int64_t*)(intptr_t)rec, (size_t)cap, (uint64_t*)(intptr_t)cnt, &k) != GS_OK) {
    throw_gs(env);
    return -1;
  }
  return (jlong)k;
}

/* replay another summary's window (rows | FAIL_BIT: the verdict is ANDed in) */
JNIEXPORT void JNICALL FN(foldRecords)(JNIEnv* env, jclass c, jlong h, jlong rec, jlong countWord) {
  (void)c;
  CHECK(gs_fold_records_device(H(h), (const int64_t*)(intptr_t)rec, (size_t)countWord, 0));
}

JNIEXPORT void JNICALL FN(setWindowServer)(JNIEnv* env, jclass c, jlong h, jboolean on) {
  (void)c;
  CHECK(gs_set_window_server(H(h), on ? 1 : 0));
}

JNIEXPORT void JNICALL FN(setBatchDedup)(JNIEnv* env, jclass c, jlong h, jboolean on) {
  (void)c;
  CHECK(gs_set_batch_dedup(H(h), on ? 1 : 0));
}

/* ---- multi-GPU group ------------------------------------------------------ */

JNIEXPORT jbyteArray JNICALL FN(groupUniqueId)(JNIEnv* env, jclass c) {
  (void)c;
  jbyte id[GS_GROUP_ID_BYTES];
  if (gs_group_unique_id(id) != GS_OK) {
    throw_gs(env);
    return NULL;
  }
  jbyteArray out = (*env)->NewByteArray(env, GS_GROUP_ID_BYTES);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, GS_GROUP_ID_BYTES, id);
  return out;
}

JNIEXPORT jlong JNICALL FN(groupCreate)(JNIEnv* env, jclass c, jlong h, jbyteArray id, jint nranks, jint rank,
                                        jlong batch) {
  (void)c;
  if ((*env)->GetArrayLength(env, id) != GS_GROUP_ID_BYTES) {
    throw_msg(env, "groupCreate: id must be GS_GROUP_ID_BYTES long");
    return 0;
  }
  jbyte buf[GS_GROUP_ID_BYTES];
  (*env)->GetByteArrayRegion(env, id, 0, GS_GROUP_ID_BYTES, buf);
  gs_group_t g = NULL;
  if (gs_group_create(&g, H(h), buf, nranks, rank, (size_t)batch) != GS_OK) {
    throw_gs(env);
    return 0;
  }
  return (jlong)(intptr_t)g;
}

JNIEXPORT void JNICALL FN(groupFold)(JNIEnv* env, jclass c, jlong g, jlong s, jlong d, jlong n) {
  (void)c;
  CHECK(gs_group_fold_device(G(g), (const int64_t*)(intptr_t)s, (const int64_t*)(intptr_t)d, (size_t)n));
}

JNIEXPORT void JNICALL FN(groupFinish)(JNIEnv* env, jclass c, jlong g) {
  (void)c;
  CHECK(gs_group_finish(G(g)));
}

JNIEXPORT void JNICALL FN(groupTreeCombine)(JNIEnv* env, jclass c, jlong g) {
  (void)c;
  CHECK(gs_group_tree_combine(G(g)));
}

/* owner-partitioned group (gs_group_create_partitioned): device addresses as longs */
JNIEXPORT jlong JNICALL FN(groupCreatePartitioned)(JNIEnv* env, jclass c, jlong h, jbyteArray id, jint nranks,
                                                   jint rank, jlong verticesHint, jlong windowEdges) {
  (void)c;
  if ((*env)->GetArrayLength(env, id) != GS_GROUP_ID_BYTES) {
    throw_msg(env, "groupCreatePartitioned: id must be GS_GROUP_ID_BYTES long");
    return 0;
  }
  jbyte buf[GS_GROUP_ID_BYTES];
  (*env)->GetByteArrayRegion(env, id, 0, GS_GROUP_ID_BYTES, buf);
  gs_group_t g = NULL;
  if (gs_group_create_partitioned(&g, H(h), buf, nranks, rank, (uint64_t)verticesHint, (size_t)windowEdges) != GS_OK) {
    throw_gs(env);
    return 0;
  }
  return (jlong)(intptr_t)g;
}

JNIEXPORT void JNICALL FN(groupPartFold)(JNIEnv* env, jclass c, jlong g, jlong s, jlong d, jlong n) {
  (void)c;
  CHECK(gs_group_part_fold_device(G(g), (const int64_t*)(intptr_t)s, (const int64_t*)(intptr_t)d, (size_t)n));
}

JNIEXPORT void JNICALL FN(groupPartCombine)(JNIEnv* env, jclass c, jlong g) {
  (void)c;
  CHECK(gs_group_part_combine(G(g)));
}

JNIEXPORT jlong JNICALL FN(groupPartLabels)(JNIEnv* env, jclass c, jlong g, jlong v, jlong label, jlong parity,
                                            jlong cap) {
  (void)c;
  size_t n = 0;
  if (gs_group_part_labels_device(G(g), (int64_t*)(intptr_t)v, (int64_t*)(intptr_t)label, (uint8_t*)(intptr_t)parity,
                                  (size_t)cap, &n) != GS_OK) {
    throw_gs(env);
    return 0;
  }
  return (jlong)n;
}

JNIEXPORT void JNICALL FN(groupPartReset)(JNIEnv* env, jclass c, jlong g) {
  (void)c;
  CHECK(gs_group_part_reset(G(g)));
}

JNIEXPORT void JNICALL FN(groupDestroy)(JNIEnv* env, jclass c, jlong g) {
  (void)env;
  (void)c;
  gs_group_destroy(G(g));
}
