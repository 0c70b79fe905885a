/*
 * JNI entry points of libgs_jni.so (native/gs_jni.c) over the C ABI in
 * include/gs_summary.h and include/gs_group.h. One static native per ABI call the
 * GPU-backed summaries make; every failure is rethrown as a RuntimeException carrying
 * gs_last_error() (the reference's `throws Exception` on foldEdges/reduce,
 * S/EdgesFold.java:47). Handles are opaque longs (gs_handle / gs_group_t).
 *
 * Not compiled in this repository's image (no JDK); the C++ host mirror
 * (gelly-streaming_amd/host/gelly_streaming.hpp) drives the same call sequence and is
 * what the tests run.
 */
package org.apache.flink.graph.streaming.summaries;

final class GsNative {
	static {
		System.loadLibrary("gs_jni");
	}

	private GsNative() {}

	static final int KIND_CC = 0;      // GS_KIND_CC: DisjointSet
	static final int KIND_SIGNED = 1;  // GS_KIND_SIGNED: Candidates
	static final long FAIL_BIT = 1L << 62;  // GS_FAIL_BIT in count words

	// ---- lifecycle (gs_create / gs_destroy / gs_reset / gs_reset_config)
	static native long create(int device, int kind, long capacityHint);
	static native void destroy(long h);
	static native void reset(long h);
	static native void resetConfig(long h);

	// ---- fold / combine (gs_fold, gs_fold_parity, gs_combine, gs_combine_exported_device)
	static native void fold(long h, long[] src, long[] dst, int n);
	static native void foldParity(long h, long[] src, long[] dst, byte[] parity, int n);
	static native void combine(long dst, long src);
	static native void markFailed(long h);

	// ---- queries (gs_find, gs_num_vertices, gs_export_labels, gs_bip_status, gs_export_colouring)
	static native Long find(long h, long v);
	static native long numVertices(long h);
	static native long tableCapacity(long h);  // gs_table_capacity: slots (the pool's size classes)
	static native long hbmBytes(int device);  // gs_hbm_bytes: device memory of every live summary (the pool's budget)
	static native long createBytes(int kind, long capacityHint);  // gs_create_bytes: what a create allocates
	static native int exportLabels(long h, long[] v, long[] label);
	static native boolean bipStatus(long h);
	static native int exportColouring(long h, long[] comp, long[] v, byte[] sign);

	// ---- checkpoint (gs_serialize / gs_deserialize)
	static native byte[] serialize(long h);
	static native void deserialize(long h, byte[] image);

	// ---- per-window change emission (gs_set_change_tracking / gs_take_changes)
	static native void setChangeTracking(long h, boolean on);
	static native int takeChanges(long h, long[] v, long[] label, byte[] parity);

	// ---- latency path (gs_set_delta_tracking / gs_fold_take_device): device addresses
	static native void setDeltaTracking(long h, boolean on);
	static native long foldTake(long h, long srcDev, long dstDev, long n, long recDev, long cap, long cntDev);
	static native void foldRecords(long h, long recDev, long countWord);
	static native void setWindowServer(long h, boolean on);  // gs_set_window_server: one resident launch

	// ---- staging (gs_set_batch_dedup): repeats of an edge within a flush are dropped first
	static native void setBatchDedup(long h, boolean on);

	// ---- multi-GPU group (include/gs_group.h)
	static native byte[] groupUniqueId();
	static native long groupCreate(long h, byte[] id, int nranks, int rank, long batchEdges);
	static native void groupFold(long g, long srcDev, long dstDev, long n);
	static native void groupFinish(long g);
	static native void groupTreeCombine(long g);
	static native void groupDestroy(long g);
	// owner-partitioned group (gs_group_create_partitioned, DESIGN.md section 5b): local forests,
	// owned label slices; device addresses as longs
	static native long groupCreatePartitioned(long h, byte[] id, int nranks, int rank, long verticesHint,
			long windowEdges);
	static native void groupPartFold(long g, long srcDev, long dstDev, long n);
	static native void groupPartCombine(long g);
	static native long groupPartLabels(long g, long vDev, long labelDev, long parityDev, long cap);
	static native void groupPartReset(long g);
}
