/*
 * What the Kryo serializer and the handle pool need from a GPU-backed summary.
 */
package org.apache.flink.graph.streaming.summaries;

interface GpuSummary {
	/** Fold the buffered per-edge callbacks as one micro-batch. */
	void flush();

	/** The gs_handle (0 once released). */
	long handle();

	/** Return the handle to the pool (the summary must not be used afterwards). */
	void release();

	/** Size the handle this summary takes at its first use for about `vertices` vertices (a
	 *  copy: its source's count); no effect once it holds a handle. */
	void sizeFor(long vertices);

	/** Vertices a gs_serialize image holds (its header: u32 magic, kind, ok, 0, u64 n). */
	static long imageVertices(byte[] image) {
		if (image == null || image.length < 24) {
			return 0;
		}
		return java.nio.ByteBuffer.wrap(image).order(java.nio.ByteOrder.LITTLE_ENDIAN).getLong(16);
	}

	/** The hint a summary's handle is created or pooled for: an explicit size, else the
	 *  pending image's vertex count, else the pool's default. */
	static long hintFor(long sized, byte[] image) {
		if (sized > 0) {
			return sized;
		}
		long n = imageVertices(image);
		return n > 0 ? n : HandlePool.CAPACITY_HINT;
	}
}
