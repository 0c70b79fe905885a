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
}
