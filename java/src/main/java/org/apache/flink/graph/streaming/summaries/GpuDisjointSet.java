/*
 * GPU-backed DisjointSet<Long>: the drop-in initial value of ConnectedComponents
 * (S/library/ConnectedComponents.java:52-54: `new GpuDisjointSet()` instead of
 * `new DisjointSet<>()`). UpdateCC.foldEdges (:83-86) and CombineCC.reduce (:116-126)
 * are unchanged: they call union, getMatches().size() and merge, which this class
 * overrides. The forest lives in HBM behind a gs_handle; union() only buffers the
 * edge, and the buffer is flushed as one micro-batch (gs_fold) when full or before
 * any read, merge or checkpoint.
 *
 * Replaces S/summaries/DisjointSet.java:44-150:
 *   getMatches  :44-46  -> LazyMatches (size = gs_num_vertices, get = gs_find)
 *   makeSet     :53-56  -> union(e, e) (a self-loop adds its vertex)
 *   find        :66-80  -> gs_find (null for a vertex never seen)
 *   union       :92-118 -> buffered, gs_fold
 *   merge       :127-131-> gs_combine (GPU partner) or union per entry (any other)
 *   toString    :134-150-> canonical grouping {min id=[members ascending], ...}
 * The labels are canonical (component minimum), so every grouping the reference's
 * HashMap order could print is the same partition (DESIGN.md section 2).
 */
package org.apache.flink.graph.streaming.summaries;

import java.util.Map;
import java.util.Set;

public class GpuDisjointSet extends DisjointSet<Long> implements GpuSummary {
	private static final long serialVersionUID = 1L;
	static final int BATCH = Integer.getInteger("gs.batch", 1 << 20);  // flush size (micro-batch)

	private transient long handle;
	private transient long[] src = new long[BATCH];
	private transient long[] dst = new long[BATCH];
	private transient int n;

	public GpuDisjointSet() {
		handle = HandlePool.CC.acquire();
	}

	public GpuDisjointSet(Set<Long> elements) {  // DisjointSet(Set<R>) :36-42
		this();
		for (Long e : elements) {
			makeSet(e);
		}
	}

	@Override
	public void union(Long e1, Long e2) {
		src[n] = e1;
		dst[n] = e2;
		if (++n == BATCH) {
			flush();
		}
	}

	@Override
	public void makeSet(Long e) {
		union(e, e);
	}

	@Override
	public Long find(Long e) {
		flush();
		return GsNative.find(handle, e);
	}

	@Override
	public void merge(DisjointSet<Long> other) {
		flush();
		if (other instanceof GpuDisjointSet) {
			GpuDisjointSet o = (GpuDisjointSet) other;
			o.flush();
			GsNative.combine(handle, o.handle);  // asynchronous, ordered behind both handles' work
			return;
		}
		for (Map.Entry<Long, Long> entry : other.getMatches().entrySet()) {  // :127-131
			union(entry.getKey(), entry.getValue());
		}
	}

	@Override
	public Map<Long, Long> getMatches() {
		flush();
		return new LazyMatches(this);
	}

	@Override
	public String toString() {
		return LazyMatches.groupByLabel(getMatches().entrySet());
	}

	/** Rows changed since the previous call (vertex, new canonical label); turns change
	 *  tracking on at the first call (gs_set_change_tracking / gs_take_changes). */
	public int takeChanges(long[] v, long[] label) {
		flush();
		return GsNative.takeChanges(handle, v, label, null);
	}

	public void setChangeTracking(boolean on) {
		flush();
		GsNative.setChangeTracking(handle, on);
	}

	// ---- GpuSummary
	@Override
	public void flush() {
		if (n > 0) {
			GsNative.fold(handle, src, dst, n);  // copied before it returns: the buffer is free again
			n = 0;
		}
	}

	@Override
	public long handle() {
		return handle;
	}

	@Override
	public void release() {
		if (handle != 0) {
			n = 0;
			HandlePool.CC.release(handle);
			handle = 0;
		}
	}

	@Override
	protected void finalize() {  // backstop (Java 8): reduce/Merger keep only the returned summary
		release();
	}
}
