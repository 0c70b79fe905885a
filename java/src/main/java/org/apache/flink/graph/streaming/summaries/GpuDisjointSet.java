/*
 * GPU-backed DisjointSet<Long>: the drop-in initial value of ConnectedComponents
 * (S/library/ConnectedComponents.java:52-54: `new GpuDisjointSet()` instead of
 * `new DisjointSet<>()`, or GpuConnectedComponents). UpdateCC.foldEdges (:83-86) and
 * CombineCC.reduce (:116-126) are unchanged: they call union, getMatches().size() and
 * merge, which this class overrides. The forest lives in HBM behind a gs_handle;
 * union() only buffers the edge, and the buffer is flushed as one micro-batch (gs_fold)
 * when full or before any read, merge or checkpoint.
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
 *
 * Java serialization (S extends Serializable, S/SummaryAggregation.java:22). Flink ships
 * the operator's functions to the TaskManagers by Java serialization, the Merger with its
 * `initialVal` and `summary` fields (SummaryAggregation.java:95-103). So:
 *   - the handle is taken from the pool at first USE, never in the constructor: the job
 *     client that builds `new GpuDisjointSet()` needs no GPU;
 *   - writeObject writes the gs_serialize image (or nothing for a summary that was never
 *     used); readObject keeps it and the first use of the copy applies it to a pooled
 *     handle (gs_deserialize). Kryo (GpuSummarySerializer) takes the same image.
 * The C++ host mirror models this path (writeObject / readObject in gelly_streaming.hpp,
 * tests/cpp/test_java_serialization.cpp, oracle-exact in tests/test_gpu_host_mirror.py).
 */
package org.apache.flink.graph.streaming.summaries;

import java.io.IOException;
import java.io.ObjectInputStream;
import java.io.ObjectOutputStream;
import java.util.Map;
import java.util.Set;

public class GpuDisjointSet extends DisjointSet<Long> implements GpuSummary {
	private static final long serialVersionUID = 2L;
	static final int BATCH = Integer.getInteger("gs.batch", 1 << 20);  // flush size (micro-batch)

	private transient long handle;   // 0 until the first use
	private transient byte[] image;  // read by readObject, applied at the first use
	private transient long sized;    // sizeFor(): the vertices the first handle is taken for (0: default)
	private transient long[] src;    // edge buffers, allocated at the first union
	private transient long[] dst;
	private transient int n;

	public GpuDisjointSet() {
	}

	public GpuDisjointSet(Set<Long> elements) {  // DisjointSet(Set<R>) :36-42
		for (Long e : elements) {
			makeSet(e);
		}
	}

	@Override
	public void union(Long e1, Long e2) {
		if (src == null) {
			src = new long[BATCH];
			dst = new long[BATCH];
		}
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
		return GsNative.find(handle(), e);
	}

	@Override
	public void merge(DisjointSet<Long> other) {
		flush();
		if (other instanceof GpuDisjointSet) {
			GpuDisjointSet o = (GpuDisjointSet) other;
			o.flush();
			GsNative.combine(handle(), o.handle());  // asynchronous, ordered behind both handles' work
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
		return GsNative.takeChanges(handle(), v, label, null);
	}

	public void setChangeTracking(boolean on) {
		flush();
		GsNative.setChangeTracking(handle(), on);
	}

	// ---- GpuSummary
	@Override
	public void flush() {
		if (n > 0) {
			GsNative.fold(handle(), src, dst, n);  // copied before it returns: the buffer is free again
			n = 0;
		}
	}

	/** The gs_handle, taken from the pool at the first use (a deserialised image applied). */
	@Override
	public long handle() {
		if (handle == 0) {
			long h = HandlePool.CC.acquire(GpuSummary.hintFor(sized, image));
			if (image != null) {
				try {
					GsNative.deserialize(h, image);
				} catch (RuntimeException e) {
					HandlePool.CC.release(h);
					throw e;
				}
				image = null;
			}
			handle = h;
		}
		return handle;
	}

	/** Size the handle taken at the first use for about `vertices` vertices (a copy: its
	 *  source's count); no effect once a handle is held. */
	@Override
	public void sizeFor(long vertices) {
		if (handle == 0) {
			sized = Math.max(vertices, 1L);
		}
	}

	/** Back to the pool: the combine dropped this summary (GpuConnectedComponents), or it
	 *  is no longer needed. It reads as a fresh, empty initial value afterwards. */
	@Override
	public void release() {
		n = 0;
		sized = 0;
		image = null;
		if (handle != 0) {
			HandlePool.CC.release(handle);
			handle = 0;
		}
	}

	// ---- Java serialization (the Merger's fields, SummaryAggregation.java:95-103)
	private void writeObject(ObjectOutputStream out) throws IOException {
		out.defaultWriteObject();
		byte[] img = image;  // not yet applied and nothing buffered on top: ship it as it came
		if (handle != 0 || n > 0) {
			// edges buffered on a deserialised copy belong in the image (ADVICE r4): flush()
			// applies the pending image to a handle first, then folds them
			flush();
			img = GsNative.serialize(handle());
		}
		out.writeObject(img);  // null: never used, the empty initial value
	}

	private void readObject(ObjectInputStream in) throws IOException, ClassNotFoundException {
		in.defaultReadObject();
		image = (byte[]) in.readObject();
		handle = 0;
		n = 0;
	}

	@Override
	protected void finalize() {  // backstop (Java 8) for summaries nobody released
		release();
	}
}
