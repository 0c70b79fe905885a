/*
 * GPU-backed Candidates: the drop-in initial value of BipartitenessCheck
 * (S/library/BipartitenessCheck.java:50-52: `new GpuCandidates(true)` instead of
 * `new Candidates(true)`). updateFunction.foldEdges (:93-95) calls
 * candidates.merge(edgeToCandidate(v1, v2)) once per edge and combineFunction.reduce
 * (:128-130) calls c1.merge(c2); both stay unchanged. The signed forest (parity of
 * every vertex to its parent in the link word) lives in HBM behind a gs_handle.
 *
 * Replaces S/summaries/Candidates.java:44-196:
 *   getSuccess :44-46    -> gs_bip_status
 *   getMap     :48-50    -> gs_export_colouring, as TreeMap<comp, TreeMap<v, SignedVertex>>
 *   add        :52-74    -> buffered edges (vertex against the component key, parity from the signs)
 *   merge      :77-139   -> one-edge candidate: buffered edge, gs_fold per micro-batch;
 *                           GpuCandidates: gs_combine (the verdict is the AND, :79-81);
 *                           any other Candidates: its components folded vertex by vertex
 *   fail       :194-196  -> the sticky device verdict; getMap() is then {} -> "(false,{})"
 * The output is the canonical colouring (components keyed by their minimum id, sign =
 * same side as that minimum), which equals the reference's exactly in its exact
 * regime and the mathematical truth everywhere (DESIGN.md section 2); the reference's
 * order-dependent quirks are not reproduced.
 *
 * Java serialization as GpuDisjointSet's: the handle is taken at the first use (the job
 * client builds the initial value without a GPU), writeObject ships the gs_serialize
 * image (verdict included) and the copy applies it at its first use; a
 * `new GpuCandidates(false)` that was never used ships its failed verdict as a field.
 */
package org.apache.flink.graph.streaming.summaries;

import java.io.IOException;
import java.io.ObjectInputStream;
import java.io.ObjectOutputStream;
import java.util.Map;
import java.util.TreeMap;

import org.apache.flink.graph.streaming.util.SignedVertex;

public class GpuCandidates extends Candidates implements GpuSummary {
	private static final long serialVersionUID = 2L;
	static final int BATCH = GpuDisjointSet.BATCH;

	private final boolean failedInitially;  // new GpuCandidates(false): applied at the first use
	private transient long handle;          // 0 until the first use
	private transient byte[] image;         // read by readObject, applied at the first use
	private transient long sized;           // sizeFor(): the vertices the first handle is taken for (0: default)
	private transient long[] src;           // edge buffers, allocated at the first edge
	private transient long[] dst;
	private transient byte[] par;
	private transient int n;
	private transient boolean plain = true;  // every buffered edge has parity 1 (a stream edge)

	public GpuCandidates() {
		this(true);
	}

	public GpuCandidates(boolean success) {
		super(success);
		failedInitially = !success;
	}

	public GpuCandidates(boolean success, Candidates input) throws Exception {  // :36-42
		this(success);
		merge(input);
	}

	private void buffer(long a, long b, boolean differentSides) {
		if (src == null) {
			src = new long[BATCH];
			dst = new long[BATCH];
			par = new byte[BATCH];
		}
		src[n] = a;
		dst[n] = b;
		par[n] = (byte) (differentSides ? 1 : 0);
		plain &= differentSides;
		if (++n == BATCH) {
			flush();
		}
	}

	@Override
	public boolean add(long component, Map<Long, SignedVertex> vertices) throws Exception {
		for (SignedVertex v : vertices.values()) {
			add(component, v);
		}
		return true;  // a conflict surfaces in the verdict (getSuccess), as merge's does
	}

	/** The component key is taken with sign true, as every Candidates built through
	 *  add / edgeToCandidate has it (the first vertex added under a key is the key). */
	@Override
	public boolean add(long component, SignedVertex vertex) throws Exception {
		buffer(component, vertex.getVertex(), !vertex.getSign());
		return true;
	}

	@Override
	public Candidates merge(Candidates input) throws Exception {
		if (input instanceof GpuCandidates) {  // combineFunction.reduce: c1.merge(c2)
			GpuCandidates o = (GpuCandidates) input;
			flush();
			o.flush();
			GsNative.combine(handle(), o.handle());  // rows + verdict, ordered behind both handles
			return this;
		}
		if (!input.getSuccess()) {  // :79-81
			flush();
			GsNative.markFailed(handle());
			return this;
		}
		for (Map.Entry<Long, Map<Long, SignedVertex>> comp : input.getMap().entrySet()) {
			Map<Long, SignedVertex> members = comp.getValue();
			SignedVertex anchor = null;
			for (SignedVertex v : members.values()) {
				if (anchor == null) {
					anchor = v;
					// a lone vertex (a self-loop's candidate) still becomes a vertex
					if (members.size() == 1) {
						buffer(v.getVertex(), v.getVertex(), true);
					}
					continue;
				}
				// edgeToCandidate(u, v) = {min: {min: +, max: -}}: one buffered stream edge
				buffer(anchor.getVertex(), v.getVertex(), anchor.getSign() != v.getSign());
			}
		}
		return this;
	}

	@Override
	public boolean getSuccess() {
		flush();
		f0 = GsNative.bipStatus(handle());
		return f0;
	}

	@Override
	public TreeMap<Long, Map<Long, SignedVertex>> getMap() {
		flush();
		TreeMap<Long, Map<Long, SignedVertex>> map = new TreeMap<>();
		int c = (int) GsNative.numVertices(handle());
		long[] comp = new long[c];
		long[] v = new long[c];
		byte[] sign = new byte[c];
		int got = GsNative.exportColouring(handle(), comp, v, sign);  // 0 rows once the verdict failed
		for (int i = 0; i < got; i++) {
			map.computeIfAbsent(comp[i], k -> new TreeMap<>()).put(v[i], new SignedVertex(v[i], sign[i] != 0));
		}
		f1 = map;
		return map;
	}

	@Override
	public String toString() {  // Tuple2.toString: "(true,{1={1=(1,true), 3=(3,false)}, ...})"
		boolean ok = getSuccess();
		getMap();
		f0 = ok;
		return super.toString();
	}

	// ---- GpuSummary
	@Override
	public void flush() {
		if (n > 0) {
			if (plain) {
				GsNative.fold(handle(), src, dst, n);  // every edge: different sides
			} else {
				GsNative.foldParity(handle(), src, dst, par, n);
			}
			n = 0;
			plain = true;
		}
	}

	/** The gs_handle, taken from the pool at the first use (a deserialised image or the
	 *  initial failed verdict applied). */
	@Override
	public long handle() {
		if (handle == 0) {
			long h = HandlePool.SIGNED.acquire(GpuSummary.hintFor(sized, image));
			try {
				if (image != null) {
					GsNative.deserialize(h, image);  // rows and verdict
				} else if (failedInitially) {
					GsNative.markFailed(h);
				}
			} catch (RuntimeException e) {
				HandlePool.SIGNED.release(h);
				throw e;
			}
			image = null;
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

	/** Back to the pool (the combine dropped this summary, GpuBipartitenessCheck); it reads
	 *  as a fresh initial value afterwards. */
	@Override
	public void release() {
		n = 0;
		sized = 0;
		plain = true;
		image = null;
		if (handle != 0) {
			HandlePool.SIGNED.release(handle);
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
		out.writeObject(img);  // null: never used (failedInitially travels as a field)
	}

	private void readObject(ObjectInputStream in) throws IOException, ClassNotFoundException {
		in.defaultReadObject();
		image = (byte[]) in.readObject();
		handle = 0;
		n = 0;
		plain = true;
	}

	@Override
	protected void finalize() {  // backstop (Java 8) for summaries nobody released
		release();
	}
}
