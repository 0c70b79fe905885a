/*
 * DisjointSet.getMatches() (S/summaries/DisjointSet.java:44-46) without materialising
 * the forest. CombineCC.reduce calls getMatches().size() on both inputs on every
 * combine (S/library/ConnectedComponents.java:117-118): size() is gs_num_vertices
 * (O(1), the sharded counters), get() is gs_find, and only iteration exports the rows
 * (vertex, canonical label), once, through gs_export_labels.
 */
package org.apache.flink.graph.streaming.summaries;

import java.util.AbstractMap;
import java.util.ArrayList;
import java.util.Collections;
import java.util.LinkedHashSet;
import java.util.List;
import java.util.Map;
import java.util.Set;
import java.util.TreeMap;

final class LazyMatches extends AbstractMap<Long, Long> {
	private final GpuDisjointSet s;
	private Set<Map.Entry<Long, Long>> rows;

	LazyMatches(GpuDisjointSet s) {
		this.s = s;
	}

	@Override
	public int size() {
		return (int) GsNative.numVertices(s.handle());
	}

	@Override
	public Long get(Object k) {
		return k instanceof Long ? GsNative.find(s.handle(), (Long) k) : null;
	}

	@Override
	public boolean containsKey(Object k) {
		return get(k) != null;
	}

	@Override
	public Set<Map.Entry<Long, Long>> entrySet() {
		if (rows == null) {
			int c = size();
			long[] v = new long[c];
			long[] l = new long[c];
			int got = GsNative.exportLabels(s.handle(), v, l);
			Set<Map.Entry<Long, Long>> r = new LinkedHashSet<>(Math.max(16, 2 * got));
			for (int i = 0; i < got; i++) {
				r.add(new AbstractMap.SimpleImmutableEntry<>(v[i], l[i]));
			}
			rows = Collections.unmodifiableSet(r);
		}
		return rows;
	}

	/**
	 * DisjointSet.toString (:134-150) in canonical form: components keyed by their
	 * minimum id in ascending order, members ascending -- "{1=[1, 2, 3, 5], 6=[6, 7]}".
	 * The reference keys each component by find(v), an arbitrary member, in HashMap
	 * order; the partition is the same.
	 */
	static String groupByLabel(Set<Map.Entry<Long, Long>> entries) {
		TreeMap<Long, List<Long>> comps = new TreeMap<>();
		for (Map.Entry<Long, Long> e : entries) {
			comps.computeIfAbsent(e.getValue(), k -> new ArrayList<>()).add(e.getKey());
		}
		for (List<Long> members : comps.values()) {
			Collections.sort(members);
		}
		return comps.toString();
	}
}
