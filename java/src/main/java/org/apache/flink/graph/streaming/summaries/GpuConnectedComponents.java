/*
 * ConnectedComponents over the GPU summary, as one class: the same operator and the same
 * constructor signature as S/library/ConnectedComponents.java:52-54
 * (`new GpuConnectedComponents<>(mergeWindowTime)` where a job had
 * `new ConnectedComponents<>(mergeWindowTime)`), with
 *   - the fold unchanged (ConnectedComponents.UpdateCC, :83-86);
 *   - the initial value `new GpuDisjointSet()` (no GPU handle until it is used on a
 *     TaskManager, so the job client needs no GPU);
 *   - CombineCC's reduce (:116-126: merge the smaller into the larger, return the
 *     larger) followed by an explicit release of the input it dropped: its handle (and
 *     its table, ~64 MiB at the default hint) goes back to the pool at once instead of
 *     waiting for the garbage collector's finalize(). The dropped input is never read
 *     again by the dataflow: the window reduce keeps the returned value, and the Merger
 *     (SummaryAggregation.java:107-119) keeps `summary = reduce(s, summary)`; an
 *     initialVal it dropped reads as a fresh empty summary afterwards, which is what it
 *     held (transient state restarts from it).
 */
package org.apache.flink.graph.streaming.summaries;

import org.apache.flink.api.common.functions.ReduceFunction;
import org.apache.flink.graph.streaming.SummaryBulkAggregation;
import org.apache.flink.graph.streaming.library.ConnectedComponents;
import org.apache.flink.types.NullValue;

public class GpuConnectedComponents extends SummaryBulkAggregation<Long, NullValue, DisjointSet<Long>, DisjointSet<Long>> {
	private static final long serialVersionUID = 1L;

	public GpuConnectedComponents(long mergeWindowTime) {
		super(new ConnectedComponents.UpdateCC<Long>(), new CombineAndRelease(), new GpuDisjointSet(), mergeWindowTime,
				false);
	}

	/** ConnectedComponents.CombineCC.reduce (:116-126) + release of the dropped input. */
	public static class CombineAndRelease implements ReduceFunction<DisjointSet<Long>> {
		private static final long serialVersionUID = 1L;

		@Override
		public DisjointSet<Long> reduce(DisjointSet<Long> s1, DisjointSet<Long> s2) throws Exception {
			int count1 = s1.getMatches().size();
			int count2 = s2.getMatches().size();
			DisjointSet<Long> keep = count1 <= count2 ? s2 : s1;
			DisjointSet<Long> drop = keep == s2 ? s1 : s2;
			keep.merge(drop);  // gs_combine: asynchronous; the pool's reset orders behind its export
			if (drop != keep && drop instanceof GpuSummary) {
				((GpuSummary) drop).release();
			}
			return keep;
		}
	}
}
