/*
 * BipartitenessCheck over the GPU summary, as one class with the reference's constructor
 * signature (S/library/BipartitenessCheck.java:50-52): the fold unchanged
 * (updateFunction, :93-95, whose edgeToCandidate GpuCandidates.merge buffers), the
 * initial value `new GpuCandidates(true)` (no GPU handle until it is used), and
 * combineFunction's reduce (:128-130: c1.merge(c2)) followed by an explicit release of
 * c2 when merge returned c1: the dataflow never reads the dropped input again
 * (GpuConnectedComponents explains why, for the Merger's fields too).
 */
package org.apache.flink.graph.streaming.summaries;

import org.apache.flink.api.common.functions.ReduceFunction;
import org.apache.flink.graph.streaming.SummaryBulkAggregation;
import org.apache.flink.graph.streaming.library.BipartitenessCheck;
import org.apache.flink.types.NullValue;

public class GpuBipartitenessCheck extends SummaryBulkAggregation<Long, NullValue, Candidates, Candidates> {
	private static final long serialVersionUID = 1L;

	public GpuBipartitenessCheck(long mergeWindowTime) {
		super(new BipartitenessCheck.updateFunction<Long>(), new MergeAndRelease(), new GpuCandidates(true),
				mergeWindowTime, false);
	}

	/** BipartitenessCheck.combineFunction.reduce (:128-130) + release of the dropped input. */
	public static class MergeAndRelease implements ReduceFunction<Candidates> {
		private static final long serialVersionUID = 1L;

		@Override
		public Candidates reduce(Candidates c1, Candidates c2) throws Exception {
			Candidates out = c1.merge(c2);
			if (out == c1 && c2 != c1 && c2 instanceof GpuSummary) {
				((GpuSummary) c2).release();
			}
			return out;
		}
	}
}
