/*
 * Native handles reused across windows. Flink copies the summary's initial value for
 * every (partition, window) fold -- the window fold state starts from
 * TypeSerializer.copy(initialValue), S/SummaryBulkAggregation.java:79-80 -- and drops
 * the partial after the all-window reduce. A fresh gs_create per copy would allocate
 * and initialise a table per window; a released handle is instead restored with
 * gs_reset_config (O(touched vertices) on the device, asynchronous; tracking,
 * pipelining and profiling back to a fresh handle's settings) and handed to the next
 * summary of the same kind.
 */
package org.apache.flink.graph.streaming.summaries;

import java.util.ArrayDeque;

final class HandlePool {
	/** Device of this TaskManager's summaries (one TaskManager per GPU). */
	static final int DEVICE = Integer.getInteger("gs.device", 0);
	/** Expected vertices per summary; the table grows past it on its own. */
	static final long CAPACITY_HINT = Long.getLong("gs.capacityHint", 1L << 20);
	static final int MAX_FREE = 64;

	static final HandlePool CC = new HandlePool(GsNative.KIND_CC);
	static final HandlePool SIGNED = new HandlePool(GsNative.KIND_SIGNED);

	private final int kind;
	private final ArrayDeque<Long> free = new ArrayDeque<>();
	private long created, reused;

	private HandlePool(int kind) {
		this.kind = kind;
	}

	synchronized long acquire() {
		Long h = free.poll();
		if (h != null) {
			reused++;
			return h;
		}
		created++;
		return GsNative.create(DEVICE, kind, CAPACITY_HINT);
	}

	synchronized void release(long h) {
		if (h == 0) {
			return;
		}
		try {
			GsNative.resetConfig(h);  // value and configuration of a fresh handle
		} catch (RuntimeException broken) {
			GsNative.destroy(h);      // a broken handle is not pooled
			return;
		}
		if (free.size() < MAX_FREE) {
			free.push(h);
		} else {
			GsNative.destroy(h);
		}
	}

	synchronized long created() {
		return created;
	}

	synchronized long reused() {
		return reused;
	}
}
