"""The JNI glue as committed source: no JDK exists in this
image, so java/ and native/gs_jni.c cannot be compiled here. These text checks keep
them consistent with each other and with the C ABI: every `native` method of
GsNative.java has exactly one JNIEXPORT of the right mangled name in gs_jni.c, every
gs_* function the glue calls is declared in include/*.h (and exported by the library,
tests/test_capi.py), and every GsNative method the summaries call exists."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "java", "src", "main", "java", "org", "apache", "flink", "graph", "streaming", "summaries")
JNI = os.path.join(ROOT, "native", "gs_jni.c")


def _read(p):
    with open(p) as f:
        return f.read()


def _declared_abi():
    names = set()
    inc = os.path.join(ROOT, "include")
    for fn in os.listdir(inc):
        if fn.endswith(".h"):
            text = re.sub(r"/\*.*?\*/", "", _read(os.path.join(inc, fn)), flags=re.S)
            names.update(re.findall(r"\b(gs_[a-z_0-9]+)\s*\(", text))
    return names


def test_every_native_method_has_one_jni_export():
    java = _read(os.path.join(PKG, "GsNative.java"))
    natives = re.findall(r"static native \S+ (\w+)\(", java)
    assert len(natives) >= 25 and len(set(natives)) == len(natives)
    c = _read(JNI)
    exports = re.findall(r"JNIEXPORT \S+ JNICALL FN\((\w+)\)", c)
    assert sorted(exports) == sorted(natives)
    assert "#define FN(name) Java_org_apache_flink_graph_streaming_summaries_GsNative_##name" in c


def test_glue_calls_only_declared_abi():
    c = re.sub(r"/\*.*?\*/", "", _read(JNI), flags=re.S)
    called = set(re.findall(r"\b(gs_[a-z_0-9]+)\s*\(", c))
    assert called, "no ABI calls found"
    missing = called - _declared_abi()
    assert not missing, missing


def test_summaries_call_existing_natives():
    natives = set(re.findall(r"static native \S+ (\w+)\(", _read(os.path.join(PKG, "GsNative.java"))))
    for fn in os.listdir(PKG):
        if fn.endswith(".java") and fn != "GsNative.java":
            used = set(re.findall(r"GsNative\.(\w+)\(", _read(os.path.join(PKG, fn))))
            assert used <= natives, (fn, used - natives)


def test_java_sources_are_complete():
    # no elided bodies left from the round-2 markdown sketch
    for fn in os.listdir(PKG):
        text = _read(os.path.join(PKG, fn))
        assert "/* ..." not in text and "{ ... }" not in text and "…" not in text, fn
        assert text.count("{") == text.count("}"), fn
    for cls in ("GpuDisjointSet", "GpuCandidates", "LazyMatches", "HandlePool", "GpuSummarySerializer", "GsNative"):
        assert os.path.exists(os.path.join(PKG, cls + ".java")), cls


def test_summaries_survive_java_serialization_by_construction():
    """the handle is taken at the first use (no HandlePool.acquire in
    a constructor: the job client needs no GPU), both summaries carry writeObject /
    readObject, and the operators release the input their combine drops. The behaviour
    itself is modelled and tested on the C++ host mirror (test_java_serialization)."""
    for cls, pool in (("GpuDisjointSet", "CC"), ("GpuCandidates", "SIGNED")):
        text = _read(os.path.join(PKG, cls + ".java"))
        assert "private void writeObject(ObjectOutputStream out)" in text, cls
        assert "private void readObject(ObjectInputStream in)" in text, cls
        ctors = re.findall(r"public %s\([^)]*\)[^{]*\{(.*?)\n\t\}" % cls, text, flags=re.S)
        assert ctors and not any("acquire" in c for c in ctors), cls
        assert text.count("HandlePool.%s.acquire(" % pool) == 1, cls  # in handle() only
    for op in ("GpuConnectedComponents", "GpuBipartitenessCheck"):
        text = _read(os.path.join(PKG, op + ".java"))
        assert ".release();" in text and "extends SummaryBulkAggregation" in text, op


def test_jni_fold_outside_critical_regions():
    """gs_fold may copy, launch and wait; JNI forbids that inside a
    Get*ArrayCritical region. The glue copies with Get<T>ArrayRegion instead."""
    c = re.sub(r"/\*.*?\*/", "", _read(JNI), flags=re.S)
    assert "GetPrimitiveArrayCritical" not in c
    assert "GetLongArrayRegion" in c and "GetByteArrayRegion" in c


def test_write_object_serialises_buffered_edges_of_a_deserialised_copy():
    """union() only buffers, so a deserialised copy (image pending, no handle) with
    fewer than BATCH buffered edges must not ship its stale image. writeObject serialises
    whenever a handle exists or edges are buffered (flush() applies the pending image first),
    the same condition as the C++ mirror (`h_ || n_ ? serialize() : image_`, modelled and
    oracle-checked in tests/cpp/test_java_serialization.cpp)."""
    for cls in ("GpuDisjointSet", "GpuCandidates"):
        text = _read(os.path.join(PKG, cls + ".java"))
        body = re.search(r"private void writeObject\(ObjectOutputStream out\)[^{]*\{(.*?)\n\t\}", text, flags=re.S)
        assert body, cls
        b = body.group(1)
        assert re.search(r"if \(handle != 0 \|\| n > 0\) \{", b), cls
        assert "img == null &&" not in b, cls
        assert "GsNative.serialize(handle())" in b and b.index("flush();") < b.index("GsNative.serialize"), cls
    mirror = _read(os.path.join(ROOT, "gelly-streaming_amd", "host", "gelly_streaming.hpp"))
    assert "h_ || n_ ? serialize() : image_" in mirror


def test_handle_pool_hbm_budget_by_construction():
    """VERDICT r4 item 3 / r5 item 2, ADVICE r5: the pool checks its budget against the
    library's count of device memory (GsNative.hbmBytes -> gs_hbm_bytes: a table that grew while
    handed out counts at once) plus the creates reserved under its lock (concurrent task slots
    cannot all pass the check); before a create would pass gs.hbmBudgetBytes it runs
    System.gc() + System.runFinalization() OUTSIDE its lock, rate-limited after a pass that
    returned nothing; device work (resetConfig, tableCapacity, destroy) never runs under the
    lock; a request takes a pooled handle of its class or any larger one before it creates.
    Copies are sized from their source's vertex count and deserialised summaries from their
    image. The behaviour is modelled on the C++ mirror (test_handle_budget)."""
    pool = _read(os.path.join(PKG, "HandlePool.java"))
    acq = re.search(r"\tlong acquire\(long hint\) \{(.*?)\n\t\}", pool, flags=re.S).group(1)
    assert "synchronized long acquire" not in pool  # not under the pool's lock
    assert "GsNative.createBytes(kind, hint)" in acq and "reserve(need, false)" in acq and "evictFor(need)" in acq
    assert acq.index("collect();") < acq.index("GsNative.create(")
    assert "take(cls, true)" in acq  # any larger pooled handle before a create
    res = re.search(r"private synchronized boolean reserve\(long need, boolean force\) \{(.*?)\n\t\}", pool,
                    flags=re.S).group(1)
    assert "GsNative.hbmBytes(DEVICE) + reserved + need > BUDGET_BYTES" in res
    col = re.search(r"private void collect\(\) \{(.*?)\n\t\}", pool, flags=re.S).group(1)
    assert "System.gc();" in col and "System.runFinalization();" in col and "GC_BACKOFF_MS" in col
    # the gc runs between two synchronized blocks, never inside one
    assert col.index("System.gc();") > col.index("before = nfree;") and "synchronized (this)" in col
    rel = re.search(r"\tvoid release\(long h\) \{(.*?)\n\t\}", pool, flags=re.S).group(1)
    assert "synchronized void release" not in pool
    assert rel.index("GsNative.resetConfig(h)") < rel.index("synchronized (this)")
    assert rel.index("GsNative.tableCapacity(h)") < rel.index("synchronized (this)")
    ser = _read(os.path.join(PKG, "GpuSummarySerializer.java"))
    copy = re.search(r"public GpuSummary copy\(.*?\n\t\}", ser, flags=re.S).group(0)
    assert "sizeFor(2 * GsNative.numVertices(original.handle()))" in copy
    assert copy.index("sizeFor(") < copy.index("c.handle()")
    for cls, p in (("GpuDisjointSet", "CC"), ("GpuCandidates", "SIGNED")):
        text = _read(os.path.join(PKG, cls + ".java"))
        assert "HandlePool.%s.acquire(GpuSummary.hintFor(sized, image))" % p in text
        # sizeFor has its own Javadoc; release() keeps "Back to the pool"
        assert re.search(r"/\*\* Back to the pool[^/]*\*/\n\t@Override\n\tpublic void release\(\)", text), cls
    assert "enableObjectReuse" in _read(os.path.join(ROOT, "INTEGRATION.md"))
