/*
 * GpuShuffleWriter — the map task's writer on the GPU path (the work Spark's SortShuffleWriter /
 * UnsafeShuffleWriter do, chosen at compat/spark_3_0/UcxShuffleManager.scala:36-50 in the
 * reference): records are serialized into fixed-width rows in a direct host buffer, staged to HBM
 * and partitioned + grouped by partition id + indexed by libsparkucx_amd's gfx950 kernels
 * (sux_write_map_output_host), which also publishes the map's directory slot (the reference's
 * writeIndexFileAndCommit + descriptor PUT, CommonUcxShuffleBlockResolver.scala:33-107).
 *
 * GpuPartitioning decides whether a dependency can take this path: its partitioner must be one
 * the kernels restate bit-exactly (RangePartitioner over byte-array keys, HashPartitioner over
 * Long/Int keys) and its serializer must be a FixedWidthRowSerializer (rows of exactly
 * `recordSize` bytes).  Anything else keeps Spark's writer; its committed data file is adopted
 * by the resolver instead.
 */
package org.apache.spark.shuffle.gpu

import java.nio.{ByteBuffer, ByteOrder}

import org.apache.spark.{HashPartitioner, Partitioner, RangePartitioner, ShuffleDependency,
  SparkConf, TaskContext}
import org.apache.spark.internal.config
import org.apache.spark.io.CompressionCodec
import org.apache.spark.scheduler.MapStatus
import org.apache.spark.shuffle.{ShuffleWriteMetricsReporter, ShuffleWriter}
import org.apache.spark.shuffle.ucx.gpu.SuxNative
import org.apache.spark.storage.BlockManagerId

/** How a dependency's partitioner maps onto a sux_partitioner_desc (P1). */
case class GpuPartitioning(kind: Int, numPartitions: Int, keyOffset: Int, keyLen: Int,
                           ascending: Boolean, rangeBounds: Array[Byte])

object GpuPartitioning {
  private val longKeys = Set("long", "java.lang.Long", "scala.Long")
  private val intKeys = Set("int", "java.lang.Integer", "scala.Int")

  /** None when the partitioner has no bit-exact restatement on the GPU.  keyClassName is the
   * dependency's key class (ShuffleDependency.keyClassName): a HashPartitioner takes the GPU
   * path only for Long / Int keys, whose hashCode the kernels restate (Long.hashCode,
   * Integer.hashCode) — an 8-byte key of another type hashes differently in Spark. */
  def of(p: Partitioner, keyLen: Int, keyClassName: String): Option[GpuPartitioning] = p match {
    case h: HashPartitioner if keyLen == 8 && longKeys(keyClassName) =>
      Some(GpuPartitioning(SuxNative.PART_HASH_LONG, h.numPartitions, 0, 8, true, null))
    case h: HashPartitioner if keyLen == 4 && intKeys(keyClassName) =>
      Some(GpuPartitioning(SuxNative.PART_HASH_INT, h.numPartitions, 0, 4, true, null))
    case _: HashPartitioner => None
    case r: RangePartitioner[_, _] if keyLen > 0 && keyLen <= 16 =>
      // the bounds RangePartitioner sampled (private; reached by reflection, as the reference
      // reaches Spark internals it needs) must be byte arrays of keyLen bytes
      val f = classOf[RangePartitioner[_, _]].getDeclaredField("rangeBounds")
      f.setAccessible(true)
      val bounds = f.get(r).asInstanceOf[Array[_]]
      if (bounds.forall { case b: Array[Byte] => b.length == keyLen; case _ => false }) {
        val asc = {
          val g = classOf[RangePartitioner[_, _]].getDeclaredField("ascending")
          g.setAccessible(true)
          g.getBoolean(r)
        }
        Some(GpuPartitioning(SuxNative.PART_RANGE_BYTES, r.numPartitions, 0, keyLen, asc,
          bounds.flatMap(_.asInstanceOf[Array[Byte]])))
      } else None
    case _ => None
  }
}

/**
 * spark.shuffle.compress as the GPU restates it.  Spark's writers wrap every partition segment in
 * SerializerManager.wrapStream, so under the default config (compress on, lz4) a reader's
 * wrapStream expects lz4-java LZ4BlockOutputStream streams in every block — the reference's reader
 * relies on exactly that (compat/spark_3_0/UcxShuffleReader.scala:61).
 *   Some((CODEC_NONE, 0))        compress off: raw data files;
 *   Some((CODEC_LZ4, blockSize)) lz4: the node compresses every partition run on the GPU into the
 *                                bytes lz4-java writes (sux_shuffle_set_codec);
 *   None                         another codec, or encrypted shuffle streams: no GPU restatement —
 *                                such a dependency keeps Spark's writer, and the GPU sort in the
 *                                reader declines it (its blocks cannot be decoded on the GPU).
 */
object GpuCodec {
  def of(conf: SparkConf): Option[(Int, Int)] =
    if (conf.get(config.IO_ENCRYPTION_ENABLED)) None
    else if (!conf.get(config.SHUFFLE_COMPRESS)) Some((SuxNative.CODEC_NONE, 0))
    else if (CompressionCodec.getShortName(conf.get(config.IO_COMPRESSION_CODEC)) == "lz4") {
      Some((SuxNative.CODEC_LZ4,
        conf.getSizeAsBytes("spark.io.compression.lz4.blockSize", "32k").toInt))
    } else None

  /** The lz4-java chunk size a reader must accept (LZ4BlockInputStream decodes any chunk up to
   * the size its token declares; the GPU decoder is bounded by the writer's block size). */
  def maxBlockSize(conf: SparkConf): Int =
    math.max(64, conf.getSizeAsBytes("spark.io.compression.lz4.blockSize", "32k").toInt)
}

/** A row codec: one record is exactly recordSize bytes, the key's keyLen bytes first. */
trait FixedWidthRows[K, V] extends Serializable {
  def recordSize: Int
  def keyLen: Int
  def write(key: K, value: V, out: ByteBuffer): Unit
  /** The inverse of write: consumes exactly recordSize bytes of `in`. */
  def read(in: ByteBuffer): (K, V)
}

/** What a GPU shuffle's handle carries to every executor (UcxGpuShuffleHandle): the row layout
 * of its dependency's serializer. */
case class GpuRowLayout(recordSize: Int, keyOffset: Int, keyLen: Int)

/**
 * The dependency's serializer for a GPU shuffle: fixed-width rows, no stream header, no length
 * prefix — the bytes the kernels partition and the bytes Spark's own writers produce with it are
 * the same, and its deserializer reads either.  A ShuffleDependency is built with it
 * (`new ShuffledRDD(...).setSerializer(new FixedWidthRowSerializer(rows))`); registerShuffle
 * finds the layout here, inside the dependency — the shuffle id does not exist before the
 * dependency's constructor runs, so nothing can be registered by id ahead of it.
 */
class FixedWidthRowSerializer[K, V](val rows: FixedWidthRows[K, V])
  extends org.apache.spark.serializer.Serializer with Serializable {

  def layout: GpuRowLayout = GpuRowLayout(rows.recordSize, 0, rows.keyLen)

  // rows are independent fixed-size byte runs: concatenations are valid streams (batch fetch)
  override def supportsRelocationOfSerializedObjects: Boolean = true

  override def newInstance(): org.apache.spark.serializer.SerializerInstance =
    new FixedWidthRowSerializerInstance(rows)
}

private class FixedWidthRowSerializerInstance[K, V](rows: FixedWidthRows[K, V])
  extends org.apache.spark.serializer.SerializerInstance {
  import java.io.{EOFException, InputStream, OutputStream}
  import org.apache.spark.serializer.{DeserializationStream, SerializationStream}
  import scala.reflect.ClassTag

  private def unsupported = throw new UnsupportedOperationException(
    "FixedWidthRowSerializer only streams (key, value) rows")
  override def serialize[T: ClassTag](t: T): ByteBuffer = unsupported
  override def deserialize[T: ClassTag](bytes: ByteBuffer): T = unsupported
  override def deserialize[T: ClassTag](bytes: ByteBuffer, loader: ClassLoader): T = unsupported

  override def serializeStream(s: OutputStream): SerializationStream = new SerializationStream {
    private val row = ByteBuffer.allocate(rows.recordSize).order(ByteOrder.LITTLE_ENDIAN)
    private var key: Any = _
    private var haveKey = false
    override def writeKey[T: ClassTag](k: T): SerializationStream = { key = k; haveKey = true; this }
    override def writeValue[T: ClassTag](v: T): SerializationStream = {
      require(haveKey, "a row is written as writeKey then writeValue")
      row.clear()
      rows.write(key.asInstanceOf[K], v.asInstanceOf[V], row)
      require(row.position() == rows.recordSize, s"row is not ${rows.recordSize} bytes")
      s.write(row.array(), 0, rows.recordSize)
      haveKey = false
      this
    }
    override def writeObject[T: ClassTag](t: T): SerializationStream = t match {
      case (k, v) => writeKey(k); writeValue(v)
      case _ => unsupported
    }
    override def flush(): Unit = s.flush()
    override def close(): Unit = s.close()
  }

  override def deserializeStream(s: InputStream): DeserializationStream = new DeserializationStream {
    private val row = ByteBuffer.allocate(rows.recordSize).order(ByteOrder.LITTLE_ENDIAN)
    /** The next row, or EOFException at a clean end of stream. */
    private def next(): (K, V) = {
      var got = 0
      while (got < rows.recordSize) {
        val r = s.read(row.array(), got, rows.recordSize - got)
        if (r < 0) {
          if (got == 0) throw new EOFException
          throw new java.io.IOException(s"truncated row: $got of ${rows.recordSize} bytes")
        }
        got += r
      }
      row.clear()
      rows.read(row)
    }
    override def readObject[T: ClassTag](): T = next().asInstanceOf[T]
    override def readKey[T: ClassTag](): T = unsupported
    override def readValue[T: ClassTag](): T = unsupported
    override def asKeyValueIterator: Iterator[(Any, Any)] = new Iterator[(Any, Any)] {
      private var pending: Option[(K, V)] = None
      private var done = false
      override def hasNext: Boolean = {
        if (pending.isEmpty && !done) {
          try pending = Some(next()) catch { case _: EOFException => done = true; s.close() }
        }
        pending.nonEmpty
      }
      override def next(): (Any, Any) = {
        if (!hasNext) throw new NoSuchElementException
        val kv = pending.get
        pending = None
        kv
      }
    }
    override def close(): Unit = s.close()
  }
}

/** A key ordering the GPU sort restates bit-exactly (sux_sort_records): when the dependency
 * orders its keys with one of these, the reader sorts on the GPU instead of ExternalSorter. */
trait GpuKeyOrdering extends Serializable {
  def sortKind: Int
  def keyLen: Int
}

/** TeraSort's order: unsigned lexicographic over keyLen-byte keys. */
class UnsignedBytesOrdering(val keyLen: Int) extends Ordering[Array[Byte]] with GpuKeyOrdering {
  require(keyLen >= 1 && keyLen <= 12, "the GPU sorts byte keys of 1..12 bytes")
  override def sortKind: Int = SuxNative.SORT_BYTES
  override def compare(a: Array[Byte], b: Array[Byte]): Int = {
    var i = 0
    while (i < keyLen) {
      val d = (a(i) & 0xff) - (b(i) & 0xff)
      if (d != 0) return d
      i += 1
    }
    0
  }
}

/** Spark's LongType order (signed), for a little-endian int64 key. */
object SignedLongOrdering extends Ordering[Long] with GpuKeyOrdering {
  override def sortKind: Int = SuxNative.SORT_LONG
  override def keyLen: Int = 8
  override def compare(a: Long, b: Long): Int = java.lang.Long.compare(a, b)
}

class GpuShuffleWriter[K, V](
    node: GpuNode,
    shuffleId: Int,
    mapId: Long,
    numPartitions: Int,
    partitioner: Long,
    rows: FixedWidthRows[K, V],
    metrics: ShuffleWriteMetricsReporter) extends ShuffleWriter[K, V] {

  private var status: MapStatus = _
  private var lengths: Array[Long] = _

  override def write(records: Iterator[Product2[K, V]]): Unit = {
    import org.apache.spark.unsafe.Platform
    val rs = rows.recordSize
    // rows are serialized into a small direct chunk and appended to native staging memory that
    // grows in long arithmetic (a ByteBuffer stops at 2 GiB; a map task's output need not)
    val chunk = ByteBuffer.allocateDirect(rs * 4096).order(ByteOrder.LITTLE_ENDIAN)
    val chunkAddr = chunk.asInstanceOf[sun.nio.ch.DirectBuffer].address()
    var cap = rs.toLong * 65536
    var base = Platform.allocateMemory(cap)
    var used = 0L
    def flushChunk(): Unit = {
      val len = chunk.position().toLong
      if (used + len > cap) {
        var bigger = cap * 2
        while (used + len > bigger) bigger *= 2
        base = Platform.reallocateMemory(base, cap, bigger)
        cap = bigger
      }
      Platform.copyMemory(null, chunkAddr, null, base + used, len)
      used += len
      chunk.clear()
    }
    var n = 0L
    val t0 = System.nanoTime()
    try {
      records.foreach { kv =>
        if (chunk.remaining() < rs) flushChunk()
        val before = chunk.position()
        rows.write(kv._1, kv._2, chunk)
        require(chunk.position() - before == rs, s"row is not $rs bytes")
        n += 1
      }
      flushChunk()
      // slot = TaskContext.getPartitionId (compat/spark_3_0/UcxShuffleBlockResolver.scala:38)
      val slot = TaskContext.getPartitionId()
      if (n > 0) {
        SuxNative.writeMapOutputHostAddr(node.handle, shuffleId, slot, partitioner, base, n,
          node.threadStream())
      }
      // under spark.shuffle.compress the node committed LZ4Block streams (GpuCodec): the index
      // file, and so these MapStatus lengths, are the compressed ones, as Spark's writers report
      lengths = new Array[Long](numPartitions)
      if (n > 0) {
        val idx = ByteBuffer.wrap(SuxNative.mapOutputIndex(node.handle, shuffleId, slot, numPartitions))
        var prev = idx.getLong(0)  // big-endian, Spark's index file bytes
        for (p <- 0 until numPartitions) {
          val next = idx.getLong(8 * (p + 1))
          lengths(p) = next - prev
          prev = next
        }
      }
    } finally {
      Platform.freeMemory(base)  // the write copied the rows to HBM before returning
    }
    metrics.incRecordsWritten(n)
    metrics.incBytesWritten(lengths.sum)  // the committed (compressed) bytes, as Spark counts them
    metrics.incWriteTime(System.nanoTime() - t0)
    status = MapStatus(blockManagerId(), lengths, mapId)
  }

  private def blockManagerId(): BlockManagerId = org.apache.spark.SparkEnv.get.blockManager.shuffleServerId

  override def stop(success: Boolean): Option[MapStatus] = if (success) Option(status) else None

  /** The committed partition lengths (the MapStatus sizes). */
  def getPartitionLengths(): Array[Long] = lengths
}
