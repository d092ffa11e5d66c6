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
 * Long/Int keys) and its rows must serialize to exactly `recordSize` bytes.  Anything else keeps
 * Spark's writer; its committed data file is adopted by the resolver instead.
 */
package org.apache.spark.shuffle.gpu

import java.nio.{ByteBuffer, ByteOrder}

import org.apache.spark.{HashPartitioner, Partitioner, RangePartitioner, ShuffleDependency, TaskContext}
import org.apache.spark.scheduler.MapStatus
import org.apache.spark.shuffle.{ShuffleWriteMetricsReporter, ShuffleWriter}
import org.apache.spark.shuffle.ucx.gpu.SuxNative
import org.apache.spark.storage.BlockManagerId

/** How a dependency's partitioner maps onto a sux_partitioner_desc (P1). */
case class GpuPartitioning(kind: Int, numPartitions: Int, keyOffset: Int, keyLen: Int,
                           ascending: Boolean, rangeBounds: Array[Byte])

object GpuPartitioning {
  /** None when the partitioner has no bit-exact restatement on the GPU. */
  def of(p: Partitioner, keyLen: Int): Option[GpuPartitioning] = p match {
    case h: HashPartitioner if keyLen == 8 =>
      Some(GpuPartitioning(SuxNative.PART_HASH_LONG, h.numPartitions, 0, 8, true, null))
    case h: HashPartitioner if keyLen == 4 =>
      Some(GpuPartitioning(SuxNative.PART_HASH_INT, h.numPartitions, 0, 4, true, null))
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

/** A row serializer writing one record as exactly recordSize bytes (key first). */
trait FixedWidthRows[K, V] extends Serializable {
  def recordSize: Int
  def keyLen: Int
  def write(key: K, value: V, out: ByteBuffer): Unit
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
    val rs = rows.recordSize
    var buf = ByteBuffer.allocateDirect(rs * 65536).order(ByteOrder.LITTLE_ENDIAN)
    var n = 0L
    val t0 = System.nanoTime()
    records.foreach { kv =>
      if (buf.remaining() < rs) {  // grow the staging buffer (map tasks are bounded by Spark)
        val bigger = ByteBuffer.allocateDirect(buf.capacity() * 2).order(ByteOrder.LITTLE_ENDIAN)
        buf.flip()
        bigger.put(buf)
        buf = bigger
      }
      val before = buf.position()
      rows.write(kv._1, kv._2, buf)
      require(buf.position() - before == rs, s"row is not $rs bytes")
      n += 1
    }
    // slot = TaskContext.getPartitionId (compat/spark_3_0/UcxShuffleBlockResolver.scala:38)
    val slot = TaskContext.getPartitionId()
    if (n > 0) {
      SuxNative.writeMapOutputHost(node.handle, shuffleId, slot, partitioner, buf, n, rs,
        node.threadStream())
    }
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
    metrics.incRecordsWritten(n)
    metrics.incBytesWritten(n * rs)
    metrics.incWriteTime(System.nanoTime() - t0)
    status = MapStatus(blockManagerId(), lengths, mapId)
  }

  private def blockManagerId(): BlockManagerId = org.apache.spark.SparkEnv.get.blockManager.shuffleServerId

  override def stop(success: Boolean): Option[MapStatus] = if (success) Option(status) else None

  /** The committed partition lengths (the MapStatus sizes). */
  def getPartitionLengths(): Array[Long] = lengths
}
