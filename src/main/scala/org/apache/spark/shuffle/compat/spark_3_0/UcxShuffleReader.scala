/*
 * UcxShuffleReader (Spark 3.0): the reduce task's read() on the GPU node.
 *
 * 1. Which (map task, reduce range) blocks it needs comes from Spark's MapOutputTracker, as in
 *    the reference (getMapSizesByExecutorId); mapTaskId -> map index (the directory slot).
 * 2. When several GPUs share the shuffle, the node-wide exchange (the all-to-all of the
 *    partitions each GPU owns, started on every executor by the driver's GpuExchangeCoordinator)
 *    must have completed: the task waits for it.  Any executor may then read any partition —
 *    its own from local HBM, another GPU's from that GPU's HBM over xGMI (a one-sided read, the
 *    reference's GET model) — so Spark may schedule the task anywhere.
 * 3. The blocks are fetched in one batch through UcxShuffleClient (one ShuffleBlockBatchId per
 *    map when the reduce range spans several partitions) — synchronous, so no progress loop and
 *    no reflection into Spark's results queue are needed.
 * 4. Rows are decoded by the dependency's serializer: for a GPU shuffle that is the
 *    FixedWidthRowSerializer whose rows the kernels wrote.  When the dependency orders its keys
 *    with an ordering the GPU restates (GpuKeyOrdering) and has no aggregator, the fetched rows
 *    are sorted on the GPU (sux_sort_records) in place of ExternalSorter; otherwise aggregation
 *    and the key sort stay Spark's (the reference's :100-154).
 */
package org.apache.spark.shuffle.compat.spark_3_0

import scala.collection.mutable

import org.apache.spark.{InterruptibleIterator, SparkEnv, SparkException, TaskContext}
import org.apache.spark.network.buffer.ManagedBuffer
import org.apache.spark.network.shuffle.BlockFetchingListener
import org.apache.spark.shuffle.{ShuffleReadMetricsReporter, ShuffleReader, UcxGpuShuffleHandle}
import org.apache.spark.shuffle.gpu.{FixedWidthRowSerializer, GpuKeyOrdering, GpuNode}
import org.apache.spark.shuffle.ucx.gpu.{DeviceManagedBuffer, SuxNative}
import org.apache.spark.shuffle.ucx.reducer.compat.spark_3_0.UcxShuffleClient
import org.apache.spark.storage.{BlockId, ShuffleBlockBatchId, ShuffleBlockId}
import org.apache.spark.util.CompletionIterator
import org.apache.spark.util.collection.ExternalSorter

class UcxShuffleReader[K, C](handle: UcxGpuShuffleHandle[K, _, C], node: GpuNode,
                             startPartition: Int, endPartition: Int, context: TaskContext,
                             readMetrics: ShuffleReadMetricsReporter) extends ShuffleReader[K, C] {

  private val dep = handle.baseHandle.dependency

  override def read(): Iterator[Product2[K, C]] = {
    val blocks = SparkEnv.get.mapOutputTracker
      .getMapSizesByExecutorId(handle.shuffleId, startPartition, endPartition).toSeq
    val mapIndex = new java.util.HashMap[java.lang.Long, Integer]()
    val wanted = mutable.ArrayBuffer[String]()
    val batch = endPartition - startPartition > 1
    blocks.foreach { case (_, bs) =>
      bs.foreach { case (id, _, idx) =>
        val mapId = id match {
          case b: ShuffleBlockId => b.mapId
          case b: ShuffleBlockBatchId => b.mapId
          case other => throw new SparkException(s"Unknown block $other")
        }
        if (!mapIndex.containsKey(mapId)) {
          mapIndex.put(mapId, Int.box(idx))
          wanted += (if (batch) ShuffleBlockBatchId(handle.shuffleId, mapId, startPartition, endPartition).name
                     else ShuffleBlockId(handle.shuffleId, mapId, startPartition).name)
        }
      }
    }
    node.awaitExchange(handle.shuffleId)

    val fetched = mutable.ArrayBuffer[(String, ManagedBuffer)]()
    var failure: Option[(String, Throwable)] = None
    val tmp = context.taskMetrics().createTempShuffleReadMetrics()
    val client = new UcxShuffleClient(handle.shuffleId, node, mapIndex, tmp)
    client.fetchBlocks("", 0, "", wanted.toArray, new BlockFetchingListener {
      override def onBlockFetchSuccess(blockId: String, data: ManagedBuffer): Unit =
        fetched += blockId -> data
      override def onBlockFetchFailure(blockId: String, e: Throwable): Unit =
        if (failure.isEmpty) failure = Some(blockId -> e)
    }, null)
    client.close()
    failure.foreach { case (id, e) =>
      fetched.foreach(_._2.release())
      throw new SparkException(s"fetch of $id failed", e)
    }
    context.taskMetrics().mergeShuffleReadMetrics()

    gpuSorted(fetched).foreach(sorted => return sorted)

    val ser = dep.serializer.newInstance()
    val serializerManager = SparkEnv.get.serializerManager
    val recordIter = fetched.iterator.flatMap { case (id, buf) =>
      readMetrics.incRemoteBlocksFetched(1)
      readMetrics.incRemoteBytesRead(buf.size())
      val in = serializerManager.wrapStream(BlockId(id), buf.createInputStream())
      CompletionIterator[(Any, Any), Iterator[(Any, Any)]](
        ser.deserializeStream(in).asKeyValueIterator, { in.close(); buf.release() })
    }
    val metricIter = CompletionIterator[(Any, Any), Iterator[(Any, Any)]](
      recordIter.map { r => readMetrics.incRecordsRead(1); r }, context.taskMetrics().mergeShuffleReadMetrics())
    val interruptible = new InterruptibleIterator[(Any, Any)](context, metricIter)

    // aggregation and ordering: Spark's reader semantics [ext]
    val aggregated: Iterator[Product2[K, C]] = dep.aggregator match {
      case Some(agg) if dep.mapSideCombine =>
        agg.combineCombinersByKey(interruptible.asInstanceOf[Iterator[(K, C)]], context)
      case Some(agg) =>
        agg.combineValuesByKey(interruptible.asInstanceOf[Iterator[(K, Nothing)]], context)
      case None => interruptible.asInstanceOf[Iterator[Product2[K, C]]]
    }
    dep.keyOrdering match {
      case Some(ord: Ordering[K]) =>
        val sorter = new ExternalSorter[K, C, C](context, ordering = Some(ord), serializer = dep.serializer)
        sorter.insertAll(aggregated)
        context.taskMetrics().incMemoryBytesSpilled(sorter.memoryBytesSpilled)
        context.taskMetrics().incDiskBytesSpilled(sorter.diskBytesSpilled)
        context.taskMetrics().incPeakExecutionMemory(sorter.peakMemoryUsedBytes)
        CompletionIterator[Product2[K, C], Iterator[Product2[K, C]]](sorter.iterator, sorter.stop())
      case None => aggregated
    }
  }

  /**
   * The GPU key sort (§8f item 1): a GPU shuffle (fixed-width rows) whose key ordering the GPU
   * restates and that has no aggregator.  Every fetched block is a slice of ONE pooled device
   * buffer, in request order (sux_fetch_blocks), so the rows are sorted where they lie, stably
   * (the map-ordered concatenation gives one deterministic order for equal keys, quirk Q4), and
   * decoded from a host copy of the sorted buffer.
   */
  private def gpuSorted(fetched: Seq[(String, ManagedBuffer)]): Option[Iterator[Product2[K, C]]] = {
    val (rows, ord) = (dep.serializer, dep.keyOrdering) match {
      case (s: FixedWidthRowSerializer[_, _], Some(o: GpuKeyOrdering))
          if dep.aggregator.isEmpty && handle.layout.exists(_.keyLen == o.keyLen) =>
        (s.rows, o)
      case _ => return None
    }
    val bufs = fetched.map(_._2).collect { case d: DeviceManagedBuffer => d }
    if (bufs.size != fetched.size || bufs.map(_.bufferHandle()).distinct.size > 1) return None
    val rs = rows.recordSize
    val total = bufs.map(_.size()).sum
    if (total == 0) {
      bufs.foreach(_.release())
      return Some(Iterator.empty)
    }
    val stream = node.threadStream()
    val t0 = System.nanoTime()
    val sorted = SuxNative.sortRecords(node.handle, ord.sortKind, bufs.head.bufferHandle(),
      total / rs, rs, handle.layout.get.keyOffset, ord.keyLen, stream)
    bufs.foreach(_.release())  // the fetched blocks' references; the pooled buffer goes back
    readMetrics.incFetchWaitTime((System.nanoTime() - t0) / 1000000)
    val out = new DeviceManagedBuffer(sorted, 0, total, stream)
    val host = out.nioByteBuffer().order(java.nio.ByteOrder.LITTLE_ENDIAN)
    out.release()
    readMetrics.incRecordsRead(total / rs)
    Some(new InterruptibleIterator[Product2[K, C]](context, new Iterator[Product2[K, C]] {
      override def hasNext: Boolean = host.remaining() >= rs
      override def next(): Product2[K, C] = {
        val slice = host.slice()
        slice.limit(rs)
        host.position(host.position() + rs)
        rows.read(slice.order(java.nio.ByteOrder.LITTLE_ENDIAN)).asInstanceOf[Product2[K, C]]
      }
    }))
  }
}
