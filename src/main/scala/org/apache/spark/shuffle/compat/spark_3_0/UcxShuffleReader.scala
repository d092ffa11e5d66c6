/*
 * UcxShuffleReader (Spark 3.0): the reduce task's read() on the GPU node.
 *
 * 1. Which (map task, reduce range) blocks it needs comes from Spark's MapOutputTracker, as in
 *    the reference (getMapSizesByExecutorId); mapTaskId -> map index (the directory slot).
 * 2. When several GPUs share the shuffle, the first reduce task of this executor runs the
 *    node-wide exchange (a collective all-to-all of the partitions each GPU owns), replacing the
 *    per-block remote GETs.
 * 3. The blocks are fetched in one batch through UcxShuffleClient (one ShuffleBlockBatchId per
 *    map when the reduce range spans several partitions) — synchronous, so no progress loop and
 *    no reflection into Spark's results queue are needed.
 * 4. Deserialization, aggregation and the key sort stay Spark's (the reference's :100-154).
 */
package org.apache.spark.shuffle.compat.spark_3_0

import scala.collection.mutable

import org.apache.spark.{InterruptibleIterator, SparkEnv, SparkException, TaskContext}
import org.apache.spark.network.buffer.ManagedBuffer
import org.apache.spark.network.shuffle.BlockFetchingListener
import org.apache.spark.shuffle.{ShuffleReadMetricsReporter, ShuffleReader, UcxGpuShuffleHandle}
import org.apache.spark.shuffle.gpu.GpuNode
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
    if (node.worldSize > 1) node.exchangeOnce(handle.shuffleId)

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
}
