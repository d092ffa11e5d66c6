/*
 * UcxShuffleManager (Spark 3.0) on the MI355X data path: spark.shuffle.manager =
 * org.apache.spark.shuffle.UcxShuffleManager, with spark.shuffle.sort.io.plugin.class =
 * org.apache.spark.shuffle.compat.spark_3_0.UcxLocalDiskShuffleDataIO, as for the reference.
 *
 * Map side: a dependency whose partitioner and rows the GPU restates bit-exactly
 * (GpuPartitioning, FixedWidthRows registered for its shuffle) is written by GpuShuffleWriter;
 * any other keeps Spark's writer, and the resolver adopts its committed data file into the
 * node's HBM.  Reduce side: UcxShuffleReader fetches through the node (after the node-wide
 * exchange when several GPUs share the shuffle).  The driver's metadata table of the reference
 * (registerShuffleCommon, CommonUcxShuffleManager.scala:39-56) becomes each node's directory,
 * sized by the number of MAP tasks (the reference sizes it by partitioner.numPartitions, quirk
 * Q1, and its PUTs overrun the table when maps outnumber reduces).
 */
package org.apache.spark.shuffle

import java.util.concurrent.ConcurrentHashMap

import org.apache.spark.{ShuffleDependency, SparkConf, SparkEnv, TaskContext}
import org.apache.spark.internal.Logging
import org.apache.spark.shuffle.compat.spark_3_0.{UcxShuffleBlockResolver, UcxShuffleReader}
import org.apache.spark.shuffle.gpu.{FixedWidthRows, GpuNode, GpuPartitioning, GpuShuffleWriter}
import org.apache.spark.shuffle.sort.SortShuffleManager
import org.apache.spark.shuffle.ucx.gpu.SuxNative
import org.apache.spark.util.ShutdownHookManager

/** Handle broadcast to the tasks: Spark's handle + what the node needs to register the shuffle. */
class UcxGpuShuffleHandle[K, V, C](shuffleId: Int, val numMaps: Int, val recordSize: Int,
                                   val baseHandle: BaseShuffleHandle[K, V, C])
  extends ShuffleHandle(shuffleId)

class UcxShuffleManager(val conf: SparkConf, isDriver: Boolean) extends SortShuffleManager(conf)
  with Logging {

  ShutdownHookManager.addShutdownHook(Int.MaxValue - 1)(() => stop())
  if (isDriver) GpuNode.startIfMissing(conf, isDriver = true)

  override val shuffleBlockResolver = new UcxShuffleBlockResolver(conf)

  /** Fixed-width row layouts by shuffle id, registered by the application (e.g. TeraSort). */
  val rowLayouts = new ConcurrentHashMap[Int, FixedWidthRows[_, _]]()

  private val registered = ConcurrentHashMap.newKeySet[Int]()
  private val partitioners = new ConcurrentHashMap[Int, java.lang.Long]()

  def startUcxNodeIfMissing(): GpuNode = GpuNode.startIfMissing(conf, isDriver)

  override def registerShuffle[K, V, C](shuffleId: Int,
                                        dependency: ShuffleDependency[K, V, C]): ShuffleHandle = {
    val base = super.registerShuffle(shuffleId, dependency).asInstanceOf[BaseShuffleHandle[K, V, C]]
    val numMaps = dependency.rdd.partitions.length  // Q1: slots per MAP task
    val rs = Option(rowLayouts.get(shuffleId)).map(_.recordSize).getOrElse(0)
    new UcxGpuShuffleHandle(shuffleId, numMaps, rs, base)
  }

  /** The executor's node learns a shuffle on its first task (register is idempotent here). */
  private def ensureRegistered(h: UcxGpuShuffleHandle[_, _, _], node: GpuNode): Unit = {
    if (registered.add(h.shuffleId)) {
      SuxNative.registerShuffle(node.handle, h.shuffleId, h.numMaps,
        h.baseHandle.dependency.partitioner.numPartitions, math.max(4, h.recordSize))
    }
  }

  override def getWriter[K, V](handle: ShuffleHandle, mapId: Long, context: TaskContext,
                               metrics: ShuffleWriteMetricsReporter): ShuffleWriter[K, V] = {
    val h = handle.asInstanceOf[UcxGpuShuffleHandle[K, V, _]]
    val node = GpuNode.get  // IllegalStateException before the executor components start
    ensureRegistered(h, node)
    val dep = h.baseHandle.dependency
    val rows = Option(rowLayouts.get(h.shuffleId)).map(_.asInstanceOf[FixedWidthRows[K, V]])
    val gpu = rows.flatMap(r => GpuPartitioning.of(dep.partitioner, r.keyLen).map(r -> _))
    gpu match {
      case Some((r, p)) =>
        val part = partitioners.computeIfAbsent(h.shuffleId, _ =>
          SuxNative.partitionerCreate(node.handle, p.kind, p.numPartitions, p.keyOffset, p.keyLen,
            42, p.ascending, p.rangeBounds))
        new GpuShuffleWriter[K, V](node, h.shuffleId, mapId, p.numPartitions, part, r, metrics)
      case None =>  // Spark's own writer; the resolver adopts its committed file
        super.getWriter[K, V](h.baseHandle, mapId, context, metrics)
    }
  }

  override def getReader[K, C](handle: ShuffleHandle, startPartition: Int, endPartition: Int,
                               context: TaskContext,
                               metrics: ShuffleReadMetricsReporter): ShuffleReader[K, C] = {
    val h = handle.asInstanceOf[UcxGpuShuffleHandle[K, _, C]]
    val node = startUcxNodeIfMissing()
    ensureRegistered(h, node)
    new UcxShuffleReader[K, C](h, node, startPartition, endPartition, context, metrics)
  }

  override def unregisterShuffle(shuffleId: Int): Boolean = {
    if (registered.remove(shuffleId)) {
      val node = GpuNode.get
      SuxNative.unregisterShuffle(node.handle, shuffleId)
      node.forget(shuffleId)
    }
    Option(partitioners.remove(shuffleId)).foreach(p => SuxNative.partitionerDestroy(p))
    rowLayouts.remove(shuffleId)
    super.unregisterShuffle(shuffleId)
  }

  override def stop(): Unit = synchronized {
    registered.forEach(id => unregisterShuffle(id))
    GpuNode.stop()
    super.stop()
  }
}
