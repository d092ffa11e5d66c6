/*
 * UcxShuffleManager (Spark 3.0) on the MI355X data path: spark.shuffle.manager =
 * org.apache.spark.shuffle.UcxShuffleManager, with spark.shuffle.sort.io.plugin.class =
 * org.apache.spark.shuffle.compat.spark_3_0.UcxLocalDiskShuffleDataIO, as for the reference.
 *
 * Map side: a dependency whose partitioner and rows the GPU restates bit-exactly
 * (GpuPartitioning, and a FixedWidthRowSerializer as the dependency's serializer — its row
 * layout travels to the executors inside UcxGpuShuffleHandle) is written by GpuShuffleWriter;
 * any other keeps Spark's writer, and the resolver adopts its committed data file into the
 * node's HBM.  Reduce side: UcxShuffleReader fetches through the node, after the node-wide
 * exchange the driver's GpuExchangeCoordinator starts on every executor as map tasks finish.  The driver's metadata table of the reference
 * (registerShuffleCommon, CommonUcxShuffleManager.scala:39-56) becomes each node's directory,
 * sized by the number of MAP tasks (the reference sizes it by partitioner.numPartitions, quirk
 * Q1, and its PUTs overrun the table when maps outnumber reduces).
 */
package org.apache.spark.shuffle

import java.util.concurrent.ConcurrentHashMap

import scala.collection.JavaConverters._

import org.apache.spark.{ShuffleDependency, SparkConf, SparkEnv, TaskContext}
import org.apache.spark.internal.Logging
import org.apache.spark.shuffle.api.ShuffleExecutorComponents
import org.apache.spark.shuffle.compat.spark_3_0.{UcxShuffleBlockResolver, UcxShuffleReader}
import org.apache.spark.shuffle.gpu.{FixedWidthRowSerializer, GpuCodec, GpuExchangeCoordinator,
  GpuNode, GpuPartitioning, GpuRowLayout, GpuShuffleWriter}
import org.apache.spark.shuffle.sort.SortShuffleManager
import org.apache.spark.shuffle.ucx.gpu.SuxNative
import org.apache.spark.util.ShutdownHookManager

/** Handle broadcast to the tasks: Spark's handle + what the node needs to register the shuffle:
 * the map count (directory slots) and, for a GPU shuffle, the row layout (a serializable POD, the
 * analog of the reference's UcxRemoteMemory in UcxShuffleHandle, CommonUcxShuffleManager.scala:99-102). */
class UcxGpuShuffleHandle[K, V, C](shuffleId: Int, val numMaps: Int,
                                   val layout: Option[GpuRowLayout],
                                   val baseHandle: BaseShuffleHandle[K, V, C])
  extends ShuffleHandle(shuffleId) {
  /** The node's record size for this shuffle (4: byte-stream data files of Spark's writers). */
  def recordSize: Int = layout.map(_.recordSize).getOrElse(4)
}

class UcxShuffleManager(val conf: SparkConf, isDriver: Boolean) extends SortShuffleManager(conf)
  with Logging {

  ShutdownHookManager.addShutdownHook(Int.MaxValue - 1)(() => stop())
  // Spark builds this manager inside SparkEnv.create, before SparkEnv.set: nothing here may need
  // SparkEnv.  The driver sets up the group's control endpoint from the plugin's driver
  // components or its first registerShuffle; an executor of a group joins in the background once
  // its SparkEnv exists (so it is in every exchange even without tasks); a lone GPU starts its
  // node with the first task, through the executor components, as the reference does.
  if (!isDriver && conf.getInt("spark.shuffle.ucx.gpu.worldSize", 1) > 1) {
    GpuNode.joinInBackground(conf, isDriver)
  }

  // compat/spark_3_0/UcxShuffleManager.scala:21,46,49,63-72 of the reference: the executor's
  // ShuffleDataIO components, initialised the first time a writer is asked for — initializeExecutor
  // starts the node (UcxLocalDiskShuffleExecutorComponents), so getWriter works on an executor
  // that has done nothing else.  Spark 3.0 initialises them nowhere else on an executor.
  private lazy val shuffleExecutorComponents: ShuffleExecutorComponents = {
    val components = ShuffleDataIOUtils.loadShuffleDataIO(conf).executor()
    val extraConfigs = conf.getAllWithPrefix(ShuffleDataIOUtils.SHUFFLE_SPARK_CONF_PREFIX).toMap
    components.initializeExecutor(conf.getAppId, SparkEnv.get.executorId, extraConfigs.asJava)
    components
  }

  override val shuffleBlockResolver = new UcxShuffleBlockResolver(conf)

  private val partitioners = new ConcurrentHashMap[Int, java.lang.Long]()

  def startUcxNodeIfMissing(): GpuNode = GpuNode.startIfMissing(conf, isDriver)

  override def registerShuffle[K, V, C](shuffleId: Int,
                                        dependency: ShuffleDependency[K, V, C]): ShuffleHandle = {
    val base = super.registerShuffle(shuffleId, dependency).asInstanceOf[BaseShuffleHandle[K, V, C]]
    val numMaps = dependency.rdd.partitions.length  // Q1: slots per MAP task
    // the row layout is a property of the dependency's serializer, so it exists when Spark calls
    // this from the ShuffleDependency constructor (before any id-keyed registration could)
    val layout = dependency.serializer match {
      case s: FixedWidthRowSerializer[_, _] => Some(s.layout)
      case _ => None
    }
    val handle = new UcxGpuShuffleHandle(shuffleId, numMaps, layout, base)
    if (isDriver) {
      GpuNode.setupDriver(conf)  // SparkEnv is set by now (a no-op for a lone GPU)
      GpuExchangeCoordinator.watch(conf, shuffleId, numMaps, dependency.partitioner.numPartitions,
        handle.recordSize)
    }
    handle
  }

  /** The executor's node learns a shuffle on its first task (register is idempotent here). */
  private def ensureRegistered(h: UcxGpuShuffleHandle[_, _, _], node: GpuNode): Unit =
    node.ensureRegistered(h.shuffleId, h.numMaps, h.baseHandle.dependency.partitioner.numPartitions,
      h.recordSize)

  override def getWriter[K, V](handle: ShuffleHandle, mapId: Long, context: TaskContext,
                               metrics: ShuffleWriteMetricsReporter): ShuffleWriter[K, V] = {
    val h = handle.asInstanceOf[UcxGpuShuffleHandle[K, V, _]]
    shuffleExecutorComponents  // Spark's SPI init; ours starts the node (initializeExecutor)
    val node = startUcxNodeIfMissing()  // and whatever plugin class is configured, so does this
    node.checkTaskDevice()
    ensureRegistered(h, node)
    val dep = h.baseHandle.dependency
    // the GPU writes only what Spark's writer would: fixed-width rows, a partitioner it restates,
    // and a codec it restates byte for byte (GpuCodec: none, or lz4 under spark.shuffle.compress)
    val rows = dep.serializer match {
      case s: FixedWidthRowSerializer[_, _] if h.layout.isDefined && GpuCodec.of(conf).isDefined =>
        Some(s.asInstanceOf[FixedWidthRowSerializer[K, V]].rows)
      case _ => None
    }
    val gpu = rows.flatMap(r =>
      GpuPartitioning.of(dep.partitioner, r.keyLen, dep.keyClassName).map(r -> _))
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
    node.checkTaskDevice()
    ensureRegistered(h, node)
    // shouldBatchFetch = true, as the reference's getReader passes (compat/spark_3_0/
    // UcxShuffleManager.scala:53-60); the reader applies fetchContinuousBlocksInBatch's guard
    new UcxShuffleReader[K, C](h, node, startPartition, endPartition, context, metrics,
      shouldBatchFetch = true)
  }

  override def unregisterShuffle(shuffleId: Int): Boolean = {
    Option(GpuNodeOrNull()).foreach(_.unregister(shuffleId))
    Option(partitioners.remove(shuffleId)).foreach(p => SuxNative.partitionerDestroy(p))
    if (isDriver) GpuExchangeCoordinator.forget(shuffleId)
    super.unregisterShuffle(shuffleId)
  }

  override def stop(): Unit = synchronized {
    Option(GpuNodeOrNull()).foreach(n => n.registeredShuffles.foreach(id => unregisterShuffle(id)))
    GpuNode.stop()
    super.stop()
  }

  private def GpuNodeOrNull(): GpuNode =
    try GpuNode.get catch { case _: IllegalStateException => null }
}
