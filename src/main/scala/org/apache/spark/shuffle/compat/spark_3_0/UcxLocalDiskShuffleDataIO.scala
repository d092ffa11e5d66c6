/*
 * The ShuffleDataIO plugin (spark.shuffle.sort.io.plugin.class).  Its driver components set up
 * the GPU group's control endpoint once SparkEnv exists; its executor components start
 * the executor's GPU node before the first writer exists (UcxShuffleManager.getWriter forces
 * them, as the reference's compat/spark_3_0/UcxShuffleManager.scala:21,46,49 does) and keep Spark's local-disk writers for
 * the dependencies the GPU writer does not take — their commit reaches UcxShuffleBlockResolver,
 * which adopts the committed file into HBM.  Asking for a writer before initializeExecutor throws
 * IllegalStateException, as the reference's components do.
 */
package org.apache.spark.shuffle.compat.spark_3_0

import java.util
import java.util.Optional

import org.apache.spark.{SparkConf, SparkEnv}
import org.apache.spark.shuffle.UcxShuffleManager
import org.apache.spark.shuffle.api.{ShuffleDriverComponents, ShuffleExecutorComponents, ShuffleMapOutputWriter, SingleSpillShuffleMapOutputWriter}
import org.apache.spark.shuffle.gpu.GpuNode
import org.apache.spark.shuffle.sort.io.{LocalDiskShuffleDataIO, LocalDiskShuffleDriverComponents, LocalDiskShuffleExecutorComponents, LocalDiskShuffleMapOutputWriter, LocalDiskSingleSpillMapOutputWriter}

case class UcxLocalDiskShuffleDataIO(sparkConf: SparkConf) extends LocalDiskShuffleDataIO(sparkConf) {
  override def executor(): ShuffleExecutorComponents = new UcxLocalDiskShuffleExecutorComponents(sparkConf)
  override def driver(): ShuffleDriverComponents = new UcxLocalDiskShuffleDriverComponents(sparkConf)
}

/** The driver's components: SparkContext calls initializeApplication after SparkEnv.set and
 * before any stage runs, the first point where the GPU group's control endpoint can exist
 * (executors that join earlier wait for it, GpuControlEndpoint.driverRef). */
class UcxLocalDiskShuffleDriverComponents(sparkConf: SparkConf)
  extends LocalDiskShuffleDriverComponents {
  override def initializeApplication(): util.Map[String, String] = {
    GpuNode.setupDriver(sparkConf)
    super.initializeApplication()
  }
}

class UcxLocalDiskShuffleExecutorComponents(sparkConf: SparkConf)
  extends LocalDiskShuffleExecutorComponents(sparkConf) {

  @volatile private var resolver: UcxShuffleBlockResolver = _

  override def initializeExecutor(appId: String, execId: String,
                                  extraConfigs: util.Map[String, String]): Unit = {
    val manager = SparkEnv.get.shuffleManager.asInstanceOf[UcxShuffleManager]
    manager.startUcxNodeIfMissing()
    resolver = manager.shuffleBlockResolver
  }

  private def initialized(): UcxShuffleBlockResolver = {
    val r = resolver
    if (r == null) {
      throw new IllegalStateException("Executor components must be initialized before getting writers.")
    }
    r
  }

  override def createMapOutputWriter(shuffleId: Int, mapTaskId: Long,
                                     numPartitions: Int): ShuffleMapOutputWriter =
    new LocalDiskShuffleMapOutputWriter(shuffleId, mapTaskId, numPartitions, initialized(), sparkConf)

  override def createSingleFileMapOutputWriter(shuffleId: Int,
                                               mapId: Long): Optional[SingleSpillShuffleMapOutputWriter] =
    Optional.of(new LocalDiskSingleSpillMapOutputWriter(shuffleId, mapId, initialized()))
}
