/*
 * The ShuffleDataIO plugin (spark.shuffle.sort.io.plugin.class).  Its executor components start
 * the executor's GPU node before the first writer exists and keep Spark's local-disk writers for
 * the dependencies the GPU writer does not take — their commit reaches UcxShuffleBlockResolver,
 * which adopts the committed file into HBM.  Asking for a writer before initializeExecutor throws
 * IllegalStateException, as the reference's components do.
 */
package org.apache.spark.shuffle.compat.spark_3_0

import java.util
import java.util.Optional

import org.apache.spark.{SparkConf, SparkEnv}
import org.apache.spark.shuffle.UcxShuffleManager
import org.apache.spark.shuffle.api.{ShuffleExecutorComponents, ShuffleMapOutputWriter, SingleSpillShuffleMapOutputWriter}
import org.apache.spark.shuffle.sort.io.{LocalDiskShuffleDataIO, LocalDiskShuffleExecutorComponents, LocalDiskShuffleMapOutputWriter, LocalDiskSingleSpillMapOutputWriter}

case class UcxLocalDiskShuffleDataIO(sparkConf: SparkConf) extends LocalDiskShuffleDataIO(sparkConf) {
  override def executor(): ShuffleExecutorComponents = new UcxLocalDiskShuffleExecutorComponents(sparkConf)
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
