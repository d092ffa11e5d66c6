/*
 * GpuNode — the executor's (or driver's) handle on libsparkucx_amd: the process singleton the
 * reference calls UcxNode (UcxNode.java:60-96), started lazily and closed at stop().
 *
 *  - configuration: the reference's spark.shuffle.ucx.* keys (UcxShuffleConf.scala:17-90) plus
 *    spark.shuffle.ucx.gpu.* (device, rank and size of the node's exchange group);
 *  - one HIP stream per task thread, the analog of getThreadLocalWorker (:147-176);
 *  - the exchange group's control plane: an all-gather over Spark RPC through the driver
 *    (GpuBootstrapEndpoint), which replaces the UCX tag messages of the reference's bootstrap;
 *  - exchangeOnce: the node-wide all-to-all of a shuffle, run by the first reduce task of every
 *    executor (a collective: each executor of the group takes part once).
 */
package org.apache.spark.shuffle.gpu

import java.util.concurrent.ConcurrentHashMap

import scala.collection.mutable

import org.apache.spark.{SparkConf, SparkEnv}
import org.apache.spark.internal.Logging
import org.apache.spark.network.util.JavaUtils
import org.apache.spark.rpc.{RpcCallContext, RpcEnv, ThreadSafeRpcEndpoint}
import org.apache.spark.shuffle.ucx.gpu.{Bootstrap, SuxNative}
import org.apache.spark.util.RpcUtils

class GpuNode private (conf: SparkConf, isDriver: Boolean) extends Logging {
  private def ucx(k: String) = "spark.shuffle.ucx." + k
  private def bytes(k: String, dflt: String): Long = JavaUtils.byteStringAsBytes(conf.get(k, dflt))

  val device: Int = conf.getInt(ucx("gpu.device"), 0)
  val rank: Int = conf.getInt(ucx("gpu.rank"), 0)
  val worldSize: Int = conf.getInt(ucx("gpu.worldSize"), 1)
  // UcxShuffleConf.scala:32-40: the directory slot is 2 * rkeySize
  val metadataBlockSize: Long = 2 * bytes(ucx("rkeySize"), "150")
  // :74-81: a bare number is MiB
  val minAllocationSize: Long = {
    val v = conf.get(ucx("memory.minAllocationSize"), "4")
    if (v.nonEmpty && v.last.isDigit) v.toLong << 20 else JavaUtils.byteStringAsBytes(v)
  }

  private val handle0: Long = SuxNative.nodeCreate(device, rank, worldSize, null,
    bytes(ucx("memory.minBufferSize"), "1024"), minAllocationSize, metadataBlockSize,
    conf.get(ucx("memory.preAllocateBuffers"), ""), isDriver)

  private val bootCtx: Long =
    if (worldSize > 1 && !isDriver) SuxNative.setBootstrap(handle0, new RpcBootstrap(conf, rank, worldSize))
    else 0L

  // spark.shuffle.ucx.gpu.tuning.<field> = <int>: the node's kernel tuning table (sux_tuning);
  // unset fields keep the measured defaults
  locally {
    val fields = SuxNative.TUNING_FIELDS.map(f => conf.getInt(ucx("gpu.tuning." + f), 0))
    if (fields.exists(_ != 0)) SuxNative.setTuning(handle0, fields)
  }

  def handle: Long = handle0

  /** Device-side failures the kernels recorded (bounded waits that timed out). */
  def check(): Unit = SuxNative.nodeCheck(handle0)

  private val streams = new ConcurrentHashMap[Long, java.lang.Long]()
  private val threadStream = ThreadLocal.withInitial[java.lang.Long](() => {
    val s = SuxNative.streamCreate(handle0)
    streams.put(Thread.currentThread().getId, s)
    s
  })

  /** This task thread's stream (getThreadLocalWorker analog). */
  def threadStream(): Long = threadStream.get()

  private val exchanged = mutable.Set[Int]()

  /** The node-wide exchange of a shuffle, once per executor (the first reduce task runs it). */
  def exchangeOnce(shuffleId: Int): Unit = exchanged.synchronized {
    if (!exchanged.contains(shuffleId)) {
      val t0 = System.nanoTime()
      SuxNative.exchange(handle0, shuffleId, threadStream())
      exchanged += shuffleId
      logInfo(s"shuffle $shuffleId exchanged in ${(System.nanoTime() - t0) / 1e6} ms")
    }
  }

  def forget(shuffleId: Int): Unit = exchanged.synchronized { exchanged -= shuffleId }

  def close(): Unit = synchronized {
    streams.values().forEach(s => SuxNative.streamDestroy(handle0, s))
    streams.clear()
    SuxNative.nodeDestroy(handle0)
    if (bootCtx != 0L) SuxNative.releaseBootstrap(bootCtx)
  }
}

object GpuNode {
  @volatile private var instance: GpuNode = _

  /** CommonUcxShuffleManager.startUcxNodeIfMissing (:67-71): lazy and synchronized. */
  def startIfMissing(conf: SparkConf, isDriver: Boolean): GpuNode = synchronized {
    if (instance == null) {
      if (isDriver && conf.getInt("spark.shuffle.ucx.gpu.worldSize", 1) > 1) {
        GpuBootstrapEndpoint.setup(SparkEnv.get.rpcEnv, conf.getInt("spark.shuffle.ucx.gpu.worldSize", 1))
      }
      instance = new GpuNode(conf, isDriver)
    }
    instance
  }

  def get: GpuNode = {
    val n = instance
    if (n == null) {
      throw new IllegalStateException("Executor components must be initialized before getting writers.")
    }
    n
  }

  def stop(): Unit = synchronized {
    if (instance != null) {
      instance.close()
      instance = null
    }
  }
}

/** Host all-gather through the driver endpoint: one ask per round, answered when all ranks
 * of the round have arrived. */
private class RpcBootstrap(conf: SparkConf, rank: Int, world: Int) extends Bootstrap {
  private var round = 0L
  private lazy val driver = RpcUtils.makeDriverRef(GpuBootstrapEndpoint.NAME, conf, SparkEnv.get.rpcEnv)

  override def allGather(mine: Array[Byte]): Array[Byte] = synchronized {
    round += 1
    driver.askSync[Array[Byte]](GpuBootstrapEndpoint.Contribute(round, rank, world, mine))
  }
}

private[gpu] object GpuBootstrapEndpoint {
  val NAME = "SparkUcxGpuBootstrap"
  case class Contribute(round: Long, rank: Int, world: Int, bytes: Array[Byte])

  def setup(rpcEnv: RpcEnv, world: Int): Unit =
    rpcEnv.setupEndpoint(NAME, new GpuBootstrapEndpoint(rpcEnv, world))
}

private class GpuBootstrapEndpoint(override val rpcEnv: RpcEnv, world: Int)
  extends ThreadSafeRpcEndpoint {
  import GpuBootstrapEndpoint.Contribute
  private val pending = mutable.Map[Long, Array[(Array[Byte], RpcCallContext)]]()

  override def receiveAndReply(context: RpcCallContext): PartialFunction[Any, Unit] = {
    case Contribute(round, rank, w, bytes) =>
      require(w == world, s"bootstrap: executor reports world $w, driver expects $world")
      val slots = pending.getOrElseUpdate(round, new Array(world))
      slots(rank) = (bytes, context)
      if (slots.forall(_ != null)) {
        val all = slots.flatMap(_._1)
        slots.foreach(_._2.reply(all))
        pending.remove(round)
      }
  }
}
