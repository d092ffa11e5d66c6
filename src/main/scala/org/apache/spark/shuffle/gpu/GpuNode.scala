/*
 * GpuNode — the executor's (or driver's) handle on libsparkucx_amd: the process singleton the
 * reference calls UcxNode (UcxNode.java:60-96), started lazily and closed at stop().
 *
 *  - configuration: the reference's spark.shuffle.ucx.* keys (UcxShuffleConf.scala:17-90) plus
 *    spark.shuffle.ucx.gpu.* (size of the node's exchange group, transport, pool cap, exchange
 *    window).  Every executor of a group reads the SAME conf: its rank comes from the driver
 *    (Hello -> Welcome, in order of first arrival, keyed by executor id: sux_group), the way the
 *    reference's executors introduce themselves with their BlockManagerId and the driver fans
 *    them out (UcxNode.java:111-145, RpcConnectionCallback.java:47-89); its GPU is the task's
 *    Spark-assigned "gpu" resource (spark.executor.resource.gpu.*), else its local index on the
 *    host (executors of one host take devices 0, 1, ... in join order);
 *  - one HIP stream per task thread, the analog of getThreadLocalWorker (:147-176);
 *  - the exchange group's control plane over Spark RPC through the driver (GpuControlEndpoint):
 *    a host all-gather matched by tag, which replaces the UCX tag messages of the reference's
 *    bootstrap, and the driver -> executor messages of GpuExchangeCoordinator.  With
 *    spark.shuffle.ucx.gpu.transport = rccl (default) the node joins the group's RCCL
 *    communicator on its exchange thread, before its first exchange window (sux_node_connect:
 *    rank 0's unique id through that all-gather, then ncclCommInitRank); with ipc the exchange
 *    pulls blocks over HIP IPC (several executors on one GPU);
 *  - lifecycle (the reference's: UcxShuffleManager.scala:21,46,49,63-72 and
 *    UcxWorkerWrapper.getConnection, UcxWorkerWrapper.scala:129-152): starting a node never waits
 *    for the other executors — Hello -> rank (the driver answers at once), node, bootstrap, then
 *    Ready; the driver relays exchange messages to an executor only after its Ready, replaying
 *    the ones it missed; the one group-wide wait (the communicator) runs on the exchange thread.
 *    An executor of a group starts its node in the background as soon as its SparkEnv exists
 *    (UcxShuffleManager), so it joins every exchange even if it never runs a task; any map task
 *    starts it too, through the executor components (getWriter), as in the reference;
 *  - the exchange: a collective over the group, so it is not run by whichever reduce task comes
 *    first (an executor without reduce tasks would never join it) but by every executor when the
 *    driver's coordinator says so — window by window as map tasks finish, the last when the map
 *    stage completes — on one exchange thread per node; reduce tasks wait for it.
 */
package org.apache.spark.shuffle.gpu

import java.util.concurrent.{ConcurrentHashMap, Executors, ThreadFactory, TimeUnit}

import scala.collection.mutable
import scala.concurrent.{Await, Promise}
import scala.concurrent.duration.Duration

import org.apache.spark.{SparkConf, SparkContext, SparkEnv, TaskContext, Success => TaskSuccess}
import org.apache.spark.internal.Logging
import org.apache.spark.network.util.JavaUtils
import org.apache.spark.rpc.{RpcCallContext, RpcEndpointRef, RpcEnv, ThreadSafeRpcEndpoint}
import org.apache.spark.scheduler.{SparkListener, SparkListenerStageCompleted,
  SparkListenerStageSubmitted, SparkListenerTaskEnd}
import org.apache.spark.shuffle.ucx.gpu.{Bootstrap, SuxNative}
import org.apache.spark.util.{RpcUtils, Utils}

/** `undo`: what the constructor acquired so far, released in reverse by GpuNode.startIfMissing if
 * a later step throws (ADVICE r05: a failed join used to leave its executor endpoint registered —
 * so every retry failed in setupEndpoint — and leak the node). */
class GpuNode private (conf: SparkConf, isDriver: Boolean, undo: mutable.ArrayBuffer[() => Unit])
  extends Logging {
  private def ucx(k: String) = "spark.shuffle.ucx." + k
  private def bytes(k: String, dflt: String): Long = JavaUtils.byteStringAsBytes(conf.get(k, dflt))

  val worldSize: Int = conf.getInt(ucx("gpu.worldSize"), 1)
  private val transport: String = conf.get(ucx("gpu.transport"), "rccl")
  require(transport == "rccl" || transport == "ipc",
    s"spark.shuffle.ucx.gpu.transport must be rccl or ipc, not $transport")
  private val member = worldSize > 1 && !isDriver

  // executors of a group register with the driver's control endpoint (which also relays the
  // coordinator's messages to them) and learn their rank from its reply.  The executor endpoint
  // holds every message it gets until the node is built (ready(), the constructor's last step);
  // the driver relays nothing to this executor before its Ready anyway (ADVICE r04).
  private val (rank0, localIndex, myEndpoint) =
    if (member) {
      val env = SparkEnv.get
      val ep = new GpuExecutorEndpoint(env.rpcEnv)
      val me = env.rpcEnv.setupEndpoint(GpuControlEndpoint.EXECUTOR + env.executorId, ep)
      undo += (() => env.rpcEnv.stop(me))
      val w = GpuControlEndpoint.driverRef(conf, env.rpcEnv)
        .askSync[GpuControlEndpoint.Welcome](
          GpuControlEndpoint.Hello(env.executorId, Utils.localHostName(), worldSize, me))
      (w.rank, w.localIndex, Some((ep, me)))
    } else (0, 0, None)
  val rank: Int = rank0

  // spark.shuffle.ucx.gpu.device pins it; else the task's "gpu" resource (Spark 3.0 resource
  // scheduling) when the node starts inside a task; else the executor's local index on its host.
  // A node started by the background join has no task: its device is checked against the first
  // task's gpu resource (checkTaskDevice) — a mismatch fails loudly instead of letting two
  // executors share a GPU or a task hand the node pointers on another device (ADVICE r05).
  val device: Int =
    if (conf.contains(ucx("gpu.device"))) conf.getInt(ucx("gpu.device"), 0)
    else GpuNode.taskGpu().getOrElse(localIndex)
  private val deviceFromTask = conf.contains(ucx("gpu.device")) || GpuNode.taskGpu().isDefined

  /** The running task's Spark "gpu" resource must be this node's device (see `device`). */
  def checkTaskDevice(): Unit = if (!deviceFromTask) {
    GpuNode.taskGpu().foreach { g =>
      if (g != device) {
        throw new IllegalStateException(s"this executor's GPU shuffle node runs on device " +
          s"$device (its local index, chosen when it joined the group before any task ran) but " +
          s"Spark assigned GPU $g to this task: set spark.shuffle.ucx.gpu.device, or give each " +
          "executor exactly one visible GPU")
      }
    }
  }

  // UcxShuffleConf.scala:32-40: the directory slot is 2 * rkeySize
  val metadataBlockSize: Long = 2 * bytes(ucx("rkeySize"), "150")
  // :74-81: a bare number is MiB
  val minAllocationSize: Long = {
    val v = conf.get(ucx("memory.minAllocationSize"), "4")
    if (v.nonEmpty && v.last.isDigit) v.toLong << 20 else JavaUtils.byteStringAsBytes(v)
  }

  private val boot: Bootstrap = if (member) new RpcBootstrap(conf, rank, worldSize) else null

  // no communicator yet: the node is built without waiting for any other executor; rccl joins
  // the group's communicator on the exchange thread (connectOnce)
  private val handle0: Long = SuxNative.nodeCreate(device, rank, worldSize, null,
    bytes(ucx("memory.minBufferSize"), "1024"), minAllocationSize, metadataBlockSize,
    conf.get(ucx("memory.preAllocateBuffers"), ""), conf.getInt(ucx("gpu.poolLimitMiB"), 0),
    isDriver)
  undo += (() => SuxNative.nodeDestroy(handle0))

  private val bootCtx: Long =
    if (member) SuxNative.setBootstrap(handle0, boot, worldSize) else 0L
  if (bootCtx != 0L) undo.prepend(() => SuxNative.releaseBootstrap(bootCtx))  // after the node

  // HBM-capacity fallback: committed map outputs spill to Spark's files.  The directory is
  // private to this executor and application (a uniquely named subdirectory of the block
  // manager's first local dir, blockmgr-<uuid> under spark.local.dir), so executors and
  // applications sharing a host never overwrite or unlink each other's files; it is deleted
  // when the node stops.  (A node of a larger group never spills: its peers read its slabs.)
  private val spillDir: java.io.File =
    if (!isDriver) {
      val root = Option(SparkEnv.get).flatMap(e => Option(e.blockManager))
        .map(_.diskBlockManager.localDirs.head)
        .getOrElse(new java.io.File(System.getProperty("java.io.tmpdir")))
      val id = Option(SparkEnv.get).map(_.executorId).getOrElse("executor")
      val d = Utils.createDirectory(root.getAbsolutePath, s"sparkucx-gpu-${conf.getAppId}-$id")
      undo += (() => Utils.deleteRecursively(d))
      SuxNative.setSpillDir(handle0, d.getAbsolutePath)
      d
    } else null

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

  // ---- shuffles this node knows (registerShuffleCommon, CommonUcxShuffleManager.scala:39-56:
  // an executor learns a shuffle from its first task, or from the coordinator's first message)
  private val registered = ConcurrentHashMap.newKeySet[Int]()

  // spark.shuffle.compress for the maps this node writes (GpuCodec; None: Spark's writer writes
  // them, and its committed files are adopted as they are)
  private val codec: Option[(Int, Int)] = GpuCodec.of(conf)

  def ensureRegistered(shuffleId: Int, numMaps: Int, numPartitions: Int, recordSize: Int): Unit =
    registered.synchronized {
      if (!registered.contains(shuffleId)) {
        SuxNative.registerShuffle(handle0, shuffleId, numMaps, numPartitions, recordSize)
        codec.foreach { case (c, bs) => SuxNative.setShuffleCodec(handle0, shuffleId, c, bs) }
        registered.add(shuffleId)
      }
    }

  def unregister(shuffleId: Int): Unit = registered.synchronized {
    if (registered.remove(shuffleId)) SuxNative.unregisterShuffle(handle0, shuffleId)
    exchanges.remove(shuffleId)
  }

  def registeredShuffles: Seq[Int] = registered.toArray(Array.empty[Integer]).toSeq.map(_.intValue)

  // ---- the exchange --------------------------------------------------------------------------
  private val exchangeThread = Executors.newSingleThreadExecutor(new ThreadFactory {
    override def newThread(r: Runnable): Thread = {
      val t = new Thread(r, s"sparkucx-gpu-exchange-$rank")
      t.setDaemon(true)
      t
    }
  })
  undo += (() => exchangeThread.shutdownNow())
  private lazy val exchangeStream: Long = SuxNative.streamCreate(handle0)
  // exchange thread only: the group's RCCL communicator, joined before the first exchange
  // (every executor of the group gets the same first window, so every rank reaches it)
  private var connected = !(member && transport == "rccl")
  private def connectOnce(): Unit = if (!connected) {
    SuxNative.nodeConnect(handle0)
    connected = true
  }
  private val exchanges = new ConcurrentHashMap[Int, Promise[Unit]]()
  private def promiseOf(id: Int): Promise[Unit] = exchanges.computeIfAbsent(id, _ => Promise[Unit]())
  private val exchangeTimeout: Duration =
    Duration(conf.getTimeAsSeconds("spark.network.timeout", "120s"), TimeUnit.SECONDS)

  /** Map tasks [first, first + count) of a shuffle are committed on every executor: enqueue
   * their exchange (sux_exchange_maps; asynchronous on the exchange stream, so the next maps'
   * kernels keep running).  Driver messages reach every executor in the same order, so the
   * collective calls match. */
  def exchangeWindow(w: GpuControlEndpoint.ExchangeWindow): Unit =
    exchangeThread.execute(() => {
      try {
        ensureRegistered(w.shuffleId, w.numMaps, w.numPartitions, w.recordSize)
        connectOnce()
        SuxNative.exchangeMaps(handle0, w.shuffleId, w.first, w.count, exchangeStream)
      } catch { case e: Throwable => promiseOf(w.shuffleId).tryFailure(e) }
    })

  /** The map stage completed: finish the shuffle's exchange (sux_exchange_wait). */
  def exchangeDone(shuffleId: Int): Unit =
    exchangeThread.execute(() => {
      try {
        SuxNative.exchangeWait(handle0, shuffleId)
        promiseOf(shuffleId).trySuccess(())
      } catch { case e: Throwable => promiseOf(shuffleId).tryFailure(e) }
    })

  /** Reduce tasks wait for the exchange (a group of one GPU has nothing to exchange). */
  def awaitExchange(shuffleId: Int): Unit =
    if (worldSize > 1) Await.result(promiseOf(shuffleId).future, exchangeTimeout)

  // the node is built: deliver what the endpoint held, then tell the driver it may relay
  myEndpoint.foreach { case (ep, me) =>
    ep.ready(this)
    GpuControlEndpoint.driverRef(conf, SparkEnv.get.rpcEnv)
      .askSync[Boolean](GpuControlEndpoint.Ready(rank, me))
  }

  def close(): Unit = synchronized {
    exchangeThread.shutdown()
    exchangeThread.awaitTermination(10, TimeUnit.SECONDS)
    streams.values().forEach(s => SuxNative.streamDestroy(handle0, s))
    streams.clear()
    SuxNative.nodeDestroy(handle0)
    if (bootCtx != 0L) SuxNative.releaseBootstrap(bootCtx)
    if (spillDir != null) Utils.deleteRecursively(spillDir)
  }
}

object GpuNode extends Logging {
  @volatile private var instance: GpuNode = _
  /** The bootstrap all-gather of rank 0's RCCL unique id (SUX_TAG_COMM_ID, made by
   * sux_node_connect): outside every shuffle's tags ((shuffle id << 32) | count, ids >= 0). */
  val COMM_ID_TAG: Long = 0xFFFFFFFF00000000L

  /** CommonUcxShuffleManager.startUcxNodeIfMissing (:67-71): lazy and synchronized.  Needs
   * SparkEnv (an executor's endpoint, the block manager's dirs), so it is never called from a
   * ShuffleManager constructor: Spark builds the manager inside SparkEnv.create. */
  def startIfMissing(conf: SparkConf, isDriver: Boolean): GpuNode = synchronized {
    if (instance == null) {
      val undo = mutable.ArrayBuffer[() => Unit]()
      try instance = new GpuNode(conf, isDriver, undo)
      catch {
        case e: Throwable =>
          // a failed start leaves nothing behind, so the next attempt (the first task, after a
          // failed background join) starts from scratch
          undo.reverseIterator.foreach(f => try f() catch { case _: Throwable => })
          throw e
      }
    }
    instance
  }

  /** The running task's Spark-assigned GPU (spark.task.resource.gpu.amount), if any. */
  def taskGpu(): Option[Int] =
    Option(TaskContext.get()).flatMap(_.resources().get("gpu"))
      .flatMap(_.addresses.headOption).map(_.toInt)

  /** Driver: the group's control endpoint (idempotent; needs SparkEnv, see ensureSetup). */
  def setupDriver(conf: SparkConf): Unit = GpuControlEndpoint.ensureSetup(conf)

  /** An executor of a group joins it as soon as its SparkEnv exists, on a daemon thread, so that
   * it takes part in every exchange even if the scheduler never gives it a task (the exchange is
   * a collective over the group).  A failed join is logged and leaves nothing registered
   * (startIfMissing's undo); the first task retries it. */
  def joinInBackground(conf: SparkConf, isDriver: Boolean): Unit = {
    val t = new Thread(() => {
      try {
        val deadline = System.currentTimeMillis() +
          conf.getTimeAsMs("spark.network.timeout", "120s")
        while (SparkEnv.get == null && System.currentTimeMillis() < deadline) Thread.sleep(20)
        if (SparkEnv.get != null) startIfMissing(conf, isDriver)
      } catch {
        case e: Throwable => logWarning("GPU group join failed; the first task retries it", e)
      }
    }, "sparkucx-gpu-join")
    t.setDaemon(true)
    t.start()
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

/** Host all-gather through the driver endpoint: one ask per collective, answered when every rank
 * contributed to the same tag. */
private class RpcBootstrap(conf: SparkConf, rank: Int, world: Int) extends Bootstrap {
  private lazy val driver = RpcUtils.makeDriverRef(GpuControlEndpoint.NAME, conf, SparkEnv.get.rpcEnv)

  override def allGather(tag: Long, mine: Array[Byte]): Array[Byte] =
    driver.askSync[Array[Byte]](GpuControlEndpoint.Contribute(tag, rank, world, mine))
}

private[gpu] object GpuControlEndpoint {
  val NAME = "SparkUcxGpuControl"
  val EXECUTOR = "SparkUcxGpuExecutor-"
  case class Contribute(tag: Long, rank: Int, world: Int, bytes: Array[Byte])
  /** An executor joins the group: every executor sends the same conf's world size. */
  case class Hello(executorId: String, host: String, world: Int, ref: RpcEndpointRef)
  case class Welcome(rank: Int, localIndex: Int, world: Int)
  /** The executor's node is built: from now on the driver relays exchange messages to it,
   * starting with every relayed message it missed. */
  case class Ready(rank: Int, ref: RpcEndpointRef)
  /** Driver-internal: a shuffle's relayed messages leave the backlog. */
  case class Forget(shuffleId: Int)
  /** Map tasks [first, first + count) of a shuffle (numMaps / numPartitions / recordSize: what an
   * executor that ran none of its tasks needs to register it before the collective). */
  case class ExchangeWindow(shuffleId: Int, numMaps: Int, numPartitions: Int, recordSize: Int,
                            first: Int, count: Int)
  case class ExchangeDone(shuffleId: Int)

  @volatile private var endpoint: RpcEndpointRef = _

  /** Driver: the control endpoint, set up once SparkEnv exists — from the plugin's driver
   * components (ShuffleDriverComponents.initializeApplication, which SparkContext calls after
   * SparkEnv.set) or from the first registerShuffle, whichever comes first.  Never from the
   * ShuffleManager's constructor: SparkEnv.get is still null there. */
  def ensureSetup(conf: SparkConf): Unit = synchronized {
    val world = conf.getInt("spark.shuffle.ucx.gpu.worldSize", 1)
    if (endpoint == null && world > 1) {
      val env = SparkEnv.get
      require(env != null, "the GPU control endpoint needs the driver's SparkEnv")
      endpoint = env.rpcEnv.setupEndpoint(NAME, new GpuControlEndpoint(env.rpcEnv, world))
    }
  }

  /** Executor: the driver's endpoint, waiting for it to exist (an executor's background join
   * can start before the driver set it up), bounded by spark.network.timeout. */
  def driverRef(conf: SparkConf, rpcEnv: RpcEnv): RpcEndpointRef = {
    val deadline = System.currentTimeMillis() + conf.getTimeAsMs("spark.network.timeout", "120s")
    var ref: RpcEndpointRef = null
    while (ref == null) {
      try ref = RpcUtils.makeDriverRef(NAME, conf, rpcEnv)
      catch {
        case e: Exception =>
          if (System.currentTimeMillis() > deadline) throw e
          Thread.sleep(200)
      }
    }
    ref
  }

  /** Driver: relay a coordinator message to every executor of the group, in order. */
  def broadcast(msg: Any): Unit = Option(endpoint).foreach(_.send(msg))
}

private class GpuControlEndpoint(override val rpcEnv: RpcEnv, world: Int)
  extends ThreadSafeRpcEndpoint {
  import GpuControlEndpoint._
  private val pending = mutable.Map[Long, Array[(Array[Byte], RpcCallContext)]]()
  // executors that are Ready (null until then) and every relayed message of the live shuffles,
  // in order: a late executor gets the ones it missed before any new one
  private val executors = new Array[RpcEndpointRef](world)
  private val backlog = mutable.ArrayBuffer[Any]()
  // ranks by first arrival, keyed by executor id (sux_group: a repeated hello gets its rank back)
  private val group: Long = SuxNative.groupCreate(world)

  override def onStop(): Unit = SuxNative.groupDestroy(group)

  override def receive: PartialFunction[Any, Unit] = {
    case m @ (_: ExchangeWindow | _: ExchangeDone) =>
      backlog += m
      executors.filter(_ != null).foreach(_.send(m))
    case Forget(id) =>
      backlog --= backlog.filter {
        case w: ExchangeWindow => w.shuffleId == id
        case d: ExchangeDone => d.shuffleId == id
        case _ => false
      }
  }

  override def receiveAndReply(context: RpcCallContext): PartialFunction[Any, Unit] = {
    case Hello(executorId, host, w, ref) =>
      if (w != world) {
        context.sendFailure(new IllegalStateException(
          s"executor $executorId expects a GPU group of $w, the driver's is $world"))
      } else {
        try {
          val Array(rank, local) = SuxNative.groupJoin(group, executorId, host)
          context.reply(Welcome(rank, local, world))
        } catch { case e: Exception => context.sendFailure(e) }
      }
    case Ready(rank, ref) =>
      if (rank < 0 || rank >= world) {
        context.sendFailure(new IllegalStateException(s"Ready from rank $rank of $world"))
      } else {
        backlog.foreach(ref.send)
        executors(rank) = ref
        context.reply(true)
      }
    case Contribute(tag, rank, w, bytes) =>
      require(w == world, s"bootstrap: executor reports world $w, driver expects $world")
      val slots = pending.getOrElseUpdate(tag, new Array(world))
      require(slots(rank) == null, s"bootstrap: rank $rank contributed twice to collective $tag")
      slots(rank) = (bytes, context)
      if (slots.forall(_ != null)) {
        pending.remove(tag)
        if (slots.exists(_._1.length != bytes.length)) {  // ranks out of step: fail them all
          val e = new IllegalStateException(s"bootstrap: contributions of different sizes to $tag")
          slots.foreach(_._2.sendFailure(e))
        } else {
          val all = slots.flatMap(_._1)
          slots.foreach(_._2.reply(all))
        }
      }
  }
}

private class GpuExecutorEndpoint(override val rpcEnv: RpcEnv) extends ThreadSafeRpcEndpoint {
  import GpuControlEndpoint._
  // messages that arrive before the node is built wait here, in order (ThreadSafeRpcEndpoint:
  // receive and ready() never run at once, both synchronized on this endpoint)
  private var node: GpuNode = _
  private val held = mutable.ArrayBuffer[Any]()

  def ready(n: GpuNode): Unit = synchronized {
    node = n
    held.foreach(deliver)
    held.clear()
  }

  private def deliver(m: Any): Unit = m match {
    case w: ExchangeWindow => node.exchangeWindow(w)
    case ExchangeDone(id) => node.exchangeDone(id)
  }

  override def receive: PartialFunction[Any, Unit] = {
    case m @ (_: ExchangeWindow | _: ExchangeDone) =>
      synchronized { if (node == null) held += m else deliver(m) }
  }
}

/**
 * Driver side: starts each GPU shuffle's exchange on every executor.  With
 * spark.shuffle.ucx.gpu.exchangeWindowMaps = w > 0, window k (maps [k w, (k+1) w)) is exchanged
 * as soon as all its map tasks have succeeded, while later map tasks still run (the overlap of
 * the exchange with the next maps; receive memory per window is bounded like the reference's
 * maxBytesInFlight, UcxShuffleReader.scala:56-70); the remaining maps and the completion follow
 * the map stage's end.  w = 0: one exchange at the stage's end.
 */
object GpuExchangeCoordinator extends Logging {
  private case class Watch(numMaps: Int, numPartitions: Int, recordSize: Int, window: Int,
                           done: mutable.BitSet, var sent: Int) {
    def msg(id: Int, first: Int, count: Int) =
      GpuControlEndpoint.ExchangeWindow(id, numMaps, numPartitions, recordSize, first, count)
  }
  private val watched = new ConcurrentHashMap[Int, Watch]()
  private val stageShuffle = new ConcurrentHashMap[Int, Int]()
  @volatile private var listening = false

  def watch(conf: SparkConf, shuffleId: Int, numMaps: Int, numPartitions: Int,
            recordSize: Int): Unit = {
    if (conf.getInt("spark.shuffle.ucx.gpu.worldSize", 1) <= 1) return
    watched.put(shuffleId, Watch(numMaps, numPartitions, recordSize,
      conf.getInt("spark.shuffle.ucx.gpu.exchangeWindowMaps", 0), mutable.BitSet(), 0))
    synchronized {
      if (!listening) {
        SparkContext.getActive.foreach(_.addSparkListener(Listener))
        listening = true
      }
    }
  }

  def forget(shuffleId: Int): Unit = {
    watched.remove(shuffleId)
    GpuControlEndpoint.broadcast(GpuControlEndpoint.Forget(shuffleId))
  }

  private def advance(id: Int, w: Watch, stageDone: Boolean): Unit = w.synchronized {
    if (w.window > 0) {
      while (w.sent < w.numMaps && (w.sent until math.min(w.numMaps, w.sent + w.window)).forall(w.done)) {
        val n = math.min(w.window, w.numMaps - w.sent)
        GpuControlEndpoint.broadcast(w.msg(id, w.sent, n))
        w.sent += n
      }
    }
    if (stageDone) {
      if (w.sent < w.numMaps) {
        GpuControlEndpoint.broadcast(w.msg(id, w.sent, w.numMaps - w.sent))
        w.sent = w.numMaps
      }
      GpuControlEndpoint.broadcast(GpuControlEndpoint.ExchangeDone(id))
      logInfo(s"shuffle $id: exchange of ${w.numMaps} map outputs started on every executor")
    }
  }

  private object Listener extends SparkListener {
    override def onStageSubmitted(e: SparkListenerStageSubmitted): Unit =
      e.stageInfo.shuffleDepId.foreach(id => stageShuffle.put(e.stageInfo.stageId, id))

    // taskInfo.index is the task's index in its TaskSet, which equals the map (partition) index
    // only in a stage's first attempt: a resubmitted attempt holds just the missing partitions.
    // Later attempts therefore mark nothing; their maps are exchanged at the stage's end.
    override def onTaskEnd(e: SparkListenerTaskEnd): Unit =
      if (e.reason == TaskSuccess && e.stageAttemptId == 0) {
        Option(stageShuffle.get(e.stageId)).flatMap(id => Option(watched.get(id)).map(id -> _))
          .foreach { case (id, w) =>
            w.synchronized { w.done += e.taskInfo.index }
            advance(id, w, stageDone = false)
          }
      }

    override def onStageCompleted(e: SparkListenerStageCompleted): Unit =
      if (e.stageInfo.failureReason.isEmpty) {
        e.stageInfo.shuffleDepId.foreach { id =>
          Option(watched.get(id)).foreach(w => advance(id, w, stageDone = true))
        }
      }
  }
}
