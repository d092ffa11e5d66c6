/*
 * UcxShuffleBlockResolver (Spark 3.0): writeIndexFileAndCommit for map outputs Spark's own
 * writers produced (dependencies the GPU writer does not take).  After Spark's commit (index
 * file + rename, IndexShuffleBlockResolver [ext]) the committed data file is mapped and adopted
 * into the node's HBM with its lengths (sux_commit_map_output), so the reduce side and the
 * node-wide exchange serve it like any GPU-written map.  The reference instead mmaps and
 * registers both files with UCX and PUTs a descriptor into the driver's table
 * (CommonUcxShuffleBlockResolver.scala:33-107); an empty data file publishes nothing (:42-45 of
 * the compat resolver), and the slot is TaskContext.getPartitionId (:38), as here.
 */
package org.apache.spark.shuffle.compat.spark_3_0

import java.io.File

import org.apache.spark.{SparkConf, TaskContext}
import org.apache.spark.shuffle.IndexShuffleBlockResolver
import org.apache.spark.shuffle.gpu.GpuNode
import org.apache.spark.shuffle.ucx.gpu.SuxNative

class UcxShuffleBlockResolver(conf: SparkConf) extends IndexShuffleBlockResolver(conf) {

  override def writeIndexFileAndCommit(shuffleId: Int, mapId: Long, lengths: Array[Long],
                                       dataTmp: File): Unit = {
    super.writeIndexFileAndCommit(shuffleId, mapId, lengths, dataTmp)
    val slot = TaskContext.getPartitionId()
    val file = getDataFile(shuffleId, mapId)
    if (file.length() == 0) return
    // the first commit of the map wins (another attempt's file has the same lengths)
    val committed = {
      val idx = new Array[Long](lengths.length)
      val index = getIndexFile(shuffleId, mapId)
      SuxNative.indexFileCommit(index.getPath, file.getPath, null, lengths, idx)
      idx
    }
    // the file is mapped natively, whatever its size: FileChannel.map stops at 2 GiB, which is
    // why the reference maps through FileChannelImpl.map0 (UnsafeUtils.mmap, UnsafeUtils.java:
    // 48-57, used at CommonUcxShuffleBlockResolver.scala:45-58)
    val node = GpuNode.get
    SuxNative.commitMapOutputFile(node.handle, shuffleId, slot, file.getPath, committed,
      node.threadStream())
  }
}
