/*
 * UcxShuffleClient — BlockStoreClient.fetchBlocks of the GPU plugin (Spark 3.0).
 *
 * The reference (this path in the reference tree) resolves each block in two RDMA rounds:
 * 16-byte offset pairs from the mapper's index file, then the block bytes into one pooled
 * buffer (UcxShuffleClient.java:50-127, OnOffsetsFetchCallback.java:44-92).  Here the map outputs
 * and their index tables live in the node's HBM (this executor's maps, or after the node-wide
 * exchange this rank's partitions of every map), so one sux_fetch_blocks call sizes every block
 * from the directory and gathers them into one pooled device buffer, in request order.  Blocks
 * are delivered as DeviceManagedBuffer slices (one pool reference each).  Unlike the reference,
 * a block that cannot be served reaches listener.onBlockFetchFailure, so Spark raises a
 * FetchFailedException and retries the stage instead of hanging.
 */
package org.apache.spark.shuffle.ucx.reducer.compat.spark_3_0;

import java.util.Map;

import org.apache.spark.executor.TempShuffleReadMetrics;
import org.apache.spark.network.shuffle.BlockFetchingListener;
import org.apache.spark.network.shuffle.BlockStoreClient;
import org.apache.spark.network.shuffle.DownloadFileManager;
import org.apache.spark.shuffle.gpu.GpuNode;
import org.apache.spark.shuffle.ucx.gpu.DeviceManagedBuffer;
import org.apache.spark.shuffle.ucx.gpu.SuxException;
import org.apache.spark.shuffle.ucx.gpu.SuxNative;
import org.apache.spark.storage.BlockId;
import org.apache.spark.storage.ShuffleBlockBatchId;
import org.apache.spark.storage.ShuffleBlockId;
import org.slf4j.Logger;
import org.slf4j.LoggerFactory;

public class UcxShuffleClient extends BlockStoreClient {
  private static final Logger logger = LoggerFactory.getLogger(UcxShuffleClient.class);
  private final int shuffleId;
  private final GpuNode node;
  private final Map<Long, Integer> mapId2PartitionId;
  private final TempShuffleReadMetrics shuffleReadMetrics;

  public UcxShuffleClient(int shuffleId, GpuNode node, Map<Long, Integer> mapId2PartitionId,
                          TempShuffleReadMetrics shuffleReadMetrics) {
    this.shuffleId = shuffleId;
    this.node = node;
    this.mapId2PartitionId = mapId2PartitionId;
    this.shuffleReadMetrics = shuffleReadMetrics;
  }

  @Override
  public void fetchBlocks(String host, int port, String execId, String[] blockIds,
                          BlockFetchingListener listener, DownloadFileManager downloadFileManager) {
    long startTime = System.currentTimeMillis();
    int[] triples = new int[3 * blockIds.length];
    int n = 0;
    String[] names = new String[blockIds.length];
    for (String name : blockIds) {
      BlockId id = BlockId.apply(name);
      long mapId;
      int start;
      int end;
      if (id instanceof ShuffleBlockId) {
        ShuffleBlockId b = (ShuffleBlockId) id;
        mapId = b.mapId();
        start = b.reduceId();
        end = start + 1;
      } else if (id instanceof ShuffleBlockBatchId) {  // a run of reduce ids of one map
        ShuffleBlockBatchId b = (ShuffleBlockBatchId) id;
        mapId = b.mapId();
        start = b.startReduceId();
        end = b.endReduceId();
      } else {
        listener.onBlockFetchFailure(name, new IllegalArgumentException("Unknown block " + name));
        continue;
      }
      Integer mapIndex = mapId2PartitionId.get(mapId);
      if (mapIndex == null) {
        listener.onBlockFetchFailure(name, new IllegalArgumentException(
            "no map index for map task " + mapId + " of shuffle " + shuffleId));
        continue;
      }
      triples[3 * n] = mapIndex;
      triples[3 * n + 1] = start;
      triples[3 * n + 2] = end;
      names[n++] = name;
    }
    if (n == 0) {
      return;
    }
    if (n < blockIds.length) {
      triples = java.util.Arrays.copyOf(triples, 3 * n);
    }
    long stream = node.threadStream();
    long[] sizes = new long[n];
    long buffer;
    try {
      buffer = SuxNative.fetchBlocks(node.handle(), shuffleId, triples, sizes, stream);
    } catch (SuxException e) {
      for (int i = 0; i < n; i++) {
        listener.onBlockFetchFailure(names[i], e);
      }
      return;
    }
    long offset = 0;
    long total = 0;
    for (int i = 0; i < n; i++) {  // one slice per block, in request order
      listener.onBlockFetchSuccess(names[i],
          new DeviceManagedBuffer(buffer, offset, sizes[i], stream));
      offset += sizes[i];
      total += sizes[i];
    }
    long ms = System.currentTimeMillis() - startTime;
    shuffleReadMetrics.incFetchWaitTime(ms);
    logger.debug("shuffle {}: fetched {} blocks, {} bytes in {} ms", shuffleId, n, total, ms);
  }

  @Override
  public void close() {
  }
}
