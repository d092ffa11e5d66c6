/*
 * SuxNative — the JNI surface of libsparkucx_amd.so (include/sparkucx_amd.h), one static native
 * method per function of src/main/native/sux_jni.c.  Handles are longs; a failed call throws
 * SuxException carrying the SUX_E* code and the library's message.
 */
package org.apache.spark.shuffle.ucx.gpu;

import java.nio.ByteBuffer;

public final class SuxNative {
  private SuxNative() {}

  static {
    // libsparkucx_amd_jni.so links libsparkucx_amd.so (rpath $ORIGIN); both ship in the jar's
    // native directory or on java.library.path
    System.loadLibrary("sparkucx_amd_jni");
    if (abiVersion() != ABI_VERSION) {
      throw new UnsatisfiedLinkError("libsparkucx_amd ABI " + abiVersion() + ", plugin built for "
          + ABI_VERSION);
    }
  }

  public static final int ABI_VERSION = 6;

  // status codes (SUX_*)
  public static final int OK = 0, EINVAL = -1, ENOMEM = -2, EHIP = -3, ECOMM = -4, ENOENT = -5,
      ESTATE = -6, ERANGE = -7, EIO = -8;
  // partitioner kinds (SUX_PART_*)
  public static final int PART_RANGE_BYTES = 1, PART_MURMUR3_LONG = 2, PART_MURMUR3_INT = 3,
      PART_MURMUR3_BYTES = 4, PART_HASH_LONG = 5, PART_HASH_INT = 6;

  // ---- node (UcxNode) ----
  public static native int abiVersion();
  public static native byte[] commUniqueId();
  /** poolLimitMiB: spark.shuffle.ucx.gpu.poolLimitMiB (0 = no cap on the device pool). */
  public static native long nodeCreate(int device, int rank, int worldSize, byte[] commId,
                                       long minBufferSize, long minAllocationSize,
                                       long metadataBlockSize, String preAllocateBuffers,
                                       int poolLimitMiB, boolean isDriver);
  public static native void nodeDestroy(long node);
  /** Returns a context to pass to releaseBootstrap once the node is destroyed.  Every reply of
   * the bootstrap must be exactly worldSize * the contribution's bytes. */
  public static native long setBootstrap(long node, Bootstrap bootstrap, int worldSize);
  // ---- executor group membership (driver) ----
  /** One per application on the driver: ranks of a GPU group's executors (sux_group). */
  public static native long groupCreate(int worldSize);
  public static native void groupDestroy(long group);
  /** {rank, localIndex}: rank by first arrival, keyed by executor id; localIndex = executors of
   * the same host that joined earlier.  SuxException(ERANGE) once the group is complete. */
  public static native int[] groupJoin(long group, String executorId, String host);
  /** HBM-capacity fallback: committed map outputs spill to Spark's files under dir. */
  public static native void setSpillDir(long node, String dir);
  public static native long spills(long node);
  /** Join the group's RCCL communicator (a collective over the group: rank 0's unique id
   * through the node's bootstrap, then ncclCommInitRank); called on the exchange thread before
   * the first exchange window, so starting a node never waits for the other executors. */
  public static native void nodeConnect(long node);

  public static native void releaseBootstrap(long ctx);
  public static native long[] poolStats(long node);
  /** sux_tuning fields in header order (TUNING_FIELDS); 0 = the measured default. */
  public static native void setTuning(long node, int[] fields);
  public static native int[] getTuning(long node);
  /** Throws SuxException(EHIP) when a kernel recorded a failure in the device error word. */
  public static native void nodeCheck(long node);
  public static final String[] TUNING_FIELDS = {
      "hist_kernel", "scatter_kernel", "coresident", "scatter_chunk", "scatter_depth",
      "hist_stage", "s6_chunk", "tiles_per_item", "small_groups", "tile_records", "onepass",
      "varlen_kernel", "varlen_tile", "sort_max_digit_bits", "sort_gather", "sort_all_passes",
      "hist_wgs_per_cu", "small_kernel", "small_waves", "scatter_order",
      "small_wgs_per_cu", "sort_msd", "exchange_self", "hist_nt", "counts_layout",
      "scatter_counters", "lz4_queue", "scatter_nt", "gather_kernel", "split_cus", "msd_direct"};
  public static native long streamCreate(long node);
  public static native void streamDestroy(long node, long stream);

  // ---- partitioner ----
  public static native long partitionerCreate(long node, int kind, int numPartitions, int keyOffset,
                                              int keyLen, int seed, boolean ascending,
                                              byte[] rangeBounds);
  public static native void partitionerDestroy(long part);

  // ---- shuffle lifecycle ----
  /** Returns the directory bytes (num_maps * metadataBlockSize). */
  public static native long registerShuffle(long node, int shuffleId, int numMaps,
                                            int numPartitions, int recordSize);
  public static native void unregisterShuffle(long node, int shuffleId);

  // ---- map side ----
  public static native void writeMapOutputHost(long node, int shuffleId, int mapIndex, long part,
                                               ByteBuffer records, long numRecords, int recordSize,
                                               long stream);
  /** Records at a raw host address (a staging area of any size, no 2 GiB ByteBuffer limit). */
  public static native void writeMapOutputHostAddr(long node, int shuffleId, int mapIndex,
                                                   long part, long hostAddr, long numRecords,
                                                   long stream);
  public static native void writeMapOutputs(long node, int shuffleId, int firstMapIndex, long part,
                                            long deviceRecords, long recordsPerMap,
                                            long numRecords, long stream);
  public static native void waitMapOutputs(long node, int shuffleId);
  public static native void commitMapOutput(long node, int shuffleId, int mapIndex,
                                            ByteBuffer data, long dataBytes, long[] lengths,
                                            long stream);
  /** A committed data file of any size by address (mmapped past FileChannel.map's 2 GiB). */
  public static native void commitMapOutputAddr(long node, int shuffleId, int mapIndex,
                                                long dataAddr, long dataBytes, long[] lengths,
                                                long stream);
  /** Spark's committed data file by path, mapped natively (any size) and adopted. */
  public static native void commitMapOutputFile(long node, int shuffleId, int mapIndex,
                                                String dataPath, long[] lengths, long stream);
  public static native byte[] mapOutputIndex(long node, int shuffleId, int mapIndex,
                                             int numPartitions);
  /** spark.shuffle.compress for the maps the node writes (SUX_CODEC_*), before the first one. */
  public static native void setShuffleCodec(long node, int shuffleId, int codec, int blockSize);
  public static final int CODEC_NONE = 0, CODEC_LZ4 = 1;

  // ---- exchange ----
  public static native void exchange(long node, int shuffleId, long stream);
  /** Asynchronous exchange of map tasks [firstMap, firstMap + numMaps) (a collective). */
  public static native void exchangeMaps(long node, int shuffleId, int firstMap, int numMaps,
                                         long stream);
  /** Completes every exchange of the shuffle enqueued by this executor (a collective). */
  public static native void exchangeWait(long node, int shuffleId);
  public static native int[] ownedPartitions(long node, int shuffleId, int rank);

  // ---- fetch ----
  public static native long fetchBlocks(long node, int shuffleId, int[] blocks, long[] sizes,
                                        long stream);
  public static native long bufferDevicePtr(long buf);
  /** The fetched blocks' LZ4Block streams (sizes[i] bytes each from offset) decoded on the GPU
   * into a new buffer; outSizes[i] receives block i's decoded size.  EIO: a corrupted stream. */
  public static native long decompressBuffer(long node, long buf, long offset, long[] sizes,
                                             int maxBlockSize, long[] outSizes, long stream);
  /** Sort n fixed-size records of a fetched buffer by key on the GPU; returns a new buffer. */
  public static native long sortRecords(long node, int keyKind, long buf, long n, int recordSize,
                                        int keyOffset, int keyLen, long stream);
  public static final int SORT_BYTES = 1, SORT_LONG = 2, SORT_INT = 3;
  public static native void bufferRead(long buf, long offset, ByteBuffer dst, long len,
                                       long stream);
  public static native void bufferRetain(long buf, int count);
  public static native void bufferRelease(long buf);

  // ---- Spark's on-disk files ----
  public static native boolean indexFileCommit(String indexPath, String dataPath, String dataTmp,
                                               long[] lengths, long[] lengthsOut);
}
