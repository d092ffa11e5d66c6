/*
 * sux_jni.c — JNI binding of libsparkucx_amd.so for the JVM plugin classes
 * (org.apache.spark.shuffle.ucx.gpu.SuxNative, src/main/java/.../gpu/SuxNative.java).
 *
 * Every native method of SuxNative is one function here and calls the C-ABI of
 * include/sparkucx_amd.h; nothing else.  Conventions:
 *   - handles (sux_node*, sux_partitioner*, sux_buffer*, hipStream_t) travel as jlong;
 *   - a negative SUX_E* status becomes a thrown org.apache.spark.shuffle.ucx.gpu.SuxException
 *     (RuntimeException, like org.openucx.jucx.UcxException in the reference) carrying the code
 *     and sux_last_error(); the caller (UcxShuffleClient) turns fetch errors into
 *     BlockFetchingListener.onBlockFetchFailure, which the reference never calls;
 *   - host byte ranges come in as direct ByteBuffers (GetDirectBufferAddress, no copy): Spark's
 *     serializer output, an mmapped data file, or a reducer's staging buffer;
 *   - the bootstrap all-gather calls back into a Java object (GpuNode's control plane over
 *     Spark RPC) on the thread that called exchange().
 *
 * Build (needs a JDK, absent from this image): src/main/native/Makefile.
 */
#define _POSIX_C_SOURCE 200809L /* O_CLOEXEC, mmap */
#include <fcntl.h>
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../../include/sparkucx_amd.h"

#define SUX_JNI_CLASS "org/apache/spark/shuffle/ucx/gpu/SuxNative"
#define SUX_EXC_CLASS "org/apache/spark/shuffle/ucx/gpu/SuxException"
#define FN(name) Java_org_apache_spark_shuffle_ucx_gpu_SuxNative_##name

/* ---- errors ------------------------------------------------------------------------------ */
static void throw_sux(JNIEnv* env, int rc, const char* what) {
  char msg[2048];
  char err[1792];
  sux_last_error(err, sizeof err);
  snprintf(msg, sizeof msg, "%s: %s", what, err);
  jclass cls = (*env)->FindClass(env, SUX_EXC_CLASS);
  if (!cls) return; /* NoClassDefFoundError already pending */
  jmethodID ctor = (*env)->GetMethodID(env, cls, "<init>", "(ILjava/lang/String;)V");
  if (!ctor) return;
  jstring js = (*env)->NewStringUTF(env, msg);
  jthrowable t = (jthrowable)(*env)->NewObject(env, cls, ctor, (jint)rc, js);
  if (t) (*env)->Throw(env, t);
}

/* returns non-zero (and leaves an exception pending) when rc is an error */
static int failed(JNIEnv* env, int rc, const char* what) {
  if (rc == SUX_OK) return 0;
  throw_sux(env, rc, what);
  return 1;
}

static void* direct(JNIEnv* env, jobject buf, jlong need, const char* what) {
  if (!buf) {
    throw_sux(env, SUX_EINVAL, what);
    return NULL;
  }
  void* p = (*env)->GetDirectBufferAddress(env, buf);
  jlong cap = (*env)->GetDirectBufferCapacity(env, buf);
  if (!p || cap < need) {
    char m[256];
    snprintf(m, sizeof m, "%s: a direct ByteBuffer of >= %lld bytes is required", what,
             (long long)need);
    (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/IllegalArgumentException"), m);
    return NULL;
  }
  return p;
}

#define NODE(h) ((sux_node*)(intptr_t)(h))
#define PART(h) ((sux_partitioner*)(intptr_t)(h))
#define BUF(h) ((sux_buffer*)(intptr_t)(h))
#define STREAM(h) ((void*)(intptr_t)(h))

/* ---- node: UcxNode ctor / close (UcxNode.java:60-96, :194-221) ---------------------------- */
JNIEXPORT jint JNICALL FN(abiVersion)(JNIEnv* env, jclass cls) {
  (void)env;
  (void)cls;
  return sux_abi_version();
}

JNIEXPORT jbyteArray JNICALL FN(commUniqueId)(JNIEnv* env, jclass cls) {
  (void)cls;
  uint8_t id[128];
  if (failed(env, sux_comm_unique_id(id), "commUniqueId")) return NULL;
  jbyteArray out = (*env)->NewByteArray(env, 128);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, 128, (const jbyte*)id);
  return out;
}

JNIEXPORT jlong JNICALL FN(nodeCreate)(JNIEnv* env, jclass cls, jint device, jint rank,
                                       jint worldSize, jbyteArray commId, jlong minBufferSize,
                                       jlong minAllocationSize, jlong metadataBlockSize,
                                       jstring preAllocateBuffers, jint poolLimitMiB,
                                       jboolean isDriver) {
  (void)cls;
  sux_conf c;
  sux_conf_init(&c);
  c.device = device;
  c.rank = rank;
  c.world_size = worldSize;
  c.min_buffer_size = (uint64_t)minBufferSize;
  c.min_allocation_size = (uint64_t)minAllocationSize;
  c.metadata_block_size = (uint64_t)metadataBlockSize;
  c.pool_limit_mib = poolLimitMiB > 0 ? (uint32_t)poolLimitMiB : 0u;
  if (commId) {
    if ((*env)->GetArrayLength(env, commId) != 128) {
      throw_sux(env, SUX_EINVAL, "nodeCreate: the RCCL unique id is 128 bytes");
      return 0;
    }
    (*env)->GetByteArrayRegion(env, commId, 0, 128, (jbyte*)c.comm_id);
  }
  if (preAllocateBuffers) {
    const char* spec = (*env)->GetStringUTFChars(env, preAllocateBuffers, NULL);
    int rc = sux_conf_set_prealloc(&c, spec);
    (*env)->ReleaseStringUTFChars(env, preAllocateBuffers, spec);
    if (failed(env, rc, "spark.shuffle.ucx.memory.preAllocateBuffers")) return 0;
  }
  sux_node* n = NULL;
  if (failed(env, sux_node_create(&c, isDriver ? 1 : 0, &n), "UcxNode")) return 0;
  return (jlong)(intptr_t)n;
}

JNIEXPORT void JNICALL FN(nodeDestroy)(JNIEnv* env, jclass cls, jlong node) {
  (void)cls;
  failed(env, sux_node_destroy(NODE(node)), "UcxNode.close");
}

/* Bootstrap: the node calls back into Bootstrap.allGather(long tag, byte[]) -> byte[]
 * (world * bytes; the tag names the collective, see sux_allgather_fn). */
typedef struct {
  JavaVM* vm;
  jobject target; /* global ref to an org.apache.spark.shuffle.ucx.gpu.Bootstrap */
  jmethodID all_gather;
  jint world;     /* the node's group size: the reply must be exactly world * bytes */
} boot_ctx;

static int boot_allgather(void* vctx, uint64_t tag, const void* send, uint64_t bytes, void* recv) {
  boot_ctx* b = (boot_ctx*)vctx;
  JNIEnv* env = NULL;
  int attached = 0;
  if ((*b->vm)->GetEnv(b->vm, (void**)&env, JNI_VERSION_1_8) != JNI_OK) {
    if ((*b->vm)->AttachCurrentThread(b->vm, (void**)&env, NULL) != JNI_OK) return -1;
    attached = 1;
  }
  int rc = -1;
  jbyteArray in = (*env)->NewByteArray(env, (jsize)bytes);
  if (in) {
    (*env)->SetByteArrayRegion(env, in, 0, (jsize)bytes, (const jbyte*)send);
    jbyteArray out =
        (jbyteArray)(*env)->CallObjectMethod(env, b->target, b->all_gather, (jlong)tag, in);
    if (!(*env)->ExceptionCheck(env) && out) {
      /* recv holds exactly world * bytes: any other reply (a contribution of another size, a
       * round matched with the wrong collective) is an error, never a longer copy */
      const jsize n = (*env)->GetArrayLength(env, out);
      if ((uint64_t)n == (uint64_t)b->world * bytes) {
        (*env)->GetByteArrayRegion(env, out, 0, n, (jbyte*)recv);
        rc = 0;
      }
    }
    if ((*env)->ExceptionCheck(env)) (*env)->ExceptionClear(env); /* reported as SUX_ECOMM */
  }
  if (attached) (*b->vm)->DetachCurrentThread(b->vm);
  return rc;
}

JNIEXPORT jlong JNICALL FN(setBootstrap)(JNIEnv* env, jclass cls, jlong node, jobject bootstrap,
                                         jint worldSize) {
  (void)cls;
  if (worldSize < 1) {
    throw_sux(env, SUX_EINVAL, "setBootstrap: world size must be >= 1");
    return 0;
  }
  boot_ctx* b = (boot_ctx*)calloc(1, sizeof *b);
  if (!b) {
    throw_sux(env, SUX_ENOMEM, "setBootstrap");
    return 0;
  }
  (*env)->GetJavaVM(env, &b->vm);
  b->target = (*env)->NewGlobalRef(env, bootstrap);
  b->world = worldSize;
  jclass bc = (*env)->GetObjectClass(env, bootstrap);
  b->all_gather = (*env)->GetMethodID(env, bc, "allGather", "(J[B)[B");
  if (!b->all_gather || failed(env, sux_node_set_bootstrap(NODE(node), boot_allgather, b),
                               "setBootstrap")) {
    (*env)->DeleteGlobalRef(env, b->target);
    free(b);
    return 0;
  }
  return (jlong)(intptr_t)b; /* freed by releaseBootstrap after nodeDestroy */
}

/* The group's RCCL communicator, joined on the exchange thread (sux_node_connect: rank 0's
 * unique id through the bootstrap above, then ncclCommInitRank) */
JNIEXPORT void JNICALL FN(nodeConnect)(JNIEnv* env, jclass cls, jlong node) {
  (void)cls;
  failed(env, sux_node_connect(NODE(node)), "nodeConnect");
}

JNIEXPORT void JNICALL FN(releaseBootstrap)(JNIEnv* env, jclass cls, jlong ctx) {
  (void)cls;
  boot_ctx* b = (boot_ctx*)(intptr_t)ctx;
  if (!b) return;
  (*env)->DeleteGlobalRef(env, b->target);
  free(b);
}

/* ---- executor group membership, on the driver (GpuControlEndpoint's Hello) ----------------- */
JNIEXPORT jlong JNICALL FN(groupCreate)(JNIEnv* env, jclass cls, jint worldSize) {
  (void)cls;
  sux_group* g = NULL;
  if (failed(env, sux_group_create(worldSize, &g), "groupCreate")) return 0;
  return (jlong)(intptr_t)g;
}

JNIEXPORT void JNICALL FN(groupDestroy)(JNIEnv* env, jclass cls, jlong group) {
  (void)cls;
  failed(env, sux_group_destroy((sux_group*)(intptr_t)group), "groupDestroy");
}

/* {rank, localIndex} of an executor (a repeated hello of the same id gets the same pair). */
JNIEXPORT jintArray JNICALL FN(groupJoin)(JNIEnv* env, jclass cls, jlong group,
                                          jstring executorId, jstring host) {
  (void)cls;
  if (!executorId || !host) {
    throw_sux(env, SUX_EINVAL, "groupJoin: executor id and host are required");
    return NULL;
  }
  const char* id = (*env)->GetStringUTFChars(env, executorId, NULL);
  const char* h = (*env)->GetStringUTFChars(env, host, NULL);
  int32_t v[2] = {-1, -1};
  int rc = sux_group_join((sux_group*)(intptr_t)group, id, h, &v[0], &v[1]);
  (*env)->ReleaseStringUTFChars(env, host, h);
  (*env)->ReleaseStringUTFChars(env, executorId, id);
  if (failed(env, rc, "groupJoin")) return NULL;
  jintArray out = (*env)->NewIntArray(env, 2);
  if (out) (*env)->SetIntArrayRegion(env, out, 0, 2, (const jint*)v);
  return out;
}

/* HBM-capacity fallback: spill committed map outputs to Spark's files under spark.local.dir. */
JNIEXPORT void JNICALL FN(setSpillDir)(JNIEnv* env, jclass cls, jlong node, jstring dir) {
  (void)cls;
  const char* d = dir ? (*env)->GetStringUTFChars(env, dir, NULL) : NULL;
  int rc = sux_node_set_spill_dir(NODE(node), d);
  if (d) (*env)->ReleaseStringUTFChars(env, dir, d);
  failed(env, rc, "setSpillDir");
}

JNIEXPORT jlong JNICALL FN(spills)(JNIEnv* env, jclass cls, jlong node) {
  (void)cls;
  uint64_t v = 0;
  if (failed(env, sux_node_spills(NODE(node), &v), "spills")) return 0;
  return (jlong)v;
}

JNIEXPORT jlongArray JNICALL FN(poolStats)(JNIEnv* env, jclass cls, jlong node) {
  (void)cls;
  uint64_t v[4] = {0, 0, 0, 0};
  if (failed(env, sux_pool_stats(NODE(node), &v[0], &v[1], &v[2], &v[3]), "poolStats")) return NULL;
  jlongArray out = (*env)->NewLongArray(env, 4);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, 4, (const jlong*)v);
  return out;
}

/* ---- kernel tuning table (sux_tuning) and the device error word ------------------------------
 * fields[] in the header's field order (hist_kernel .. split_cus); 0 keeps the default. */
#define SUX_TUNING_FIELDS ((int)(sizeof(sux_tuning) / sizeof(int32_t)) - 1)
JNIEXPORT void JNICALL FN(setTuning)(JNIEnv* env, jclass cls, jlong node, jintArray fields) {
  (void)cls;
  sux_tuning t;
  memset(&t, 0, sizeof t);
  const jsize n = fields ? (*env)->GetArrayLength(env, fields) : 0;
  if (n > SUX_TUNING_FIELDS) {
    throw_sux(env, SUX_EINVAL, "setTuning: more fields than sux_tuning has");
    return;
  }
  if (n) (*env)->GetIntArrayRegion(env, fields, 0, n, (jint*)&t);
  failed(env, sux_node_set_tuning(NODE(node), &t), "setTuning");
}

JNIEXPORT jintArray JNICALL FN(getTuning)(JNIEnv* env, jclass cls, jlong node) {
  (void)cls;
  sux_tuning t;
  if (failed(env, sux_node_get_tuning(NODE(node), &t), "getTuning")) return NULL;
  jintArray out = (*env)->NewIntArray(env, SUX_TUNING_FIELDS);
  if (out) (*env)->SetIntArrayRegion(env, out, 0, SUX_TUNING_FIELDS, (const jint*)&t);
  return out;
}

JNIEXPORT void JNICALL FN(nodeCheck)(JNIEnv* env, jclass cls, jlong node) {
  (void)cls;
  failed(env, sux_node_check(NODE(node)), "nodeCheck");
}

/* ---- per-task-thread stream (UcxNode.getThreadLocalWorker, UcxNode.java:147-176) --------- */
JNIEXPORT jlong JNICALL FN(streamCreate)(JNIEnv* env, jclass cls, jlong node) {
  (void)cls;
  void* s = NULL;
  /* complement of 0 reserved CUs = an ordinary stream on every CU */
  if (failed(env, sux_stream_create(NODE(node), 0, 1, &s), "streamCreate")) return 0;
  return (jlong)(intptr_t)s;
}

JNIEXPORT void JNICALL FN(streamDestroy)(JNIEnv* env, jclass cls, jlong node, jlong stream) {
  (void)cls;
  failed(env, sux_stream_destroy(NODE(node), STREAM(stream)), "streamDestroy");
}

/* ---- partitioner (the dependency's Partitioner, P1) --------------------------------------- */
JNIEXPORT jlong JNICALL FN(partitionerCreate)(JNIEnv* env, jclass cls, jlong node, jint kind,
                                              jint numPartitions, jint keyOffset, jint keyLen,
                                              jint seed, jboolean ascending,
                                              jbyteArray rangeBounds) {
  (void)cls;
  sux_partitioner_desc d;
  memset(&d, 0, sizeof d);
  d.kind = kind;
  d.num_partitions = numPartitions;
  d.key_offset = keyOffset;
  d.key_len = keyLen;
  d.seed = seed;
  d.ascending = ascending ? 1 : 0;
  jbyte* b = NULL;
  if (rangeBounds) {
    b = (*env)->GetByteArrayElements(env, rangeBounds, NULL);
    d.range_bounds = (const uint8_t*)b;
  }
  sux_partitioner* p = NULL;
  int rc = sux_partitioner_create(NODE(node), &d, &p);
  if (b) (*env)->ReleaseByteArrayElements(env, rangeBounds, b, JNI_ABORT);
  if (failed(env, rc, "partitioner")) return 0;
  return (jlong)(intptr_t)p;
}

JNIEXPORT void JNICALL FN(partitionerDestroy)(JNIEnv* env, jclass cls, jlong part) {
  (void)cls;
  failed(env, sux_partitioner_destroy(PART(part)), "partitionerDestroy");
}

/* ---- shuffle lifecycle (CommonUcxShuffleManager.scala:39-91) ------------------------------ */
JNIEXPORT jlong JNICALL FN(registerShuffle)(JNIEnv* env, jclass cls, jlong node, jint shuffleId,
                                            jint numMaps, jint numPartitions, jint recordSize) {
  (void)cls;
  sux_handle_desc h;
  if (failed(env, sux_register_shuffle(NODE(node), shuffleId, numMaps, numPartitions, recordSize, &h),
             "registerShuffle"))
    return 0;
  return (jlong)h.directory_bytes;
}

JNIEXPORT void JNICALL FN(unregisterShuffle)(JNIEnv* env, jclass cls, jlong node, jint shuffleId) {
  (void)cls;
  failed(env, sux_unregister_shuffle(NODE(node), shuffleId), "unregisterShuffle");
}

/* ---- map side (getWriter(...).write + writeIndexFileAndCommit) ----------------------------- */
JNIEXPORT void JNICALL FN(writeMapOutputHost)(JNIEnv* env, jclass cls, jlong node, jint shuffleId,
                                              jint mapIndex, jlong part, jobject records,
                                              jlong numRecords, jint recordSize, jlong stream) {
  (void)cls;
  void* p = direct(env, records, numRecords * (jlong)recordSize, "writeMapOutputHost");
  if (!p && numRecords) return;
  failed(env, sux_write_map_output_host(NODE(node), shuffleId, mapIndex, PART(part), p,
                                        (uint64_t)numRecords, STREAM(stream)),
         "ShuffleWriter.write");
}

/* The same from a raw host address (records of any size: a staging area the writer grew past
 * the 2 GiB a ByteBuffer can hold, Platform.allocateMemory / UnsafeUtils.mmap addresses). */
JNIEXPORT void JNICALL FN(writeMapOutputHostAddr)(JNIEnv* env, jclass cls, jlong node,
                                                  jint shuffleId, jint mapIndex, jlong part,
                                                  jlong hostAddr, jlong numRecords,
                                                  jlong stream) {
  (void)cls;
  if (numRecords < 0 || (numRecords > 0 && hostAddr == 0)) {
    throw_sux(env, SUX_EINVAL, "writeMapOutputHostAddr: bad address or record count");
    return;
  }
  failed(env, sux_write_map_output_host(NODE(node), shuffleId, mapIndex, PART(part),
                                        (const void*)(intptr_t)hostAddr, (uint64_t)numRecords,
                                        STREAM(stream)),
         "ShuffleWriter.write");
}

JNIEXPORT void JNICALL FN(writeMapOutputs)(JNIEnv* env, jclass cls, jlong node, jint shuffleId,
                                           jint firstMapIndex, jlong part, jlong deviceRecords,
                                           jlong recordsPerMap, jlong numRecords, jlong stream) {
  (void)cls;
  failed(env, sux_write_map_outputs(NODE(node), shuffleId, firstMapIndex, PART(part),
                                    (const void*)(intptr_t)deviceRecords, (uint64_t)recordsPerMap,
                                    (uint64_t)numRecords, STREAM(stream)),
         "writeMapOutputs");
}

JNIEXPORT void JNICALL FN(waitMapOutputs)(JNIEnv* env, jclass cls, jlong node, jint shuffleId) {
  (void)cls;
  failed(env, sux_wait_map_outputs(NODE(node), shuffleId), "waitMapOutputs");
}

JNIEXPORT void JNICALL FN(commitMapOutput)(JNIEnv* env, jclass cls, jlong node, jint shuffleId,
                                           jint mapIndex, jobject data, jlong dataBytes,
                                           jlongArray lengths, jlong stream) {
  (void)cls;
  void* p = dataBytes ? direct(env, data, dataBytes, "writeIndexFileAndCommit") : NULL;
  if (!p && dataBytes) return;
  jlong* len = (*env)->GetLongArrayElements(env, lengths, NULL);
  int rc = sux_commit_map_output(NODE(node), shuffleId, mapIndex, p, (uint64_t)dataBytes,
                                 (const int64_t*)len, STREAM(stream));
  (*env)->ReleaseLongArrayElements(env, lengths, len, JNI_ABORT);
  failed(env, rc, "writeIndexFileAndCommit");
}

/* writeIndexFileAndCommit of a data file of any size, by address: Spark's committed file
 * mapped past FileChannel.map's 2 GiB limit (the reference's UnsafeUtils.mmap,
 * UnsafeUtils.java:48-57, used at CommonUcxShuffleBlockResolver.scala:45-52). */
JNIEXPORT void JNICALL FN(commitMapOutputAddr)(JNIEnv* env, jclass cls, jlong node,
                                               jint shuffleId, jint mapIndex, jlong dataAddr,
                                               jlong dataBytes, jlongArray lengths, jlong stream) {
  (void)cls;
  if (dataBytes < 0 || (dataBytes > 0 && dataAddr == 0) || !lengths) {
    throw_sux(env, SUX_EINVAL, "commitMapOutputAddr: bad address, size or lengths");
    return;
  }
  jlong* len = (*env)->GetLongArrayElements(env, lengths, NULL);
  int rc = sux_commit_map_output(NODE(node), shuffleId, mapIndex, (const void*)(intptr_t)dataAddr,
                                 (uint64_t)dataBytes, (const int64_t*)len, STREAM(stream));
  (*env)->ReleaseLongArrayElements(env, lengths, len, JNI_ABORT);
  failed(env, rc, "writeIndexFileAndCommit");
}

/* writeIndexFileAndCommit of Spark's committed data file by path: mapped here (any size — the
 * reference maps files past 2 GiB through FileChannelImpl.map0, UnsafeUtils.java:48-57), adopted
 * into the node's HBM (sux_commit_map_output copies it before returning) and unmapped. */
JNIEXPORT void JNICALL FN(commitMapOutputFile)(JNIEnv* env, jclass cls, jlong node,
                                               jint shuffleId, jint mapIndex, jstring dataPath,
                                               jlongArray lengths, jlong stream) {
  (void)cls;
  if (!dataPath || !lengths) {
    throw_sux(env, SUX_EINVAL, "commitMapOutputFile: path and lengths are required");
    return;
  }
  const char* path = (*env)->GetStringUTFChars(env, dataPath, NULL);
  char what[512];
  snprintf(what, sizeof what, "writeIndexFileAndCommit(%s)", path);
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  (*env)->ReleaseStringUTFChars(env, dataPath, path);
  struct stat st;
  if (fd < 0 || fstat(fd, &st) != 0) {
    if (fd >= 0) close(fd);
    throw_sux(env, SUX_EIO, what);
    return;
  }
  void* p = NULL;
  if (st.st_size > 0) {
    p = mmap(NULL, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);
    if (p == MAP_FAILED) {
      close(fd);
      throw_sux(env, SUX_EIO, what);
      return;
    }
  }
  jlong* len = (*env)->GetLongArrayElements(env, lengths, NULL);
  int rc = sux_commit_map_output(NODE(node), shuffleId, mapIndex, p, (uint64_t)st.st_size,
                                 (const int64_t*)len, STREAM(stream));
  (*env)->ReleaseLongArrayElements(env, lengths, len, JNI_ABORT);
  if (p) munmap(p, (size_t)st.st_size);
  close(fd);
  failed(env, rc, what);
}

JNIEXPORT jbyteArray JNICALL FN(mapOutputIndex)(JNIEnv* env, jclass cls, jlong node,
                                                jint shuffleId, jint mapIndex, jint numPartitions) {
  (void)cls;
  const jsize n = 8 * (numPartitions + 1);
  uint8_t* tmp = (uint8_t*)malloc((size_t)n);
  if (!tmp) {
    throw_sux(env, SUX_ENOMEM, "mapOutputIndex");
    return NULL;
  }
  int rc = sux_map_output_index(NODE(node), shuffleId, mapIndex, tmp, (uint64_t)n);
  jbyteArray out = NULL;
  if (!failed(env, rc, "mapOutputIndex")) {
    out = (*env)->NewByteArray(env, n);
    if (out) (*env)->SetByteArrayRegion(env, out, 0, n, (const jbyte*)tmp);
  }
  free(tmp);
  return out;
}

/* spark.shuffle.compress for the maps this node writes (GpuShuffleWriter): SUX_CODEC_LZ4 with
 * spark.io.compression.lz4.blockSize, or SUX_CODEC_NONE; before the shuffle's first map output. */
JNIEXPORT void JNICALL FN(setShuffleCodec)(JNIEnv* env, jclass cls, jlong node, jint shuffleId,
                                           jint codec, jint blockSize) {
  (void)cls;
  failed(env, sux_shuffle_set_codec(NODE(node), shuffleId, codec, blockSize), "setShuffleCodec");
}

/* ---- exchange (the all-to-all that replaces the reducers' remote GETs) -------------------- */
JNIEXPORT void JNICALL FN(exchange)(JNIEnv* env, jclass cls, jlong node, jint shuffleId,
                                    jlong stream) {
  (void)cls;
  failed(env, sux_exchange(NODE(node), shuffleId, STREAM(stream)), "exchange");
}

/* The exchange of one window of map tasks, asynchronous (stream-ordered), and its completion. */
JNIEXPORT void JNICALL FN(exchangeMaps)(JNIEnv* env, jclass cls, jlong node, jint shuffleId,
                                        jint firstMap, jint numMaps, jlong stream) {
  (void)cls;
  failed(env, sux_exchange_maps(NODE(node), shuffleId, firstMap, numMaps, STREAM(stream)),
         "exchangeMaps");
}

JNIEXPORT void JNICALL FN(exchangeWait)(JNIEnv* env, jclass cls, jlong node, jint shuffleId) {
  (void)cls;
  failed(env, sux_exchange_wait(NODE(node), shuffleId), "exchangeWait");
}

JNIEXPORT jintArray JNICALL FN(ownedPartitions)(JNIEnv* env, jclass cls, jlong node,
                                                jint shuffleId, jint rank) {
  (void)cls;
  int32_t se[2];
  if (failed(env, sux_owned_partitions(NODE(node), shuffleId, rank, &se[0], &se[1]),
             "ownedPartitions"))
    return NULL;
  jintArray out = (*env)->NewIntArray(env, 2);
  if (out) (*env)->SetIntArrayRegion(env, out, 0, 2, (const jint*)se);
  return out;
}

/* ---- fetch: UcxShuffleClient.fetchBlocks (reducer/compat/spark_3_0/UcxShuffleClient.java:94) */
/* blocks = {mapIndex, startReduce, endReduce} triples; sizes[i] <- bytes of block i; returns
 * the pooled buffer (one reference per block, OnBlocksFetchCallback.java:35-53). */
JNIEXPORT jlong JNICALL FN(fetchBlocks)(JNIEnv* env, jclass cls, jlong node, jint shuffleId,
                                        jintArray blocks, jlongArray sizes, jlong stream) {
  (void)cls;
  const jsize n3 = (*env)->GetArrayLength(env, blocks);
  if (n3 % 3 != 0 || (*env)->GetArrayLength(env, sizes) < n3 / 3) {
    throw_sux(env, SUX_EINVAL, "fetchBlocks: blocks are (map, start, end) triples");
    return 0;
  }
  const int32_t n = n3 / 3;
  sux_block_id* ids = (sux_block_id*)calloc((size_t)(n ? n : 1), sizeof *ids);
  int64_t* sz = (int64_t*)calloc((size_t)(n ? n : 1), sizeof *sz);
  jint* b = (*env)->GetIntArrayElements(env, blocks, NULL);
  if (!ids || !sz || !b) {
    free(ids);
    free(sz);
    if (b) (*env)->ReleaseIntArrayElements(env, blocks, b, JNI_ABORT);
    throw_sux(env, SUX_ENOMEM, "fetchBlocks");
    return 0;
  }
  for (int32_t i = 0; i < n; ++i) {
    ids[i].map_index = b[3 * i];
    ids[i].start_reduce = b[3 * i + 1];
    ids[i].end_reduce = b[3 * i + 2];
  }
  (*env)->ReleaseIntArrayElements(env, blocks, b, JNI_ABORT);
  sux_buffer* out = NULL;
  int rc = sux_fetch_blocks(NODE(node), shuffleId, ids, n, sz, &out, STREAM(stream));
  if (rc == SUX_OK) (*env)->SetLongArrayRegion(env, sizes, 0, n, (const jlong*)sz);
  free(ids);
  free(sz);
  if (failed(env, rc, "fetchBlocks")) return 0;
  return (jlong)(intptr_t)out;
}

/* The reader's key sort on the GPU (the ExternalSorter step, UcxShuffleReader.scala:138-154 in
 * the reference): `n` fixed-size records of a fetched buffer -> a new pooled buffer in ascending
 * key order, stable (sux_sort_records); the workspace is a pooled buffer released here. */
JNIEXPORT jlong JNICALL FN(sortRecords)(JNIEnv* env, jclass cls, jlong node, jint keyKind,
                                        jlong buf, jlong n, jint recordSize, jint keyOffset,
                                        jint keyLen, jlong stream) {
  (void)cls;
  void* src = NULL;
  uint64_t size = 0;
  if (failed(env, sux_buffer_info(BUF(buf), &src, &size, NULL), "sortRecords")) return 0;
  if ((uint64_t)n * (uint64_t)recordSize > size) {
    throw_sux(env, SUX_EINVAL, "sortRecords: the buffer holds fewer records");
    return 0;
  }
  uint64_t ws_bytes = 0;
  if (failed(env, sux_sort_workspace_size((uint64_t)n, (uint32_t)recordSize, &ws_bytes),
             "sortRecords"))
    return 0;
  sux_buffer* out = NULL;
  sux_buffer* ws = NULL;
  if (failed(env, sux_buffer_alloc(NODE(node), (uint64_t)n * (uint64_t)recordSize, &out),
             "sortRecords"))
    return 0;
  if (failed(env, sux_buffer_alloc(NODE(node), ws_bytes, &ws), "sortRecords")) {
    sux_buffer_release(out);
    return 0;
  }
  void* dst = NULL;
  void* w = NULL;
  sux_buffer_info(out, &dst, NULL, NULL);
  sux_buffer_info(ws, &w, NULL, NULL);
  int rc = sux_sort_records(NODE(node), keyKind, src, (uint64_t)n, (uint32_t)recordSize,
                            keyOffset, keyLen, dst, w, ws_bytes, STREAM(stream));
  /* the workspace may go back to the pool only after the stream ran the sort (release does not
   * wait): a one-byte read-back synchronises the stream */
  if (rc == SUX_OK && n > 0) {
    uint8_t first;
    rc = sux_buffer_read(out, 0, &first, 1, STREAM(stream));
  }
  sux_buffer_release(ws);
  if (failed(env, rc, "sortRecords")) {
    sux_buffer_release(out);
    return 0;
  }
  return (jlong)(intptr_t)out;
}

/* The reader's GPU sort of a compressed shuffle: the fetched blocks (sizes[i] bytes each,
 * consecutive from `offset` in the pooled buffer) decoded as LZ4Block streams into a new pooled
 * buffer (sux_buffer_decompress); outSizes[i] <- block i's decoded bytes.  A corrupted stream is
 * SuxException(EIO), the IOException Spark's LZ4BlockInputStream throws. */
JNIEXPORT jlong JNICALL FN(decompressBuffer)(JNIEnv* env, jclass cls, jlong node, jlong buf,
                                             jlong offset, jlongArray sizes, jint maxBlockSize,
                                             jlongArray outSizes, jlong stream) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, sizes);
  if (outSizes && (*env)->GetArrayLength(env, outSizes) < n) {
    throw_sux(env, SUX_EINVAL, "decompressBuffer: outSizes is shorter than sizes");
    return 0;
  }
  int64_t* os = (int64_t*)calloc((size_t)(n ? n : 1), sizeof *os);
  jlong* sz = (*env)->GetLongArrayElements(env, sizes, NULL);
  if (!os || !sz) {
    free(os);
    if (sz) (*env)->ReleaseLongArrayElements(env, sizes, sz, JNI_ABORT);
    throw_sux(env, SUX_ENOMEM, "decompressBuffer");
    return 0;
  }
  sux_buffer* out = NULL;
  int rc = sux_buffer_decompress(NODE(node), BUF(buf), (uint64_t)offset, (const int64_t*)sz, n,
                                 maxBlockSize, &out, os, STREAM(stream));
  (*env)->ReleaseLongArrayElements(env, sizes, sz, JNI_ABORT);
  if (rc == SUX_OK && outSizes) (*env)->SetLongArrayRegion(env, outSizes, 0, n, (const jlong*)os);
  free(os);
  if (failed(env, rc, "decompressBuffer")) return 0;
  return (jlong)(intptr_t)out;
}

JNIEXPORT jlong JNICALL FN(bufferDevicePtr)(JNIEnv* env, jclass cls, jlong buf) {
  (void)cls;
  void* p = NULL;
  if (failed(env, sux_buffer_info(BUF(buf), &p, NULL, NULL), "bufferDevicePtr")) return 0;
  return (jlong)(intptr_t)p;
}

JNIEXPORT void JNICALL FN(bufferRead)(JNIEnv* env, jclass cls, jlong buf, jlong offset,
                                      jobject dst, jlong len, jlong stream) {
  (void)cls;
  void* p = direct(env, dst, len, "bufferRead");
  if (!p && len) return;
  failed(env, sux_buffer_read(BUF(buf), (uint64_t)offset, p, (uint64_t)len, STREAM(stream)),
         "ManagedBuffer.nioByteBuffer");
}

JNIEXPORT void JNICALL FN(bufferRetain)(JNIEnv* env, jclass cls, jlong buf, jint count) {
  (void)cls;
  failed(env, sux_buffer_retain(BUF(buf), count), "ManagedBuffer.retain");
}

JNIEXPORT void JNICALL FN(bufferRelease)(JNIEnv* env, jclass cls, jlong buf) {
  (void)cls;
  failed(env, sux_buffer_release(BUF(buf)), "ManagedBuffer.release");
}

/* ---- Spark's on-disk files (local-disk fallback / external shuffle service) -------------- */
JNIEXPORT jboolean JNICALL FN(indexFileCommit)(JNIEnv* env, jclass cls, jstring indexPath,
                                               jstring dataPath, jstring dataTmp,
                                               jlongArray lengths, jlongArray lengthsOut) {
  (void)cls;
  const char* ip = (*env)->GetStringUTFChars(env, indexPath, NULL);
  const char* dp = (*env)->GetStringUTFChars(env, dataPath, NULL);
  const char* tp = dataTmp ? (*env)->GetStringUTFChars(env, dataTmp, NULL) : NULL;
  const jsize R = (*env)->GetArrayLength(env, lengths);
  jlong* len = (*env)->GetLongArrayElements(env, lengths, NULL);
  jlong* out = lengthsOut ? (*env)->GetLongArrayElements(env, lengthsOut, NULL) : NULL;
  int32_t reused = 0;
  int rc = sux_index_file_commit(ip, dp, tp, (const int64_t*)len, R, (int64_t*)out, &reused);
  if (out) (*env)->ReleaseLongArrayElements(env, lengthsOut, out, rc == SUX_OK ? 0 : JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, lengths, len, JNI_ABORT);
  if (tp) (*env)->ReleaseStringUTFChars(env, dataTmp, tp);
  (*env)->ReleaseStringUTFChars(env, dataPath, dp);
  (*env)->ReleaseStringUTFChars(env, indexPath, ip);
  if (failed(env, rc, "writeIndexFileAndCommit")) return JNI_FALSE;
  return reused ? JNI_TRUE : JNI_FALSE;
}
