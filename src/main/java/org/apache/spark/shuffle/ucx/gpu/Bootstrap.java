/*
 * Bootstrap — the control plane the node's exchange uses when no RCCL communicator spans the
 * executors: a host all-gather over Spark RPC.  It replaces the reference's UCX tag messages
 * through the driver (UcxNode.startExecutor, UcxNode.java:130-145; RpcConnectionCallback.java).
 */
package org.apache.spark.shuffle.ucx.gpu;

public interface Bootstrap {
  /**
   * Every executor of the node's group passes the same number of bytes under the same tag;
   * returns the concatenation of all contributions in rank order.  The tag names the collective
   * ((shuffle id << 32) | the shuffle's all-gather sequence number, equal on every executor), so
   * the control plane matches contributions by tag, never by arrival order.
   */
  byte[] allGather(long tag, byte[] mine);
}
