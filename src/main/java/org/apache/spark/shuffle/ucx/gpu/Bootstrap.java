/*
 * Bootstrap — the control plane the node's exchange uses when no RCCL communicator spans the
 * executors: a host all-gather over Spark RPC.  It replaces the reference's UCX tag messages
 * through the driver (UcxNode.startExecutor, UcxNode.java:130-145; RpcConnectionCallback.java).
 */
package org.apache.spark.shuffle.ucx.gpu;

public interface Bootstrap {
  /**
   * Every executor of the node's group passes the same number of bytes; returns the
   * concatenation of all contributions in rank order.
   */
  byte[] allGather(byte[] mine);
}
