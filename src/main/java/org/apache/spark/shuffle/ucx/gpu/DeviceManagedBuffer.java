/*
 * DeviceManagedBuffer — one block of a fetch: a slice [offset, offset + size) of the pooled
 * device buffer sux_fetch_blocks filled.  Every block holds one reference of that buffer; the
 * last release() returns it to the node's pool — the refcounted NioManagedBuffer slices of
 * OnBlocksFetchCallback.java:33-57.  The bytes reach the JVM when Spark's stream reads them
 * (nioByteBuffer / createInputStream copy the slice to host memory once).
 */
package org.apache.spark.shuffle.ucx.gpu;

import java.io.IOException;
import java.io.InputStream;
import java.nio.ByteBuffer;

import io.netty.buffer.Unpooled;
import org.apache.spark.network.buffer.ManagedBuffer;
import org.apache.spark.network.buffer.NioManagedBuffer;

public final class DeviceManagedBuffer extends ManagedBuffer {
  private final long buffer;  // sux_buffer*
  private final long offset;
  private final long size;
  private final long stream;
  private ByteBuffer host;    // lazily read copy

  public DeviceManagedBuffer(long buffer, long offset, long size, long stream) {
    this.buffer = buffer;
    this.offset = offset;
    this.size = size;
    this.stream = stream;
  }

  /** The pooled sux_buffer this block is a slice of (a GPU consumer of several blocks). */
  public long bufferHandle() {
    return buffer;
  }

  /** Offset of the block in that buffer. */
  public long offset() {
    return offset;
  }

  /** Device address of the block (for a GPU consumer: no host copy at all). */
  public long devicePointer() {
    return SuxNative.bufferDevicePtr(buffer) + offset;
  }

  @Override
  public long size() {
    return size;
  }

  @Override
  public synchronized ByteBuffer nioByteBuffer() throws IOException {
    if (host == null) {
      if (size > Integer.MAX_VALUE) {
        throw new IOException("block of " + size + " bytes exceeds a ByteBuffer");
      }
      ByteBuffer b = ByteBuffer.allocateDirect((int) size);
      SuxNative.bufferRead(buffer, offset, b, size, stream);
      host = b;
    }
    return host.duplicate();
  }

  @Override
  public InputStream createInputStream() throws IOException {
    return new NioManagedBuffer(nioByteBuffer()).createInputStream();
  }

  @Override
  public ManagedBuffer retain() {
    SuxNative.bufferRetain(buffer, 1);
    return this;
  }

  @Override
  public ManagedBuffer release() {
    SuxNative.bufferRelease(buffer);
    return this;
  }

  @Override
  public Object convertToNetty() throws IOException {
    return Unpooled.wrappedBuffer(nioByteBuffer());
  }
}
