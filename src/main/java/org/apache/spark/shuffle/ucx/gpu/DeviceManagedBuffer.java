/*
 * DeviceManagedBuffer — one block of a fetch: a slice [offset, offset + size) of the pooled
 * device buffer sux_fetch_blocks filled.  Every block holds one reference of that buffer; the
 * last release() returns it to the node's pool — the refcounted NioManagedBuffer slices of
 * OnBlocksFetchCallback.java:33-57.  The bytes reach the JVM when Spark's stream reads them:
 * nioByteBuffer copies the slice to host memory once; createInputStream streams a block larger
 * than one chunk through a bounded direct buffer (a reduce block may pass the 2 GiB a ByteBuffer
 * holds, and the reader's memory stays bounded like the reference's maxBytesInFlight,
 * UcxShuffleReader.scala:56-70).
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

  /** Bytes a streamed block is staged in at a time. */
  static final int CHUNK = 8 << 20;

  @Override
  public InputStream createInputStream() throws IOException {
    synchronized (this) {
      if (host != null || size <= CHUNK) {
        return new NioManagedBuffer(nioByteBuffer()).createInputStream();
      }
    }
    return new DeviceInputStream();
  }

  /** The block read from the device chunk by chunk into one direct buffer. */
  private final class DeviceInputStream extends InputStream {
    private final ByteBuffer stage = ByteBuffer.allocateDirect(CHUNK);
    private long staged = 0;  // block bytes staged so far

    DeviceInputStream() {
      stage.limit(0);
    }

    private boolean fill() {
      if (stage.hasRemaining()) {
        return true;
      }
      if (staged >= size) {
        return false;
      }
      long len = Math.min(CHUNK, size - staged);
      stage.clear();
      SuxNative.bufferRead(buffer, offset + staged, stage, len, stream);  // at the buffer's start
      stage.limit((int) len);
      staged += len;
      return true;
    }

    @Override
    public int read() {
      return fill() ? stage.get() & 0xff : -1;
    }

    @Override
    public int read(byte[] b, int off, int len) {
      if (len == 0) {
        return 0;
      }
      if (!fill()) {
        return -1;
      }
      int n = Math.min(len, stage.remaining());
      stage.get(b, off, n);
      return n;
    }

    @Override
    public long skip(long n) {
      long done = 0;
      while (done < n && fill()) {
        int k = (int) Math.min(n - done, stage.remaining());
        stage.position(stage.position() + k);
        done += k;
      }
      return done;
    }

    @Override
    public int available() {
      return stage.remaining();
    }
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
