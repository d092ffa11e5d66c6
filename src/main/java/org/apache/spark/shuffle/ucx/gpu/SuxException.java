/*
 * SuxException — a failed libsparkucx_amd call: the SUX_E* status and the library's message.
 * A RuntimeException, as org.openucx.jucx.UcxException is in the reference.
 */
package org.apache.spark.shuffle.ucx.gpu;

public class SuxException extends RuntimeException {
  private final int code;

  public SuxException(int code, String message) {
    super(message);
    this.code = code;
  }

  public int code() {
    return code;
  }

  /** True when the block was not found here (SUX_ENOENT): Spark should see a fetch failure. */
  public boolean isMissingBlock() {
    return code == SuxNative.ENOENT;
  }
}
