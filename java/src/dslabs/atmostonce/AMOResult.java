package dslabs.atmostonce;

import dslabs.framework.Result;
import lombok.Data;

/** The result of the client's command `sequenceNum` (the device's Reply: seq + 24-bit result). */
@Data
public final class AMOResult implements Result {
  private final Result result;
  private final int sequenceNum;
}
