package dslabs.clientserver;

import dslabs.framework.Timer;
import lombok.Data;

/** Re-sends the client's command `sequenceNum` while it has no result (device: type 2, 100 ms). */
@Data
final class ClientTimer implements Timer {
  static final int CLIENT_RETRY_MILLIS = 100;

  private final int sequenceNum;
}
