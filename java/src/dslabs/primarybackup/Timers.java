package dslabs.primarybackup;

import dslabs.framework.Timer;
import lombok.Data;

/* lab2 timers (DESIGN.md §12) as the reference stub declares them
 * (labs/lab2-primarybackup/src/dslabs/primarybackup/Timers.java: Lombok @Data), the client's with
 * this solution's field. */

/** The ViewServer's liveness check, re-set on every fire (device: type 9, 100 ms). */
@Data
final class PingCheckTimer implements Timer {
  static final int PING_CHECK_MILLIS = 100;
}

/** A server's ping to the ViewServer, re-set on every fire (device: type 10, 25 ms). */
@Data
final class PingTimer implements Timer {
  static final int PING_MILLIS = 25;
}

/** A client's retry of its command `seq` (device: type 11, 100 ms, head of the client's queue). */
@Data
final class ClientTimer implements Timer {
  static final int CLIENT_RETRY_MILLIS = 100;
  private final int seq;
}
