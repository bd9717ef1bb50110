package dslabs.primarybackup;

import dslabs.framework.Timer;

/* lab2 timers (DESIGN.md §12) as records, with the reference's names and periods
 * (labs/lab2-primarybackup/src/dslabs/primarybackup/Timers.java). */

/** The ViewServer's liveness check, re-set on every fire (device: type 9, 100 ms). */
record PingCheckTimer() implements Timer {
  static final int PING_CHECK_MILLIS = 100;
}

/** A server's ping to the ViewServer, re-set on every fire (device: type 10, 25 ms). */
record PingTimer() implements Timer {
  static final int PING_MILLIS = 25;
}

/** A client's retry of its command `seq` (device: type 11, 100 ms, head of the client's queue). */
record ClientTimer(int seq) implements Timer {
  static final int CLIENT_RETRY_MILLIS = 100;
}
