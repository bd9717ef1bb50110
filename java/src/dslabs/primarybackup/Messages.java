package dslabs.primarybackup;

import dslabs.atmostonce.AMOApplication;
import dslabs.atmostonce.AMOCommand;
import dslabs.atmostonce.AMOResult;
import dslabs.framework.Application;
import dslabs.framework.Message;

/*
 * lab2 messages (DESIGN.md §12) as records: the same names, components and equality as the
 * reference's (labs/lab2-primarybackup/src/dslabs/primarybackup/Messages.java) plus this solution's
 * primary-backup messages. Device records (dslabs_amd/csrc/protocols/pb.hpp): type:4 | from | to |
 * payload, types 0 Ping .. 8 ForwardAck.
 */

/* ViewServer messages */
record Ping(int viewNum) implements Message {}

record GetView() implements Message {}

record ViewReply(View view) implements Message {}

/* Primary-backup messages */

/** A client's command to the primary it knows (device: type 3, the command's sequence number). */
record Request(AMOCommand command) implements Message {}

/** The primary's answer (device: type 4, seq | result:10 @2). */
record Reply(AMOResult result) implements Message {}

/** The primary's application, sent to the backup of a new view (device: type 5, view | app:40 @8). */
record StateTransfer(View view, AMOApplication<Application> app) implements Message {}

/** The backup installed the view's state (device: type 6, viewNum). */
record StateTransferAck(int viewNum) implements Message {}

/** A client command the primary forwards to its backup (device: type 7, viewNum | client @4 | seq @7). */
record Forward(int viewNum, AMOCommand command) implements Message {}

/** The backup executed the forwarded command (device: type 8, as Forward). */
record ForwardAck(int viewNum, AMOCommand command) implements Message {}
