package dslabs.primarybackup;

import dslabs.atmostonce.AMOApplication;
import dslabs.atmostonce.AMOCommand;
import dslabs.atmostonce.AMOResult;
import dslabs.framework.Application;
import dslabs.framework.Message;
import lombok.Data;

/*
 * lab2 messages (DESIGN.md §12): the reference stub's ViewServer messages as it declares them
 * (labs/lab2-primarybackup/src/dslabs/primarybackup/Messages.java: Lombok @Data, fluent accessors)
 * plus this solution's primary-backup messages in the same form. Device records
 * (dslabs_amd/csrc/protocols/pb.hpp): type:4 | from | to | payload, types 0 Ping .. 8 ForwardAck.
 */

/* ViewServer messages */
@Data
class Ping implements Message {
  private final int viewNum;
}

@Data
class GetView implements Message {}

@Data
class ViewReply implements Message {
  private final View view;
}

/* Primary-backup messages */

/** A client's command to the primary it knows (device: type 3, the command's sequence number). */
@Data
class Request implements Message {
  private final AMOCommand command;
}

/** The primary's answer (device: type 4, seq | result:10 @2). */
@Data
class Reply implements Message {
  private final AMOResult result;
}

/** The primary's application, sent to the backup of a new view (device: type 5, view | app:40 @8). */
@Data
class StateTransfer implements Message {
  private final View view;
  private final AMOApplication<Application> app;
}

/** The backup installed the view's state (device: type 6, viewNum). */
@Data
class StateTransferAck implements Message {
  private final int viewNum;
}

/** A client command the primary forwards to its backup (device: type 7, viewNum | client @4 | seq @7). */
@Data
class Forward implements Message {
  private final int viewNum;
  private final AMOCommand command;
}

/** The backup executed the forwarded command (device: type 8, as Forward). */
@Data
class ForwardAck implements Message {
  private final int viewNum;
  private final AMOCommand command;
}
