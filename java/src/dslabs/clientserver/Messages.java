package dslabs.clientserver;

import dslabs.atmostonce.AMOCommand;
import dslabs.atmostonce.AMOResult;
import dslabs.framework.Message;
import lombok.Data;

/** A client's command to the server (device: type 0, the command's sequence number). */
@Data
class Request implements Message {
  private final AMOCommand command;
}

/** The server's answer (device: type 1, sequence number + 24-bit result, amokv.hpp). */
@Data
class Reply implements Message {
  private final AMOResult result;
}
