package dslabs.atmostonce;

import dslabs.framework.Address;
import dslabs.framework.Command;
import lombok.Data;

/**
 * A client's command tagged with the client and its sequence number (DESIGN.md §11). On the
 * device a Request carries only the sequence number: the command is the sender's workload command
 * of that number (dslabs_amd/csrc/protocols/amokv.hpp).
 */
@Data
public final class AMOCommand implements Command {
  private final Command command;
  private final Address clientAddress;
  private final int sequenceNum;

  @Override
  public boolean readOnly() {
    return command.readOnly();
  }
}
