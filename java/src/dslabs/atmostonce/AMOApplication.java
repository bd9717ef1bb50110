package dslabs.atmostonce;

import dslabs.framework.Address;
import dslabs.framework.Application;
import dslabs.framework.Command;
import dslabs.framework.Result;
import java.util.HashMap;
import java.util.Map;
import lombok.EqualsAndHashCode;
import lombok.Getter;
import lombok.NonNull;
import lombok.RequiredArgsConstructor;
import lombok.ToString;

/**
 * At-most-once wrapper (DESIGN.md §11): per client, the last executed sequence number and its
 * result. A command newer than the client's last executes; the last one again returns the cached
 * result; an older one is superseded (null: the server does not reply). The device keeps the same
 * table as the server's AMO words (w3..w5 = seq:2 | result:24, dslabs_amd/csrc/protocols/amokv.hpp).
 */
@EqualsAndHashCode
@ToString
@RequiredArgsConstructor
public final class AMOApplication<T extends Application> implements Application {
  @Getter @NonNull private final T application;

  private final Map<Address, AMOResult> lastResults = new HashMap<>();

  @Override
  public AMOResult execute(Command command) {
    if (!(command instanceof AMOCommand)) {
      throw new IllegalArgumentException();
    }
    AMOCommand amo = (AMOCommand) command;
    AMOResult last = lastResults.get(amo.clientAddress());
    if (last != null && amo.sequenceNum() <= last.sequenceNum()) {
      return amo.sequenceNum() == last.sequenceNum() ? last : null;
    }
    AMOResult r = new AMOResult(application.execute(amo.command()), amo.sequenceNum());
    lastResults.put(amo.clientAddress(), r);
    return r;
  }

  public Result executeReadOnly(Command command) {
    if (!command.readOnly()) {
      throw new IllegalArgumentException();
    }
    if (command instanceof AMOCommand) {
      return execute(command);
    }
    return application.execute(command);
  }

  public boolean alreadyExecuted(AMOCommand amoCommand) {
    AMOResult last = lastResults.get(amoCommand.clientAddress());
    return last != null && amoCommand.sequenceNum() <= last.sequenceNum();
  }
}
