package dslabs.clientserver;

import dslabs.atmostonce.AMOCommand;
import dslabs.framework.Address;
import dslabs.framework.Client;
import dslabs.framework.Command;
import dslabs.framework.Node;
import dslabs.framework.Result;
import lombok.EqualsAndHashCode;
import lombok.ToString;

/**
 * lab1 client (DESIGN.md §11): each command gets the next sequence number, goes to the server
 * with a ClientTimer that re-sends it while it has no result; the reply for the current sequence
 * number is the result. Device form: the client words of dslabs_amd/csrc/protocols/amokv.hpp
 * (seq, hasResult, the current result and the ClientTimer queue).
 */
@ToString(callSuper = true)
@EqualsAndHashCode(callSuper = true)
class SimpleClient extends Node implements Client {
  private final Address serverAddress;

  private int sequenceNum;
  private AMOCommand pending;
  private Result result;

  /* -----------------------------------------------------------------------------------------------
   *  Construction and Initialization
   * ---------------------------------------------------------------------------------------------*/
  public SimpleClient(Address address, Address serverAddress) {
    super(address);
    this.serverAddress = serverAddress;
  }

  @Override
  public synchronized void init() {
    // No initialization necessary
  }

  /* -----------------------------------------------------------------------------------------------
   *  Client Methods
   * ---------------------------------------------------------------------------------------------*/
  @Override
  public synchronized void sendCommand(Command command) {
    sequenceNum++;
    pending = new AMOCommand(command, address(), sequenceNum);
    result = null;
    send(new Request(pending), serverAddress);
    set(new ClientTimer(sequenceNum), ClientTimer.CLIENT_RETRY_MILLIS);
  }

  @Override
  public synchronized boolean hasResult() {
    return result != null;
  }

  @Override
  public synchronized Result getResult() throws InterruptedException {
    while (result == null) wait();
    return result;
  }

  /* -----------------------------------------------------------------------------------------------
   *  Message Handlers
   * ---------------------------------------------------------------------------------------------*/
  private synchronized void handleReply(Reply m, Address sender) {
    if (result != null || m.result().sequenceNum() != sequenceNum) return;
    result = m.result().result();
    notifyAll();
  }

  /* -----------------------------------------------------------------------------------------------
   *  Timer Handlers
   * ---------------------------------------------------------------------------------------------*/
  private synchronized void onClientTimer(ClientTimer t) {
    if (result != null || t.sequenceNum() != sequenceNum) return;
    send(new Request(pending), serverAddress);
    set(t, ClientTimer.CLIENT_RETRY_MILLIS);
  }
}
