package dslabs.primarybackup;

import static dslabs.primarybackup.ClientTimer.CLIENT_RETRY_MILLIS;

import dslabs.atmostonce.AMOCommand;
import dslabs.framework.Address;
import dslabs.framework.Client;
import dslabs.framework.Command;
import dslabs.framework.Node;
import dslabs.framework.Result;
import lombok.EqualsAndHashCode;
import lombok.ToString;

/**
 * lab2 client (DESIGN.md §12): lab1's client plus a cached view. It asks the ViewServer when it
 * knows no primary; its timer asks again and re-sends; a newer ViewReply re-sends the pending
 * command to the new primary. Device form: the client words of dslabs_amd/csrc/protocols/pb.hpp.
 */
@ToString(callSuper = true)
@EqualsAndHashCode(callSuper = true)
class PBClient extends Node implements Client {
  private final Address viewServer;

  private int viewNum = ViewServer.STARTUP_VIEWNUM;
  private Address primary;
  private int seq;
  private AMOCommand pending;
  private Result result;

  /* -----------------------------------------------------------------------------------------------
   *  Construction and Initialization
   * ---------------------------------------------------------------------------------------------*/
  public PBClient(Address address, Address viewServer) {
    super(address);
    this.viewServer = viewServer;
  }

  @Override
  public synchronized void init() {}

  /* -----------------------------------------------------------------------------------------------
   *  Client Methods
   * ---------------------------------------------------------------------------------------------*/
  @Override
  public synchronized void sendCommand(Command command) {
    seq++;
    result = null;
    pending = new AMOCommand(command, address(), seq);
    sendPending();
    set(new ClientTimer(seq), CLIENT_RETRY_MILLIS);
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
    if (!waiting() || m.result().sequenceNum() != seq) return;
    result = m.result().result();
    notifyAll();
  }

  private synchronized void handleViewReply(ViewReply m, Address sender) {
    if (m.view().viewNum() <= viewNum) return;
    viewNum = m.view().viewNum();
    primary = m.view().primary();
    if (waiting()) sendPending();
  }

  /* -----------------------------------------------------------------------------------------------
   *  Timer Handlers
   * ---------------------------------------------------------------------------------------------*/
  private synchronized void onClientTimer(ClientTimer t) {
    if (!waiting() || t.seq() != seq) return;
    send(new GetView(), viewServer);
    if (primary != null) send(new Request(pending), primary);
    set(t, CLIENT_RETRY_MILLIS);
  }

  /* -----------------------------------------------------------------------------------------------
   *  Utils
   * ---------------------------------------------------------------------------------------------*/
  private boolean waiting() {
    return seq > 0 && result == null;
  }

  private void sendPending() {
    if (primary != null) send(new Request(pending), primary);
    else send(new GetView(), viewServer);
  }
}
