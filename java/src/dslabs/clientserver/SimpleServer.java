package dslabs.clientserver;

import dslabs.atmostonce.AMOApplication;
import dslabs.atmostonce.AMOResult;
import dslabs.framework.Address;
import dslabs.framework.Application;
import dslabs.framework.Node;
import lombok.EqualsAndHashCode;
import lombok.ToString;

/**
 * lab1 server (DESIGN.md §11): executes each request through an at-most-once application and
 * replies, except to a superseded request (an older sequence number than the client's last).
 * Device form: the server words of dslabs_amd/csrc/protocols/amokv.hpp (3 key values + the AMO table).
 */
@ToString(callSuper = true)
@EqualsAndHashCode(callSuper = true)
class SimpleServer extends Node {
  private final AMOApplication<Application> app;

  /* -----------------------------------------------------------------------------------------------
   *  Construction and Initialization
   * ---------------------------------------------------------------------------------------------*/
  public SimpleServer(Address address, Application app) {
    super(address);
    this.app = new AMOApplication<>(app);
  }

  @Override
  public void init() {
    // No initialization necessary
  }

  /* -----------------------------------------------------------------------------------------------
   *  Message Handlers
   * ---------------------------------------------------------------------------------------------*/
  private void handleRequest(Request m, Address sender) {
    AMOResult r = app.execute(m.command());
    if (r != null) send(new Reply(r), sender);
  }
}
