package dslabs.primarybackup;

import static dslabs.primarybackup.PingTimer.PING_MILLIS;

import dslabs.atmostonce.AMOApplication;
import dslabs.atmostonce.AMOResult;
import dslabs.framework.Address;
import dslabs.framework.Application;
import dslabs.framework.Node;
import dslabs.framework.testing.utils.Cloning;
import lombok.EqualsAndHashCode;
import lombok.ToString;

/**
 * lab2 primary / backup server (DESIGN.md §12): pings the ViewServer every 25 ms with its latest
 * view number, or the last started one while it is the primary of a view whose backup has not
 * acknowledged the state transfer. A new view with this server as primary and a backup sends the
 * application to the backup, which installs it once and acknowledges. The primary serves client
 * requests only once started; with a backup it forwards each and executes it when the backup has.
 * Device form: the server words of dslabs_amd/csrc/protocols/pb.hpp (view, started, lastStarted,
 * the two keys' values and the AMO table).
 */
@ToString(callSuper = true)
@EqualsAndHashCode(callSuper = true)
class PBServer extends Node {
  private final Address viewServer;

  private AMOApplication<Application> app;
  private View view = new View(ViewServer.STARTUP_VIEWNUM, null, null);
  private boolean started;
  private int lastStarted = ViewServer.STARTUP_VIEWNUM;

  /* -----------------------------------------------------------------------------------------------
   *  Construction and Initialization
   * ---------------------------------------------------------------------------------------------*/
  PBServer(Address address, Address viewServer, Application app) {
    super(address);
    this.viewServer = viewServer;
    this.app = new AMOApplication<>(app);
  }

  @Override
  public void init() {
    send(new Ping(ViewServer.STARTUP_VIEWNUM), viewServer);
    set(new PingTimer(), PING_MILLIS);
  }

  /* -----------------------------------------------------------------------------------------------
   *  Message Handlers
   * ---------------------------------------------------------------------------------------------*/
  private void handleRequest(Request m, Address sender) {
    if (!isPrimary() || !started) return;
    if (view.backup() == null) {
      AMOResult r = app.execute(m.command());
      if (r != null) send(new Reply(r), sender);
    } else {
      send(new Forward(view.viewNum(), m.command()), view.backup());
    }
  }

  private void handleViewReply(ViewReply m, Address sender) {
    View v = m.view();
    if (v.viewNum() <= view.viewNum()) return;
    view = v;
    started = false;
    if (!address().equals(v.primary())) return;
    if (v.backup() == null) {
      started = true;
      lastStarted = v.viewNum();
    } else {
      send(new StateTransfer(v, Cloning.clone(app)), v.backup());
    }
  }

  private void handleStateTransfer(StateTransfer m, Address sender) {
    View v = m.view();
    if (v.viewNum() < view.viewNum() || !address().equals(v.backup()) || !sender.equals(v.primary())) return;
    // installed once per view: a redelivered transfer must not undo the forwarded operations since
    if (v.viewNum() == view.viewNum() && started) return;
    view = v;
    started = true;
    app = Cloning.clone(m.app());
    send(new StateTransferAck(v.viewNum()), sender);
  }

  private void handleStateTransferAck(StateTransferAck m, Address sender) {
    if (isPrimary() && !started && m.viewNum() == view.viewNum()) {
      started = true;
      lastStarted = view.viewNum();
    }
  }

  private void handleForward(Forward m, Address sender) {
    if (m.viewNum() != view.viewNum() || !address().equals(view.backup()) || !sender.equals(view.primary())) return;
    app.execute(m.command());
    send(new ForwardAck(m.viewNum(), m.command()), sender);
  }

  private void handleForwardAck(ForwardAck m, Address sender) {
    if (!isPrimary() || !started || m.viewNum() != view.viewNum()) return;
    AMOResult r = app.execute(m.command());
    if (r != null) send(new Reply(r), m.command().clientAddress());
  }

  /* -----------------------------------------------------------------------------------------------
   *  Timer Handlers
   * ---------------------------------------------------------------------------------------------*/
  private void onPingTimer(PingTimer t) {
    send(new Ping(isPrimary() && !started ? lastStarted : view.viewNum()), viewServer);
    set(t, PING_MILLIS);
  }

  /* -----------------------------------------------------------------------------------------------
   *  Utils
   * ---------------------------------------------------------------------------------------------*/
  private boolean isPrimary() {
    return address().equals(view.primary());
  }
}
