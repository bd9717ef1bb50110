package dslabs.primarybackup;

import static dslabs.primarybackup.PingCheckTimer.PING_CHECK_MILLIS;

import dslabs.framework.Address;
import dslabs.framework.Node;
import java.util.HashSet;
import java.util.Set;
import lombok.EqualsAndHashCode;
import lombok.ToString;

/**
 * lab2 ViewServer (DESIGN.md §12, labs/lab2-primarybackup/README.md:161-216): the first pinging
 * server is primary of view 1; a server is dead when it did not ping between the last two checks;
 * the view changes only after its primary acknowledged it (Ping(current viewNum)); on a check a
 * dead primary is replaced by a live backup (stuck otherwise), a dead backup is dropped, a missing
 * backup is filled from the lowest live idle server; a ping also fills a missing backup at once.
 * Device form: the viewserver word of dslabs_amd/csrc/protocols/pb.hpp (view, acked, the two ping
 * sets). The oracle's and the device's restatements pass ViewServerTest 01-12.
 */
@ToString(callSuper = true)
@EqualsAndHashCode(callSuper = true)
class ViewServer extends Node {
  static final int STARTUP_VIEWNUM = 0;
  private static final int INITIAL_VIEWNUM = 1;

  private View view = new View(STARTUP_VIEWNUM, null, null);
  private boolean acked;
  private Set<Address> pingedSinceCheck = new HashSet<>();  // device: recent
  private Set<Address> pingedLastPeriod = new HashSet<>();  // device: aliveLast

  /* -----------------------------------------------------------------------------------------------
   *  Construction and Initialization
   * ---------------------------------------------------------------------------------------------*/
  public ViewServer(Address address) {
    super(address);
  }

  @Override
  public void init() {
    set(new PingCheckTimer(), PING_CHECK_MILLIS);
  }

  /* -----------------------------------------------------------------------------------------------
   *  Message Handlers
   * ---------------------------------------------------------------------------------------------*/
  private void handlePing(Ping m, Address sender) {
    pingedSinceCheck.add(sender);
    if (view.viewNum() == STARTUP_VIEWNUM) {
      view = new View(INITIAL_VIEWNUM, sender, null);
      acked = false;
    }
    if (sender.equals(view.primary()) && m.viewNum() == view.viewNum()) acked = true;
    if (acked && view.backup() == null) {
      Set<Address> live = new HashSet<>(pingedSinceCheck);
      live.addAll(pingedLastPeriod);
      Address idle = lowestIdle(live, view.primary(), null);
      if (idle != null) newView(view.primary(), idle);
    }
    send(new ViewReply(view), sender);
  }

  private void handleGetView(GetView m, Address sender) {
    send(new ViewReply(view), sender);
  }

  /* -----------------------------------------------------------------------------------------------
   *  Timer Handlers
   * ---------------------------------------------------------------------------------------------*/
  private void onPingCheckTimer(PingCheckTimer t) {
    Set<Address> alive = pingedSinceCheck;
    pingedLastPeriod = alive;
    pingedSinceCheck = new HashSet<>();
    if (acked && view.viewNum() != STARTUP_VIEWNUM) {
      Address p = view.primary(), b = view.backup();
      boolean bAlive = b != null && alive.contains(b);
      if (!alive.contains(p)) {
        if (bAlive) newView(b, lowestIdle(alive, b, null));
      } else if (b != null && !bAlive) {
        newView(p, lowestIdle(alive, p, null));
      } else if (b == null) {
        Address idle = lowestIdle(alive, p, null);
        if (idle != null) newView(p, idle);
      }
    }
    set(t, PING_CHECK_MILLIS);
  }

  /* -----------------------------------------------------------------------------------------------
   *  Utils
   * ---------------------------------------------------------------------------------------------*/
  private void newView(Address primary, Address backup) {
    view = new View(view.viewNum() + 1, primary, backup);
    acked = false;
  }

  /** The live server, other than p and b, whose address sorts first (device: the lowest server id). */
  private static Address lowestIdle(Set<Address> live, Address p, Address b) {
    Address best = null;
    for (Address a : live)
      if (!a.equals(p) && !a.equals(b) && (best == null || a.toString().compareTo(best.toString()) < 0)) best = a;
    return best;
  }
}
