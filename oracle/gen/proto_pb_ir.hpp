// GENERATED from the protocol IR (dslabs_amd/ir/specs/pb.py) by dslabs_amd/ir/gen_oracle.py; do not edit.
// oracle/ -- TEST INFRASTRUCTURE ONLY (see oracle_core.hpp).
#pragma once
#include "../oracle_core.hpp"

namespace oracle {
namespace pb_ir {

struct Params {
  int servers = 2;
  int clients = 1;
  int ncmds = 2;
  int op[2][3] = {};
  int key[2][3] = {};
  int sym[2][3] = {};
  int expected[2][3] = {};
};
// Params from the engine's parameter vector (dsl_protocol_desc.params order)
inline Params from_vector(const std::vector<long long>& v) {
  Params p;
  size_t q = 0;
  if (q < v.size()) p.servers = (int)v[q];
  q++;
  if (q < v.size()) p.clients = (int)v[q];
  q++;
  if (q < v.size()) p.ncmds = (int)v[q];
  q++;
  for (int r = 0; r < 2; r++)
    for (int c = 0; c < 3; c++, q++) p.op[r][c] = q < v.size() ? (int)v[q] : 0;
  for (int r = 0; r < 2; r++)
    for (int c = 0; c < 3; c++, q++) p.key[r][c] = q < v.size() ? (int)v[q] : 0;
  for (int r = 0; r < 2; r++)
    for (int c = 0; c < 3; c++, q++) p.sym[r][c] = q < v.size() ? (int)v[q] : 0;
  for (int r = 0; r < 2; r++)
    for (int c = 0; c < 3; c++, q++) p.expected[r][c] = q < v.size() ? (int)v[q] : -1;
  return p;
}
// node index of a kind's first instance: kinds in declaration order, instances consecutive
inline int first_viewserver(const Params& prm) { (void)prm; return 0; }
inline int first_server(const Params& prm) { (void)prm; return 0 + 1; }
inline int first_client(const Params& prm) { (void)prm; return 0 + 1 + prm.servers; }
inline int wsize(int c, const Params& prm) { (void)c; (void)prm; return prm.ncmds; }

struct N_viewserver : Node {
  Params prm;
  int self = 0;
  int vnum = 0;
  int vp = 0;
  int vb = 0;
  int acked = 0;
  int recent = 0;
  int alive = 0;
  std::shared_ptr<Node> clone() const override { return std::make_shared<N_viewserver>(*this); }
  void key(std::string& out) const override {
    out += "viewserver{";
    out += std::to_string(vnum) + ",";
    out += std::to_string(vp) + ",";
    out += std::to_string(vb) + ",";
    out += std::to_string(acked) + ",";
    out += std::to_string(recent) + ",";
    out += std::to_string(alive) + ",";
    out += "}";
  }
  std::string str() const override {
    return std::string("viewserver(") + "vnum=" + std::to_string(vnum) + ", " + "vp=" + std::to_string(vp) + ", " + "vb=" + std::to_string(vb) + ", " + "acked=" + std::to_string(acked) + ", " + "recent=" + std::to_string(recent) + ", " + "alive=" + std::to_string(alive) + ")";
  }
  void init(Ctx& ctx) override {
    ctx.set(Rec{"PingCheckTimer", {}}, 100, 100);
  }
  void handleMessage(const Rec& m, int from, int, Ctx& ctx) override {
    (void)from; (void)ctx;
    if (m.type == "Ping") {
      const int l_frm = from;
      if (((l_frm < 1) || (l_frm > prm.servers))) {
        throw HandlerException("Ping from a node that is not a server");
      }
      recent = (recent | (1 << (l_frm - 1)));
      if ((vnum == 0)) {
        vnum = 1;
        vp = l_frm;
        vb = 0;
        acked = 0;
      }
      if (((l_frm == vp) && (std::stoi(m.f[0]) == vnum))) {
        acked = 1;
      }
      if (((acked == 1) && (vb == 0))) {
        const int l_live = (recent | alive);
        int l_pidle = 0;
        if (((((3 <= prm.servers) && (((l_live >> 2) & 1) == 1)) && (3 != vp)) && (3 != 0))) {
          l_pidle = 3;
        }
        if (((((2 <= prm.servers) && (((l_live >> 1) & 1) == 1)) && (2 != vp)) && (2 != 0))) {
          l_pidle = 2;
        }
        if (((((1 <= prm.servers) && (((l_live >> 0) & 1) == 1)) && (1 != vp)) && (1 != 0))) {
          l_pidle = 1;
        }
        if ((l_pidle != 0)) {
          if (((vnum + 1) > 15)) {
            // view number past 15: bounded on the device only
          }
          vnum = (vnum + 1);
          vp = vp;
          vb = l_pidle;
          acked = 0;
        }
      }
      ctx.send(Rec{"ViewReply", {std::to_string(vnum), std::to_string(vp), std::to_string(vb)}}, l_frm);
      return;
    }
    if (m.type == "GetView") {
      ctx.send(Rec{"ViewReply", {std::to_string(vnum), std::to_string(vp), std::to_string(vb)}}, from);
      return;
    }
    throw HandlerException("no handler");
  }
  void onTimer(const Rec& t, Ctx& ctx) override {
    (void)ctx;
    if (t.type == "PingCheckTimer") {
      const int l_alv = recent;
      alive = l_alv;
      recent = 0;
      if (((acked == 1) && (vnum != 0))) {
        const int l_pp = vp;
        const int l_bb = vb;
        const int l_palive = ((l_alv >> (l_pp - 1)) & 1);
        const int l_balive = ((l_bb != 0) && (((l_alv >> (l_bb - 1)) & 1) == 1));
        if ((l_palive == 0)) {
          if (l_balive) {
            int l_cidle1 = 0;
            if (((((3 <= prm.servers) && (((l_alv >> 2) & 1) == 1)) && (3 != l_bb)) && (3 != 0))) {
              l_cidle1 = 3;
            }
            if (((((2 <= prm.servers) && (((l_alv >> 1) & 1) == 1)) && (2 != l_bb)) && (2 != 0))) {
              l_cidle1 = 2;
            }
            if (((((1 <= prm.servers) && (((l_alv >> 0) & 1) == 1)) && (1 != l_bb)) && (1 != 0))) {
              l_cidle1 = 1;
            }
            if (((vnum + 1) > 15)) {
              // view number past 15: bounded on the device only
            }
            vnum = (vnum + 1);
            vp = l_bb;
            vb = l_cidle1;
            acked = 0;
          }
        }
        if ((((l_palive == 1) && (l_bb != 0)) && (!l_balive))) {
          int l_cidle2 = 0;
          if (((((3 <= prm.servers) && (((l_alv >> 2) & 1) == 1)) && (3 != l_pp)) && (3 != 0))) {
            l_cidle2 = 3;
          }
          if (((((2 <= prm.servers) && (((l_alv >> 1) & 1) == 1)) && (2 != l_pp)) && (2 != 0))) {
            l_cidle2 = 2;
          }
          if (((((1 <= prm.servers) && (((l_alv >> 0) & 1) == 1)) && (1 != l_pp)) && (1 != 0))) {
            l_cidle2 = 1;
          }
          if (((vnum + 1) > 15)) {
            // view number past 15: bounded on the device only
          }
          vnum = (vnum + 1);
          vp = l_pp;
          vb = l_cidle2;
          acked = 0;
        }
        if (((l_palive == 1) && (l_bb == 0))) {
          int l_cidle3 = 0;
          if (((((3 <= prm.servers) && (((l_alv >> 2) & 1) == 1)) && (3 != l_pp)) && (3 != 0))) {
            l_cidle3 = 3;
          }
          if (((((2 <= prm.servers) && (((l_alv >> 1) & 1) == 1)) && (2 != l_pp)) && (2 != 0))) {
            l_cidle3 = 2;
          }
          if (((((1 <= prm.servers) && (((l_alv >> 0) & 1) == 1)) && (1 != l_pp)) && (1 != 0))) {
            l_cidle3 = 1;
          }
          if ((l_cidle3 != 0)) {
            if (((vnum + 1) > 15)) {
              // view number past 15: bounded on the device only
            }
            vnum = (vnum + 1);
            vp = l_pp;
            vb = l_cidle3;
            acked = 0;
          }
        }
      }
      ctx.set(Rec{"PingCheckTimer", {}}, 100, 100);
      return;
    }
    throw HandlerException("no timer handler");
  }
};

struct N_server : Node {
  Params prm;
  int self = 0;
  int vnum = 0;
  int vp = 0;
  int vb = 0;
  int started = 0;
  int last = 0;
  std::vector<int> kv = std::vector<int>(2, 0);
  std::vector<int> amo = std::vector<int>(2, 0);
  std::shared_ptr<Node> clone() const override { return std::make_shared<N_server>(*this); }
  void key(std::string& out) const override {
    out += "server{";
    out += std::to_string(vnum) + ",";
    out += std::to_string(vp) + ",";
    out += std::to_string(vb) + ",";
    out += std::to_string(started) + ",";
    out += std::to_string(last) + ",";
    for (int x : kv) out += std::to_string(x) + ",";
    for (int x : amo) out += std::to_string(x) + ",";
    out += "}";
  }
  std::string str() const override {
    return std::string("server(") + "vnum=" + std::to_string(vnum) + ", " + "vp=" + std::to_string(vp) + ", " + "vb=" + std::to_string(vb) + ", " + "started=" + std::to_string(started) + ", " + "last=" + std::to_string(last) + ")";
  }
  void init(Ctx& ctx) override {
    ctx.send(Rec{"Ping", {std::to_string(0)}}, (first_viewserver(prm) + 1 - 1));
    ctx.set(Rec{"PingTimer", {}}, 25, 25);
  }
  void handleMessage(const Rec& m, int from, int, Ctx& ctx) override {
    (void)from; (void)ctx;
    if (m.type == "ViewReply") {
      if ((std::stoi(m.f[0]) <= vnum)) {
        return;
      }
      vnum = std::stoi(m.f[0]);
      vp = std::stoi(m.f[1]);
      vb = std::stoi(m.f[2]);
      started = 0;
      if ((std::stoi(m.f[1]) == self)) {
        if ((std::stoi(m.f[2]) == 0)) {
          started = 1;
          last = std::stoi(m.f[0]);
        } else {
          ctx.send(Rec{"StateTransfer", {std::to_string(std::stoi(m.f[0])), std::to_string(std::stoi(m.f[1])), std::to_string(std::stoi(m.f[2])), std::to_string(kv[0]), std::to_string(kv[1]), std::to_string(amo[0]), std::to_string(amo[1])}}, std::stoi(m.f[2]));
        }
      }
      return;
    }
    if (m.type == "Request") {
      const int l_seq = std::stoi(m.f[0]);
      const int l_c = (from - (first_client(prm) + 1 - 1));
      if (((((l_c < 0) || (l_c >= prm.clients)) || (l_seq < 1)) || (l_seq > prm.ncmds))) {
        throw HandlerException("request from an unknown client or command");
      }
      if (((vp != self) || (started == 0))) {
        return;
      }
      if ((vb == 0)) {
        int l_r = -1;
        const int l_amo = amo[l_c];
        const int l_lastseq = (l_amo & 3);
        l_r = -1;
        if ((l_seq == l_lastseq)) {
          l_r = (l_amo >> 2);
        }
        if ((l_seq > l_lastseq)) {
          const int l_k = (l_seq - 1);
          const int l_op = prm.op[l_c][l_k];
          const int l_key = prm.key[l_c][l_k];
          const int l_sym = prm.sym[l_c][l_k];
          const int l_v = kv[l_key];
          if ((l_op == 0)) {
            if (((l_v & 3) != 0)) {
              l_r = ((l_v << 2) | 1);
            } else {
              l_r = 2;
            }
          }
          if ((l_op == 1)) {
            kv[l_key] = ((l_sym << 2) | 1);
            l_r = 3;
          }
          if ((l_op == 2)) {
            const int l_n = (l_v & 3);
            if ((l_n >= 3)) {
              // value longer than 3 tokens: bounded on the device only
            }
            const int l_v2 = (((l_v - l_n) | (l_n + 1)) | (l_sym << ((l_n * 2) + 2)));
            kv[l_key] = l_v2;
            l_r = (l_v2 << 2);
          }
          amo[l_c] = (l_seq | (l_r << 2));
        }
        if ((l_r >= 0)) {
          ctx.send(Rec{"Reply", {std::to_string(l_seq), std::to_string(l_r)}}, from);
        }
      } else {
        ctx.send(Rec{"Forward", {std::to_string(vnum), std::to_string(from), std::to_string(l_seq)}}, vb);
      }
      return;
    }
    if (m.type == "StateTransfer") {
      if ((((std::stoi(m.f[0]) < vnum) || (std::stoi(m.f[2]) != self)) || (std::stoi(m.f[1]) != from))) {
        return;
      }
      if (((std::stoi(m.f[0]) == vnum) && (started == 1))) {
        return;
      }
      vnum = std::stoi(m.f[0]);
      vp = std::stoi(m.f[1]);
      vb = std::stoi(m.f[2]);
      started = 1;
      kv[0] = std::stoi(m.f[3]);
      kv[1] = std::stoi(m.f[4]);
      amo[0] = std::stoi(m.f[5]);
      amo[1] = std::stoi(m.f[6]);
      ctx.send(Rec{"StateTransferAck", {std::to_string(std::stoi(m.f[0]))}}, from);
      return;
    }
    if (m.type == "StateTransferAck") {
      if ((((vp == self) && (started == 0)) && (std::stoi(m.f[0]) == vnum))) {
        started = 1;
        last = vnum;
      }
      return;
    }
    if (m.type == "Forward") {
      const int l_seq = std::stoi(m.f[2]);
      const int l_ca = std::stoi(m.f[1]);
      const int l_c = (l_ca - (first_client(prm) + 1 - 1));
      if (((((l_c < 0) || (l_c >= prm.clients)) || (l_seq < 1)) || (l_seq > prm.ncmds))) {
        throw HandlerException("forward of an unknown client or command");
      }
      if ((((vnum != std::stoi(m.f[0])) || (vb != self)) || (vp != from))) {
        return;
      }
      int l_r = -1;
      const int l_amo = amo[l_c];
      const int l_lastseq = (l_amo & 3);
      l_r = -1;
      if ((l_seq == l_lastseq)) {
        l_r = (l_amo >> 2);
      }
      if ((l_seq > l_lastseq)) {
        const int l_k = (l_seq - 1);
        const int l_op = prm.op[l_c][l_k];
        const int l_key = prm.key[l_c][l_k];
        const int l_sym = prm.sym[l_c][l_k];
        const int l_v = kv[l_key];
        if ((l_op == 0)) {
          if (((l_v & 3) != 0)) {
            l_r = ((l_v << 2) | 1);
          } else {
            l_r = 2;
          }
        }
        if ((l_op == 1)) {
          kv[l_key] = ((l_sym << 2) | 1);
          l_r = 3;
        }
        if ((l_op == 2)) {
          const int l_n = (l_v & 3);
          if ((l_n >= 3)) {
            // value longer than 3 tokens: bounded on the device only
          }
          const int l_v2 = (((l_v - l_n) | (l_n + 1)) | (l_sym << ((l_n * 2) + 2)));
          kv[l_key] = l_v2;
          l_r = (l_v2 << 2);
        }
        amo[l_c] = (l_seq | (l_r << 2));
      }
      ctx.send(Rec{"ForwardAck", {std::to_string(std::stoi(m.f[0])), std::to_string(l_ca), std::to_string(l_seq)}}, from);
      return;
    }
    if (m.type == "ForwardAck") {
      const int l_seq = std::stoi(m.f[2]);
      const int l_ca = std::stoi(m.f[1]);
      const int l_c = (l_ca - (first_client(prm) + 1 - 1));
      if (((((l_c < 0) || (l_c >= prm.clients)) || (l_seq < 1)) || (l_seq > prm.ncmds))) {
        throw HandlerException("forward of an unknown client or command");
      }
      if ((((vp != self) || (started == 0)) || (vnum != std::stoi(m.f[0])))) {
        return;
      }
      int l_r = -1;
      const int l_amo = amo[l_c];
      const int l_lastseq = (l_amo & 3);
      l_r = -1;
      if ((l_seq == l_lastseq)) {
        l_r = (l_amo >> 2);
      }
      if ((l_seq > l_lastseq)) {
        const int l_k = (l_seq - 1);
        const int l_op = prm.op[l_c][l_k];
        const int l_key = prm.key[l_c][l_k];
        const int l_sym = prm.sym[l_c][l_k];
        const int l_v = kv[l_key];
        if ((l_op == 0)) {
          if (((l_v & 3) != 0)) {
            l_r = ((l_v << 2) | 1);
          } else {
            l_r = 2;
          }
        }
        if ((l_op == 1)) {
          kv[l_key] = ((l_sym << 2) | 1);
          l_r = 3;
        }
        if ((l_op == 2)) {
          const int l_n = (l_v & 3);
          if ((l_n >= 3)) {
            // value longer than 3 tokens: bounded on the device only
          }
          const int l_v2 = (((l_v - l_n) | (l_n + 1)) | (l_sym << ((l_n * 2) + 2)));
          kv[l_key] = l_v2;
          l_r = (l_v2 << 2);
        }
        amo[l_c] = (l_seq | (l_r << 2));
      }
      if ((l_r >= 0)) {
        ctx.send(Rec{"Reply", {std::to_string(l_seq), std::to_string(l_r)}}, l_ca);
      }
      return;
    }
    throw HandlerException("no handler");
  }
  void onTimer(const Rec& t, Ctx& ctx) override {
    (void)ctx;
    if (t.type == "PingTimer") {
      const int l_n = vnum;
      if (((vp == self) && (started == 0))) {
        ctx.send(Rec{"Ping", {std::to_string(last)}}, (first_viewserver(prm) + 1 - 1));
      } else {
        ctx.send(Rec{"Ping", {std::to_string(l_n)}}, (first_viewserver(prm) + 1 - 1));
      }
      ctx.set(Rec{"PingTimer", {}}, 25, 25);
      return;
    }
    throw HandlerException("no timer handler");
  }
};

struct N_client : Client {
  Params prm;
  int self = 0;
  int cvnum = 0;
  int cprim = 0;
  int seq = 0;
  int result = 0;
  std::shared_ptr<Node> clone() const override { return std::make_shared<N_client>(*this); }
  void key(std::string& out) const override {
    out += "client{";
    out += std::to_string(cvnum) + ",";
    out += std::to_string(cprim) + ",";
    out += std::to_string(seq) + ",";
    out += std::to_string(result) + ",";
    out += "}";
  }
  std::string str() const override {
    return std::string("client(") + "cvnum=" + std::to_string(cvnum) + ", " + "cprim=" + std::to_string(cprim) + ", " + "seq=" + std::to_string(seq) + ", " + "result=" + std::to_string(result) + ")";
  }
  void handleMessage(const Rec& m, int from, int, Ctx& ctx) override {
    (void)from; (void)ctx;
    if (m.type == "ViewReply") {
      if ((std::stoi(m.f[0]) > cvnum)) {
        cvnum = std::stoi(m.f[0]);
        cprim = std::stoi(m.f[1]);
        if (((seq > 0) && (result == 0))) {
          if ((cprim != 0)) {
            ctx.send(Rec{"Request", {std::to_string(seq)}}, cprim);
          } else {
            ctx.send(Rec{"GetView", {}}, (first_viewserver(prm) + 1 - 1));
          }
        }
      }
      return;
    }
    if (m.type == "Reply") {
      if ((((seq > 0) && (result == 0)) && (std::stoi(m.f[0]) == seq))) {
        result = std::stoi(m.f[1]);
      }
      return;
    }
    throw HandlerException("no handler");
  }
  void onTimer(const Rec& t, Ctx& ctx) override {
    (void)ctx;
    if (t.type == "ClientTimer") {
      if ((((seq > 0) && (result == 0)) && (std::stoi(t.f[0]) == seq))) {
        ctx.send(Rec{"GetView", {}}, (first_viewserver(prm) + 1 - 1));
        if ((cprim != 0)) {
          ctx.send(Rec{"Request", {std::to_string(std::stoi(t.f[0]))}}, cprim);
        }
        ctx.set(Rec{"ClientTimer", {std::to_string(std::stoi(t.f[0]))}}, 100, 100);
      }
      return;
    }
    throw HandlerException("no timer handler");
  }
  void sendCommand(const Rec& c, Ctx& ctx) override {
    const int cmd = std::stoi(c.f[0]);
    seq = cmd;
    result = 0;
    if ((cprim != 0)) {
      ctx.send(Rec{"Request", {std::to_string(cmd)}}, cprim);
    } else {
      ctx.send(Rec{"GetView", {}}, (first_viewserver(prm) + 1 - 1));
    }
    ctx.set(Rec{"ClientTimer", {std::to_string(cmd)}}, 100, 100);
  }
  bool hasResult() const override { return result != 0; }
  Rec getResult() const override { return Rec{"Result", {std::to_string(result)}}; }
};

// Addresses: node kinds in declaration order, instances consecutive.
inline std::shared_ptr<State> initial(const Params& prm, Names& names) {
  std::vector<std::shared_ptr<Node>> nodes;
  std::vector<Kind> kinds;
  for (int c = 1; c <= 1; c++) {
    names.addr.push_back("viewserver");
    auto n = std::make_shared<N_viewserver>();
    n->prm = prm;
    n->self = (int)nodes.size();
    nodes.push_back(n);
    kinds.push_back(Kind::Server);
  }
  for (int c = 1; c <= prm.servers; c++) {
    names.addr.push_back("server" + std::to_string(c));
    auto n = std::make_shared<N_server>();
    n->prm = prm;
    n->self = (int)nodes.size();
    nodes.push_back(n);
    kinds.push_back(Kind::Server);
  }
  for (int c = 1; c <= prm.clients; c++) {
    names.addr.push_back("client" + std::to_string(c));
    auto n = std::make_shared<N_client>();
    n->prm = prm;
    n->self = (int)nodes.size();
    auto cw = std::make_shared<ClientWorker>();
    cw->client = n;
    cw->addrName = names.addr.back();
    const int ci = c - 1;
    cw->workload.cmds = {"%i"};
    if (prm.expected[ci][1 - 1] >= 0) cw->workload.results = {"%i"};  // a workload with expected results
    cw->workload.numTimes = wsize(ci, prm);
    cw->workload.parser = [ci, prm](const std::string& c, const std::string& r) {
      (void)ci; (void)prm;
      (void)r;
      const int k = std::stoi(c);  // command k (1-based); the results template may be absent
      return std::make_pair(Rec{"Command", {c}}, Rec{"Result", {std::to_string(prm.expected[ci][k - 1])}});
    };
    nodes.push_back(cw);
    kinds.push_back(Kind::ClientWorker);
  }
  return makeInitial(nodes, kinds);
}

inline const N_viewserver* n_viewserver(const State& s, int a) { return dynamic_cast<const N_viewserver*>(s.nodes[a].get()); }
inline const N_server* n_server(const State& s, int a) { return dynamic_cast<const N_server*>(s.nodes[a].get()); }
inline const N_client* n_client(const State& s, int a) { return dynamic_cast<const N_client*>(s.cw(a)->client.get()); }
// network() = the network and the dropped messages (SearchState.java:153-157)
template <class F>
inline bool any_net_(const State& s, F f) {
  for (auto& e : s.network)
    if (f(e)) return true;
  for (auto& e : s.dropped)
    if (f(e)) return true;
  return false;
}
// the protocol's state predicates by their oracle CLI names (StatePredicate); a predicate with
// integer arguments is NAME:a0[:a1]
inline std::optional<Predicate> predicate(const std::string& name, const Params& prm) {
  std::vector<std::string> parts_;
  for (size_t i = 0, j; i <= name.size(); i = j + 1) {
    j = name.find(':', i);
    if (j == std::string::npos) j = name.size();
    parts_.push_back(name.substr(i, j - i));
  }
  const std::string base_ = parts_[0];
  const int a0_ = parts_.size() > 1 ? std::stoi(parts_[1]) : 0, a1_ = parts_.size() > 2 ? std::stoi(parts_[2]) : 0;
  (void)a0_; (void)a1_;
  if ((base_ == "hasViewReply") && parts_.size() == 2) {
    return Predicate{"ViewReply with viewNum", [prm, a0_, a1_](const State& s) {
      (void)s; (void)a0_; (void)a1_;
      PredResult res_;
      if (any_net_(s, [&](const Envelope& e) { return e.m.type == "ViewReply" && ((std::stoi(e.m.f[0]) >= a0_)); })) {
        { res_.value = true; return res_; }
      }
      { res_.value = false; return res_; }
      return res_;
    }};
  }
  if ((base_ == "hasViewReplyExact") && parts_.size() == 2) {
    return Predicate{"ViewReply with View", [prm, a0_, a1_](const State& s) {
      (void)s; (void)a0_; (void)a1_;
      PredResult res_;
      if (any_net_(s, [&](const Envelope& e) { return e.m.type == "ViewReply" && ((((std::stoi(e.m.f[0]) | (std::stoi(e.m.f[1]) << 4)) | (std::stoi(e.m.f[2]) << 6)) == a0_)); })) {
        { res_.value = true; return res_; }
      }
      { res_.value = false; return res_; }
      return res_;
    }};
  }
  if ((base_ == "viewRepliesSent") && parts_.size() == 3) {
    return Predicate{"ViewReply for View sent to nodes, primary ack sent", [prm, a0_, a1_](const State& s) {
      (void)s; (void)a0_; (void)a1_;
      PredResult res_;
      const int l_view = a0_;
      const int l_prim = ((l_view >> 4) & 3);
      const int l_num = (l_view & 15);
      if ((!any_net_(s, [&](const Envelope& e) { return e.m.type == "Ping" && ((((e.from == l_prim) && (e.to == 0)) && (std::stoi(e.m.f[0]) == l_num))); }))) {
        { res_.value = false; return res_; }
      }
      if (((((a1_ >> 0) & 1) == 1) && (!any_net_(s, [&](const Envelope& e) { return e.m.type == "ViewReply" && (((e.to == 0) && (((std::stoi(e.m.f[0]) | (std::stoi(e.m.f[1]) << 4)) | (std::stoi(e.m.f[2]) << 6)) == l_view))); })))) {
        { res_.value = false; return res_; }
      }
      if (((((a1_ >> 1) & 1) == 1) && (!any_net_(s, [&](const Envelope& e) { return e.m.type == "ViewReply" && (((e.to == 1) && (((std::stoi(e.m.f[0]) | (std::stoi(e.m.f[1]) << 4)) | (std::stoi(e.m.f[2]) << 6)) == l_view))); })))) {
        { res_.value = false; return res_; }
      }
      if (((((a1_ >> 2) & 1) == 1) && (!any_net_(s, [&](const Envelope& e) { return e.m.type == "ViewReply" && (((e.to == 2) && (((std::stoi(e.m.f[0]) | (std::stoi(e.m.f[1]) << 4)) | (std::stoi(e.m.f[2]) << 6)) == l_view))); })))) {
        { res_.value = false; return res_; }
      }
      if (((((a1_ >> 3) & 1) == 1) && (!any_net_(s, [&](const Envelope& e) { return e.m.type == "ViewReply" && (((e.to == 3) && (((std::stoi(e.m.f[0]) | (std::stoi(e.m.f[1]) << 4)) | (std::stoi(e.m.f[2]) << 6)) == l_view))); })))) {
        { res_.value = false; return res_; }
      }
      if (((((a1_ >> 4) & 1) == 1) && (!any_net_(s, [&](const Envelope& e) { return e.m.type == "ViewReply" && (((e.to == 4) && (((std::stoi(e.m.f[0]) | (std::stoi(e.m.f[1]) << 4)) | (std::stoi(e.m.f[2]) << 6)) == l_view))); })))) {
        { res_.value = false; return res_; }
      }
      if (((((a1_ >> 5) & 1) == 1) && (!any_net_(s, [&](const Envelope& e) { return e.m.type == "ViewReply" && (((e.to == 5) && (((std::stoi(e.m.f[0]) | (std::stoi(e.m.f[1]) << 4)) | (std::stoi(e.m.f[2]) << 6)) == l_view))); })))) {
        { res_.value = false; return res_; }
      }
      { res_.value = true; return res_; }
      return res_;
    }};
  }
  return std::nullopt;
}

}  // namespace pb_ir
}  // namespace oracle
