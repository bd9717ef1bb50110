// GENERATED from the protocol IR (dslabs_amd/ir/specs/multipaxos.py) by dslabs_amd/ir/gen_oracle.py; do not edit.
// oracle/ -- TEST INFRASTRUCTURE ONLY (see oracle_core.hpp).
#pragma once
#include "../oracle_core.hpp"

namespace oracle {
namespace multipaxos_ir {

struct Params {
  int servers = 3;
  int clients = 2;
  int ncmd[2][1] = {};
  int op[2][3] = {};
  int val[2][3] = {};
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
  for (int r = 0; r < 2; r++)
    for (int c = 0; c < 1; c++, q++) p.ncmd[r][c] = q < v.size() ? (int)v[q] : 0;
  for (int r = 0; r < 2; r++)
    for (int c = 0; c < 3; c++, q++) p.op[r][c] = q < v.size() ? (int)v[q] : 0;
  for (int r = 0; r < 2; r++)
    for (int c = 0; c < 3; c++, q++) p.val[r][c] = q < v.size() ? (int)v[q] : 0;
  for (int r = 0; r < 2; r++)
    for (int c = 0; c < 3; c++, q++) p.expected[r][c] = q < v.size() ? (int)v[q] : -1;
  return p;
}
// node index of a kind's first instance: kinds in declaration order, instances consecutive
inline int first_server(const Params& prm) { (void)prm; return 0; }
inline int first_client(const Params& prm) { (void)prm; return 0 + prm.servers; }
inline int wsize(int c, const Params& prm) { (void)c; (void)prm; return prm.ncmd[c][0]; }

struct N_server : Node {
  Params prm;
  int self = 0;
  int round = 0;
  int leader = 0;
  int active = 0;
  int electing = 0;
  int heard = 0;
  int missed = 0;
  int p1bvotes = 0;
  int slotout = 0;
  int slotin = 0;
  std::vector<int> log = std::vector<int>(4, 0);
  std::vector<int> p1blog = std::vector<int>(4, 0);
  std::vector<int> votes = std::vector<int>(4, 0);
  std::shared_ptr<Node> clone() const override { return std::make_shared<N_server>(*this); }
  void key(std::string& out) const override {
    out += "server{";
    out += std::to_string(round) + ",";
    out += std::to_string(leader) + ",";
    out += std::to_string(active) + ",";
    out += std::to_string(electing) + ",";
    out += std::to_string(heard) + ",";
    out += std::to_string(missed) + ",";
    out += std::to_string(p1bvotes) + ",";
    out += std::to_string(slotout) + ",";
    out += std::to_string(slotin) + ",";
    for (int x : log) out += std::to_string(x) + ",";
    for (int x : p1blog) out += std::to_string(x) + ",";
    for (int x : votes) out += std::to_string(x) + ",";
    out += "}";
  }
  std::string str() const override {
    return std::string("server(") + "round=" + std::to_string(round) + ", " + "leader=" + std::to_string(leader) + ", " + "active=" + std::to_string(active) + ", " + "electing=" + std::to_string(electing) + ", " + "heard=" + std::to_string(heard) + ", " + "missed=" + std::to_string(missed) + ", " + "p1bvotes=" + std::to_string(p1bvotes) + ", " + "slotout=" + std::to_string(slotout) + ", " + "slotin=" + std::to_string(slotin) + ")";
  }
  void init(Ctx& ctx) override {
    slotout = 1;
    slotin = 1;
    if (((self - first_server(prm)) == 0)) {
      active = 1;
    }
    ctx.set(Rec{"Tick", {}}, 100, 100);
  }
  void handleMessage(const Rec& m, int from, int, Ctx& ctx) override {
    (void)from; (void)ctx;
    int fl_ = 0;
    bool handled = false;
    if (m.type == "Request") {
      handled = true;
      [&]() {
        const int l_cmd = std::stoi(m.f[0]);
        const int l_c = ((l_cmd >= 4) ? 1 : 0);
        const int l_q = (l_cmd - (((l_cmd >= 4) ? 1 : 0) * 3));
        const int l_upto0 = slotout;
        int l_kv1 = 0;
        int l_ls02 = 0;
        int l_ls13 = 0;
        int l_r4 = 0;
        const int l_cmd5 = ((log[0] >> 8) & 7);
        const int l_c6 = ((l_cmd5 >= 4) ? 1 : 0);
        const int l_q7 = (l_cmd5 - (((l_cmd5 >= 4) ? 1 : 0) * 3));
        if ((((1 < l_upto0) && (l_cmd5 != 0)) && ((l_c6 ? l_ls13 : l_ls02) < l_q7))) {
          const int l_c8 = ((l_cmd5 >= 4) ? 1 : 0);
          const int l_op9 = prm.op[l_c8][((l_cmd5 - (((l_cmd5 >= 4) ? 1 : 0) * 3)) - 1)];
          const int l_v10 = prm.val[l_c8][((l_cmd5 - (((l_cmd5 >= 4) ? 1 : 0) * 3)) - 1)];
          int l_x11 = 0;
          if ((l_op9 == 1)) {
            l_kv1 = (1 | (l_v10 << 3));
            l_x11 = 7;
          }
          if ((l_op9 == 2)) {
            const int l_len12 = (l_kv1 & 7);
            l_kv1 = (((l_len12 + 1) | (l_kv1 & -8)) | (l_v10 << (3 + (l_len12 * 2))));
            l_x11 = l_kv1;
          }
          if ((l_op9 == 3)) {
            l_x11 = (((l_kv1 & 7) != 0) ? l_kv1 : 6);
          }
          if ((l_c6 != 0)) {
            l_ls13 = l_q7;
          } else {
            l_ls02 = l_q7;
          }
          if (((l_c6 == l_c) && (l_q7 == l_q))) {
            l_r4 = l_x11;
          }
        }
        const int l_cmd13 = ((log[1] >> 8) & 7);
        const int l_c14 = ((l_cmd13 >= 4) ? 1 : 0);
        const int l_q15 = (l_cmd13 - (((l_cmd13 >= 4) ? 1 : 0) * 3));
        if ((((2 < l_upto0) && (l_cmd13 != 0)) && ((l_c14 ? l_ls13 : l_ls02) < l_q15))) {
          const int l_c16 = ((l_cmd13 >= 4) ? 1 : 0);
          const int l_op17 = prm.op[l_c16][((l_cmd13 - (((l_cmd13 >= 4) ? 1 : 0) * 3)) - 1)];
          const int l_v18 = prm.val[l_c16][((l_cmd13 - (((l_cmd13 >= 4) ? 1 : 0) * 3)) - 1)];
          int l_x19 = 0;
          if ((l_op17 == 1)) {
            l_kv1 = (1 | (l_v18 << 3));
            l_x19 = 7;
          }
          if ((l_op17 == 2)) {
            const int l_len20 = (l_kv1 & 7);
            l_kv1 = (((l_len20 + 1) | (l_kv1 & -8)) | (l_v18 << (3 + (l_len20 * 2))));
            l_x19 = l_kv1;
          }
          if ((l_op17 == 3)) {
            l_x19 = (((l_kv1 & 7) != 0) ? l_kv1 : 6);
          }
          if ((l_c14 != 0)) {
            l_ls13 = l_q15;
          } else {
            l_ls02 = l_q15;
          }
          if (((l_c14 == l_c) && (l_q15 == l_q))) {
            l_r4 = l_x19;
          }
        }
        const int l_cmd21 = ((log[2] >> 8) & 7);
        const int l_c22 = ((l_cmd21 >= 4) ? 1 : 0);
        const int l_q23 = (l_cmd21 - (((l_cmd21 >= 4) ? 1 : 0) * 3));
        if ((((3 < l_upto0) && (l_cmd21 != 0)) && ((l_c22 ? l_ls13 : l_ls02) < l_q23))) {
          const int l_c24 = ((l_cmd21 >= 4) ? 1 : 0);
          const int l_op25 = prm.op[l_c24][((l_cmd21 - (((l_cmd21 >= 4) ? 1 : 0) * 3)) - 1)];
          const int l_v26 = prm.val[l_c24][((l_cmd21 - (((l_cmd21 >= 4) ? 1 : 0) * 3)) - 1)];
          int l_x27 = 0;
          if ((l_op25 == 1)) {
            l_kv1 = (1 | (l_v26 << 3));
            l_x27 = 7;
          }
          if ((l_op25 == 2)) {
            const int l_len28 = (l_kv1 & 7);
            l_kv1 = (((l_len28 + 1) | (l_kv1 & -8)) | (l_v26 << (3 + (l_len28 * 2))));
            l_x27 = l_kv1;
          }
          if ((l_op25 == 3)) {
            l_x27 = (((l_kv1 & 7) != 0) ? l_kv1 : 6);
          }
          if ((l_c22 != 0)) {
            l_ls13 = l_q23;
          } else {
            l_ls02 = l_q23;
          }
          if (((l_c22 == l_c) && (l_q23 == l_q))) {
            l_r4 = l_x27;
          }
        }
        const int l_cmd29 = ((log[3] >> 8) & 7);
        const int l_c30 = ((l_cmd29 >= 4) ? 1 : 0);
        const int l_q31 = (l_cmd29 - (((l_cmd29 >= 4) ? 1 : 0) * 3));
        if ((((4 < l_upto0) && (l_cmd29 != 0)) && ((l_c30 ? l_ls13 : l_ls02) < l_q31))) {
          const int l_c32 = ((l_cmd29 >= 4) ? 1 : 0);
          const int l_op33 = prm.op[l_c32][((l_cmd29 - (((l_cmd29 >= 4) ? 1 : 0) * 3)) - 1)];
          const int l_v34 = prm.val[l_c32][((l_cmd29 - (((l_cmd29 >= 4) ? 1 : 0) * 3)) - 1)];
          int l_x35 = 0;
          if ((l_op33 == 1)) {
            l_kv1 = (1 | (l_v34 << 3));
            l_x35 = 7;
          }
          if ((l_op33 == 2)) {
            const int l_len36 = (l_kv1 & 7);
            l_kv1 = (((l_len36 + 1) | (l_kv1 & -8)) | (l_v34 << (3 + (l_len36 * 2))));
            l_x35 = l_kv1;
          }
          if ((l_op33 == 3)) {
            l_x35 = (((l_kv1 & 7) != 0) ? l_kv1 : 6);
          }
          if ((l_c30 != 0)) {
            l_ls13 = l_q31;
          } else {
            l_ls02 = l_q31;
          }
          if (((l_c30 == l_c) && (l_q31 == l_q))) {
            l_r4 = l_x35;
          }
        }
        const int l_ls = (l_c ? l_ls13 : l_ls02);
        if ((l_ls >= l_q)) {
          if (((active != 0) && (l_ls == l_q))) {
            ctx.send(Rec{"Reply", {std::to_string(l_q), std::to_string(l_r4)}}, (first_client(prm) + (l_c + 1) - 1));
          }
          return;
        }
        int l_slot = slotin;
        int l_inlog = 0;
        const int l_e37 = log[0];
        if ((((l_e37 & 3) != 0) && (2 > l_slot))) {
          l_slot = 2;
        }
        if ((((l_e37 & 3) != 0) && (((l_e37 >> 8) & 7) == l_cmd))) {
          l_inlog = 1;
        }
        const int l_e38 = log[1];
        if ((((l_e38 & 3) != 0) && (3 > l_slot))) {
          l_slot = 3;
        }
        if ((((l_e38 & 3) != 0) && (((l_e38 >> 8) & 7) == l_cmd))) {
          l_inlog = 1;
        }
        const int l_e39 = log[2];
        if ((((l_e39 & 3) != 0) && (4 > l_slot))) {
          l_slot = 4;
        }
        if ((((l_e39 & 3) != 0) && (((l_e39 >> 8) & 7) == l_cmd))) {
          l_inlog = 1;
        }
        const int l_e40 = log[3];
        if ((((l_e40 & 3) != 0) && (5 > l_slot))) {
          l_slot = 5;
        }
        if ((((l_e40 & 3) != 0) && (((l_e40 >> 8) & 7) == l_cmd))) {
          l_inlog = 1;
        }
        if ((((active == 0) || (l_slot > 4)) || (l_inlog != 0))) {
          return;
        }
        slotin = (l_slot + 1);
        log[(l_slot - 1)] = ((1 | (((round << 2) | leader) << 2)) | (l_cmd << 8));
        votes[(l_slot - 1)] = (1 << (self - first_server(prm)));
        if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
          ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(l_slot), std::to_string(l_cmd)}}, (first_server(prm) + 1 - 1));
        }
        if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
          ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(l_slot), std::to_string(l_cmd)}}, (first_server(prm) + 2 - 1));
        }
        if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
          ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(l_slot), std::to_string(l_cmd)}}, (first_server(prm) + 3 - 1));
        }
        if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
          const int l_ccmd41 = ((log[(l_slot - 1)] >> 8) & 7);
          log[(l_slot - 1)] = ((2 | (0 << 2)) | (l_ccmd41 << 8));
          votes[(l_slot - 1)] = 0;
          if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
            ctx.send(Rec{"Decision", {std::to_string(l_slot), std::to_string(l_ccmd41)}}, (first_server(prm) + 1 - 1));
          }
          if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
            ctx.send(Rec{"Decision", {std::to_string(l_slot), std::to_string(l_ccmd41)}}, (first_server(prm) + 2 - 1));
          }
          if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
            ctx.send(Rec{"Decision", {std::to_string(l_slot), std::to_string(l_ccmd41)}}, (first_server(prm) + 3 - 1));
          }
        }
        if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
          fl_ |= 1;
        }
      }();
    }
    if (m.type == "P1a") {
      handled = true;
      [&]() {
        const int l_b = ((std::stoi(m.f[0]) << 2) | std::stoi(m.f[1]));
        if ((l_b < ((round << 2) | leader))) {
          return;
        }
        if ((l_b > ((round << 2) | leader))) {
          round = (l_b >> 2);
          leader = (l_b & 3);
          active = 0;
          electing = 0;
          p1bvotes = 0;
          votes[0] = 0;
          p1blog[0] = 0;
          votes[1] = 0;
          p1blog[1] = 0;
          votes[2] = 0;
          p1blog[2] = 0;
          votes[3] = 0;
          p1blog[3] = 0;
        }
        heard = 1;
        ctx.send(Rec{"P1b", {std::to_string(std::stoi(m.f[0])), std::to_string(std::stoi(m.f[1])), std::to_string(log[0]), std::to_string(log[1]), std::to_string(log[2]), std::to_string(log[3])}}, from);
      }();
    }
    if (m.type == "P1b") {
      handled = true;
      [&]() {
        const int l_b = ((std::stoi(m.f[0]) << 2) | std::stoi(m.f[1]));
        if (((electing == 0) || (l_b != ((round << 2) | leader)))) {
          return;
        }
        const int l_v = (p1bvotes | (1 << (from - (first_server(prm) + 1 - 1))));
        p1bvotes = l_v;
        const int l_me42 = std::stoi(m.f[2]);
        const int l_mm43 = p1blog[0];
        if (((l_me42 & 3) == 2)) {
          p1blog[0] = ((2 | (0 << 2)) | (((l_me42 >> 8) & 7) << 8));
        } else {
          if (((((l_me42 & 3) == 1) && ((l_mm43 & 3) != 2)) && (((l_mm43 & 3) == 0) || (((l_mm43 >> 2) & 63) < ((l_me42 >> 2) & 63))))) {
            p1blog[0] = l_me42;
          }
        }
        const int l_me44 = std::stoi(m.f[3]);
        const int l_mm45 = p1blog[1];
        if (((l_me44 & 3) == 2)) {
          p1blog[1] = ((2 | (0 << 2)) | (((l_me44 >> 8) & 7) << 8));
        } else {
          if (((((l_me44 & 3) == 1) && ((l_mm45 & 3) != 2)) && (((l_mm45 & 3) == 0) || (((l_mm45 >> 2) & 63) < ((l_me44 >> 2) & 63))))) {
            p1blog[1] = l_me44;
          }
        }
        const int l_me46 = std::stoi(m.f[4]);
        const int l_mm47 = p1blog[2];
        if (((l_me46 & 3) == 2)) {
          p1blog[2] = ((2 | (0 << 2)) | (((l_me46 >> 8) & 7) << 8));
        } else {
          if (((((l_me46 & 3) == 1) && ((l_mm47 & 3) != 2)) && (((l_mm47 & 3) == 0) || (((l_mm47 >> 2) & 63) < ((l_me46 >> 2) & 63))))) {
            p1blog[2] = l_me46;
          }
        }
        const int l_me48 = std::stoi(m.f[5]);
        const int l_mm49 = p1blog[3];
        if (((l_me48 & 3) == 2)) {
          p1blog[3] = ((2 | (0 << 2)) | (((l_me48 >> 8) & 7) << 8));
        } else {
          if (((((l_me48 & 3) == 1) && ((l_mm49 & 3) != 2)) && (((l_mm49 & 3) == 0) || (((l_mm49 >> 2) & 63) < ((l_me48 >> 2) & 63))))) {
            p1blog[3] = l_me48;
          }
        }
        if ((!(((((l_v & 1) + ((l_v >> 1) & 1)) + ((l_v >> 2) & 1)) * 2) > prm.servers))) {
          return;
        }
        fl_ |= 2;
      }();
    }
    if (m.type == "P2a") {
      handled = true;
      [&]() {
        const int l_b = ((std::stoi(m.f[0]) << 2) | std::stoi(m.f[1]));
        if ((l_b < ((round << 2) | leader))) {
          return;
        }
        if ((l_b > ((round << 2) | leader))) {
          round = (l_b >> 2);
          leader = (l_b & 3);
          active = 0;
          electing = 0;
          p1bvotes = 0;
          votes[0] = 0;
          p1blog[0] = 0;
          votes[1] = 0;
          p1blog[1] = 0;
          votes[2] = 0;
          p1blog[2] = 0;
          votes[3] = 0;
          p1blog[3] = 0;
        }
        heard = 1;
        const int l_slot = std::stoi(m.f[2]);
        if (((log[(l_slot - 1)] & 3) != 2)) {
          log[(l_slot - 1)] = ((1 | (l_b << 2)) | (std::stoi(m.f[3]) << 8));
        }
        ctx.send(Rec{"P2b", {std::to_string(std::stoi(m.f[0])), std::to_string(std::stoi(m.f[1])), std::to_string(l_slot)}}, from);
      }();
    }
    if (m.type == "P2b") {
      handled = true;
      [&]() {
        const int l_b = ((std::stoi(m.f[0]) << 2) | std::stoi(m.f[1]));
        const int l_slot = std::stoi(m.f[2]);
        if ((((active == 0) || (l_b != ((round << 2) | leader))) || ((log[(l_slot - 1)] & 3) != 1))) {
          return;
        }
        const int l_v = (votes[(l_slot - 1)] | (1 << (from - (first_server(prm) + 1 - 1))));
        votes[(l_slot - 1)] = l_v;
        if ((!(((((l_v & 1) + ((l_v >> 1) & 1)) + ((l_v >> 2) & 1)) * 2) > prm.servers))) {
          return;
        }
        const int l_ccmd50 = ((log[(l_slot - 1)] >> 8) & 7);
        log[(l_slot - 1)] = ((2 | (0 << 2)) | (l_ccmd50 << 8));
        votes[(l_slot - 1)] = 0;
        if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
          ctx.send(Rec{"Decision", {std::to_string(l_slot), std::to_string(l_ccmd50)}}, (first_server(prm) + 1 - 1));
        }
        if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
          ctx.send(Rec{"Decision", {std::to_string(l_slot), std::to_string(l_ccmd50)}}, (first_server(prm) + 2 - 1));
        }
        if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
          ctx.send(Rec{"Decision", {std::to_string(l_slot), std::to_string(l_ccmd50)}}, (first_server(prm) + 3 - 1));
        }
        fl_ |= 1;
      }();
    }
    if (m.type == "Decision") {
      handled = true;
      [&]() {
        const int l_slot = std::stoi(m.f[0]);
        if (((log[(l_slot - 1)] & 3) == 2)) {
          return;
        }
        log[(l_slot - 1)] = ((2 | (0 << 2)) | (std::stoi(m.f[1]) << 8));
        votes[(l_slot - 1)] = 0;
        fl_ |= 1;
      }();
    }
    if (m.type == "Heartbeat") {
      handled = true;
      [&]() {
        const int l_b = ((std::stoi(m.f[0]) << 2) | std::stoi(m.f[1]));
        if ((l_b < ((round << 2) | leader))) {
          return;
        }
        if ((l_b > ((round << 2) | leader))) {
          round = (l_b >> 2);
          leader = (l_b & 3);
          active = 0;
          electing = 0;
          p1bvotes = 0;
          votes[0] = 0;
          p1blog[0] = 0;
          votes[1] = 0;
          p1blog[1] = 0;
          votes[2] = 0;
          p1blog[2] = 0;
          votes[3] = 0;
          p1blog[3] = 0;
        }
        heard = 1;
      }();
    }
    if (!handled) throw HandlerException("no handler");
    if (fl_) {
      if (((fl_ >> 1) & 1)) {
        active = 1;
        electing = 0;
        p1bvotes = 0;
        const int l_mg51 = p1blog[0];
        const int l_mg52 = p1blog[1];
        const int l_mg53 = p1blog[2];
        const int l_mg54 = p1blog[3];
        int l_last55 = 0;
        if ((((l_mg51 & 3) != 0) || ((log[0] & 3) != 0))) {
          l_last55 = 1;
        }
        if ((((l_mg52 & 3) != 0) || ((log[1] & 3) != 0))) {
          l_last55 = 2;
        }
        if ((((l_mg53 & 3) != 0) || ((log[2] & 3) != 0))) {
          l_last55 = 3;
        }
        if ((((l_mg54 & 3) != 0) || ((log[3] & 3) != 0))) {
          l_last55 = 4;
        }
        p1blog[0] = 0;
        p1blog[1] = 0;
        p1blog[2] = 0;
        p1blog[3] = 0;
        if (((1 <= l_last55) && ((log[0] & 3) != 2))) {
          if (((l_mg51 & 3) == 2)) {
            log[0] = ((2 | (0 << 2)) | (((l_mg51 >> 8) & 7) << 8));
            votes[0] = 0;
          } else {
            log[(1 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg51 & 3) == 1) ? ((l_mg51 >> 8) & 7) : 0) << 8));
            votes[(1 - 1)] = (1 << (self - first_server(prm)));
            if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(1), std::to_string((((l_mg51 & 3) == 1) ? ((l_mg51 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
            }
            if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(1), std::to_string((((l_mg51 & 3) == 1) ? ((l_mg51 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
            }
            if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(1), std::to_string((((l_mg51 & 3) == 1) ? ((l_mg51 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
            }
            if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
              const int l_ccmd56 = ((log[(1 - 1)] >> 8) & 7);
              log[(1 - 1)] = ((2 | (0 << 2)) | (l_ccmd56 << 8));
              votes[(1 - 1)] = 0;
              if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(1), std::to_string(l_ccmd56)}}, (first_server(prm) + 1 - 1));
              }
              if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(1), std::to_string(l_ccmd56)}}, (first_server(prm) + 2 - 1));
              }
              if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(1), std::to_string(l_ccmd56)}}, (first_server(prm) + 3 - 1));
              }
            }
          }
        }
        if (((2 <= l_last55) && ((log[1] & 3) != 2))) {
          if (((l_mg52 & 3) == 2)) {
            log[1] = ((2 | (0 << 2)) | (((l_mg52 >> 8) & 7) << 8));
            votes[1] = 0;
          } else {
            log[(2 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg52 & 3) == 1) ? ((l_mg52 >> 8) & 7) : 0) << 8));
            votes[(2 - 1)] = (1 << (self - first_server(prm)));
            if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(2), std::to_string((((l_mg52 & 3) == 1) ? ((l_mg52 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
            }
            if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(2), std::to_string((((l_mg52 & 3) == 1) ? ((l_mg52 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
            }
            if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(2), std::to_string((((l_mg52 & 3) == 1) ? ((l_mg52 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
            }
            if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
              const int l_ccmd57 = ((log[(2 - 1)] >> 8) & 7);
              log[(2 - 1)] = ((2 | (0 << 2)) | (l_ccmd57 << 8));
              votes[(2 - 1)] = 0;
              if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(2), std::to_string(l_ccmd57)}}, (first_server(prm) + 1 - 1));
              }
              if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(2), std::to_string(l_ccmd57)}}, (first_server(prm) + 2 - 1));
              }
              if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(2), std::to_string(l_ccmd57)}}, (first_server(prm) + 3 - 1));
              }
            }
          }
        }
        if (((3 <= l_last55) && ((log[2] & 3) != 2))) {
          if (((l_mg53 & 3) == 2)) {
            log[2] = ((2 | (0 << 2)) | (((l_mg53 >> 8) & 7) << 8));
            votes[2] = 0;
          } else {
            log[(3 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg53 & 3) == 1) ? ((l_mg53 >> 8) & 7) : 0) << 8));
            votes[(3 - 1)] = (1 << (self - first_server(prm)));
            if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(3), std::to_string((((l_mg53 & 3) == 1) ? ((l_mg53 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
            }
            if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(3), std::to_string((((l_mg53 & 3) == 1) ? ((l_mg53 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
            }
            if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(3), std::to_string((((l_mg53 & 3) == 1) ? ((l_mg53 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
            }
            if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
              const int l_ccmd58 = ((log[(3 - 1)] >> 8) & 7);
              log[(3 - 1)] = ((2 | (0 << 2)) | (l_ccmd58 << 8));
              votes[(3 - 1)] = 0;
              if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(3), std::to_string(l_ccmd58)}}, (first_server(prm) + 1 - 1));
              }
              if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(3), std::to_string(l_ccmd58)}}, (first_server(prm) + 2 - 1));
              }
              if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(3), std::to_string(l_ccmd58)}}, (first_server(prm) + 3 - 1));
              }
            }
          }
        }
        if (((4 <= l_last55) && ((log[3] & 3) != 2))) {
          if (((l_mg54 & 3) == 2)) {
            log[3] = ((2 | (0 << 2)) | (((l_mg54 >> 8) & 7) << 8));
            votes[3] = 0;
          } else {
            log[(4 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg54 & 3) == 1) ? ((l_mg54 >> 8) & 7) : 0) << 8));
            votes[(4 - 1)] = (1 << (self - first_server(prm)));
            if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(4), std::to_string((((l_mg54 & 3) == 1) ? ((l_mg54 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
            }
            if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(4), std::to_string((((l_mg54 & 3) == 1) ? ((l_mg54 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
            }
            if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(4), std::to_string((((l_mg54 & 3) == 1) ? ((l_mg54 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
            }
            if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
              const int l_ccmd59 = ((log[(4 - 1)] >> 8) & 7);
              log[(4 - 1)] = ((2 | (0 << 2)) | (l_ccmd59 << 8));
              votes[(4 - 1)] = 0;
              if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(4), std::to_string(l_ccmd59)}}, (first_server(prm) + 1 - 1));
              }
              if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(4), std::to_string(l_ccmd59)}}, (first_server(prm) + 2 - 1));
              }
              if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(4), std::to_string(l_ccmd59)}}, (first_server(prm) + 3 - 1));
              }
            }
          }
        }
        slotin = (l_last55 + 1);
      }
      const int l_so060 = slotout;
      const int l_act61 = active;
      int l_kv62 = 0;
      int l_ls063 = 0;
      int l_ls164 = 0;
      int l_so65 = l_so060;
      int l_run66 = 1;
      const int l_e67 = log[0];
      const int l_cmd68 = ((l_e67 >> 8) & 7);
      const int l_c69 = ((l_cmd68 >= 4) ? 1 : 0);
      const int l_q70 = (l_cmd68 - (((l_cmd68 >= 4) ? 1 : 0) * 3));
      const int l_before71 = (1 < l_so060);
      const int l_now72 = (((!l_before71) && (l_run66 != 0)) && ((l_e67 & 3) == 2));
      l_run66 = (((l_run66 != 0) && (l_before71 || l_now72)) ? 1 : 0);
      if ((((l_before71 || l_now72) && (l_cmd68 != 0)) && ((l_c69 ? l_ls164 : l_ls063) < l_q70))) {
        const int l_c73 = ((l_cmd68 >= 4) ? 1 : 0);
        const int l_op74 = prm.op[l_c73][((l_cmd68 - (((l_cmd68 >= 4) ? 1 : 0) * 3)) - 1)];
        const int l_v75 = prm.val[l_c73][((l_cmd68 - (((l_cmd68 >= 4) ? 1 : 0) * 3)) - 1)];
        int l_x76 = 0;
        if ((l_op74 == 1)) {
          l_kv62 = (1 | (l_v75 << 3));
          l_x76 = 7;
        }
        if ((l_op74 == 2)) {
          const int l_len77 = (l_kv62 & 7);
          l_kv62 = (((l_len77 + 1) | (l_kv62 & -8)) | (l_v75 << (3 + (l_len77 * 2))));
          l_x76 = l_kv62;
        }
        if ((l_op74 == 3)) {
          l_x76 = (((l_kv62 & 7) != 0) ? l_kv62 : 6);
        }
        if ((l_c69 != 0)) {
          l_ls164 = l_q70;
        } else {
          l_ls063 = l_q70;
        }
        if ((l_now72 && (l_act61 != 0))) {
          ctx.send(Rec{"Reply", {std::to_string(l_q70), std::to_string(l_x76)}}, (first_client(prm) + (l_c69 + 1) - 1));
        }
      }
      if (l_now72) {
        l_so65 = 2;
      }
      const int l_e78 = log[1];
      const int l_cmd79 = ((l_e78 >> 8) & 7);
      const int l_c80 = ((l_cmd79 >= 4) ? 1 : 0);
      const int l_q81 = (l_cmd79 - (((l_cmd79 >= 4) ? 1 : 0) * 3));
      const int l_before82 = (2 < l_so060);
      const int l_now83 = (((!l_before82) && (l_run66 != 0)) && ((l_e78 & 3) == 2));
      l_run66 = (((l_run66 != 0) && (l_before82 || l_now83)) ? 1 : 0);
      if ((((l_before82 || l_now83) && (l_cmd79 != 0)) && ((l_c80 ? l_ls164 : l_ls063) < l_q81))) {
        const int l_c84 = ((l_cmd79 >= 4) ? 1 : 0);
        const int l_op85 = prm.op[l_c84][((l_cmd79 - (((l_cmd79 >= 4) ? 1 : 0) * 3)) - 1)];
        const int l_v86 = prm.val[l_c84][((l_cmd79 - (((l_cmd79 >= 4) ? 1 : 0) * 3)) - 1)];
        int l_x87 = 0;
        if ((l_op85 == 1)) {
          l_kv62 = (1 | (l_v86 << 3));
          l_x87 = 7;
        }
        if ((l_op85 == 2)) {
          const int l_len88 = (l_kv62 & 7);
          l_kv62 = (((l_len88 + 1) | (l_kv62 & -8)) | (l_v86 << (3 + (l_len88 * 2))));
          l_x87 = l_kv62;
        }
        if ((l_op85 == 3)) {
          l_x87 = (((l_kv62 & 7) != 0) ? l_kv62 : 6);
        }
        if ((l_c80 != 0)) {
          l_ls164 = l_q81;
        } else {
          l_ls063 = l_q81;
        }
        if ((l_now83 && (l_act61 != 0))) {
          ctx.send(Rec{"Reply", {std::to_string(l_q81), std::to_string(l_x87)}}, (first_client(prm) + (l_c80 + 1) - 1));
        }
      }
      if (l_now83) {
        l_so65 = 3;
      }
      const int l_e89 = log[2];
      const int l_cmd90 = ((l_e89 >> 8) & 7);
      const int l_c91 = ((l_cmd90 >= 4) ? 1 : 0);
      const int l_q92 = (l_cmd90 - (((l_cmd90 >= 4) ? 1 : 0) * 3));
      const int l_before93 = (3 < l_so060);
      const int l_now94 = (((!l_before93) && (l_run66 != 0)) && ((l_e89 & 3) == 2));
      l_run66 = (((l_run66 != 0) && (l_before93 || l_now94)) ? 1 : 0);
      if ((((l_before93 || l_now94) && (l_cmd90 != 0)) && ((l_c91 ? l_ls164 : l_ls063) < l_q92))) {
        const int l_c95 = ((l_cmd90 >= 4) ? 1 : 0);
        const int l_op96 = prm.op[l_c95][((l_cmd90 - (((l_cmd90 >= 4) ? 1 : 0) * 3)) - 1)];
        const int l_v97 = prm.val[l_c95][((l_cmd90 - (((l_cmd90 >= 4) ? 1 : 0) * 3)) - 1)];
        int l_x98 = 0;
        if ((l_op96 == 1)) {
          l_kv62 = (1 | (l_v97 << 3));
          l_x98 = 7;
        }
        if ((l_op96 == 2)) {
          const int l_len99 = (l_kv62 & 7);
          l_kv62 = (((l_len99 + 1) | (l_kv62 & -8)) | (l_v97 << (3 + (l_len99 * 2))));
          l_x98 = l_kv62;
        }
        if ((l_op96 == 3)) {
          l_x98 = (((l_kv62 & 7) != 0) ? l_kv62 : 6);
        }
        if ((l_c91 != 0)) {
          l_ls164 = l_q92;
        } else {
          l_ls063 = l_q92;
        }
        if ((l_now94 && (l_act61 != 0))) {
          ctx.send(Rec{"Reply", {std::to_string(l_q92), std::to_string(l_x98)}}, (first_client(prm) + (l_c91 + 1) - 1));
        }
      }
      if (l_now94) {
        l_so65 = 4;
      }
      const int l_e100 = log[3];
      const int l_cmd101 = ((l_e100 >> 8) & 7);
      const int l_c102 = ((l_cmd101 >= 4) ? 1 : 0);
      const int l_q103 = (l_cmd101 - (((l_cmd101 >= 4) ? 1 : 0) * 3));
      const int l_before104 = (4 < l_so060);
      const int l_now105 = (((!l_before104) && (l_run66 != 0)) && ((l_e100 & 3) == 2));
      l_run66 = (((l_run66 != 0) && (l_before104 || l_now105)) ? 1 : 0);
      if ((((l_before104 || l_now105) && (l_cmd101 != 0)) && ((l_c102 ? l_ls164 : l_ls063) < l_q103))) {
        const int l_c106 = ((l_cmd101 >= 4) ? 1 : 0);
        const int l_op107 = prm.op[l_c106][((l_cmd101 - (((l_cmd101 >= 4) ? 1 : 0) * 3)) - 1)];
        const int l_v108 = prm.val[l_c106][((l_cmd101 - (((l_cmd101 >= 4) ? 1 : 0) * 3)) - 1)];
        int l_x109 = 0;
        if ((l_op107 == 1)) {
          l_kv62 = (1 | (l_v108 << 3));
          l_x109 = 7;
        }
        if ((l_op107 == 2)) {
          const int l_len110 = (l_kv62 & 7);
          l_kv62 = (((l_len110 + 1) | (l_kv62 & -8)) | (l_v108 << (3 + (l_len110 * 2))));
          l_x109 = l_kv62;
        }
        if ((l_op107 == 3)) {
          l_x109 = (((l_kv62 & 7) != 0) ? l_kv62 : 6);
        }
        if ((l_c102 != 0)) {
          l_ls164 = l_q103;
        } else {
          l_ls063 = l_q103;
        }
        if ((l_now105 && (l_act61 != 0))) {
          ctx.send(Rec{"Reply", {std::to_string(l_q103), std::to_string(l_x109)}}, (first_client(prm) + (l_c102 + 1) - 1));
        }
      }
      if (l_now105) {
        l_so65 = 5;
      }
      slotout = l_so65;
    }
  }
  void onTimer(const Rec& t, Ctx& ctx) override {
    (void)ctx;
    if (t.type == "Tick") {
      if ((active != 0)) {
        if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
          ctx.send(Rec{"Heartbeat", {std::to_string(round), std::to_string(leader)}}, (first_server(prm) + 1 - 1));
        }
        if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
          ctx.send(Rec{"Heartbeat", {std::to_string(round), std::to_string(leader)}}, (first_server(prm) + 2 - 1));
        }
        if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
          ctx.send(Rec{"Heartbeat", {std::to_string(round), std::to_string(leader)}}, (first_server(prm) + 3 - 1));
        }
      } else {
        if ((heard != 0)) {
          heard = 0;
          missed = 0;
        } else {
          const int l_mis = (((missed + 1) > 2) ? 2 : (missed + 1));
          missed = l_mis;
          if (((l_mis >= 2) && (round < 15))) {
            missed = 0;
            heard = 0;
            round = (round + 1);
            leader = (self - first_server(prm));
            electing = 1;
            active = 0;
            votes[0] = 0;
            p1blog[0] = 0;
            votes[1] = 0;
            p1blog[1] = 0;
            votes[2] = 0;
            p1blog[2] = 0;
            votes[3] = 0;
            p1blog[3] = 0;
            p1bvotes = (1 << (self - first_server(prm)));
            const int l_me111 = log[0];
            const int l_mm112 = p1blog[0];
            if (((l_me111 & 3) == 2)) {
              p1blog[0] = ((2 | (0 << 2)) | (((l_me111 >> 8) & 7) << 8));
            } else {
              if (((((l_me111 & 3) == 1) && ((l_mm112 & 3) != 2)) && (((l_mm112 & 3) == 0) || (((l_mm112 >> 2) & 63) < ((l_me111 >> 2) & 63))))) {
                p1blog[0] = l_me111;
              }
            }
            const int l_me113 = log[1];
            const int l_mm114 = p1blog[1];
            if (((l_me113 & 3) == 2)) {
              p1blog[1] = ((2 | (0 << 2)) | (((l_me113 >> 8) & 7) << 8));
            } else {
              if (((((l_me113 & 3) == 1) && ((l_mm114 & 3) != 2)) && (((l_mm114 & 3) == 0) || (((l_mm114 >> 2) & 63) < ((l_me113 >> 2) & 63))))) {
                p1blog[1] = l_me113;
              }
            }
            const int l_me115 = log[2];
            const int l_mm116 = p1blog[2];
            if (((l_me115 & 3) == 2)) {
              p1blog[2] = ((2 | (0 << 2)) | (((l_me115 >> 8) & 7) << 8));
            } else {
              if (((((l_me115 & 3) == 1) && ((l_mm116 & 3) != 2)) && (((l_mm116 & 3) == 0) || (((l_mm116 >> 2) & 63) < ((l_me115 >> 2) & 63))))) {
                p1blog[2] = l_me115;
              }
            }
            const int l_me117 = log[3];
            const int l_mm118 = p1blog[3];
            if (((l_me117 & 3) == 2)) {
              p1blog[3] = ((2 | (0 << 2)) | (((l_me117 >> 8) & 7) << 8));
            } else {
              if (((((l_me117 & 3) == 1) && ((l_mm118 & 3) != 2)) && (((l_mm118 & 3) == 0) || (((l_mm118 >> 2) & 63) < ((l_me117 >> 2) & 63))))) {
                p1blog[3] = l_me117;
              }
            }
            if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
              ctx.send(Rec{"P1a", {std::to_string(round), std::to_string(leader)}}, (first_server(prm) + 1 - 1));
            }
            if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
              ctx.send(Rec{"P1a", {std::to_string(round), std::to_string(leader)}}, (first_server(prm) + 2 - 1));
            }
            if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
              ctx.send(Rec{"P1a", {std::to_string(round), std::to_string(leader)}}, (first_server(prm) + 3 - 1));
            }
            if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
              active = 1;
              electing = 0;
              p1bvotes = 0;
              const int l_mg119 = p1blog[0];
              const int l_mg120 = p1blog[1];
              const int l_mg121 = p1blog[2];
              const int l_mg122 = p1blog[3];
              int l_last123 = 0;
              if ((((l_mg119 & 3) != 0) || ((log[0] & 3) != 0))) {
                l_last123 = 1;
              }
              if ((((l_mg120 & 3) != 0) || ((log[1] & 3) != 0))) {
                l_last123 = 2;
              }
              if ((((l_mg121 & 3) != 0) || ((log[2] & 3) != 0))) {
                l_last123 = 3;
              }
              if ((((l_mg122 & 3) != 0) || ((log[3] & 3) != 0))) {
                l_last123 = 4;
              }
              p1blog[0] = 0;
              p1blog[1] = 0;
              p1blog[2] = 0;
              p1blog[3] = 0;
              if (((1 <= l_last123) && ((log[0] & 3) != 2))) {
                if (((l_mg119 & 3) == 2)) {
                  log[0] = ((2 | (0 << 2)) | (((l_mg119 >> 8) & 7) << 8));
                  votes[0] = 0;
                } else {
                  log[(1 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg119 & 3) == 1) ? ((l_mg119 >> 8) & 7) : 0) << 8));
                  votes[(1 - 1)] = (1 << (self - first_server(prm)));
                  if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(1), std::to_string((((l_mg119 & 3) == 1) ? ((l_mg119 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
                  }
                  if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(1), std::to_string((((l_mg119 & 3) == 1) ? ((l_mg119 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
                  }
                  if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(1), std::to_string((((l_mg119 & 3) == 1) ? ((l_mg119 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
                  }
                  if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
                    const int l_ccmd124 = ((log[(1 - 1)] >> 8) & 7);
                    log[(1 - 1)] = ((2 | (0 << 2)) | (l_ccmd124 << 8));
                    votes[(1 - 1)] = 0;
                    if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(1), std::to_string(l_ccmd124)}}, (first_server(prm) + 1 - 1));
                    }
                    if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(1), std::to_string(l_ccmd124)}}, (first_server(prm) + 2 - 1));
                    }
                    if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(1), std::to_string(l_ccmd124)}}, (first_server(prm) + 3 - 1));
                    }
                  }
                }
              }
              if (((2 <= l_last123) && ((log[1] & 3) != 2))) {
                if (((l_mg120 & 3) == 2)) {
                  log[1] = ((2 | (0 << 2)) | (((l_mg120 >> 8) & 7) << 8));
                  votes[1] = 0;
                } else {
                  log[(2 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg120 & 3) == 1) ? ((l_mg120 >> 8) & 7) : 0) << 8));
                  votes[(2 - 1)] = (1 << (self - first_server(prm)));
                  if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(2), std::to_string((((l_mg120 & 3) == 1) ? ((l_mg120 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
                  }
                  if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(2), std::to_string((((l_mg120 & 3) == 1) ? ((l_mg120 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
                  }
                  if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(2), std::to_string((((l_mg120 & 3) == 1) ? ((l_mg120 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
                  }
                  if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
                    const int l_ccmd125 = ((log[(2 - 1)] >> 8) & 7);
                    log[(2 - 1)] = ((2 | (0 << 2)) | (l_ccmd125 << 8));
                    votes[(2 - 1)] = 0;
                    if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(2), std::to_string(l_ccmd125)}}, (first_server(prm) + 1 - 1));
                    }
                    if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(2), std::to_string(l_ccmd125)}}, (first_server(prm) + 2 - 1));
                    }
                    if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(2), std::to_string(l_ccmd125)}}, (first_server(prm) + 3 - 1));
                    }
                  }
                }
              }
              if (((3 <= l_last123) && ((log[2] & 3) != 2))) {
                if (((l_mg121 & 3) == 2)) {
                  log[2] = ((2 | (0 << 2)) | (((l_mg121 >> 8) & 7) << 8));
                  votes[2] = 0;
                } else {
                  log[(3 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg121 & 3) == 1) ? ((l_mg121 >> 8) & 7) : 0) << 8));
                  votes[(3 - 1)] = (1 << (self - first_server(prm)));
                  if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(3), std::to_string((((l_mg121 & 3) == 1) ? ((l_mg121 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
                  }
                  if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(3), std::to_string((((l_mg121 & 3) == 1) ? ((l_mg121 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
                  }
                  if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(3), std::to_string((((l_mg121 & 3) == 1) ? ((l_mg121 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
                  }
                  if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
                    const int l_ccmd126 = ((log[(3 - 1)] >> 8) & 7);
                    log[(3 - 1)] = ((2 | (0 << 2)) | (l_ccmd126 << 8));
                    votes[(3 - 1)] = 0;
                    if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(3), std::to_string(l_ccmd126)}}, (first_server(prm) + 1 - 1));
                    }
                    if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(3), std::to_string(l_ccmd126)}}, (first_server(prm) + 2 - 1));
                    }
                    if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(3), std::to_string(l_ccmd126)}}, (first_server(prm) + 3 - 1));
                    }
                  }
                }
              }
              if (((4 <= l_last123) && ((log[3] & 3) != 2))) {
                if (((l_mg122 & 3) == 2)) {
                  log[3] = ((2 | (0 << 2)) | (((l_mg122 >> 8) & 7) << 8));
                  votes[3] = 0;
                } else {
                  log[(4 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg122 & 3) == 1) ? ((l_mg122 >> 8) & 7) : 0) << 8));
                  votes[(4 - 1)] = (1 << (self - first_server(prm)));
                  if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(4), std::to_string((((l_mg122 & 3) == 1) ? ((l_mg122 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
                  }
                  if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(4), std::to_string((((l_mg122 & 3) == 1) ? ((l_mg122 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
                  }
                  if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(4), std::to_string((((l_mg122 & 3) == 1) ? ((l_mg122 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
                  }
                  if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
                    const int l_ccmd127 = ((log[(4 - 1)] >> 8) & 7);
                    log[(4 - 1)] = ((2 | (0 << 2)) | (l_ccmd127 << 8));
                    votes[(4 - 1)] = 0;
                    if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(4), std::to_string(l_ccmd127)}}, (first_server(prm) + 1 - 1));
                    }
                    if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(4), std::to_string(l_ccmd127)}}, (first_server(prm) + 2 - 1));
                    }
                    if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(4), std::to_string(l_ccmd127)}}, (first_server(prm) + 3 - 1));
                    }
                  }
                }
              }
              slotin = (l_last123 + 1);
              const int l_so0128 = slotout;
              const int l_act129 = active;
              int l_kv130 = 0;
              int l_ls0131 = 0;
              int l_ls1132 = 0;
              int l_so133 = l_so0128;
              int l_run134 = 1;
              const int l_e135 = log[0];
              const int l_cmd136 = ((l_e135 >> 8) & 7);
              const int l_c137 = ((l_cmd136 >= 4) ? 1 : 0);
              const int l_q138 = (l_cmd136 - (((l_cmd136 >= 4) ? 1 : 0) * 3));
              const int l_before139 = (1 < l_so0128);
              const int l_now140 = (((!l_before139) && (l_run134 != 0)) && ((l_e135 & 3) == 2));
              l_run134 = (((l_run134 != 0) && (l_before139 || l_now140)) ? 1 : 0);
              if ((((l_before139 || l_now140) && (l_cmd136 != 0)) && ((l_c137 ? l_ls1132 : l_ls0131) < l_q138))) {
                const int l_c141 = ((l_cmd136 >= 4) ? 1 : 0);
                const int l_op142 = prm.op[l_c141][((l_cmd136 - (((l_cmd136 >= 4) ? 1 : 0) * 3)) - 1)];
                const int l_v143 = prm.val[l_c141][((l_cmd136 - (((l_cmd136 >= 4) ? 1 : 0) * 3)) - 1)];
                int l_x144 = 0;
                if ((l_op142 == 1)) {
                  l_kv130 = (1 | (l_v143 << 3));
                  l_x144 = 7;
                }
                if ((l_op142 == 2)) {
                  const int l_len145 = (l_kv130 & 7);
                  l_kv130 = (((l_len145 + 1) | (l_kv130 & -8)) | (l_v143 << (3 + (l_len145 * 2))));
                  l_x144 = l_kv130;
                }
                if ((l_op142 == 3)) {
                  l_x144 = (((l_kv130 & 7) != 0) ? l_kv130 : 6);
                }
                if ((l_c137 != 0)) {
                  l_ls1132 = l_q138;
                } else {
                  l_ls0131 = l_q138;
                }
                if ((l_now140 && (l_act129 != 0))) {
                  ctx.send(Rec{"Reply", {std::to_string(l_q138), std::to_string(l_x144)}}, (first_client(prm) + (l_c137 + 1) - 1));
                }
              }
              if (l_now140) {
                l_so133 = 2;
              }
              const int l_e146 = log[1];
              const int l_cmd147 = ((l_e146 >> 8) & 7);
              const int l_c148 = ((l_cmd147 >= 4) ? 1 : 0);
              const int l_q149 = (l_cmd147 - (((l_cmd147 >= 4) ? 1 : 0) * 3));
              const int l_before150 = (2 < l_so0128);
              const int l_now151 = (((!l_before150) && (l_run134 != 0)) && ((l_e146 & 3) == 2));
              l_run134 = (((l_run134 != 0) && (l_before150 || l_now151)) ? 1 : 0);
              if ((((l_before150 || l_now151) && (l_cmd147 != 0)) && ((l_c148 ? l_ls1132 : l_ls0131) < l_q149))) {
                const int l_c152 = ((l_cmd147 >= 4) ? 1 : 0);
                const int l_op153 = prm.op[l_c152][((l_cmd147 - (((l_cmd147 >= 4) ? 1 : 0) * 3)) - 1)];
                const int l_v154 = prm.val[l_c152][((l_cmd147 - (((l_cmd147 >= 4) ? 1 : 0) * 3)) - 1)];
                int l_x155 = 0;
                if ((l_op153 == 1)) {
                  l_kv130 = (1 | (l_v154 << 3));
                  l_x155 = 7;
                }
                if ((l_op153 == 2)) {
                  const int l_len156 = (l_kv130 & 7);
                  l_kv130 = (((l_len156 + 1) | (l_kv130 & -8)) | (l_v154 << (3 + (l_len156 * 2))));
                  l_x155 = l_kv130;
                }
                if ((l_op153 == 3)) {
                  l_x155 = (((l_kv130 & 7) != 0) ? l_kv130 : 6);
                }
                if ((l_c148 != 0)) {
                  l_ls1132 = l_q149;
                } else {
                  l_ls0131 = l_q149;
                }
                if ((l_now151 && (l_act129 != 0))) {
                  ctx.send(Rec{"Reply", {std::to_string(l_q149), std::to_string(l_x155)}}, (first_client(prm) + (l_c148 + 1) - 1));
                }
              }
              if (l_now151) {
                l_so133 = 3;
              }
              const int l_e157 = log[2];
              const int l_cmd158 = ((l_e157 >> 8) & 7);
              const int l_c159 = ((l_cmd158 >= 4) ? 1 : 0);
              const int l_q160 = (l_cmd158 - (((l_cmd158 >= 4) ? 1 : 0) * 3));
              const int l_before161 = (3 < l_so0128);
              const int l_now162 = (((!l_before161) && (l_run134 != 0)) && ((l_e157 & 3) == 2));
              l_run134 = (((l_run134 != 0) && (l_before161 || l_now162)) ? 1 : 0);
              if ((((l_before161 || l_now162) && (l_cmd158 != 0)) && ((l_c159 ? l_ls1132 : l_ls0131) < l_q160))) {
                const int l_c163 = ((l_cmd158 >= 4) ? 1 : 0);
                const int l_op164 = prm.op[l_c163][((l_cmd158 - (((l_cmd158 >= 4) ? 1 : 0) * 3)) - 1)];
                const int l_v165 = prm.val[l_c163][((l_cmd158 - (((l_cmd158 >= 4) ? 1 : 0) * 3)) - 1)];
                int l_x166 = 0;
                if ((l_op164 == 1)) {
                  l_kv130 = (1 | (l_v165 << 3));
                  l_x166 = 7;
                }
                if ((l_op164 == 2)) {
                  const int l_len167 = (l_kv130 & 7);
                  l_kv130 = (((l_len167 + 1) | (l_kv130 & -8)) | (l_v165 << (3 + (l_len167 * 2))));
                  l_x166 = l_kv130;
                }
                if ((l_op164 == 3)) {
                  l_x166 = (((l_kv130 & 7) != 0) ? l_kv130 : 6);
                }
                if ((l_c159 != 0)) {
                  l_ls1132 = l_q160;
                } else {
                  l_ls0131 = l_q160;
                }
                if ((l_now162 && (l_act129 != 0))) {
                  ctx.send(Rec{"Reply", {std::to_string(l_q160), std::to_string(l_x166)}}, (first_client(prm) + (l_c159 + 1) - 1));
                }
              }
              if (l_now162) {
                l_so133 = 4;
              }
              const int l_e168 = log[3];
              const int l_cmd169 = ((l_e168 >> 8) & 7);
              const int l_c170 = ((l_cmd169 >= 4) ? 1 : 0);
              const int l_q171 = (l_cmd169 - (((l_cmd169 >= 4) ? 1 : 0) * 3));
              const int l_before172 = (4 < l_so0128);
              const int l_now173 = (((!l_before172) && (l_run134 != 0)) && ((l_e168 & 3) == 2));
              l_run134 = (((l_run134 != 0) && (l_before172 || l_now173)) ? 1 : 0);
              if ((((l_before172 || l_now173) && (l_cmd169 != 0)) && ((l_c170 ? l_ls1132 : l_ls0131) < l_q171))) {
                const int l_c174 = ((l_cmd169 >= 4) ? 1 : 0);
                const int l_op175 = prm.op[l_c174][((l_cmd169 - (((l_cmd169 >= 4) ? 1 : 0) * 3)) - 1)];
                const int l_v176 = prm.val[l_c174][((l_cmd169 - (((l_cmd169 >= 4) ? 1 : 0) * 3)) - 1)];
                int l_x177 = 0;
                if ((l_op175 == 1)) {
                  l_kv130 = (1 | (l_v176 << 3));
                  l_x177 = 7;
                }
                if ((l_op175 == 2)) {
                  const int l_len178 = (l_kv130 & 7);
                  l_kv130 = (((l_len178 + 1) | (l_kv130 & -8)) | (l_v176 << (3 + (l_len178 * 2))));
                  l_x177 = l_kv130;
                }
                if ((l_op175 == 3)) {
                  l_x177 = (((l_kv130 & 7) != 0) ? l_kv130 : 6);
                }
                if ((l_c170 != 0)) {
                  l_ls1132 = l_q171;
                } else {
                  l_ls0131 = l_q171;
                }
                if ((l_now173 && (l_act129 != 0))) {
                  ctx.send(Rec{"Reply", {std::to_string(l_q171), std::to_string(l_x177)}}, (first_client(prm) + (l_c170 + 1) - 1));
                }
              }
              if (l_now173) {
                l_so133 = 5;
              }
              slotout = l_so133;
            }
          }
        }
      }
      ctx.set(Rec{"Tick", {}}, 100, 100);
      return;
    }
    throw HandlerException("no timer handler");
  }
};

struct N_client : Client {
  Params prm;
  int self = 0;
  int seq = 0;
  int pending = 0;
  int result = 0;
  std::shared_ptr<Node> clone() const override { return std::make_shared<N_client>(*this); }
  void key(std::string& out) const override {
    out += "client{";
    out += std::to_string(seq) + ",";
    out += std::to_string(pending) + ",";
    out += std::to_string(result) + ",";
    out += "}";
  }
  std::string str() const override {
    return std::string("client(") + "seq=" + std::to_string(seq) + ", " + "pending=" + std::to_string(pending) + ", " + "result=" + std::to_string(result) + ")";
  }
  void handleMessage(const Rec& m, int from, int, Ctx& ctx) override {
    (void)from; (void)ctx;
    if (m.type == "Reply") {
      if (((pending != 0) && (std::stoi(m.f[0]) == seq))) {
        result = std::stoi(m.f[1]);
        pending = 0;
      }
      return;
    }
    throw HandlerException("no handler");
  }
  void onTimer(const Rec& t, Ctx& ctx) override {
    (void)ctx;
    if (t.type == "ClientTimer") {
      if (((pending != 0) && (std::stoi(t.f[0]) == seq))) {
        const int l_cid179 = (((self - first_client(prm)) * 3) + std::stoi(t.f[0]));
        if ((0 < prm.servers)) {
          ctx.send(Rec{"Request", {std::to_string(l_cid179)}}, (first_server(prm) + 1 - 1));
        }
        if ((1 < prm.servers)) {
          ctx.send(Rec{"Request", {std::to_string(l_cid179)}}, (first_server(prm) + 2 - 1));
        }
        if ((2 < prm.servers)) {
          ctx.send(Rec{"Request", {std::to_string(l_cid179)}}, (first_server(prm) + 3 - 1));
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
    pending = 1;
    result = 0;
    const int l_cid180 = (((self - first_client(prm)) * 3) + cmd);
    if ((0 < prm.servers)) {
      ctx.send(Rec{"Request", {std::to_string(l_cid180)}}, (first_server(prm) + 1 - 1));
    }
    if ((1 < prm.servers)) {
      ctx.send(Rec{"Request", {std::to_string(l_cid180)}}, (first_server(prm) + 2 - 1));
    }
    if ((2 < prm.servers)) {
      ctx.send(Rec{"Request", {std::to_string(l_cid180)}}, (first_server(prm) + 3 - 1));
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
  if ((base_ == "LOGS_CONSISTENT_ALL_SLOTS" || base_ == "LOGS_CONSISTENT") && parts_.size() == 1) {
    return Predicate{"Non-empty log slots consistent", [prm, a0_, a1_](const State& s) {
      (void)s; (void)a0_; (void)a1_;
      PredResult res_;
      int l_isch181 = 0;
      int l_confl182 = 0;
      int l_chosen183 = 0;
      int l_count184 = 0;
      if ((0 < prm.servers)) {
        const int l_e185 = n_server(s, first_server(prm) + 0)->log[0];
        if (((l_e185 & 3) == 2)) {
          const int l_x186 = ((((l_e185 >> 8) & 7) != 0) ? ((prm.op[((((l_e185 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e185 >> 8) & 7) - (((((l_e185 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e185 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e185 >> 8) & 7) - (((((l_e185 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch181 != 0) && (l_x186 != l_chosen183))) {
            l_confl182 = 1;
          }
          l_chosen183 = l_x186;
          l_isch181 = 1;
        }
      }
      if ((1 < prm.servers)) {
        const int l_e187 = n_server(s, first_server(prm) + 1)->log[0];
        if (((l_e187 & 3) == 2)) {
          const int l_x188 = ((((l_e187 >> 8) & 7) != 0) ? ((prm.op[((((l_e187 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e187 >> 8) & 7) - (((((l_e187 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e187 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e187 >> 8) & 7) - (((((l_e187 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch181 != 0) && (l_x188 != l_chosen183))) {
            l_confl182 = 1;
          }
          l_chosen183 = l_x188;
          l_isch181 = 1;
        }
      }
      if ((2 < prm.servers)) {
        const int l_e189 = n_server(s, first_server(prm) + 2)->log[0];
        if (((l_e189 & 3) == 2)) {
          const int l_x190 = ((((l_e189 >> 8) & 7) != 0) ? ((prm.op[((((l_e189 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e189 >> 8) & 7) - (((((l_e189 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e189 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e189 >> 8) & 7) - (((((l_e189 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch181 != 0) && (l_x190 != l_chosen183))) {
            l_confl182 = 1;
          }
          l_chosen183 = l_x190;
          l_isch181 = 1;
        }
      }
      if ((0 < prm.servers)) {
        const int l_e191 = n_server(s, first_server(prm) + 0)->log[0];
        if ((((l_e191 & 3) != 0) && (((l_e191 & 3) != 1) || (((((l_e191 >> 8) & 7) != 0) ? ((prm.op[((((l_e191 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e191 >> 8) & 7) - (((((l_e191 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e191 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e191 >> 8) & 7) - (((((l_e191 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen183)))) {
          l_count184 = (l_count184 + 1);
        }
      }
      if ((1 < prm.servers)) {
        const int l_e192 = n_server(s, first_server(prm) + 1)->log[0];
        if ((((l_e192 & 3) != 0) && (((l_e192 & 3) != 1) || (((((l_e192 >> 8) & 7) != 0) ? ((prm.op[((((l_e192 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e192 >> 8) & 7) - (((((l_e192 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e192 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e192 >> 8) & 7) - (((((l_e192 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen183)))) {
          l_count184 = (l_count184 + 1);
        }
      }
      if ((2 < prm.servers)) {
        const int l_e193 = n_server(s, first_server(prm) + 2)->log[0];
        if ((((l_e193 & 3) != 0) && (((l_e193 & 3) != 1) || (((((l_e193 >> 8) & 7) != 0) ? ((prm.op[((((l_e193 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e193 >> 8) & 7) - (((((l_e193 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e193 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e193 >> 8) & 7) - (((((l_e193 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen183)))) {
          l_count184 = (l_count184 + 1);
        }
      }
      if (((l_isch181 != 0) && ((l_confl182 != 0) || ((l_count184 * 2) <= prm.servers)))) {
        { res_.value = false; return res_; }
      }
      int l_isch194 = 0;
      int l_confl195 = 0;
      int l_chosen196 = 0;
      int l_count197 = 0;
      if ((0 < prm.servers)) {
        const int l_e198 = n_server(s, first_server(prm) + 0)->log[1];
        if (((l_e198 & 3) == 2)) {
          const int l_x199 = ((((l_e198 >> 8) & 7) != 0) ? ((prm.op[((((l_e198 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e198 >> 8) & 7) - (((((l_e198 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e198 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e198 >> 8) & 7) - (((((l_e198 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch194 != 0) && (l_x199 != l_chosen196))) {
            l_confl195 = 1;
          }
          l_chosen196 = l_x199;
          l_isch194 = 1;
        }
      }
      if ((1 < prm.servers)) {
        const int l_e200 = n_server(s, first_server(prm) + 1)->log[1];
        if (((l_e200 & 3) == 2)) {
          const int l_x201 = ((((l_e200 >> 8) & 7) != 0) ? ((prm.op[((((l_e200 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e200 >> 8) & 7) - (((((l_e200 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e200 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e200 >> 8) & 7) - (((((l_e200 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch194 != 0) && (l_x201 != l_chosen196))) {
            l_confl195 = 1;
          }
          l_chosen196 = l_x201;
          l_isch194 = 1;
        }
      }
      if ((2 < prm.servers)) {
        const int l_e202 = n_server(s, first_server(prm) + 2)->log[1];
        if (((l_e202 & 3) == 2)) {
          const int l_x203 = ((((l_e202 >> 8) & 7) != 0) ? ((prm.op[((((l_e202 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e202 >> 8) & 7) - (((((l_e202 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e202 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e202 >> 8) & 7) - (((((l_e202 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch194 != 0) && (l_x203 != l_chosen196))) {
            l_confl195 = 1;
          }
          l_chosen196 = l_x203;
          l_isch194 = 1;
        }
      }
      if ((0 < prm.servers)) {
        const int l_e204 = n_server(s, first_server(prm) + 0)->log[1];
        if ((((l_e204 & 3) != 0) && (((l_e204 & 3) != 1) || (((((l_e204 >> 8) & 7) != 0) ? ((prm.op[((((l_e204 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e204 >> 8) & 7) - (((((l_e204 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e204 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e204 >> 8) & 7) - (((((l_e204 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen196)))) {
          l_count197 = (l_count197 + 1);
        }
      }
      if ((1 < prm.servers)) {
        const int l_e205 = n_server(s, first_server(prm) + 1)->log[1];
        if ((((l_e205 & 3) != 0) && (((l_e205 & 3) != 1) || (((((l_e205 >> 8) & 7) != 0) ? ((prm.op[((((l_e205 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e205 >> 8) & 7) - (((((l_e205 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e205 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e205 >> 8) & 7) - (((((l_e205 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen196)))) {
          l_count197 = (l_count197 + 1);
        }
      }
      if ((2 < prm.servers)) {
        const int l_e206 = n_server(s, first_server(prm) + 2)->log[1];
        if ((((l_e206 & 3) != 0) && (((l_e206 & 3) != 1) || (((((l_e206 >> 8) & 7) != 0) ? ((prm.op[((((l_e206 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e206 >> 8) & 7) - (((((l_e206 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e206 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e206 >> 8) & 7) - (((((l_e206 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen196)))) {
          l_count197 = (l_count197 + 1);
        }
      }
      if (((l_isch194 != 0) && ((l_confl195 != 0) || ((l_count197 * 2) <= prm.servers)))) {
        { res_.value = false; return res_; }
      }
      int l_isch207 = 0;
      int l_confl208 = 0;
      int l_chosen209 = 0;
      int l_count210 = 0;
      if ((0 < prm.servers)) {
        const int l_e211 = n_server(s, first_server(prm) + 0)->log[2];
        if (((l_e211 & 3) == 2)) {
          const int l_x212 = ((((l_e211 >> 8) & 7) != 0) ? ((prm.op[((((l_e211 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e211 >> 8) & 7) - (((((l_e211 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e211 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e211 >> 8) & 7) - (((((l_e211 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch207 != 0) && (l_x212 != l_chosen209))) {
            l_confl208 = 1;
          }
          l_chosen209 = l_x212;
          l_isch207 = 1;
        }
      }
      if ((1 < prm.servers)) {
        const int l_e213 = n_server(s, first_server(prm) + 1)->log[2];
        if (((l_e213 & 3) == 2)) {
          const int l_x214 = ((((l_e213 >> 8) & 7) != 0) ? ((prm.op[((((l_e213 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e213 >> 8) & 7) - (((((l_e213 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e213 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e213 >> 8) & 7) - (((((l_e213 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch207 != 0) && (l_x214 != l_chosen209))) {
            l_confl208 = 1;
          }
          l_chosen209 = l_x214;
          l_isch207 = 1;
        }
      }
      if ((2 < prm.servers)) {
        const int l_e215 = n_server(s, first_server(prm) + 2)->log[2];
        if (((l_e215 & 3) == 2)) {
          const int l_x216 = ((((l_e215 >> 8) & 7) != 0) ? ((prm.op[((((l_e215 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e215 >> 8) & 7) - (((((l_e215 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e215 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e215 >> 8) & 7) - (((((l_e215 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch207 != 0) && (l_x216 != l_chosen209))) {
            l_confl208 = 1;
          }
          l_chosen209 = l_x216;
          l_isch207 = 1;
        }
      }
      if ((0 < prm.servers)) {
        const int l_e217 = n_server(s, first_server(prm) + 0)->log[2];
        if ((((l_e217 & 3) != 0) && (((l_e217 & 3) != 1) || (((((l_e217 >> 8) & 7) != 0) ? ((prm.op[((((l_e217 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e217 >> 8) & 7) - (((((l_e217 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e217 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e217 >> 8) & 7) - (((((l_e217 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen209)))) {
          l_count210 = (l_count210 + 1);
        }
      }
      if ((1 < prm.servers)) {
        const int l_e218 = n_server(s, first_server(prm) + 1)->log[2];
        if ((((l_e218 & 3) != 0) && (((l_e218 & 3) != 1) || (((((l_e218 >> 8) & 7) != 0) ? ((prm.op[((((l_e218 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e218 >> 8) & 7) - (((((l_e218 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e218 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e218 >> 8) & 7) - (((((l_e218 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen209)))) {
          l_count210 = (l_count210 + 1);
        }
      }
      if ((2 < prm.servers)) {
        const int l_e219 = n_server(s, first_server(prm) + 2)->log[2];
        if ((((l_e219 & 3) != 0) && (((l_e219 & 3) != 1) || (((((l_e219 >> 8) & 7) != 0) ? ((prm.op[((((l_e219 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e219 >> 8) & 7) - (((((l_e219 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e219 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e219 >> 8) & 7) - (((((l_e219 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen209)))) {
          l_count210 = (l_count210 + 1);
        }
      }
      if (((l_isch207 != 0) && ((l_confl208 != 0) || ((l_count210 * 2) <= prm.servers)))) {
        { res_.value = false; return res_; }
      }
      int l_isch220 = 0;
      int l_confl221 = 0;
      int l_chosen222 = 0;
      int l_count223 = 0;
      if ((0 < prm.servers)) {
        const int l_e224 = n_server(s, first_server(prm) + 0)->log[3];
        if (((l_e224 & 3) == 2)) {
          const int l_x225 = ((((l_e224 >> 8) & 7) != 0) ? ((prm.op[((((l_e224 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e224 >> 8) & 7) - (((((l_e224 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e224 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e224 >> 8) & 7) - (((((l_e224 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch220 != 0) && (l_x225 != l_chosen222))) {
            l_confl221 = 1;
          }
          l_chosen222 = l_x225;
          l_isch220 = 1;
        }
      }
      if ((1 < prm.servers)) {
        const int l_e226 = n_server(s, first_server(prm) + 1)->log[3];
        if (((l_e226 & 3) == 2)) {
          const int l_x227 = ((((l_e226 >> 8) & 7) != 0) ? ((prm.op[((((l_e226 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e226 >> 8) & 7) - (((((l_e226 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e226 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e226 >> 8) & 7) - (((((l_e226 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch220 != 0) && (l_x227 != l_chosen222))) {
            l_confl221 = 1;
          }
          l_chosen222 = l_x227;
          l_isch220 = 1;
        }
      }
      if ((2 < prm.servers)) {
        const int l_e228 = n_server(s, first_server(prm) + 2)->log[3];
        if (((l_e228 & 3) == 2)) {
          const int l_x229 = ((((l_e228 >> 8) & 7) != 0) ? ((prm.op[((((l_e228 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e228 >> 8) & 7) - (((((l_e228 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e228 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e228 >> 8) & 7) - (((((l_e228 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch220 != 0) && (l_x229 != l_chosen222))) {
            l_confl221 = 1;
          }
          l_chosen222 = l_x229;
          l_isch220 = 1;
        }
      }
      if ((0 < prm.servers)) {
        const int l_e230 = n_server(s, first_server(prm) + 0)->log[3];
        if ((((l_e230 & 3) != 0) && (((l_e230 & 3) != 1) || (((((l_e230 >> 8) & 7) != 0) ? ((prm.op[((((l_e230 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e230 >> 8) & 7) - (((((l_e230 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e230 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e230 >> 8) & 7) - (((((l_e230 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen222)))) {
          l_count223 = (l_count223 + 1);
        }
      }
      if ((1 < prm.servers)) {
        const int l_e231 = n_server(s, first_server(prm) + 1)->log[3];
        if ((((l_e231 & 3) != 0) && (((l_e231 & 3) != 1) || (((((l_e231 >> 8) & 7) != 0) ? ((prm.op[((((l_e231 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e231 >> 8) & 7) - (((((l_e231 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e231 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e231 >> 8) & 7) - (((((l_e231 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen222)))) {
          l_count223 = (l_count223 + 1);
        }
      }
      if ((2 < prm.servers)) {
        const int l_e232 = n_server(s, first_server(prm) + 2)->log[3];
        if ((((l_e232 & 3) != 0) && (((l_e232 & 3) != 1) || (((((l_e232 >> 8) & 7) != 0) ? ((prm.op[((((l_e232 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e232 >> 8) & 7) - (((((l_e232 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e232 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e232 >> 8) & 7) - (((((l_e232 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen222)))) {
          l_count223 = (l_count223 + 1);
        }
      }
      if (((l_isch220 != 0) && ((l_confl221 != 0) || ((l_count223 * 2) <= prm.servers)))) {
        { res_.value = false; return res_; }
      }
      { res_.value = true; return res_; }
      return res_;
    }};
  }
  if ((base_ == "slotValid") && parts_.size() == 2) {
    return Predicate{"Logs consistent for slot", [prm, a0_, a1_](const State& s) {
      (void)s; (void)a0_; (void)a1_;
      PredResult res_;
      const int l_i = a0_;
      if ((l_i < 1)) {
        { res_.value = false; return res_; }
      }
      if ((l_i > 4)) {
        { res_.value = true; return res_; }
      }
      int l_isch = 0;
      int l_confl = 0;
      int l_chosen = 0;
      int l_count = 0;
      if ((0 < prm.servers)) {
        const int l_e233 = n_server(s, first_server(prm) + 0)->log[(l_i - 1)];
        if (((l_e233 & 3) == 2)) {
          const int l_x234 = ((((l_e233 >> 8) & 7) != 0) ? ((prm.op[((((l_e233 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e233 >> 8) & 7) - (((((l_e233 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e233 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e233 >> 8) & 7) - (((((l_e233 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch != 0) && (l_x234 != l_chosen))) {
            l_confl = 1;
          }
          l_chosen = l_x234;
          l_isch = 1;
        }
      }
      if ((1 < prm.servers)) {
        const int l_e235 = n_server(s, first_server(prm) + 1)->log[(l_i - 1)];
        if (((l_e235 & 3) == 2)) {
          const int l_x236 = ((((l_e235 >> 8) & 7) != 0) ? ((prm.op[((((l_e235 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e235 >> 8) & 7) - (((((l_e235 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e235 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e235 >> 8) & 7) - (((((l_e235 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch != 0) && (l_x236 != l_chosen))) {
            l_confl = 1;
          }
          l_chosen = l_x236;
          l_isch = 1;
        }
      }
      if ((2 < prm.servers)) {
        const int l_e237 = n_server(s, first_server(prm) + 2)->log[(l_i - 1)];
        if (((l_e237 & 3) == 2)) {
          const int l_x238 = ((((l_e237 >> 8) & 7) != 0) ? ((prm.op[((((l_e237 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e237 >> 8) & 7) - (((((l_e237 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e237 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e237 >> 8) & 7) - (((((l_e237 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch != 0) && (l_x238 != l_chosen))) {
            l_confl = 1;
          }
          l_chosen = l_x238;
          l_isch = 1;
        }
      }
      if ((0 < prm.servers)) {
        const int l_e239 = n_server(s, first_server(prm) + 0)->log[(l_i - 1)];
        if ((((l_e239 & 3) != 0) && (((l_e239 & 3) != 1) || (((((l_e239 >> 8) & 7) != 0) ? ((prm.op[((((l_e239 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e239 >> 8) & 7) - (((((l_e239 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e239 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e239 >> 8) & 7) - (((((l_e239 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen)))) {
          l_count = (l_count + 1);
        }
      }
      if ((1 < prm.servers)) {
        const int l_e240 = n_server(s, first_server(prm) + 1)->log[(l_i - 1)];
        if ((((l_e240 & 3) != 0) && (((l_e240 & 3) != 1) || (((((l_e240 >> 8) & 7) != 0) ? ((prm.op[((((l_e240 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e240 >> 8) & 7) - (((((l_e240 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e240 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e240 >> 8) & 7) - (((((l_e240 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen)))) {
          l_count = (l_count + 1);
        }
      }
      if ((2 < prm.servers)) {
        const int l_e241 = n_server(s, first_server(prm) + 2)->log[(l_i - 1)];
        if ((((l_e241 & 3) != 0) && (((l_e241 & 3) != 1) || (((((l_e241 >> 8) & 7) != 0) ? ((prm.op[((((l_e241 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e241 >> 8) & 7) - (((((l_e241 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e241 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e241 >> 8) & 7) - (((((l_e241 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen)))) {
          l_count = (l_count + 1);
        }
      }
      if (((l_isch != 0) && ((l_confl != 0) || ((l_count * 2) <= prm.servers)))) {
        { res_.value = false; return res_; }
      }
      { res_.value = true; return res_; }
      return res_;
    }};
  }
  if ((base_ == "hasStatus") && parts_.size() == 3) {
    return Predicate{"Server has status in slot", [prm, a0_, a1_](const State& s) {
      (void)s; (void)a0_; (void)a1_;
      PredResult res_;
      const int l_k242 = (a0_ - (first_server(prm) + 1 - 1));
      if (((l_k242 < 0) || (l_k242 >= prm.servers))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_slot243 = (a1_ >> 4);
      int l_se244 = 0;
      if (((l_slot243 >= 1) && (l_slot243 <= 4))) {
        l_se244 = n_server(s, first_server(prm) + l_k242)->log[(l_slot243 - 1)];
      }
      if (((l_se244 & 3) == (a1_ & 15))) {
        { res_.value = true; return res_; }
      }
      { res_.value = false; return res_; }
      return res_;
    }};
  }
  if ((base_ == "hasCommand") && parts_.size() == 3) {
    return Predicate{"Server has command in slot", [prm, a0_, a1_](const State& s) {
      (void)s; (void)a0_; (void)a1_;
      PredResult res_;
      const int l_k245 = (a0_ - (first_server(prm) + 1 - 1));
      if (((l_k245 < 0) || (l_k245 >= prm.servers))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_slot246 = (a1_ >> 8);
      int l_se247 = 0;
      if (((l_slot246 >= 1) && (l_slot246 <= 4))) {
        l_se247 = n_server(s, first_server(prm) + l_k245)->log[(l_slot246 - 1)];
      }
      const int l_cc = (((l_se247 & 3) == 0) ? 0 : ((((l_se247 >> 8) & 7) != 0) ? ((prm.op[((((l_se247 >> 8) & 7) >= 4) ? 1 : 0)][((((l_se247 >> 8) & 7) - (((((l_se247 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_se247 >> 8) & 7) >= 4) ? 1 : 0)][((((l_se247 >> 8) & 7) - (((((l_se247 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0));
      if ((l_cc == (a1_ & 255))) {
        { res_.value = true; return res_; }
      }
      { res_.value = false; return res_; }
      return res_;
    }};
  }
  if ((base_ == "APPENDS_LINEARIZABLE") && parts_.size() == 1) {
    return Predicate{"Sequence of appends to the same key is linearizable", [prm, a0_, a1_](const State& s) {
      (void)s; (void)a0_; (void)a1_;
      PredResult res_;
      const int l_pres248 = ((0 < prm.clients) && (0 < (int)s.cw(first_client(prm) + 0)->results.size()));
      if ((l_pres248 && (prm.op[0][0] != 2))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_res249 = (l_pres248 ? std::stoi(s.cw(first_client(prm) + 0)->results[0].f[0]) : 0);
      const int l_rlen250 = (l_res249 & 7);
      if ((l_pres248 && (((l_rlen250 == 0) || (l_rlen250 > 4)) || (((l_res249 >> (1 + (l_rlen250 * 2))) & 3) != prm.val[0][0])))) {
        { res_.value = false; return res_; }
      }
      const int l_pres251 = ((0 < prm.clients) && (1 < (int)s.cw(first_client(prm) + 0)->results.size()));
      if ((l_pres251 && (prm.op[0][1] != 2))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_res252 = (l_pres251 ? std::stoi(s.cw(first_client(prm) + 0)->results[1].f[0]) : 0);
      const int l_rlen253 = (l_res252 & 7);
      if ((l_pres251 && (((l_rlen253 == 0) || (l_rlen253 > 4)) || (((l_res252 >> (1 + (l_rlen253 * 2))) & 3) != prm.val[0][1])))) {
        { res_.value = false; return res_; }
      }
      const int l_pres254 = ((0 < prm.clients) && (2 < (int)s.cw(first_client(prm) + 0)->results.size()));
      if ((l_pres254 && (prm.op[0][2] != 2))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_res255 = (l_pres254 ? std::stoi(s.cw(first_client(prm) + 0)->results[2].f[0]) : 0);
      const int l_rlen256 = (l_res255 & 7);
      if ((l_pres254 && (((l_rlen256 == 0) || (l_rlen256 > 4)) || (((l_res255 >> (1 + (l_rlen256 * 2))) & 3) != prm.val[0][2])))) {
        { res_.value = false; return res_; }
      }
      const int l_pres257 = ((1 < prm.clients) && (0 < (int)s.cw(first_client(prm) + 1)->results.size()));
      if ((l_pres257 && (prm.op[1][0] != 2))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_res258 = (l_pres257 ? std::stoi(s.cw(first_client(prm) + 1)->results[0].f[0]) : 0);
      const int l_rlen259 = (l_res258 & 7);
      if ((l_pres257 && (((l_rlen259 == 0) || (l_rlen259 > 4)) || (((l_res258 >> (1 + (l_rlen259 * 2))) & 3) != prm.val[1][0])))) {
        { res_.value = false; return res_; }
      }
      const int l_pres260 = ((1 < prm.clients) && (1 < (int)s.cw(first_client(prm) + 1)->results.size()));
      if ((l_pres260 && (prm.op[1][1] != 2))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_res261 = (l_pres260 ? std::stoi(s.cw(first_client(prm) + 1)->results[1].f[0]) : 0);
      const int l_rlen262 = (l_res261 & 7);
      if ((l_pres260 && (((l_rlen262 == 0) || (l_rlen262 > 4)) || (((l_res261 >> (1 + (l_rlen262 * 2))) & 3) != prm.val[1][1])))) {
        { res_.value = false; return res_; }
      }
      const int l_pres263 = ((1 < prm.clients) && (2 < (int)s.cw(first_client(prm) + 1)->results.size()));
      if ((l_pres263 && (prm.op[1][2] != 2))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_res264 = (l_pres263 ? std::stoi(s.cw(first_client(prm) + 1)->results[2].f[0]) : 0);
      const int l_rlen265 = (l_res264 & 7);
      if ((l_pres263 && (((l_rlen265 == 0) || (l_rlen265 > 4)) || (((l_res264 >> (1 + (l_rlen265 * 2))) & 3) != prm.val[1][2])))) {
        { res_.value = false; return res_; }
      }
      if ((l_pres248 && l_pres251)) {
        if ((l_rlen250 == l_rlen253)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res249 >> 3) & ((1 << (((l_rlen250 < l_rlen253) ? l_rlen250 : l_rlen253) * 2)) - 1)) != ((l_res252 >> 3) & ((1 << (((l_rlen250 < l_rlen253) ? l_rlen250 : l_rlen253) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres248 && l_pres254)) {
        if ((l_rlen250 == l_rlen256)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res249 >> 3) & ((1 << (((l_rlen250 < l_rlen256) ? l_rlen250 : l_rlen256) * 2)) - 1)) != ((l_res255 >> 3) & ((1 << (((l_rlen250 < l_rlen256) ? l_rlen250 : l_rlen256) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres248 && l_pres257)) {
        if ((l_rlen250 == l_rlen259)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res249 >> 3) & ((1 << (((l_rlen250 < l_rlen259) ? l_rlen250 : l_rlen259) * 2)) - 1)) != ((l_res258 >> 3) & ((1 << (((l_rlen250 < l_rlen259) ? l_rlen250 : l_rlen259) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres248 && l_pres260)) {
        if ((l_rlen250 == l_rlen262)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res249 >> 3) & ((1 << (((l_rlen250 < l_rlen262) ? l_rlen250 : l_rlen262) * 2)) - 1)) != ((l_res261 >> 3) & ((1 << (((l_rlen250 < l_rlen262) ? l_rlen250 : l_rlen262) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres248 && l_pres263)) {
        if ((l_rlen250 == l_rlen265)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res249 >> 3) & ((1 << (((l_rlen250 < l_rlen265) ? l_rlen250 : l_rlen265) * 2)) - 1)) != ((l_res264 >> 3) & ((1 << (((l_rlen250 < l_rlen265) ? l_rlen250 : l_rlen265) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres251 && l_pres254)) {
        if ((l_rlen253 == l_rlen256)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res252 >> 3) & ((1 << (((l_rlen253 < l_rlen256) ? l_rlen253 : l_rlen256) * 2)) - 1)) != ((l_res255 >> 3) & ((1 << (((l_rlen253 < l_rlen256) ? l_rlen253 : l_rlen256) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres251 && l_pres257)) {
        if ((l_rlen253 == l_rlen259)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res252 >> 3) & ((1 << (((l_rlen253 < l_rlen259) ? l_rlen253 : l_rlen259) * 2)) - 1)) != ((l_res258 >> 3) & ((1 << (((l_rlen253 < l_rlen259) ? l_rlen253 : l_rlen259) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres251 && l_pres260)) {
        if ((l_rlen253 == l_rlen262)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res252 >> 3) & ((1 << (((l_rlen253 < l_rlen262) ? l_rlen253 : l_rlen262) * 2)) - 1)) != ((l_res261 >> 3) & ((1 << (((l_rlen253 < l_rlen262) ? l_rlen253 : l_rlen262) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres251 && l_pres263)) {
        if ((l_rlen253 == l_rlen265)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res252 >> 3) & ((1 << (((l_rlen253 < l_rlen265) ? l_rlen253 : l_rlen265) * 2)) - 1)) != ((l_res264 >> 3) & ((1 << (((l_rlen253 < l_rlen265) ? l_rlen253 : l_rlen265) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres254 && l_pres257)) {
        if ((l_rlen256 == l_rlen259)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res255 >> 3) & ((1 << (((l_rlen256 < l_rlen259) ? l_rlen256 : l_rlen259) * 2)) - 1)) != ((l_res258 >> 3) & ((1 << (((l_rlen256 < l_rlen259) ? l_rlen256 : l_rlen259) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres254 && l_pres260)) {
        if ((l_rlen256 == l_rlen262)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res255 >> 3) & ((1 << (((l_rlen256 < l_rlen262) ? l_rlen256 : l_rlen262) * 2)) - 1)) != ((l_res261 >> 3) & ((1 << (((l_rlen256 < l_rlen262) ? l_rlen256 : l_rlen262) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres254 && l_pres263)) {
        if ((l_rlen256 == l_rlen265)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res255 >> 3) & ((1 << (((l_rlen256 < l_rlen265) ? l_rlen256 : l_rlen265) * 2)) - 1)) != ((l_res264 >> 3) & ((1 << (((l_rlen256 < l_rlen265) ? l_rlen256 : l_rlen265) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres257 && l_pres260)) {
        if ((l_rlen259 == l_rlen262)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res258 >> 3) & ((1 << (((l_rlen259 < l_rlen262) ? l_rlen259 : l_rlen262) * 2)) - 1)) != ((l_res261 >> 3) & ((1 << (((l_rlen259 < l_rlen262) ? l_rlen259 : l_rlen262) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres257 && l_pres263)) {
        if ((l_rlen259 == l_rlen265)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res258 >> 3) & ((1 << (((l_rlen259 < l_rlen265) ? l_rlen259 : l_rlen265) * 2)) - 1)) != ((l_res264 >> 3) & ((1 << (((l_rlen259 < l_rlen265) ? l_rlen259 : l_rlen265) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres260 && l_pres263)) {
        if ((l_rlen262 == l_rlen265)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res261 >> 3) & ((1 << (((l_rlen262 < l_rlen265) ? l_rlen262 : l_rlen265) * 2)) - 1)) != ((l_res264 >> 3) & ((1 << (((l_rlen262 < l_rlen265) ? l_rlen262 : l_rlen265) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      { res_.value = true; return res_; }
      return res_;
    }};
  }
  return std::nullopt;
}

}  // namespace multipaxos_ir
}  // namespace oracle
