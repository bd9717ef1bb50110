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
        const int l_upto179 = slotout;
        int l_kv180 = 0;
        int l_ls0181 = 0;
        int l_ls1182 = 0;
        int l_r183 = 0;
        const int l_cmd184 = ((log[0] >> 8) & 7);
        const int l_c185 = ((l_cmd184 >= 4) ? 1 : 0);
        const int l_q186 = (l_cmd184 - (((l_cmd184 >= 4) ? 1 : 0) * 3));
        if ((((1 < l_upto179) && (l_cmd184 != 0)) && ((l_c185 ? l_ls1182 : l_ls0181) < l_q186))) {
          const int l_c187 = ((l_cmd184 >= 4) ? 1 : 0);
          const int l_op188 = prm.op[l_c187][((l_cmd184 - (((l_cmd184 >= 4) ? 1 : 0) * 3)) - 1)];
          const int l_v189 = prm.val[l_c187][((l_cmd184 - (((l_cmd184 >= 4) ? 1 : 0) * 3)) - 1)];
          int l_x190 = 0;
          if ((l_op188 == 1)) {
            l_kv180 = (1 | (l_v189 << 3));
            l_x190 = 7;
          }
          if ((l_op188 == 2)) {
            const int l_len191 = (l_kv180 & 7);
            l_kv180 = (((l_len191 + 1) | (l_kv180 & -8)) | (l_v189 << (3 + (l_len191 * 2))));
            l_x190 = l_kv180;
          }
          if ((l_op188 == 3)) {
            l_x190 = (((l_kv180 & 7) != 0) ? l_kv180 : 6);
          }
          if ((l_c185 != 0)) {
            l_ls1182 = l_q186;
          } else {
            l_ls0181 = l_q186;
          }
          if (((l_c185 == l_c) && (l_q186 == l_q))) {
            l_r183 = l_x190;
          }
        }
        const int l_cmd192 = ((log[1] >> 8) & 7);
        const int l_c193 = ((l_cmd192 >= 4) ? 1 : 0);
        const int l_q194 = (l_cmd192 - (((l_cmd192 >= 4) ? 1 : 0) * 3));
        if ((((2 < l_upto179) && (l_cmd192 != 0)) && ((l_c193 ? l_ls1182 : l_ls0181) < l_q194))) {
          const int l_c195 = ((l_cmd192 >= 4) ? 1 : 0);
          const int l_op196 = prm.op[l_c195][((l_cmd192 - (((l_cmd192 >= 4) ? 1 : 0) * 3)) - 1)];
          const int l_v197 = prm.val[l_c195][((l_cmd192 - (((l_cmd192 >= 4) ? 1 : 0) * 3)) - 1)];
          int l_x198 = 0;
          if ((l_op196 == 1)) {
            l_kv180 = (1 | (l_v197 << 3));
            l_x198 = 7;
          }
          if ((l_op196 == 2)) {
            const int l_len199 = (l_kv180 & 7);
            l_kv180 = (((l_len199 + 1) | (l_kv180 & -8)) | (l_v197 << (3 + (l_len199 * 2))));
            l_x198 = l_kv180;
          }
          if ((l_op196 == 3)) {
            l_x198 = (((l_kv180 & 7) != 0) ? l_kv180 : 6);
          }
          if ((l_c193 != 0)) {
            l_ls1182 = l_q194;
          } else {
            l_ls0181 = l_q194;
          }
          if (((l_c193 == l_c) && (l_q194 == l_q))) {
            l_r183 = l_x198;
          }
        }
        const int l_cmd200 = ((log[2] >> 8) & 7);
        const int l_c201 = ((l_cmd200 >= 4) ? 1 : 0);
        const int l_q202 = (l_cmd200 - (((l_cmd200 >= 4) ? 1 : 0) * 3));
        if ((((3 < l_upto179) && (l_cmd200 != 0)) && ((l_c201 ? l_ls1182 : l_ls0181) < l_q202))) {
          const int l_c203 = ((l_cmd200 >= 4) ? 1 : 0);
          const int l_op204 = prm.op[l_c203][((l_cmd200 - (((l_cmd200 >= 4) ? 1 : 0) * 3)) - 1)];
          const int l_v205 = prm.val[l_c203][((l_cmd200 - (((l_cmd200 >= 4) ? 1 : 0) * 3)) - 1)];
          int l_x206 = 0;
          if ((l_op204 == 1)) {
            l_kv180 = (1 | (l_v205 << 3));
            l_x206 = 7;
          }
          if ((l_op204 == 2)) {
            const int l_len207 = (l_kv180 & 7);
            l_kv180 = (((l_len207 + 1) | (l_kv180 & -8)) | (l_v205 << (3 + (l_len207 * 2))));
            l_x206 = l_kv180;
          }
          if ((l_op204 == 3)) {
            l_x206 = (((l_kv180 & 7) != 0) ? l_kv180 : 6);
          }
          if ((l_c201 != 0)) {
            l_ls1182 = l_q202;
          } else {
            l_ls0181 = l_q202;
          }
          if (((l_c201 == l_c) && (l_q202 == l_q))) {
            l_r183 = l_x206;
          }
        }
        const int l_cmd208 = ((log[3] >> 8) & 7);
        const int l_c209 = ((l_cmd208 >= 4) ? 1 : 0);
        const int l_q210 = (l_cmd208 - (((l_cmd208 >= 4) ? 1 : 0) * 3));
        if ((((4 < l_upto179) && (l_cmd208 != 0)) && ((l_c209 ? l_ls1182 : l_ls0181) < l_q210))) {
          const int l_c211 = ((l_cmd208 >= 4) ? 1 : 0);
          const int l_op212 = prm.op[l_c211][((l_cmd208 - (((l_cmd208 >= 4) ? 1 : 0) * 3)) - 1)];
          const int l_v213 = prm.val[l_c211][((l_cmd208 - (((l_cmd208 >= 4) ? 1 : 0) * 3)) - 1)];
          int l_x214 = 0;
          if ((l_op212 == 1)) {
            l_kv180 = (1 | (l_v213 << 3));
            l_x214 = 7;
          }
          if ((l_op212 == 2)) {
            const int l_len215 = (l_kv180 & 7);
            l_kv180 = (((l_len215 + 1) | (l_kv180 & -8)) | (l_v213 << (3 + (l_len215 * 2))));
            l_x214 = l_kv180;
          }
          if ((l_op212 == 3)) {
            l_x214 = (((l_kv180 & 7) != 0) ? l_kv180 : 6);
          }
          if ((l_c209 != 0)) {
            l_ls1182 = l_q210;
          } else {
            l_ls0181 = l_q210;
          }
          if (((l_c209 == l_c) && (l_q210 == l_q))) {
            l_r183 = l_x214;
          }
        }
        const int l_ls = (l_c ? l_ls1182 : l_ls0181);
        if ((l_ls >= l_q)) {
          if (((active != 0) && (l_ls == l_q))) {
            ctx.send(Rec{"Reply", {std::to_string(l_q), std::to_string(l_r183)}}, (first_client(prm) + (l_c + 1) - 1));
          }
          return;
        }
        int l_slot = slotin;
        int l_inlog = 0;
        const int l_e216 = log[0];
        if ((((l_e216 & 3) != 0) && (2 > l_slot))) {
          l_slot = 2;
        }
        if ((((l_e216 & 3) != 0) && (((l_e216 >> 8) & 7) == l_cmd))) {
          l_inlog = 1;
        }
        const int l_e217 = log[1];
        if ((((l_e217 & 3) != 0) && (3 > l_slot))) {
          l_slot = 3;
        }
        if ((((l_e217 & 3) != 0) && (((l_e217 >> 8) & 7) == l_cmd))) {
          l_inlog = 1;
        }
        const int l_e218 = log[2];
        if ((((l_e218 & 3) != 0) && (4 > l_slot))) {
          l_slot = 4;
        }
        if ((((l_e218 & 3) != 0) && (((l_e218 >> 8) & 7) == l_cmd))) {
          l_inlog = 1;
        }
        const int l_e219 = log[3];
        if ((((l_e219 & 3) != 0) && (5 > l_slot))) {
          l_slot = 5;
        }
        if ((((l_e219 & 3) != 0) && (((l_e219 >> 8) & 7) == l_cmd))) {
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
          const int l_ccmd220 = ((log[(l_slot - 1)] >> 8) & 7);
          log[(l_slot - 1)] = ((2 | (0 << 2)) | (l_ccmd220 << 8));
          votes[(l_slot - 1)] = 0;
          if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
            ctx.send(Rec{"Decision", {std::to_string(l_slot), std::to_string(l_ccmd220)}}, (first_server(prm) + 1 - 1));
          }
          if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
            ctx.send(Rec{"Decision", {std::to_string(l_slot), std::to_string(l_ccmd220)}}, (first_server(prm) + 2 - 1));
          }
          if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
            ctx.send(Rec{"Decision", {std::to_string(l_slot), std::to_string(l_ccmd220)}}, (first_server(prm) + 3 - 1));
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
        const int l_me221 = std::stoi(m.f[2]);
        const int l_mm222 = p1blog[0];
        if (((l_me221 & 3) == 2)) {
          p1blog[0] = ((2 | (0 << 2)) | (((l_me221 >> 8) & 7) << 8));
        } else {
          if (((((l_me221 & 3) == 1) && ((l_mm222 & 3) != 2)) && (((l_mm222 & 3) == 0) || (((l_mm222 >> 2) & 63) < ((l_me221 >> 2) & 63))))) {
            p1blog[0] = l_me221;
          }
        }
        const int l_me223 = std::stoi(m.f[3]);
        const int l_mm224 = p1blog[1];
        if (((l_me223 & 3) == 2)) {
          p1blog[1] = ((2 | (0 << 2)) | (((l_me223 >> 8) & 7) << 8));
        } else {
          if (((((l_me223 & 3) == 1) && ((l_mm224 & 3) != 2)) && (((l_mm224 & 3) == 0) || (((l_mm224 >> 2) & 63) < ((l_me223 >> 2) & 63))))) {
            p1blog[1] = l_me223;
          }
        }
        const int l_me225 = std::stoi(m.f[4]);
        const int l_mm226 = p1blog[2];
        if (((l_me225 & 3) == 2)) {
          p1blog[2] = ((2 | (0 << 2)) | (((l_me225 >> 8) & 7) << 8));
        } else {
          if (((((l_me225 & 3) == 1) && ((l_mm226 & 3) != 2)) && (((l_mm226 & 3) == 0) || (((l_mm226 >> 2) & 63) < ((l_me225 >> 2) & 63))))) {
            p1blog[2] = l_me225;
          }
        }
        const int l_me227 = std::stoi(m.f[5]);
        const int l_mm228 = p1blog[3];
        if (((l_me227 & 3) == 2)) {
          p1blog[3] = ((2 | (0 << 2)) | (((l_me227 >> 8) & 7) << 8));
        } else {
          if (((((l_me227 & 3) == 1) && ((l_mm228 & 3) != 2)) && (((l_mm228 & 3) == 0) || (((l_mm228 >> 2) & 63) < ((l_me227 >> 2) & 63))))) {
            p1blog[3] = l_me227;
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
        const int l_ccmd229 = ((log[(l_slot - 1)] >> 8) & 7);
        log[(l_slot - 1)] = ((2 | (0 << 2)) | (l_ccmd229 << 8));
        votes[(l_slot - 1)] = 0;
        if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
          ctx.send(Rec{"Decision", {std::to_string(l_slot), std::to_string(l_ccmd229)}}, (first_server(prm) + 1 - 1));
        }
        if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
          ctx.send(Rec{"Decision", {std::to_string(l_slot), std::to_string(l_ccmd229)}}, (first_server(prm) + 2 - 1));
        }
        if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
          ctx.send(Rec{"Decision", {std::to_string(l_slot), std::to_string(l_ccmd229)}}, (first_server(prm) + 3 - 1));
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
        const int l_mg230 = p1blog[0];
        const int l_mg231 = p1blog[1];
        const int l_mg232 = p1blog[2];
        const int l_mg233 = p1blog[3];
        int l_last234 = 0;
        if ((((l_mg230 & 3) != 0) || ((log[0] & 3) != 0))) {
          l_last234 = 1;
        }
        if ((((l_mg231 & 3) != 0) || ((log[1] & 3) != 0))) {
          l_last234 = 2;
        }
        if ((((l_mg232 & 3) != 0) || ((log[2] & 3) != 0))) {
          l_last234 = 3;
        }
        if ((((l_mg233 & 3) != 0) || ((log[3] & 3) != 0))) {
          l_last234 = 4;
        }
        p1blog[0] = 0;
        p1blog[1] = 0;
        p1blog[2] = 0;
        p1blog[3] = 0;
        if (((1 <= l_last234) && ((log[0] & 3) != 2))) {
          if (((l_mg230 & 3) == 2)) {
            log[0] = ((2 | (0 << 2)) | (((l_mg230 >> 8) & 7) << 8));
            votes[0] = 0;
          } else {
            log[(1 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg230 & 3) == 1) ? ((l_mg230 >> 8) & 7) : 0) << 8));
            votes[(1 - 1)] = (1 << (self - first_server(prm)));
            if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(1), std::to_string((((l_mg230 & 3) == 1) ? ((l_mg230 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
            }
            if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(1), std::to_string((((l_mg230 & 3) == 1) ? ((l_mg230 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
            }
            if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(1), std::to_string((((l_mg230 & 3) == 1) ? ((l_mg230 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
            }
            if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
              const int l_ccmd235 = ((log[(1 - 1)] >> 8) & 7);
              log[(1 - 1)] = ((2 | (0 << 2)) | (l_ccmd235 << 8));
              votes[(1 - 1)] = 0;
              if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(1), std::to_string(l_ccmd235)}}, (first_server(prm) + 1 - 1));
              }
              if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(1), std::to_string(l_ccmd235)}}, (first_server(prm) + 2 - 1));
              }
              if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(1), std::to_string(l_ccmd235)}}, (first_server(prm) + 3 - 1));
              }
            }
          }
        }
        if (((2 <= l_last234) && ((log[1] & 3) != 2))) {
          if (((l_mg231 & 3) == 2)) {
            log[1] = ((2 | (0 << 2)) | (((l_mg231 >> 8) & 7) << 8));
            votes[1] = 0;
          } else {
            log[(2 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg231 & 3) == 1) ? ((l_mg231 >> 8) & 7) : 0) << 8));
            votes[(2 - 1)] = (1 << (self - first_server(prm)));
            if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(2), std::to_string((((l_mg231 & 3) == 1) ? ((l_mg231 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
            }
            if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(2), std::to_string((((l_mg231 & 3) == 1) ? ((l_mg231 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
            }
            if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(2), std::to_string((((l_mg231 & 3) == 1) ? ((l_mg231 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
            }
            if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
              const int l_ccmd236 = ((log[(2 - 1)] >> 8) & 7);
              log[(2 - 1)] = ((2 | (0 << 2)) | (l_ccmd236 << 8));
              votes[(2 - 1)] = 0;
              if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(2), std::to_string(l_ccmd236)}}, (first_server(prm) + 1 - 1));
              }
              if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(2), std::to_string(l_ccmd236)}}, (first_server(prm) + 2 - 1));
              }
              if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(2), std::to_string(l_ccmd236)}}, (first_server(prm) + 3 - 1));
              }
            }
          }
        }
        if (((3 <= l_last234) && ((log[2] & 3) != 2))) {
          if (((l_mg232 & 3) == 2)) {
            log[2] = ((2 | (0 << 2)) | (((l_mg232 >> 8) & 7) << 8));
            votes[2] = 0;
          } else {
            log[(3 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg232 & 3) == 1) ? ((l_mg232 >> 8) & 7) : 0) << 8));
            votes[(3 - 1)] = (1 << (self - first_server(prm)));
            if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(3), std::to_string((((l_mg232 & 3) == 1) ? ((l_mg232 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
            }
            if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(3), std::to_string((((l_mg232 & 3) == 1) ? ((l_mg232 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
            }
            if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(3), std::to_string((((l_mg232 & 3) == 1) ? ((l_mg232 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
            }
            if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
              const int l_ccmd237 = ((log[(3 - 1)] >> 8) & 7);
              log[(3 - 1)] = ((2 | (0 << 2)) | (l_ccmd237 << 8));
              votes[(3 - 1)] = 0;
              if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(3), std::to_string(l_ccmd237)}}, (first_server(prm) + 1 - 1));
              }
              if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(3), std::to_string(l_ccmd237)}}, (first_server(prm) + 2 - 1));
              }
              if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(3), std::to_string(l_ccmd237)}}, (first_server(prm) + 3 - 1));
              }
            }
          }
        }
        if (((4 <= l_last234) && ((log[3] & 3) != 2))) {
          if (((l_mg233 & 3) == 2)) {
            log[3] = ((2 | (0 << 2)) | (((l_mg233 >> 8) & 7) << 8));
            votes[3] = 0;
          } else {
            log[(4 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg233 & 3) == 1) ? ((l_mg233 >> 8) & 7) : 0) << 8));
            votes[(4 - 1)] = (1 << (self - first_server(prm)));
            if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(4), std::to_string((((l_mg233 & 3) == 1) ? ((l_mg233 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
            }
            if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(4), std::to_string((((l_mg233 & 3) == 1) ? ((l_mg233 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
            }
            if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
              ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(4), std::to_string((((l_mg233 & 3) == 1) ? ((l_mg233 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
            }
            if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
              const int l_ccmd238 = ((log[(4 - 1)] >> 8) & 7);
              log[(4 - 1)] = ((2 | (0 << 2)) | (l_ccmd238 << 8));
              votes[(4 - 1)] = 0;
              if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(4), std::to_string(l_ccmd238)}}, (first_server(prm) + 1 - 1));
              }
              if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(4), std::to_string(l_ccmd238)}}, (first_server(prm) + 2 - 1));
              }
              if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                ctx.send(Rec{"Decision", {std::to_string(4), std::to_string(l_ccmd238)}}, (first_server(prm) + 3 - 1));
              }
            }
          }
        }
        slotin = (l_last234 + 1);
      }
      const int l_so0239 = slotout;
      const int l_act240 = active;
      int l_kv241 = 0;
      int l_ls0242 = 0;
      int l_ls1243 = 0;
      int l_so244 = l_so0239;
      int l_run245 = 1;
      const int l_e246 = log[0];
      const int l_cmd247 = ((l_e246 >> 8) & 7);
      const int l_c248 = ((l_cmd247 >= 4) ? 1 : 0);
      const int l_q249 = (l_cmd247 - (((l_cmd247 >= 4) ? 1 : 0) * 3));
      const int l_before250 = (1 < l_so0239);
      const int l_now251 = (((!l_before250) && (l_run245 != 0)) && ((l_e246 & 3) == 2));
      l_run245 = (((l_run245 != 0) && (l_before250 || l_now251)) ? 1 : 0);
      if ((((l_before250 || l_now251) && (l_cmd247 != 0)) && ((l_c248 ? l_ls1243 : l_ls0242) < l_q249))) {
        const int l_c252 = ((l_cmd247 >= 4) ? 1 : 0);
        const int l_op253 = prm.op[l_c252][((l_cmd247 - (((l_cmd247 >= 4) ? 1 : 0) * 3)) - 1)];
        const int l_v254 = prm.val[l_c252][((l_cmd247 - (((l_cmd247 >= 4) ? 1 : 0) * 3)) - 1)];
        int l_x255 = 0;
        if ((l_op253 == 1)) {
          l_kv241 = (1 | (l_v254 << 3));
          l_x255 = 7;
        }
        if ((l_op253 == 2)) {
          const int l_len256 = (l_kv241 & 7);
          l_kv241 = (((l_len256 + 1) | (l_kv241 & -8)) | (l_v254 << (3 + (l_len256 * 2))));
          l_x255 = l_kv241;
        }
        if ((l_op253 == 3)) {
          l_x255 = (((l_kv241 & 7) != 0) ? l_kv241 : 6);
        }
        if ((l_c248 != 0)) {
          l_ls1243 = l_q249;
        } else {
          l_ls0242 = l_q249;
        }
        if ((l_now251 && (l_act240 != 0))) {
          ctx.send(Rec{"Reply", {std::to_string(l_q249), std::to_string(l_x255)}}, (first_client(prm) + (l_c248 + 1) - 1));
        }
      }
      if (l_now251) {
        l_so244 = 2;
      }
      const int l_e257 = log[1];
      const int l_cmd258 = ((l_e257 >> 8) & 7);
      const int l_c259 = ((l_cmd258 >= 4) ? 1 : 0);
      const int l_q260 = (l_cmd258 - (((l_cmd258 >= 4) ? 1 : 0) * 3));
      const int l_before261 = (2 < l_so0239);
      const int l_now262 = (((!l_before261) && (l_run245 != 0)) && ((l_e257 & 3) == 2));
      l_run245 = (((l_run245 != 0) && (l_before261 || l_now262)) ? 1 : 0);
      if ((((l_before261 || l_now262) && (l_cmd258 != 0)) && ((l_c259 ? l_ls1243 : l_ls0242) < l_q260))) {
        const int l_c263 = ((l_cmd258 >= 4) ? 1 : 0);
        const int l_op264 = prm.op[l_c263][((l_cmd258 - (((l_cmd258 >= 4) ? 1 : 0) * 3)) - 1)];
        const int l_v265 = prm.val[l_c263][((l_cmd258 - (((l_cmd258 >= 4) ? 1 : 0) * 3)) - 1)];
        int l_x266 = 0;
        if ((l_op264 == 1)) {
          l_kv241 = (1 | (l_v265 << 3));
          l_x266 = 7;
        }
        if ((l_op264 == 2)) {
          const int l_len267 = (l_kv241 & 7);
          l_kv241 = (((l_len267 + 1) | (l_kv241 & -8)) | (l_v265 << (3 + (l_len267 * 2))));
          l_x266 = l_kv241;
        }
        if ((l_op264 == 3)) {
          l_x266 = (((l_kv241 & 7) != 0) ? l_kv241 : 6);
        }
        if ((l_c259 != 0)) {
          l_ls1243 = l_q260;
        } else {
          l_ls0242 = l_q260;
        }
        if ((l_now262 && (l_act240 != 0))) {
          ctx.send(Rec{"Reply", {std::to_string(l_q260), std::to_string(l_x266)}}, (first_client(prm) + (l_c259 + 1) - 1));
        }
      }
      if (l_now262) {
        l_so244 = 3;
      }
      const int l_e268 = log[2];
      const int l_cmd269 = ((l_e268 >> 8) & 7);
      const int l_c270 = ((l_cmd269 >= 4) ? 1 : 0);
      const int l_q271 = (l_cmd269 - (((l_cmd269 >= 4) ? 1 : 0) * 3));
      const int l_before272 = (3 < l_so0239);
      const int l_now273 = (((!l_before272) && (l_run245 != 0)) && ((l_e268 & 3) == 2));
      l_run245 = (((l_run245 != 0) && (l_before272 || l_now273)) ? 1 : 0);
      if ((((l_before272 || l_now273) && (l_cmd269 != 0)) && ((l_c270 ? l_ls1243 : l_ls0242) < l_q271))) {
        const int l_c274 = ((l_cmd269 >= 4) ? 1 : 0);
        const int l_op275 = prm.op[l_c274][((l_cmd269 - (((l_cmd269 >= 4) ? 1 : 0) * 3)) - 1)];
        const int l_v276 = prm.val[l_c274][((l_cmd269 - (((l_cmd269 >= 4) ? 1 : 0) * 3)) - 1)];
        int l_x277 = 0;
        if ((l_op275 == 1)) {
          l_kv241 = (1 | (l_v276 << 3));
          l_x277 = 7;
        }
        if ((l_op275 == 2)) {
          const int l_len278 = (l_kv241 & 7);
          l_kv241 = (((l_len278 + 1) | (l_kv241 & -8)) | (l_v276 << (3 + (l_len278 * 2))));
          l_x277 = l_kv241;
        }
        if ((l_op275 == 3)) {
          l_x277 = (((l_kv241 & 7) != 0) ? l_kv241 : 6);
        }
        if ((l_c270 != 0)) {
          l_ls1243 = l_q271;
        } else {
          l_ls0242 = l_q271;
        }
        if ((l_now273 && (l_act240 != 0))) {
          ctx.send(Rec{"Reply", {std::to_string(l_q271), std::to_string(l_x277)}}, (first_client(prm) + (l_c270 + 1) - 1));
        }
      }
      if (l_now273) {
        l_so244 = 4;
      }
      const int l_e279 = log[3];
      const int l_cmd280 = ((l_e279 >> 8) & 7);
      const int l_c281 = ((l_cmd280 >= 4) ? 1 : 0);
      const int l_q282 = (l_cmd280 - (((l_cmd280 >= 4) ? 1 : 0) * 3));
      const int l_before283 = (4 < l_so0239);
      const int l_now284 = (((!l_before283) && (l_run245 != 0)) && ((l_e279 & 3) == 2));
      l_run245 = (((l_run245 != 0) && (l_before283 || l_now284)) ? 1 : 0);
      if ((((l_before283 || l_now284) && (l_cmd280 != 0)) && ((l_c281 ? l_ls1243 : l_ls0242) < l_q282))) {
        const int l_c285 = ((l_cmd280 >= 4) ? 1 : 0);
        const int l_op286 = prm.op[l_c285][((l_cmd280 - (((l_cmd280 >= 4) ? 1 : 0) * 3)) - 1)];
        const int l_v287 = prm.val[l_c285][((l_cmd280 - (((l_cmd280 >= 4) ? 1 : 0) * 3)) - 1)];
        int l_x288 = 0;
        if ((l_op286 == 1)) {
          l_kv241 = (1 | (l_v287 << 3));
          l_x288 = 7;
        }
        if ((l_op286 == 2)) {
          const int l_len289 = (l_kv241 & 7);
          l_kv241 = (((l_len289 + 1) | (l_kv241 & -8)) | (l_v287 << (3 + (l_len289 * 2))));
          l_x288 = l_kv241;
        }
        if ((l_op286 == 3)) {
          l_x288 = (((l_kv241 & 7) != 0) ? l_kv241 : 6);
        }
        if ((l_c281 != 0)) {
          l_ls1243 = l_q282;
        } else {
          l_ls0242 = l_q282;
        }
        if ((l_now284 && (l_act240 != 0))) {
          ctx.send(Rec{"Reply", {std::to_string(l_q282), std::to_string(l_x288)}}, (first_client(prm) + (l_c281 + 1) - 1));
        }
      }
      if (l_now284) {
        l_so244 = 5;
      }
      slotout = l_so244;
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
            const int l_me290 = log[0];
            const int l_mm291 = p1blog[0];
            if (((l_me290 & 3) == 2)) {
              p1blog[0] = ((2 | (0 << 2)) | (((l_me290 >> 8) & 7) << 8));
            } else {
              if (((((l_me290 & 3) == 1) && ((l_mm291 & 3) != 2)) && (((l_mm291 & 3) == 0) || (((l_mm291 >> 2) & 63) < ((l_me290 >> 2) & 63))))) {
                p1blog[0] = l_me290;
              }
            }
            const int l_me292 = log[1];
            const int l_mm293 = p1blog[1];
            if (((l_me292 & 3) == 2)) {
              p1blog[1] = ((2 | (0 << 2)) | (((l_me292 >> 8) & 7) << 8));
            } else {
              if (((((l_me292 & 3) == 1) && ((l_mm293 & 3) != 2)) && (((l_mm293 & 3) == 0) || (((l_mm293 >> 2) & 63) < ((l_me292 >> 2) & 63))))) {
                p1blog[1] = l_me292;
              }
            }
            const int l_me294 = log[2];
            const int l_mm295 = p1blog[2];
            if (((l_me294 & 3) == 2)) {
              p1blog[2] = ((2 | (0 << 2)) | (((l_me294 >> 8) & 7) << 8));
            } else {
              if (((((l_me294 & 3) == 1) && ((l_mm295 & 3) != 2)) && (((l_mm295 & 3) == 0) || (((l_mm295 >> 2) & 63) < ((l_me294 >> 2) & 63))))) {
                p1blog[2] = l_me294;
              }
            }
            const int l_me296 = log[3];
            const int l_mm297 = p1blog[3];
            if (((l_me296 & 3) == 2)) {
              p1blog[3] = ((2 | (0 << 2)) | (((l_me296 >> 8) & 7) << 8));
            } else {
              if (((((l_me296 & 3) == 1) && ((l_mm297 & 3) != 2)) && (((l_mm297 & 3) == 0) || (((l_mm297 >> 2) & 63) < ((l_me296 >> 2) & 63))))) {
                p1blog[3] = l_me296;
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
              const int l_mg298 = p1blog[0];
              const int l_mg299 = p1blog[1];
              const int l_mg300 = p1blog[2];
              const int l_mg301 = p1blog[3];
              int l_last302 = 0;
              if ((((l_mg298 & 3) != 0) || ((log[0] & 3) != 0))) {
                l_last302 = 1;
              }
              if ((((l_mg299 & 3) != 0) || ((log[1] & 3) != 0))) {
                l_last302 = 2;
              }
              if ((((l_mg300 & 3) != 0) || ((log[2] & 3) != 0))) {
                l_last302 = 3;
              }
              if ((((l_mg301 & 3) != 0) || ((log[3] & 3) != 0))) {
                l_last302 = 4;
              }
              p1blog[0] = 0;
              p1blog[1] = 0;
              p1blog[2] = 0;
              p1blog[3] = 0;
              if (((1 <= l_last302) && ((log[0] & 3) != 2))) {
                if (((l_mg298 & 3) == 2)) {
                  log[0] = ((2 | (0 << 2)) | (((l_mg298 >> 8) & 7) << 8));
                  votes[0] = 0;
                } else {
                  log[(1 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg298 & 3) == 1) ? ((l_mg298 >> 8) & 7) : 0) << 8));
                  votes[(1 - 1)] = (1 << (self - first_server(prm)));
                  if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(1), std::to_string((((l_mg298 & 3) == 1) ? ((l_mg298 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
                  }
                  if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(1), std::to_string((((l_mg298 & 3) == 1) ? ((l_mg298 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
                  }
                  if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(1), std::to_string((((l_mg298 & 3) == 1) ? ((l_mg298 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
                  }
                  if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
                    const int l_ccmd303 = ((log[(1 - 1)] >> 8) & 7);
                    log[(1 - 1)] = ((2 | (0 << 2)) | (l_ccmd303 << 8));
                    votes[(1 - 1)] = 0;
                    if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(1), std::to_string(l_ccmd303)}}, (first_server(prm) + 1 - 1));
                    }
                    if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(1), std::to_string(l_ccmd303)}}, (first_server(prm) + 2 - 1));
                    }
                    if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(1), std::to_string(l_ccmd303)}}, (first_server(prm) + 3 - 1));
                    }
                  }
                }
              }
              if (((2 <= l_last302) && ((log[1] & 3) != 2))) {
                if (((l_mg299 & 3) == 2)) {
                  log[1] = ((2 | (0 << 2)) | (((l_mg299 >> 8) & 7) << 8));
                  votes[1] = 0;
                } else {
                  log[(2 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg299 & 3) == 1) ? ((l_mg299 >> 8) & 7) : 0) << 8));
                  votes[(2 - 1)] = (1 << (self - first_server(prm)));
                  if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(2), std::to_string((((l_mg299 & 3) == 1) ? ((l_mg299 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
                  }
                  if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(2), std::to_string((((l_mg299 & 3) == 1) ? ((l_mg299 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
                  }
                  if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(2), std::to_string((((l_mg299 & 3) == 1) ? ((l_mg299 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
                  }
                  if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
                    const int l_ccmd304 = ((log[(2 - 1)] >> 8) & 7);
                    log[(2 - 1)] = ((2 | (0 << 2)) | (l_ccmd304 << 8));
                    votes[(2 - 1)] = 0;
                    if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(2), std::to_string(l_ccmd304)}}, (first_server(prm) + 1 - 1));
                    }
                    if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(2), std::to_string(l_ccmd304)}}, (first_server(prm) + 2 - 1));
                    }
                    if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(2), std::to_string(l_ccmd304)}}, (first_server(prm) + 3 - 1));
                    }
                  }
                }
              }
              if (((3 <= l_last302) && ((log[2] & 3) != 2))) {
                if (((l_mg300 & 3) == 2)) {
                  log[2] = ((2 | (0 << 2)) | (((l_mg300 >> 8) & 7) << 8));
                  votes[2] = 0;
                } else {
                  log[(3 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg300 & 3) == 1) ? ((l_mg300 >> 8) & 7) : 0) << 8));
                  votes[(3 - 1)] = (1 << (self - first_server(prm)));
                  if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(3), std::to_string((((l_mg300 & 3) == 1) ? ((l_mg300 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
                  }
                  if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(3), std::to_string((((l_mg300 & 3) == 1) ? ((l_mg300 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
                  }
                  if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(3), std::to_string((((l_mg300 & 3) == 1) ? ((l_mg300 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
                  }
                  if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
                    const int l_ccmd305 = ((log[(3 - 1)] >> 8) & 7);
                    log[(3 - 1)] = ((2 | (0 << 2)) | (l_ccmd305 << 8));
                    votes[(3 - 1)] = 0;
                    if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(3), std::to_string(l_ccmd305)}}, (first_server(prm) + 1 - 1));
                    }
                    if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(3), std::to_string(l_ccmd305)}}, (first_server(prm) + 2 - 1));
                    }
                    if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(3), std::to_string(l_ccmd305)}}, (first_server(prm) + 3 - 1));
                    }
                  }
                }
              }
              if (((4 <= l_last302) && ((log[3] & 3) != 2))) {
                if (((l_mg301 & 3) == 2)) {
                  log[3] = ((2 | (0 << 2)) | (((l_mg301 >> 8) & 7) << 8));
                  votes[3] = 0;
                } else {
                  log[(4 - 1)] = ((1 | (((round << 2) | leader) << 2)) | ((((l_mg301 & 3) == 1) ? ((l_mg301 >> 8) & 7) : 0) << 8));
                  votes[(4 - 1)] = (1 << (self - first_server(prm)));
                  if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(4), std::to_string((((l_mg301 & 3) == 1) ? ((l_mg301 >> 8) & 7) : 0))}}, (first_server(prm) + 1 - 1));
                  }
                  if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(4), std::to_string((((l_mg301 & 3) == 1) ? ((l_mg301 >> 8) & 7) : 0))}}, (first_server(prm) + 2 - 1));
                  }
                  if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                    ctx.send(Rec{"P2a", {std::to_string(round), std::to_string(leader), std::to_string(4), std::to_string((((l_mg301 & 3) == 1) ? ((l_mg301 >> 8) & 7) : 0))}}, (first_server(prm) + 3 - 1));
                  }
                  if (((((((1 << (self - first_server(prm))) & 1) + (((1 << (self - first_server(prm))) >> 1) & 1)) + (((1 << (self - first_server(prm))) >> 2) & 1)) * 2) > prm.servers)) {
                    const int l_ccmd306 = ((log[(4 - 1)] >> 8) & 7);
                    log[(4 - 1)] = ((2 | (0 << 2)) | (l_ccmd306 << 8));
                    votes[(4 - 1)] = 0;
                    if (((0 < prm.servers) && (0 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(4), std::to_string(l_ccmd306)}}, (first_server(prm) + 1 - 1));
                    }
                    if (((1 < prm.servers) && (1 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(4), std::to_string(l_ccmd306)}}, (first_server(prm) + 2 - 1));
                    }
                    if (((2 < prm.servers) && (2 != (self - first_server(prm))))) {
                      ctx.send(Rec{"Decision", {std::to_string(4), std::to_string(l_ccmd306)}}, (first_server(prm) + 3 - 1));
                    }
                  }
                }
              }
              slotin = (l_last302 + 1);
              const int l_so0307 = slotout;
              const int l_act308 = active;
              int l_kv309 = 0;
              int l_ls0310 = 0;
              int l_ls1311 = 0;
              int l_so312 = l_so0307;
              int l_run313 = 1;
              const int l_e314 = log[0];
              const int l_cmd315 = ((l_e314 >> 8) & 7);
              const int l_c316 = ((l_cmd315 >= 4) ? 1 : 0);
              const int l_q317 = (l_cmd315 - (((l_cmd315 >= 4) ? 1 : 0) * 3));
              const int l_before318 = (1 < l_so0307);
              const int l_now319 = (((!l_before318) && (l_run313 != 0)) && ((l_e314 & 3) == 2));
              l_run313 = (((l_run313 != 0) && (l_before318 || l_now319)) ? 1 : 0);
              if ((((l_before318 || l_now319) && (l_cmd315 != 0)) && ((l_c316 ? l_ls1311 : l_ls0310) < l_q317))) {
                const int l_c320 = ((l_cmd315 >= 4) ? 1 : 0);
                const int l_op321 = prm.op[l_c320][((l_cmd315 - (((l_cmd315 >= 4) ? 1 : 0) * 3)) - 1)];
                const int l_v322 = prm.val[l_c320][((l_cmd315 - (((l_cmd315 >= 4) ? 1 : 0) * 3)) - 1)];
                int l_x323 = 0;
                if ((l_op321 == 1)) {
                  l_kv309 = (1 | (l_v322 << 3));
                  l_x323 = 7;
                }
                if ((l_op321 == 2)) {
                  const int l_len324 = (l_kv309 & 7);
                  l_kv309 = (((l_len324 + 1) | (l_kv309 & -8)) | (l_v322 << (3 + (l_len324 * 2))));
                  l_x323 = l_kv309;
                }
                if ((l_op321 == 3)) {
                  l_x323 = (((l_kv309 & 7) != 0) ? l_kv309 : 6);
                }
                if ((l_c316 != 0)) {
                  l_ls1311 = l_q317;
                } else {
                  l_ls0310 = l_q317;
                }
                if ((l_now319 && (l_act308 != 0))) {
                  ctx.send(Rec{"Reply", {std::to_string(l_q317), std::to_string(l_x323)}}, (first_client(prm) + (l_c316 + 1) - 1));
                }
              }
              if (l_now319) {
                l_so312 = 2;
              }
              const int l_e325 = log[1];
              const int l_cmd326 = ((l_e325 >> 8) & 7);
              const int l_c327 = ((l_cmd326 >= 4) ? 1 : 0);
              const int l_q328 = (l_cmd326 - (((l_cmd326 >= 4) ? 1 : 0) * 3));
              const int l_before329 = (2 < l_so0307);
              const int l_now330 = (((!l_before329) && (l_run313 != 0)) && ((l_e325 & 3) == 2));
              l_run313 = (((l_run313 != 0) && (l_before329 || l_now330)) ? 1 : 0);
              if ((((l_before329 || l_now330) && (l_cmd326 != 0)) && ((l_c327 ? l_ls1311 : l_ls0310) < l_q328))) {
                const int l_c331 = ((l_cmd326 >= 4) ? 1 : 0);
                const int l_op332 = prm.op[l_c331][((l_cmd326 - (((l_cmd326 >= 4) ? 1 : 0) * 3)) - 1)];
                const int l_v333 = prm.val[l_c331][((l_cmd326 - (((l_cmd326 >= 4) ? 1 : 0) * 3)) - 1)];
                int l_x334 = 0;
                if ((l_op332 == 1)) {
                  l_kv309 = (1 | (l_v333 << 3));
                  l_x334 = 7;
                }
                if ((l_op332 == 2)) {
                  const int l_len335 = (l_kv309 & 7);
                  l_kv309 = (((l_len335 + 1) | (l_kv309 & -8)) | (l_v333 << (3 + (l_len335 * 2))));
                  l_x334 = l_kv309;
                }
                if ((l_op332 == 3)) {
                  l_x334 = (((l_kv309 & 7) != 0) ? l_kv309 : 6);
                }
                if ((l_c327 != 0)) {
                  l_ls1311 = l_q328;
                } else {
                  l_ls0310 = l_q328;
                }
                if ((l_now330 && (l_act308 != 0))) {
                  ctx.send(Rec{"Reply", {std::to_string(l_q328), std::to_string(l_x334)}}, (first_client(prm) + (l_c327 + 1) - 1));
                }
              }
              if (l_now330) {
                l_so312 = 3;
              }
              const int l_e336 = log[2];
              const int l_cmd337 = ((l_e336 >> 8) & 7);
              const int l_c338 = ((l_cmd337 >= 4) ? 1 : 0);
              const int l_q339 = (l_cmd337 - (((l_cmd337 >= 4) ? 1 : 0) * 3));
              const int l_before340 = (3 < l_so0307);
              const int l_now341 = (((!l_before340) && (l_run313 != 0)) && ((l_e336 & 3) == 2));
              l_run313 = (((l_run313 != 0) && (l_before340 || l_now341)) ? 1 : 0);
              if ((((l_before340 || l_now341) && (l_cmd337 != 0)) && ((l_c338 ? l_ls1311 : l_ls0310) < l_q339))) {
                const int l_c342 = ((l_cmd337 >= 4) ? 1 : 0);
                const int l_op343 = prm.op[l_c342][((l_cmd337 - (((l_cmd337 >= 4) ? 1 : 0) * 3)) - 1)];
                const int l_v344 = prm.val[l_c342][((l_cmd337 - (((l_cmd337 >= 4) ? 1 : 0) * 3)) - 1)];
                int l_x345 = 0;
                if ((l_op343 == 1)) {
                  l_kv309 = (1 | (l_v344 << 3));
                  l_x345 = 7;
                }
                if ((l_op343 == 2)) {
                  const int l_len346 = (l_kv309 & 7);
                  l_kv309 = (((l_len346 + 1) | (l_kv309 & -8)) | (l_v344 << (3 + (l_len346 * 2))));
                  l_x345 = l_kv309;
                }
                if ((l_op343 == 3)) {
                  l_x345 = (((l_kv309 & 7) != 0) ? l_kv309 : 6);
                }
                if ((l_c338 != 0)) {
                  l_ls1311 = l_q339;
                } else {
                  l_ls0310 = l_q339;
                }
                if ((l_now341 && (l_act308 != 0))) {
                  ctx.send(Rec{"Reply", {std::to_string(l_q339), std::to_string(l_x345)}}, (first_client(prm) + (l_c338 + 1) - 1));
                }
              }
              if (l_now341) {
                l_so312 = 4;
              }
              const int l_e347 = log[3];
              const int l_cmd348 = ((l_e347 >> 8) & 7);
              const int l_c349 = ((l_cmd348 >= 4) ? 1 : 0);
              const int l_q350 = (l_cmd348 - (((l_cmd348 >= 4) ? 1 : 0) * 3));
              const int l_before351 = (4 < l_so0307);
              const int l_now352 = (((!l_before351) && (l_run313 != 0)) && ((l_e347 & 3) == 2));
              l_run313 = (((l_run313 != 0) && (l_before351 || l_now352)) ? 1 : 0);
              if ((((l_before351 || l_now352) && (l_cmd348 != 0)) && ((l_c349 ? l_ls1311 : l_ls0310) < l_q350))) {
                const int l_c353 = ((l_cmd348 >= 4) ? 1 : 0);
                const int l_op354 = prm.op[l_c353][((l_cmd348 - (((l_cmd348 >= 4) ? 1 : 0) * 3)) - 1)];
                const int l_v355 = prm.val[l_c353][((l_cmd348 - (((l_cmd348 >= 4) ? 1 : 0) * 3)) - 1)];
                int l_x356 = 0;
                if ((l_op354 == 1)) {
                  l_kv309 = (1 | (l_v355 << 3));
                  l_x356 = 7;
                }
                if ((l_op354 == 2)) {
                  const int l_len357 = (l_kv309 & 7);
                  l_kv309 = (((l_len357 + 1) | (l_kv309 & -8)) | (l_v355 << (3 + (l_len357 * 2))));
                  l_x356 = l_kv309;
                }
                if ((l_op354 == 3)) {
                  l_x356 = (((l_kv309 & 7) != 0) ? l_kv309 : 6);
                }
                if ((l_c349 != 0)) {
                  l_ls1311 = l_q350;
                } else {
                  l_ls0310 = l_q350;
                }
                if ((l_now352 && (l_act308 != 0))) {
                  ctx.send(Rec{"Reply", {std::to_string(l_q350), std::to_string(l_x356)}}, (first_client(prm) + (l_c349 + 1) - 1));
                }
              }
              if (l_now352) {
                l_so312 = 5;
              }
              slotout = l_so312;
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
        const int l_cid358 = (((self - first_client(prm)) * 3) + std::stoi(t.f[0]));
        if ((0 < prm.servers)) {
          ctx.send(Rec{"Request", {std::to_string(l_cid358)}}, (first_server(prm) + 1 - 1));
        }
        if ((1 < prm.servers)) {
          ctx.send(Rec{"Request", {std::to_string(l_cid358)}}, (first_server(prm) + 2 - 1));
        }
        if ((2 < prm.servers)) {
          ctx.send(Rec{"Request", {std::to_string(l_cid358)}}, (first_server(prm) + 3 - 1));
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
    const int l_cid359 = (((self - first_client(prm)) * 3) + cmd);
    if ((0 < prm.servers)) {
      ctx.send(Rec{"Request", {std::to_string(l_cid359)}}, (first_server(prm) + 1 - 1));
    }
    if ((1 < prm.servers)) {
      ctx.send(Rec{"Request", {std::to_string(l_cid359)}}, (first_server(prm) + 2 - 1));
    }
    if ((2 < prm.servers)) {
      ctx.send(Rec{"Request", {std::to_string(l_cid359)}}, (first_server(prm) + 3 - 1));
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
      int l_isch360 = 0;
      int l_confl361 = 0;
      int l_chosen362 = 0;
      int l_count363 = 0;
      if ((0 < prm.servers)) {
        const int l_e364 = n_server(s, first_server(prm) + 0)->log[0];
        if (((l_e364 & 3) == 2)) {
          const int l_x365 = ((((l_e364 >> 8) & 7) != 0) ? ((prm.op[((((l_e364 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e364 >> 8) & 7) - (((((l_e364 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e364 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e364 >> 8) & 7) - (((((l_e364 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch360 != 0) && (l_x365 != l_chosen362))) {
            l_confl361 = 1;
          }
          l_chosen362 = l_x365;
          l_isch360 = 1;
        }
      }
      if ((1 < prm.servers)) {
        const int l_e366 = n_server(s, first_server(prm) + 1)->log[0];
        if (((l_e366 & 3) == 2)) {
          const int l_x367 = ((((l_e366 >> 8) & 7) != 0) ? ((prm.op[((((l_e366 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e366 >> 8) & 7) - (((((l_e366 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e366 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e366 >> 8) & 7) - (((((l_e366 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch360 != 0) && (l_x367 != l_chosen362))) {
            l_confl361 = 1;
          }
          l_chosen362 = l_x367;
          l_isch360 = 1;
        }
      }
      if ((2 < prm.servers)) {
        const int l_e368 = n_server(s, first_server(prm) + 2)->log[0];
        if (((l_e368 & 3) == 2)) {
          const int l_x369 = ((((l_e368 >> 8) & 7) != 0) ? ((prm.op[((((l_e368 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e368 >> 8) & 7) - (((((l_e368 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e368 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e368 >> 8) & 7) - (((((l_e368 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch360 != 0) && (l_x369 != l_chosen362))) {
            l_confl361 = 1;
          }
          l_chosen362 = l_x369;
          l_isch360 = 1;
        }
      }
      if ((0 < prm.servers)) {
        const int l_e370 = n_server(s, first_server(prm) + 0)->log[0];
        if ((((l_e370 & 3) != 0) && (((l_e370 & 3) != 1) || (((((l_e370 >> 8) & 7) != 0) ? ((prm.op[((((l_e370 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e370 >> 8) & 7) - (((((l_e370 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e370 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e370 >> 8) & 7) - (((((l_e370 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen362)))) {
          l_count363 = (l_count363 + 1);
        }
      }
      if ((1 < prm.servers)) {
        const int l_e371 = n_server(s, first_server(prm) + 1)->log[0];
        if ((((l_e371 & 3) != 0) && (((l_e371 & 3) != 1) || (((((l_e371 >> 8) & 7) != 0) ? ((prm.op[((((l_e371 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e371 >> 8) & 7) - (((((l_e371 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e371 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e371 >> 8) & 7) - (((((l_e371 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen362)))) {
          l_count363 = (l_count363 + 1);
        }
      }
      if ((2 < prm.servers)) {
        const int l_e372 = n_server(s, first_server(prm) + 2)->log[0];
        if ((((l_e372 & 3) != 0) && (((l_e372 & 3) != 1) || (((((l_e372 >> 8) & 7) != 0) ? ((prm.op[((((l_e372 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e372 >> 8) & 7) - (((((l_e372 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e372 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e372 >> 8) & 7) - (((((l_e372 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen362)))) {
          l_count363 = (l_count363 + 1);
        }
      }
      if (((l_isch360 != 0) && ((l_confl361 != 0) || ((l_count363 * 2) <= prm.servers)))) {
        { res_.value = false; return res_; }
      }
      int l_isch373 = 0;
      int l_confl374 = 0;
      int l_chosen375 = 0;
      int l_count376 = 0;
      if ((0 < prm.servers)) {
        const int l_e377 = n_server(s, first_server(prm) + 0)->log[1];
        if (((l_e377 & 3) == 2)) {
          const int l_x378 = ((((l_e377 >> 8) & 7) != 0) ? ((prm.op[((((l_e377 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e377 >> 8) & 7) - (((((l_e377 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e377 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e377 >> 8) & 7) - (((((l_e377 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch373 != 0) && (l_x378 != l_chosen375))) {
            l_confl374 = 1;
          }
          l_chosen375 = l_x378;
          l_isch373 = 1;
        }
      }
      if ((1 < prm.servers)) {
        const int l_e379 = n_server(s, first_server(prm) + 1)->log[1];
        if (((l_e379 & 3) == 2)) {
          const int l_x380 = ((((l_e379 >> 8) & 7) != 0) ? ((prm.op[((((l_e379 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e379 >> 8) & 7) - (((((l_e379 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e379 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e379 >> 8) & 7) - (((((l_e379 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch373 != 0) && (l_x380 != l_chosen375))) {
            l_confl374 = 1;
          }
          l_chosen375 = l_x380;
          l_isch373 = 1;
        }
      }
      if ((2 < prm.servers)) {
        const int l_e381 = n_server(s, first_server(prm) + 2)->log[1];
        if (((l_e381 & 3) == 2)) {
          const int l_x382 = ((((l_e381 >> 8) & 7) != 0) ? ((prm.op[((((l_e381 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e381 >> 8) & 7) - (((((l_e381 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e381 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e381 >> 8) & 7) - (((((l_e381 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch373 != 0) && (l_x382 != l_chosen375))) {
            l_confl374 = 1;
          }
          l_chosen375 = l_x382;
          l_isch373 = 1;
        }
      }
      if ((0 < prm.servers)) {
        const int l_e383 = n_server(s, first_server(prm) + 0)->log[1];
        if ((((l_e383 & 3) != 0) && (((l_e383 & 3) != 1) || (((((l_e383 >> 8) & 7) != 0) ? ((prm.op[((((l_e383 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e383 >> 8) & 7) - (((((l_e383 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e383 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e383 >> 8) & 7) - (((((l_e383 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen375)))) {
          l_count376 = (l_count376 + 1);
        }
      }
      if ((1 < prm.servers)) {
        const int l_e384 = n_server(s, first_server(prm) + 1)->log[1];
        if ((((l_e384 & 3) != 0) && (((l_e384 & 3) != 1) || (((((l_e384 >> 8) & 7) != 0) ? ((prm.op[((((l_e384 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e384 >> 8) & 7) - (((((l_e384 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e384 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e384 >> 8) & 7) - (((((l_e384 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen375)))) {
          l_count376 = (l_count376 + 1);
        }
      }
      if ((2 < prm.servers)) {
        const int l_e385 = n_server(s, first_server(prm) + 2)->log[1];
        if ((((l_e385 & 3) != 0) && (((l_e385 & 3) != 1) || (((((l_e385 >> 8) & 7) != 0) ? ((prm.op[((((l_e385 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e385 >> 8) & 7) - (((((l_e385 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e385 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e385 >> 8) & 7) - (((((l_e385 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen375)))) {
          l_count376 = (l_count376 + 1);
        }
      }
      if (((l_isch373 != 0) && ((l_confl374 != 0) || ((l_count376 * 2) <= prm.servers)))) {
        { res_.value = false; return res_; }
      }
      int l_isch386 = 0;
      int l_confl387 = 0;
      int l_chosen388 = 0;
      int l_count389 = 0;
      if ((0 < prm.servers)) {
        const int l_e390 = n_server(s, first_server(prm) + 0)->log[2];
        if (((l_e390 & 3) == 2)) {
          const int l_x391 = ((((l_e390 >> 8) & 7) != 0) ? ((prm.op[((((l_e390 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e390 >> 8) & 7) - (((((l_e390 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e390 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e390 >> 8) & 7) - (((((l_e390 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch386 != 0) && (l_x391 != l_chosen388))) {
            l_confl387 = 1;
          }
          l_chosen388 = l_x391;
          l_isch386 = 1;
        }
      }
      if ((1 < prm.servers)) {
        const int l_e392 = n_server(s, first_server(prm) + 1)->log[2];
        if (((l_e392 & 3) == 2)) {
          const int l_x393 = ((((l_e392 >> 8) & 7) != 0) ? ((prm.op[((((l_e392 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e392 >> 8) & 7) - (((((l_e392 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e392 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e392 >> 8) & 7) - (((((l_e392 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch386 != 0) && (l_x393 != l_chosen388))) {
            l_confl387 = 1;
          }
          l_chosen388 = l_x393;
          l_isch386 = 1;
        }
      }
      if ((2 < prm.servers)) {
        const int l_e394 = n_server(s, first_server(prm) + 2)->log[2];
        if (((l_e394 & 3) == 2)) {
          const int l_x395 = ((((l_e394 >> 8) & 7) != 0) ? ((prm.op[((((l_e394 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e394 >> 8) & 7) - (((((l_e394 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e394 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e394 >> 8) & 7) - (((((l_e394 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch386 != 0) && (l_x395 != l_chosen388))) {
            l_confl387 = 1;
          }
          l_chosen388 = l_x395;
          l_isch386 = 1;
        }
      }
      if ((0 < prm.servers)) {
        const int l_e396 = n_server(s, first_server(prm) + 0)->log[2];
        if ((((l_e396 & 3) != 0) && (((l_e396 & 3) != 1) || (((((l_e396 >> 8) & 7) != 0) ? ((prm.op[((((l_e396 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e396 >> 8) & 7) - (((((l_e396 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e396 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e396 >> 8) & 7) - (((((l_e396 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen388)))) {
          l_count389 = (l_count389 + 1);
        }
      }
      if ((1 < prm.servers)) {
        const int l_e397 = n_server(s, first_server(prm) + 1)->log[2];
        if ((((l_e397 & 3) != 0) && (((l_e397 & 3) != 1) || (((((l_e397 >> 8) & 7) != 0) ? ((prm.op[((((l_e397 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e397 >> 8) & 7) - (((((l_e397 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e397 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e397 >> 8) & 7) - (((((l_e397 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen388)))) {
          l_count389 = (l_count389 + 1);
        }
      }
      if ((2 < prm.servers)) {
        const int l_e398 = n_server(s, first_server(prm) + 2)->log[2];
        if ((((l_e398 & 3) != 0) && (((l_e398 & 3) != 1) || (((((l_e398 >> 8) & 7) != 0) ? ((prm.op[((((l_e398 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e398 >> 8) & 7) - (((((l_e398 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e398 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e398 >> 8) & 7) - (((((l_e398 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen388)))) {
          l_count389 = (l_count389 + 1);
        }
      }
      if (((l_isch386 != 0) && ((l_confl387 != 0) || ((l_count389 * 2) <= prm.servers)))) {
        { res_.value = false; return res_; }
      }
      int l_isch399 = 0;
      int l_confl400 = 0;
      int l_chosen401 = 0;
      int l_count402 = 0;
      if ((0 < prm.servers)) {
        const int l_e403 = n_server(s, first_server(prm) + 0)->log[3];
        if (((l_e403 & 3) == 2)) {
          const int l_x404 = ((((l_e403 >> 8) & 7) != 0) ? ((prm.op[((((l_e403 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e403 >> 8) & 7) - (((((l_e403 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e403 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e403 >> 8) & 7) - (((((l_e403 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch399 != 0) && (l_x404 != l_chosen401))) {
            l_confl400 = 1;
          }
          l_chosen401 = l_x404;
          l_isch399 = 1;
        }
      }
      if ((1 < prm.servers)) {
        const int l_e405 = n_server(s, first_server(prm) + 1)->log[3];
        if (((l_e405 & 3) == 2)) {
          const int l_x406 = ((((l_e405 >> 8) & 7) != 0) ? ((prm.op[((((l_e405 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e405 >> 8) & 7) - (((((l_e405 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e405 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e405 >> 8) & 7) - (((((l_e405 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch399 != 0) && (l_x406 != l_chosen401))) {
            l_confl400 = 1;
          }
          l_chosen401 = l_x406;
          l_isch399 = 1;
        }
      }
      if ((2 < prm.servers)) {
        const int l_e407 = n_server(s, first_server(prm) + 2)->log[3];
        if (((l_e407 & 3) == 2)) {
          const int l_x408 = ((((l_e407 >> 8) & 7) != 0) ? ((prm.op[((((l_e407 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e407 >> 8) & 7) - (((((l_e407 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e407 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e407 >> 8) & 7) - (((((l_e407 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch399 != 0) && (l_x408 != l_chosen401))) {
            l_confl400 = 1;
          }
          l_chosen401 = l_x408;
          l_isch399 = 1;
        }
      }
      if ((0 < prm.servers)) {
        const int l_e409 = n_server(s, first_server(prm) + 0)->log[3];
        if ((((l_e409 & 3) != 0) && (((l_e409 & 3) != 1) || (((((l_e409 >> 8) & 7) != 0) ? ((prm.op[((((l_e409 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e409 >> 8) & 7) - (((((l_e409 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e409 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e409 >> 8) & 7) - (((((l_e409 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen401)))) {
          l_count402 = (l_count402 + 1);
        }
      }
      if ((1 < prm.servers)) {
        const int l_e410 = n_server(s, first_server(prm) + 1)->log[3];
        if ((((l_e410 & 3) != 0) && (((l_e410 & 3) != 1) || (((((l_e410 >> 8) & 7) != 0) ? ((prm.op[((((l_e410 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e410 >> 8) & 7) - (((((l_e410 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e410 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e410 >> 8) & 7) - (((((l_e410 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen401)))) {
          l_count402 = (l_count402 + 1);
        }
      }
      if ((2 < prm.servers)) {
        const int l_e411 = n_server(s, first_server(prm) + 2)->log[3];
        if ((((l_e411 & 3) != 0) && (((l_e411 & 3) != 1) || (((((l_e411 >> 8) & 7) != 0) ? ((prm.op[((((l_e411 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e411 >> 8) & 7) - (((((l_e411 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e411 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e411 >> 8) & 7) - (((((l_e411 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen401)))) {
          l_count402 = (l_count402 + 1);
        }
      }
      if (((l_isch399 != 0) && ((l_confl400 != 0) || ((l_count402 * 2) <= prm.servers)))) {
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
        const int l_e412 = n_server(s, first_server(prm) + 0)->log[(l_i - 1)];
        if (((l_e412 & 3) == 2)) {
          const int l_x413 = ((((l_e412 >> 8) & 7) != 0) ? ((prm.op[((((l_e412 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e412 >> 8) & 7) - (((((l_e412 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e412 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e412 >> 8) & 7) - (((((l_e412 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch != 0) && (l_x413 != l_chosen))) {
            l_confl = 1;
          }
          l_chosen = l_x413;
          l_isch = 1;
        }
      }
      if ((1 < prm.servers)) {
        const int l_e414 = n_server(s, first_server(prm) + 1)->log[(l_i - 1)];
        if (((l_e414 & 3) == 2)) {
          const int l_x415 = ((((l_e414 >> 8) & 7) != 0) ? ((prm.op[((((l_e414 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e414 >> 8) & 7) - (((((l_e414 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e414 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e414 >> 8) & 7) - (((((l_e414 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch != 0) && (l_x415 != l_chosen))) {
            l_confl = 1;
          }
          l_chosen = l_x415;
          l_isch = 1;
        }
      }
      if ((2 < prm.servers)) {
        const int l_e416 = n_server(s, first_server(prm) + 2)->log[(l_i - 1)];
        if (((l_e416 & 3) == 2)) {
          const int l_x417 = ((((l_e416 >> 8) & 7) != 0) ? ((prm.op[((((l_e416 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e416 >> 8) & 7) - (((((l_e416 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e416 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e416 >> 8) & 7) - (((((l_e416 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0);
          if (((l_isch != 0) && (l_x417 != l_chosen))) {
            l_confl = 1;
          }
          l_chosen = l_x417;
          l_isch = 1;
        }
      }
      if ((0 < prm.servers)) {
        const int l_e418 = n_server(s, first_server(prm) + 0)->log[(l_i - 1)];
        if ((((l_e418 & 3) != 0) && (((l_e418 & 3) != 1) || (((((l_e418 >> 8) & 7) != 0) ? ((prm.op[((((l_e418 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e418 >> 8) & 7) - (((((l_e418 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e418 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e418 >> 8) & 7) - (((((l_e418 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen)))) {
          l_count = (l_count + 1);
        }
      }
      if ((1 < prm.servers)) {
        const int l_e419 = n_server(s, first_server(prm) + 1)->log[(l_i - 1)];
        if ((((l_e419 & 3) != 0) && (((l_e419 & 3) != 1) || (((((l_e419 >> 8) & 7) != 0) ? ((prm.op[((((l_e419 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e419 >> 8) & 7) - (((((l_e419 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e419 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e419 >> 8) & 7) - (((((l_e419 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen)))) {
          l_count = (l_count + 1);
        }
      }
      if ((2 < prm.servers)) {
        const int l_e420 = n_server(s, first_server(prm) + 2)->log[(l_i - 1)];
        if ((((l_e420 & 3) != 0) && (((l_e420 & 3) != 1) || (((((l_e420 >> 8) & 7) != 0) ? ((prm.op[((((l_e420 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e420 >> 8) & 7) - (((((l_e420 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_e420 >> 8) & 7) >= 4) ? 1 : 0)][((((l_e420 >> 8) & 7) - (((((l_e420 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0) == l_chosen)))) {
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
      const int l_k421 = (a0_ - (first_server(prm) + 1 - 1));
      if (((l_k421 < 0) || (l_k421 >= prm.servers))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_slot422 = (a1_ >> 4);
      int l_se423 = 0;
      if (((l_slot422 >= 1) && (l_slot422 <= 4))) {
        l_se423 = n_server(s, first_server(prm) + l_k421)->log[(l_slot422 - 1)];
      }
      if (((l_se423 & 3) == (a1_ & 15))) {
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
      const int l_k424 = (a0_ - (first_server(prm) + 1 - 1));
      if (((l_k424 < 0) || (l_k424 >= prm.servers))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_slot425 = (a1_ >> 8);
      int l_se426 = 0;
      if (((l_slot425 >= 1) && (l_slot425 <= 4))) {
        l_se426 = n_server(s, first_server(prm) + l_k424)->log[(l_slot425 - 1)];
      }
      const int l_cc = (((l_se426 & 3) == 0) ? 0 : ((((l_se426 >> 8) & 7) != 0) ? ((prm.op[((((l_se426 >> 8) & 7) >= 4) ? 1 : 0)][((((l_se426 >> 8) & 7) - (((((l_se426 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)] << 2) | prm.val[((((l_se426 >> 8) & 7) >= 4) ? 1 : 0)][((((l_se426 >> 8) & 7) - (((((l_se426 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)]) : 0));
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
      const int l_pres427 = ((0 < prm.clients) && (0 < (int)s.cw(first_client(prm) + 0)->results.size()));
      if ((l_pres427 && (prm.op[0][0] != 2))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_res428 = (l_pres427 ? std::stoi(s.cw(first_client(prm) + 0)->results[0].f[0]) : 0);
      const int l_rlen429 = (l_res428 & 7);
      if ((l_pres427 && (((l_rlen429 == 0) || (l_rlen429 > 4)) || (((l_res428 >> (1 + (l_rlen429 * 2))) & 3) != prm.val[0][0])))) {
        { res_.value = false; return res_; }
      }
      const int l_pres430 = ((0 < prm.clients) && (1 < (int)s.cw(first_client(prm) + 0)->results.size()));
      if ((l_pres430 && (prm.op[0][1] != 2))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_res431 = (l_pres430 ? std::stoi(s.cw(first_client(prm) + 0)->results[1].f[0]) : 0);
      const int l_rlen432 = (l_res431 & 7);
      if ((l_pres430 && (((l_rlen432 == 0) || (l_rlen432 > 4)) || (((l_res431 >> (1 + (l_rlen432 * 2))) & 3) != prm.val[0][1])))) {
        { res_.value = false; return res_; }
      }
      const int l_pres433 = ((0 < prm.clients) && (2 < (int)s.cw(first_client(prm) + 0)->results.size()));
      if ((l_pres433 && (prm.op[0][2] != 2))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_res434 = (l_pres433 ? std::stoi(s.cw(first_client(prm) + 0)->results[2].f[0]) : 0);
      const int l_rlen435 = (l_res434 & 7);
      if ((l_pres433 && (((l_rlen435 == 0) || (l_rlen435 > 4)) || (((l_res434 >> (1 + (l_rlen435 * 2))) & 3) != prm.val[0][2])))) {
        { res_.value = false; return res_; }
      }
      const int l_pres436 = ((1 < prm.clients) && (0 < (int)s.cw(first_client(prm) + 1)->results.size()));
      if ((l_pres436 && (prm.op[1][0] != 2))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_res437 = (l_pres436 ? std::stoi(s.cw(first_client(prm) + 1)->results[0].f[0]) : 0);
      const int l_rlen438 = (l_res437 & 7);
      if ((l_pres436 && (((l_rlen438 == 0) || (l_rlen438 > 4)) || (((l_res437 >> (1 + (l_rlen438 * 2))) & 3) != prm.val[1][0])))) {
        { res_.value = false; return res_; }
      }
      const int l_pres439 = ((1 < prm.clients) && (1 < (int)s.cw(first_client(prm) + 1)->results.size()));
      if ((l_pres439 && (prm.op[1][1] != 2))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_res440 = (l_pres439 ? std::stoi(s.cw(first_client(prm) + 1)->results[1].f[0]) : 0);
      const int l_rlen441 = (l_res440 & 7);
      if ((l_pres439 && (((l_rlen441 == 0) || (l_rlen441 > 4)) || (((l_res440 >> (1 + (l_rlen441 * 2))) & 3) != prm.val[1][1])))) {
        { res_.value = false; return res_; }
      }
      const int l_pres442 = ((1 < prm.clients) && (2 < (int)s.cw(first_client(prm) + 1)->results.size()));
      if ((l_pres442 && (prm.op[1][2] != 2))) {
        throw std::runtime_error("predicate threw");
      }
      const int l_res443 = (l_pres442 ? std::stoi(s.cw(first_client(prm) + 1)->results[2].f[0]) : 0);
      const int l_rlen444 = (l_res443 & 7);
      if ((l_pres442 && (((l_rlen444 == 0) || (l_rlen444 > 4)) || (((l_res443 >> (1 + (l_rlen444 * 2))) & 3) != prm.val[1][2])))) {
        { res_.value = false; return res_; }
      }
      if ((l_pres427 && l_pres430)) {
        if ((l_rlen429 == l_rlen432)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res428 >> 3) & ((1 << (((l_rlen429 < l_rlen432) ? l_rlen429 : l_rlen432) * 2)) - 1)) != ((l_res431 >> 3) & ((1 << (((l_rlen429 < l_rlen432) ? l_rlen429 : l_rlen432) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres427 && l_pres433)) {
        if ((l_rlen429 == l_rlen435)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res428 >> 3) & ((1 << (((l_rlen429 < l_rlen435) ? l_rlen429 : l_rlen435) * 2)) - 1)) != ((l_res434 >> 3) & ((1 << (((l_rlen429 < l_rlen435) ? l_rlen429 : l_rlen435) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres427 && l_pres436)) {
        if ((l_rlen429 == l_rlen438)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res428 >> 3) & ((1 << (((l_rlen429 < l_rlen438) ? l_rlen429 : l_rlen438) * 2)) - 1)) != ((l_res437 >> 3) & ((1 << (((l_rlen429 < l_rlen438) ? l_rlen429 : l_rlen438) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres427 && l_pres439)) {
        if ((l_rlen429 == l_rlen441)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res428 >> 3) & ((1 << (((l_rlen429 < l_rlen441) ? l_rlen429 : l_rlen441) * 2)) - 1)) != ((l_res440 >> 3) & ((1 << (((l_rlen429 < l_rlen441) ? l_rlen429 : l_rlen441) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres427 && l_pres442)) {
        if ((l_rlen429 == l_rlen444)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res428 >> 3) & ((1 << (((l_rlen429 < l_rlen444) ? l_rlen429 : l_rlen444) * 2)) - 1)) != ((l_res443 >> 3) & ((1 << (((l_rlen429 < l_rlen444) ? l_rlen429 : l_rlen444) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres430 && l_pres433)) {
        if ((l_rlen432 == l_rlen435)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res431 >> 3) & ((1 << (((l_rlen432 < l_rlen435) ? l_rlen432 : l_rlen435) * 2)) - 1)) != ((l_res434 >> 3) & ((1 << (((l_rlen432 < l_rlen435) ? l_rlen432 : l_rlen435) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres430 && l_pres436)) {
        if ((l_rlen432 == l_rlen438)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res431 >> 3) & ((1 << (((l_rlen432 < l_rlen438) ? l_rlen432 : l_rlen438) * 2)) - 1)) != ((l_res437 >> 3) & ((1 << (((l_rlen432 < l_rlen438) ? l_rlen432 : l_rlen438) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres430 && l_pres439)) {
        if ((l_rlen432 == l_rlen441)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res431 >> 3) & ((1 << (((l_rlen432 < l_rlen441) ? l_rlen432 : l_rlen441) * 2)) - 1)) != ((l_res440 >> 3) & ((1 << (((l_rlen432 < l_rlen441) ? l_rlen432 : l_rlen441) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres430 && l_pres442)) {
        if ((l_rlen432 == l_rlen444)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res431 >> 3) & ((1 << (((l_rlen432 < l_rlen444) ? l_rlen432 : l_rlen444) * 2)) - 1)) != ((l_res443 >> 3) & ((1 << (((l_rlen432 < l_rlen444) ? l_rlen432 : l_rlen444) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres433 && l_pres436)) {
        if ((l_rlen435 == l_rlen438)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res434 >> 3) & ((1 << (((l_rlen435 < l_rlen438) ? l_rlen435 : l_rlen438) * 2)) - 1)) != ((l_res437 >> 3) & ((1 << (((l_rlen435 < l_rlen438) ? l_rlen435 : l_rlen438) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres433 && l_pres439)) {
        if ((l_rlen435 == l_rlen441)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res434 >> 3) & ((1 << (((l_rlen435 < l_rlen441) ? l_rlen435 : l_rlen441) * 2)) - 1)) != ((l_res440 >> 3) & ((1 << (((l_rlen435 < l_rlen441) ? l_rlen435 : l_rlen441) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres433 && l_pres442)) {
        if ((l_rlen435 == l_rlen444)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res434 >> 3) & ((1 << (((l_rlen435 < l_rlen444) ? l_rlen435 : l_rlen444) * 2)) - 1)) != ((l_res443 >> 3) & ((1 << (((l_rlen435 < l_rlen444) ? l_rlen435 : l_rlen444) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres436 && l_pres439)) {
        if ((l_rlen438 == l_rlen441)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res437 >> 3) & ((1 << (((l_rlen438 < l_rlen441) ? l_rlen438 : l_rlen441) * 2)) - 1)) != ((l_res440 >> 3) & ((1 << (((l_rlen438 < l_rlen441) ? l_rlen438 : l_rlen441) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres436 && l_pres442)) {
        if ((l_rlen438 == l_rlen444)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res437 >> 3) & ((1 << (((l_rlen438 < l_rlen444) ? l_rlen438 : l_rlen444) * 2)) - 1)) != ((l_res443 >> 3) & ((1 << (((l_rlen438 < l_rlen444) ? l_rlen438 : l_rlen444) * 2)) - 1)))) {
          { res_.value = false; return res_; }
        }
      }
      if ((l_pres439 && l_pres442)) {
        if ((l_rlen441 == l_rlen444)) {
          { res_.value = false; return res_; }
        }
        if ((((l_res440 >> 3) & ((1 << (((l_rlen441 < l_rlen444) ? l_rlen441 : l_rlen444) * 2)) - 1)) != ((l_res443 >> 3) & ((1 << (((l_rlen441 < l_rlen444) ? l_rlen441 : l_rlen444) * 2)) - 1)))) {
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
