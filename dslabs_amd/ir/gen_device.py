"""IR -> packed device protocol (a csrc/protocols/*.hpp struct with the interface nodestate.hpp
and the kernels use: layout constants, Params, record encoding, init / events / handlers,
ClientWorker loop, predicates, event descriptions). Every field access is a constant-offset
bit-field access (field_get / field_put); list elements use select chains, so nothing here is a
dynamically indexed private array."""
from __future__ import annotations

from typing import List

from .core import (Assign, Expr, ForS, IfS, LetS, SetFlagS, SetVarS, VarS, NodeKind, OverflowS, Protocol, RetPV, RetS, SendS,
                   SetAtS, SetTimerS, Stmt, ThrowS, lit, record, record_pred)


def _ind(n):
    return "  " * n


def _rec_expr(p: Protocol, s: SendS) -> str:
    parts = [f"((Rec){s.msg.index} << {p.type_off})", f"((Rec)(i) << {p.from_off})",
             f"((Rec)({s.to.dev}) << {p.to_off})"]
    for (n, b, off), v in zip(s.msg.offs, s.vals):
        parts.append(f"((Rec)(({v.dev}) & {(1 << b) - 1}) << {off})")
    return " | ".join(parts)


def _timer_entry(p: Protocol, t, vals: List[Expr]) -> str:
    parts, off = [], 0
    for (n, b), v in zip(t.fields, vals):
        parts.append(f"((({v.dev}) & {(1 << b) - 1}) << {off})")
        off += b
    fb = max([sum(b for _, b in x.fields) for x in p.timers] + [0])
    if len(p.timers) > 1:
        parts.append(f"({t.index} << {fb})")
    return " | ".join(parts) if parts else "0"


def lget(k: NodeKind, f, w: str, j: str) -> str:
    """Element j of a list / array field: a window read when it spans at most two words."""
    return f"arr_{k.name}_{f.name}({w}, {j})" if f.window_words() <= 2 else f"get({w}, {f.elem(j)}, {f.bits})"


def lput(k: NodeKind, f, w: str, j: str, v: str) -> str:
    return f"arr_put_{k.name}_{f.name}({w}, {j}, {v})" if f.window_words() <= 2 else f"put({w}, {f.elem(j)}, {f.bits}, {v})"


def _stmts(p: Protocol, k: NodeKind, ss: List[Stmt], d: int) -> List[str]:
    out = []
    for s in ss:
        if isinstance(s, Assign):
            out.append(f"{_ind(d)}put(w, {s.fld.off}, {s.fld.bits}, {s.value.dev});")
        elif isinstance(s, SendS):
            out.append(f"{_ind(d)}out.send({_rec_expr(p, s)});")
        elif isinstance(s, SetTimerS):
            if k.fixed_timer is s.timer:  # the queue stays [T] (Protocol.fixed_timer): nothing is stored
                out.append(f"{_ind(d)}// set {s.timer.name}: the queue stays [{s.timer.name}]")
            else:
                out.append(f"{_ind(d)}if (!push_timer_{k.name}(w, {_timer_entry(p, s.timer, s.vals)})) return STEP_OVERFLOW;")
        elif isinstance(s, ThrowS):
            out.append(f"{_ind(d)}return STEP_EXCEPTION;  // {s.what}")
        elif isinstance(s, VarS):
            out.append(f"{_ind(d)}int {s.name} = {s.value.dev};")
        elif isinstance(s, SetVarS):
            out.append(f"{_ind(d)}{s.name} = {s.value.dev};")
        elif isinstance(s, LetS):
            out.append(f"{_ind(d)}const int {s.name} = {s.value.dev};")
        elif isinstance(s, SetAtS):
            if s.fld.window_words() <= 2:
                out.append(f"{_ind(d)}arr_put_{k.name}_{s.fld.name}(w, {s.index.dev}, {s.value.dev});")
            else:
                out.append(f"{_ind(d)}put(w, {s.fld.elem(s.index.dev)}, {s.fld.bits}, {s.value.dev});")
        elif isinstance(s, RetS):
            out.append(f"{_ind(d)}return STEP_OK;")
        elif isinstance(s, OverflowS):
            out.append(f"{_ind(d)}return STEP_OVERFLOW;  // {s.what}")
        elif isinstance(s, RetPV):
            out.append(f"{_ind(d)}return PV_{s.value};")
        elif isinstance(s, SetFlagS):
            out.append(f"{_ind(d)}fl |= {1 << s.bit};")
        elif isinstance(s, ForS):
            out.append(f"{_ind(d)}#pragma unroll 1")
            out.append(f"{_ind(d)}for (int {s.var} = {s.lo.dev}; {s.var} < {s.hi.dev}; {s.var}++) {{")
            out += _stmts(p, k, s.body, d + 1)
            out.append(f"{_ind(d)}}}")
        elif isinstance(s, IfS):
            out.append(f"{_ind(d)}if ({s.cond.dev}) {{")
            out += _stmts(p, k, s.then, d + 1)
            if s.other:
                out.append(f"{_ind(d)}}} else {{")
                out += _stmts(p, k, s.other, d + 1)
            out.append(f"{_ind(d)}}}")
    return out


def generate(p: Protocol, source: str) -> str:
    p.layout()
    N = p.cxx_name
    rec_t = "uint32_t" if p.rec_bits == 32 else "uint64_t"
    L = []
    a = L.append
    a(f"// {N} -- GENERATED from the protocol IR ({source}) by dslabs_amd/ir/gen_device.py; do not edit.")
    for line in p.doc.strip().splitlines():
        a(f"// {line}")
    a("#pragma once")
    a('#include "../../nodestate.hpp"')
    a("")
    a("namespace dsl {")
    a("")
    a(f"struct {N} {{")
    a(f"  static constexpr int kNodes = {p.max_nodes}, kNodeWords = {p.node_words}, kNetCap = {p.net_cap}, "
      f"kMaxSends = {p.max_sends};")
    if p.sends_distinct:
        a("  static constexpr bool kSendsDistinct = true;  // checked by tests/hostcheck (dup_sends)")
    if p.net_preds():
        a("  static constexpr bool kNetPreds = true;  // a predicate reads the network (view_any_record)")
    a(f"  using Self = {N};")
    a(f"  static constexpr int kMsgClasses = {len(p.messages)};")
    a(f"  using Rec = {rec_t};")
    a(f"  using State = StateOf<{N}>;")
    a("  struct Params {")
    for q in p.params:
        a(f"    int32_t {q.name};")
    for t in p.tables:
        a(f"    int32_t {t.name}[{t.rows}][{t.cols}];")
    for t in p.tables:
        if t.packed_bits():
            a(f"    uint64_t {t.name}_pk;  // {t.name}[r][c] at bit {t.packed_bits()} * (r * {t.cols} + c) (from_desc)")
    a("  };")
    a("  static DSL_HD int get(const uint32_t* w, int bit, int width) { return field_get<kNodeWords>(w, bit, width); }")
    a("  static DSL_HD void put(uint32_t* w, int bit, int width, int v) { field_put<kNodeWords>(w, bit, width, v); }")
    # array fields within one or two words: a 32- / 64-bit window and shifts (no select chain)
    for k in p.kinds:
        for f in k.fields:
            if not (f.cap and f.window_words() <= 2):
                continue
            w0 = f.off // 32
            win = f"(uint64_t)w[{w0}]" + (f" | ((uint64_t)w[{w0 + 1}] << 32)" if f.window_words() == 2 else "")
            m = (1 << f.bits) - 1
            a(f"  static DSL_HD int arr_{k.name}_{f.name}(const uint32_t* w, int j) {{")
            a(f"    return (int)((({win}) >> ({f.off % 32} + {f.elem_rel('j')})) & {m}u);")
            a("  }")
            a(f"  static DSL_HD void arr_put_{k.name}_{f.name}(uint32_t* w, int j, int v) {{")
            a(f"    const int sh = {f.off % 32} + {f.elem_rel('j')};")
            a(f"    const uint64_t x = (({win}) & ~((uint64_t){m}u << sh)) | ((uint64_t)((uint32_t)v & {m}u) << sh);")
            a(f"    w[{w0}] = (uint32_t)x;")
            if f.window_words() == 2:
                a(f"    w[{w0 + 1}] = (uint32_t)(x >> 32);")
            a("  }")
    am = (1 << p.addr_bits) - 1
    a(f"  static DSL_HD int rec_type(Rec r) {{ return (int)(r >> {p.type_off}); }}")
    a(f"  static DSL_HD int rec_from(Rec r) {{ return (int)((r >> {p.from_off}) & {am}); }}")
    a(f"  static DSL_HD int rec_to(Rec r) {{ return (int)((r >> {p.to_off}) & {am}); }}")
    a("  static DSL_HD int msg_class(Rec r) { return rec_type(r); }")
    # node kinds
    a("  // node index -> kind: kinds are laid out in declaration order, instances consecutive")
    cnt = lambda k: str(k.count) if isinstance(k.count, int) else f"p.{k.count}"
    a("  static DSL_HD int num_nodes(const Params& p) { return " + " + ".join(cnt(k) for k in p.kinds) + "; }")
    for ki, k in enumerate(p.kinds):
        first = " + ".join(["0"] + [cnt(x) for x in p.kinds[:ki]])
        a(f"  static DSL_HD int first_{k.name}(const Params& p) {{ (void)p; return {first}; }}")
        a(f"  static DSL_HD bool is_{k.name}(int i, const Params& p) {{ return i >= first_{k.name}(p) && "
          f"i < first_{k.name}(p) + {cnt(k)}; }}")
    # commands per client (ClientWorker's workload size), c = client index from 0
    from .core import Handler
    if callable(p.workload_size):
        ws = lit(p.workload_size(Handler(p, p.kinds[0]), Expr("c", "c"))).dev
    else:
        ws = f"p.{p.workload_size}" if p.workload_size else "0"
    a(f"  static DSL_HD int wsize(int c, const Params& p) {{ (void)c; (void)p; return {ws}; }}")
    # timer queues
    fb = max([sum(b for _, b in t.fields) for t in p.timers] + [0])
    a("  // timer entries: fields from bit 0 in declaration order, the type above them")
    a("  static DSL_HD void tbounds(int type, int& mn, int& mx) {")
    for t in p.timers:
        a(f"    if (type == {t.index}) {{ mn = {t.millis[0]}; mx = {t.millis[1]}; }}")
    a("  }")
    a(f"  static DSL_HD int ttype(int e) {{ return {'e >> ' + str(fb) if len(p.timers) > 1 else '0'}; }}")
    for k in p.kinds:
        if not k.timer_cap or k.fixed_timer is not None:
            continue
        tf = next(f for f in k.fields if f.name == "_timers")
        a(f"  static DSL_HD bool push_timer_{k.name}(uint32_t* w, int e) {{")
        a(f"    const int n = get(w, {tf.len_off}, {tf.len_bits});")
        a(f"    if (n >= {tf.cap}) return false;")
        a(f"    {lput(k, tf, 'w', 'n', 'e')};")
        a(f"    put(w, {tf.len_off}, {tf.len_bits}, n + 1);")
        a("    return true;")
        a("  }")
        # deliverable entries (TimerQueue.deliverable): yield in order; skip min >= min(max yielded)
        a(f"  // TimerQueue.deliverable(): the index of deliverable entry j (-1: none), or their count (j < 0)")
        a(f"  static DSL_HD int deliverable_{k.name}(const uint32_t* w, int j) {{")
        a(f"    const int n = get(w, {tf.len_off}, {tf.len_bits});")
        if all(t.millis[0] == t.millis[1] == p.timers[0].millis[0] for t in p.timers):
            # every timer has the same fixed duration (min == max == d): an entry after the head has
            # min d >= the head's max d, so only the head is ever deliverable -- constant time
            a("    return j < 0 ? (n > 0 ? 1 : 0) : (j == 0 && n > 0 ? 0 : -1);  // only the head (equal fixed durations)")
            a("  }")
            a(f"  static DSL_HD int deliverable_general_{k.name}(const uint32_t* w, int j) {{")
            a(f"    const int n = get(w, {tf.len_off}, {tf.len_bits});")
        a("    int mm = 0x7fffffff, c = 0;")
        a(f"    for (int q = 0; q < n; q++) {{")
        a(f"      int mn = 0, mx = 0;")
        a(f"      tbounds(ttype({lget(k, tf, 'w', 'q')}), mn, mx);")
        a("      if (q > 0 && mn >= mm) continue;")
        a("      if (c == j) return q;")
        a("      c++;")
        a("      if (mx < mm) mm = mx;")
        a("    }")
        a("    return j < 0 ? c : -1;")
        a("  }")
        a(f"  static DSL_HD void remove_timer_{k.name}(uint32_t* w, int e) {{  // the first equal entry")
        a(f"    const int n = get(w, {tf.len_off}, {tf.len_bits});")
        a("    int q0 = n;")
        a(f"    for (int q = n - 1; q >= 0; q--)")
        a(f"      if ({lget(k, tf, 'w', 'q')} == e) q0 = q;")
        a("    if (q0 >= n) return;")
        a(f"    for (int q = q0; q + 1 < n; q++) {lput(k, tf, 'w', 'q', lget(k, tf, 'w', 'q + 1'))};")
        a(f"    {lput(k, tf, 'w', 'n - 1', '0')};")
        a(f"    put(w, {tf.len_off}, {tf.len_bits}, n - 1);")
        a("  }")
    # client worker
    from .core import Expr as E
    for k in p.kinds:
        if not k.client:
            continue
        rf = next(f for f in k.fields if f.name == k.result_field)
        rl = next(f for f in k.fields if f.name == "_results")
        body = record(p, k, k.send_command_fn, cmd=E("cmd", "cmd"))
        a("  template <class O>")
        a(f"  static DSL_HD int send_command_{k.name}(int i, uint32_t* w, int cmd, O& out, const Params& p) {{")
        a("    (void)p;")
        L.extend(_stmts(p, k, body, 2))
        a("    return STEP_OK;")
        a("  }")
        a("  // ClientWorker.sendNextCommandWhilePossible (waitingOnResult == |results| < workload size)")
        a("  template <class O>")
        a(f"  static DSL_HD void client_worker_{k.name}(int i, uint32_t* w, O& out, const Params& p) {{")
        a(f"    int n = get(w, {rl.len_off}, {rl.len_bits});")
        a(f"    const int res = get(w, {rf.off}, {rf.bits});")
        a(f"    const int ws = wsize(i - first_{k.name}(p), p);")
        a(f"    if (n < ws && res != 0) {{")
        a(f"      if (n >= {rl.cap}) {{ out.overflow = true; return; }}")
        a(f"      {lput(k, rl, 'w', 'n', 'res')};")
        a("      n++;")
        a(f"      put(w, {rl.len_off}, {rl.len_bits}, n);")
        a(f"      if (n < ws && send_command_{k.name}(i, w, n + 1, out, p) != STEP_OK) out.overflow = true;")
        a("    }")
        a("  }")
    # init
    a("  template <class O>")
    a("  static DSL_HD void init_node(int i, uint32_t* w, O& out, const Params& p) {")
    for k in p.kinds:
        a(f"    if (is_{k.name}(i, p)) {{")
        if k.init_fn:
            a(f"      if (init_{k.name}(i, w, out, p) != STEP_OK) out.overflow = true;")
        if k.client:  # ClientWorker.init: the first command
            a(f"      if (wsize(i - first_{k.name}(p), p) > 0 && send_command_{k.name}(i, w, 1, out, p) != STEP_OK) out.overflow = true;")
        a("      return;")
        a("    }")
    a("  }")
    a("  static DSL_HD int num_timer_events(int i, const uint32_t* w, const Params& p) {")
    for k in p.kinds:
        if k.fixed_timer is not None:
            a(f"    if (is_{k.name}(i, p)) return 1;  // [{k.fixed_timer.name}] in every state")
        elif k.timer_cap:
            a(f"    if (is_{k.name}(i, p)) return deliverable_{k.name}(w, -1);")
    a("    (void)i; (void)w; (void)p;")
    a("    return 0;")
    a("  }")
    # handler bodies (one function each: an early return still reaches the ClientWorker loop)
    for k in p.kinds:
        if k.init_fn:
            a("  template <class O>")
            a(f"  static DSL_HD int init_{k.name}(int i, uint32_t* w, O& out, const Params& p) {{")
            a("    (void)i; (void)p; (void)out;")
            L.extend(_stmts(p, k, record(p, k, k.init_fn), 2))
            a("    return STEP_OK;")
            a("  }")
        for m in p.messages:
            fn = k.handlers.get(m.name)
            if fn is None:
                continue
            a("  template <class O>")
            a(f"  static DSL_HD int hm_{k.name}_{m.name}(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {{")
            a("    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;")
            L.extend(_stmts(p, k, record(p, k, fn, event=m), 2))
            a("    return STEP_OK;")
            a("  }")
        for t in p.timers:
            fn = k.timer_handlers.get(t.name)
            if fn is None:
                continue
            a("  template <class O>")
            a(f"  static DSL_HD int ht_{k.name}_{t.name}(int i, uint32_t* w, int e, O& out, const Params& p) {{")
            a("    (void)i; (void)w; (void)out; (void)p;")
            off = 0
            for n, b in t.fields:
                a(f"    const int tf_{n} = (e >> {off}) & {(1 << b) - 1};")
                off += b
            L.extend(_stmts(p, k, record(p, k, fn, event=t, is_timer=True), 2))
            a("    return STEP_OK;")
            a("  }")
        if k.tail_fn:
            a("  template <class O>")
            a(f"  static DSL_HD int tail_{k.name}(int i, uint32_t* w, int fl, O& out, const Params& p) {{")
            a("    (void)i; (void)w; (void)out; (void)p;")
            L.extend(_stmts(p, k, record(p, k, k.tail_fn), 2))
            a("    return STEP_OK;")
            a("  }")
  # message handlers
    a("  template <class O>")
    a("  static DSL_HD int on_message(int i, uint32_t* w, Rec r, O& out, const Params& p) {")
    a("    (void)w; (void)out;")
    for k in p.kinds:
        a(f"    if (is_{k.name}(i, p)) {{")
        a("      int fl = 0, rc;")
        first = True
        for m in p.messages:
            fn = k.handlers.get(m.name)
            if fn is None:
                continue
            a(f"      {'if' if first else 'else if'} (rec_type(r) == {m.index}) rc = hm_{k.name}_{m.name}(i, w, r, out, p, fl);  // {m.name}")
            first = False
        if first:
            a("      return STEP_EXCEPTION;  // no handler for any message")
        else:
            a("      else return STEP_EXCEPTION;  // no handler for this message (Node.handleMessage throws)")
            if k.tail_fn:
                a(f"      if (rc == STEP_OK && fl) rc = tail_{k.name}(i, w, fl, out, p);  // the handlers' common tail")
            if k.client:
                a(f"      if (rc == STEP_OK) client_worker_{k.name}(i, w, out, p);")
            a("      return rc;")
        a("    }")
    a("    return STEP_EXCEPTION;")
    a("  }")
    # timer handlers
    a("  template <class O>")
    a("  static DSL_HD int on_timer(int i, uint32_t* w, int j, O& out, const Params& p) {")
    a("    (void)w; (void)j; (void)out;")
    for k in p.kinds:
        if not k.timer_cap:
            continue
        if k.fixed_timer is not None:  # stepTimer's remove and the handler's re-set cancel out
            t = k.fixed_timer
            a(f"    if (is_{k.name}(i, p)) {{")
            a("      if (j != 0) return STEP_NULL;")
            a(f"      return ht_{k.name}_{t.name}(i, w, {_timer_entry(p, t, [])}, out, p);  // {t.name}")
            a("    }")
            continue
        tf = next(f for f in k.fields if f.name == "_timers")
        a(f"    if (is_{k.name}(i, p)) {{")
        a(f"      const int q = deliverable_{k.name}(w, j);")
        a("      if (q < 0) return STEP_NULL;")
        a(f"      const int e = {lget(k, tf, 'w', 'q')};")
        for t in p.timers:
            fn = k.timer_handlers.get(t.name)
            if fn is None:
                continue
            a(f"      if (ttype(e) == {t.index}) {{  // {t.name}")
            a(f"        const int rc = ht_{k.name}_{t.name}(i, w, e, out, p);")
            a("        if (rc != STEP_OK) return rc;")
            if k.client:
                a(f"        client_worker_{k.name}(i, w, out, p);")
            a(f"        remove_timer_{k.name}(w, e);  // SearchState.stepTimer: the first equal entry")
            a("        return STEP_OK;")
            a("      }")
        a("      return STEP_EXCEPTION;  // no handler for this timer")
        a("    }")
    a("    return STEP_EXCEPTION;")
    a("  }")
    # predicates (ClientWorker)
    ck = [k for k in p.kinds if k.client]
    a("  static DSL_HD int eval(const DevPred& pr, const NodeView& v, const Params& p) {")
    if ck:
        k = ck[0]
        rl = next(f for f in k.fields if f.name == "_results")
        exp = lit(p.expected_result(E("(c - c0)", "(c - c0)"), E("(j + 1)", "(j + 1)"))).dev
        fc, nc = f"first_{k.name}(p)", cnt(k)
        a(f"    const int c0 = {fc}, nc = {nc};")
        a("    switch (pr.id) {")
        a("      case DSL_PRED_RESULTS_OK:  // every result equals the workload's expected result")
        a("        for (int c = c0; c < c0 + nc; c++) {")
        a("          const uint32_t* w = v.node(c);")
        a(f"          const int n = get(w, {rl.len_off}, {rl.len_bits});")
        a(f"          for (int j = 0; j < n; j++) {{")
        a(f"            const int x = {exp};")
        a(f"            if (x >= 0 && {lget(k, rl, 'w', 'j')} != x) return PV_FALSE;")
        a("          }")
        a("        }")
        a("        return PV_TRUE;")
        a("      case DSL_PRED_CLIENTS_DONE:")
        a("        for (int c = c0; c < c0 + nc; c++)")
        a(f"          if (get(v.node(c), {rl.len_off}, {rl.len_bits}) < wsize(c - c0, p)) return PV_FALSE;")
        a("        return PV_TRUE;")
        a("      case DSL_PRED_CLIENT_DONE:")
        a("        if (pr.arg0 < c0 || pr.arg0 >= c0 + nc) return PV_THREW;")
        a(f"        return get(v.node((int)pr.arg0), {rl.len_off}, {rl.len_bits}) >= wsize((int)pr.arg0 - c0, p) ? PV_TRUE : PV_FALSE;")
        a("      case DSL_PRED_NONE_DECIDED:")
        a("        for (int c = c0; c < c0 + nc; c++)")
        a(f"          if (get(v.node(c), {rl.len_off}, {rl.len_bits}) > 0) return PV_FALSE;")
        a("        return PV_TRUE;")
        a("      case DSL_PRED_CLIENT_HAS_RESULTS:")
        a("        if (pr.arg0 < c0 || pr.arg0 >= c0 + nc) return PV_THREW;")
        a(f"        return get(v.node((int)pr.arg0), {rl.len_off}, {rl.len_bits}) == pr.arg1 ? PV_TRUE : PV_FALSE;")
        for pd in p.predicates:
            for pid in pd.ids:
                a(f"      case {pid}:  // {' / '.join(pd.names)}")
            a("      {")
            cached = []
            body = _stmts(p, k, record_pred(p, pd.fn, cached), 4)
            for kn, inst in cached:  # register copies of the constant instances' words (DCE keeps the used ones)
                a(f"        uint32_t pn_{kn}_{inst}[kNodeWords];")
                a(f"        {{ const uint32_t* q_ = v.node(first_{kn}(p) + {inst});  // < kNodes: in bounds for any run")
                a(f"          for (int w_ = 0; w_ < kNodeWords; w_++) pn_{kn}_{inst}[w_] = q_[w_]; }}")
            L.extend(body)
            a("        return PV_TRUE;")
            a("      }")
        a("      default:")
        a("        return PV_THREW;")
        a("    }")
    else:
        a("    (void)pr; (void)v; (void)p;")
        a("    return PV_THREW;")
    a("  }")
    a("  static uint32_t pred_reads(const DevPred& pr, const Params& p) {")
    a("    (void)pr; (void)p;")
    mask = lambda kk: f"(((1u << ({cnt(kk)})) - 1u) << first_{kk.name}(p))"
    for pd in p.predicates:
        m = " | ".join(mask(p.kind(n)) for n in pd.reads) or "kReadsAll"
        a("    if (" + " || ".join(f"pr.id == {pid}" for pid in pd.ids) + f") return {m};")
    if ck:
        k = ck[0]
        a(f"    const uint32_t clients = {mask(k)};")
        a("    return (pr.id >= DSL_PRED_RESULTS_OK && pr.id <= DSL_PRED_CLIENT_HAS_RESULTS) ? clients : kReadsAll;")
    else:
        a("    return kReadsAll;")
    a("  }")
    # incremental judge: a predicate keeps the parent's value when the words of the fields it reads
    # are equal in the old and new node (all of a node's words when it declares none)
    def bits_of(kk, names):
        """word -> mask of the bits the fields occupy (a list: its length and its elements)."""
        m = {}
        def add(bit, width):
            while width > 0:
                w, o = bit // 32, bit % 32
                n = min(width, 32 - o)
                m[w] = m.get(w, 0) | (((1 << n) - 1) << o)
                bit, width = bit + n, width - n
        for n in names:
            fd = next(f for f in kk.fields if f.name == n)
            if fd.cap:
                if not fd.array:
                    add(fd.len_off, fd.len_bits)
                for j in range(fd.cap):
                    add(fd.off + (j // fd.per) * 32 + (j % fd.per) * fd.bits, fd.bits)
            else:
                add(fd.off, fd.bits)
        return m

    def same_cond(m):
        parts = [f"(a[{w}] ^ b[{w}])" if mask == 0xffffffff else f"((a[{w}] ^ b[{w}]) & {mask:#x}u)"
                 for w, mask in sorted(m.items())]
        return " | ".join(parts) or "0u"
    if p.predicates or ck:
        # a predicate keeps the parent's value when the BITS of the fields it reads are unchanged
        a("  static DSL_HD bool pred_same(const DevPred& pr, const uint32_t* a, const uint32_t* b) {")
        for pd in p.predicates:
            m = {}
            for n, fl in pd.reads.items():
                for w, mask in bits_of(p.kind(n), fl).items():
                    m[w] = m.get(w, 0) | mask
            a("    if (" + " || ".join(f"pr.id == {pid}" for pid in pd.ids) + f") return ({same_cond(m)}) == 0;")
        if ck:
            k = ck[0]
            a(f"    if (pr.id >= DSL_PRED_RESULTS_OK && pr.id <= DSL_PRED_CLIENT_HAS_RESULTS) return ({same_cond(bits_of(k, ['_results']))}) == 0;")
        a("    return same_words<kNodeWords>(a, b);")
        a("  }")
    ids = [pid for pd in p.predicates for pid in pd.ids]
    extra = "".join(f" || id == {pid}" for pid in ids)
    a(f"  static bool known_predicate(int id) {{ return (id >= DSL_PRED_RESULTS_OK && id <= DSL_PRED_CLIENT_HAS_RESULTS){extra}; }}")
    # no-op filter (nodestate.hpp NoopFilter), branch-free: every declared case evaluated, selected by kind and type
    if any(k.noop_fns for k in p.kinds):
        a("  static DSL_HD bool surely_noop(int i, const uint32_t* row, Rec r, const Params& p) {")
        a(f"    const uint32_t* w = row + i * kNodeWords;")
        a("    bool x = false;")
        for k in p.kinds:
            if not k.noop_fns:
                continue
            for m in p.messages:
                fn = k.noop_fns.get(m.name)
                if fn is None:
                    continue
                from .core import Handler as H
                h = H(p, k, m)
                e = lit(fn(h))
                assert not h.stmts, "a no-op filter is one expression (no statements)"
                a(f"    x = (is_{k.name}(i, p) && rec_type(r) == {m.index}) ? (bool)({e.dev}) : x;  // {k.name} <- {m.name}")
        a("    return x;")
        a("  }")
    a("  static bool valid(const Params& p) {")
    conds = [f"p.{q.name} >= {q.lo} && p.{q.name} <= {q.hi}" for q in p.params]
    for k in p.kinds:
        if not isinstance(k.count, int):
            conds.append(f"p.{k.count} >= 1 && p.{k.count} <= {k.max_count}")
    for t in p.tables:
        a(f"    for (int r = 0; r < {t.rows}; r++)")
        a(f"      for (int c = 0; c < {t.cols}; c++)")
        a(f"        if (p.{t.name}[r][c] < {t.lo} || p.{t.name}[r][c] > {t.hi}) return false;")
    a("    return " + (" &&\n           ".join(conds) if conds else "true") + ";")
    a("  }")
    a("  static Params from_desc(const dsl_protocol_desc& d) {")
    a("    Params p{};")
    for qi, q in enumerate(p.params):
        a(f"    p.{q.name} = d.n_params > {qi} ? (int32_t)d.params[{qi}] : {q.default};")
    base = len(p.params)
    for t in p.tables:
        a(f"    for (int r = 0; r < {t.rows}; r++)")
        a(f"      for (int c = 0; c < {t.cols}; c++) {{")
        a(f"        const int q = {base} + r * {t.cols} + c;")
        a(f"        p.{t.name}[r][c] = d.n_params > q ? (int32_t)d.params[q] : {t.default};")
        a("      }")
        base += t.rows * t.cols
    for t in p.tables:
        b = t.packed_bits()
        if b:
            a(f"    for (int r = 0; r < {t.rows}; r++)")
            a(f"      for (int c = 0; c < {t.cols}; c++)")
            a(f"        p.{t.name}_pk |= (uint64_t)((uint32_t)p.{t.name}[r][c] & {(1 << b) - 1}u) << ({b} * (r * {t.cols} + c));")
    a("    return p;")
    a("  }")
    # descriptions
    a("  static void describe_message(Rec r, dsl_event* e) {")
    a("    e->from = rec_from(r);")
    a("    e->to = rec_to(r);")
    a("    e->type = rec_type(r);")
    a("    e->n_fields = 0;")
    for m in p.messages:
        a(f"    if (e->type == {m.index}) {{")
        a(f"      e->n_fields = {len(m.fields)};")
        for fi, (n, b, off) in enumerate(m.offs):
            a(f"      e->fields[{fi}] = (int64_t)((r >> {off}) & {(1 << b) - 1}u);")
        a("    }")
    a("  }")
    a("  static void describe_timer(int i, const uint32_t* w, int j, const Params& p, dsl_event* e) {")
    a("    e->is_timer = 1;")
    a("    e->from = e->to = i;")
    a("    (void)w; (void)j; (void)p;")
    for k in p.kinds:
        if not k.timer_cap:
            continue
        a(f"    if (is_{k.name}(i, p)) {{")
        if k.fixed_timer is not None:
            a("      if (j != 0) return;")
            a(f"      const int x = {_timer_entry(p, k.fixed_timer, [])};")
        else:
            tf = next(f for f in k.fields if f.name == "_timers")
            a(f"      const int q = deliverable_{k.name}(w, j);")
            a("      if (q < 0) return;")
            a(f"      const int x = {lget(k, tf, 'w', 'q')};")
        a(f"      e->type = {len(p.messages)} + ttype(x);")
        a("      int mn = 0, mx = 0;")
        a("      tbounds(ttype(x), mn, mx);")
        a("      e->timer_min = mn;")
        a("      e->timer_max = mx;")
        for t in p.timers:
            a(f"      if (ttype(x) == {t.index}) {{")
            a(f"        e->n_fields = {len(t.fields)};")
            off = 0
            for fi, (n, b) in enumerate(t.fields):
                a(f"        e->fields[{fi}] = (x >> {off}) & {(1 << b) - 1};")
                off += b
            a("      }")
        a("    }")
    a("  }")
    a("};")
    a("")
    a("}  // namespace dsl")
    return "\n".join(L) + "\n"
