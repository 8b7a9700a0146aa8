// compile.hpp — host-side lowering of descriptor expression trees to device bytecode (expr.hpp).
#pragma once
#include <cstring>
#include <functional>
#include <string>

#include "expr.hpp"
#include "json.hpp"

namespace sg {

using sgjson::J;

inline Ty ty_of(const std::string& s) {
  if (s == "STRING") return T_STRING;
  if (s == "INT") return T_INT;
  if (s == "LONG") return T_LONG;
  if (s == "FLOAT") return T_FLOAT;
  if (s == "DOUBLE") return T_DOUBLE;
  if (s == "BOOL") return T_BOOL;
  return T_OBJECT;
}

struct CompileError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// slot_map(slot, chain) -> loader slot id, or -1 if the reference always resolves to null
// (e.g. `e2[1]` of a single-event state).  strings(s) -> dictionary id.
struct Compiler {
  Prog& p;
  std::function<int(int, int)> slot_map;
  std::function<int(const std::string&)> intern;
  // optional: lowers a leaf (var / agg) to a loader (slot, attr) instead (host selector programs)
  std::function<bool(const J&, int&, int&)> leaf = nullptr;

  // registers are a stack: a node's result takes the lowest register of its subtree, the
  // interpreter reads every operand before it writes the destination (expr.hpp run)
  int sp = 0;
  int reg() {
    if (sp >= MAX_REG) throw CompileError("expression needs more than 16 registers");
    const int r = sp++;
    if (sp > p.nreg) p.nreg = sp;
    return r;
  }
  void emit(uint8_t op, int dst, int a, int b, int32_t imm) {
    if (p.n >= MAX_INS) throw CompileError("expression longer than 48 instructions");
    p.ins[p.n++] = Ins{op, (uint8_t)dst, (uint8_t)a, (uint8_t)b, imm};
  }
  int cconst(int64_t v) {
    for (int i = 0; i < MAX_CONST; i++) {
      if (i >= nconst) break;
      if (p.consts[i] == v) return i;
    }
    if (nconst >= MAX_CONST) throw CompileError("too many constants");
    p.consts[nconst] = v;
    return nconst++;
  }
  int nconst = 0;

  int convert(int r, Ty from, Ty to) {
    if (from == to) return r;
    int d = reg();
    emit(BC_CVT, d, r, 0, (from << 4) | to);
    return d;
  }

  // returns register holding the value; *t = its type
  int node(const J& e, Ty* t) {
    const int base = sp;
    const std::string& op = e["op"].s;
    Ty et = ty_of(e["t"].s);
    *t = et;
    int lslot, lattr;
    if (leaf && leaf(e, lslot, lattr)) {
      int d = reg();
      emit(BC_LD, d, lslot, 0, lattr);
      return d;
    }
    if (op == "const") {
      int d = reg();
      const J& v = e["v"];
      int64_t raw = 0;
      bool isnull = false;
      switch (et) {
        case T_INT: raw = (int32_t)v.as_int(); break;
        case T_LONG: raw = v.as_int(); break;
        case T_FLOAT: raw = f_bits((float)v.n); break;
        case T_DOUBLE: raw = d_bits(v.n); break;
        case T_BOOL: raw = v.b ? 1 : 0; break;
        case T_STRING: raw = intern(v.s); break;
        default: isnull = true;
      }
      emit(BC_CONST, d, 0, isnull ? 1 : 0, cconst(raw));
      return d;
    }
    if (op == "var") {
      int d = reg();
      int s = slot_map((int)e["slot"].as_int(), (int)e["chain"].as_int());
      if (s < 0) emit(BC_NULL, d, 0, 0, 0);
      else emit(BC_LD, d, s, 0, (int32_t)e["attr"].as_int());
      return d;
    }
    if (op == "outvar") {             // an output attribute (having / order by): host loader slot 255
      int d = reg();
      emit(BC_LD, d, 255, 0, (int32_t)e["attr"].as_int());
      return d;
    }
    if (op == "and" || op == "or") {
      Ty ta, tb;
      int a = node(e["a"], &ta), b = node(e["b"], &tb);
      sp = base;
      int d = reg();
      emit(op == "and" ? BC_AND : BC_OR, d, a, b, 0);
      return d;
    }
    if (op == "not" || op == "isnull") {
      Ty ta;
      int a = node(e["a"], &ta);
      sp = base;
      int d = reg();
      emit(op == "not" ? BC_NOT : BC_ISNULL, d, a, 0, 0);
      return d;
    }
    static const char* cmps[] = {">", "<", ">=", "<=", "==", "!="};
    for (int c = 0; c < 6; c++) {
      if (op == cmps[c]) {
        Ty ct = ty_of(e["ct"].s);
        if (ct == T_OBJECT) throw CompileError("compare on OBJECT type");
        Ty ta, tb;
        int a = node(e["a"], &ta), b = node(e["b"], &tb);
        if (ct != T_STRING && ct != T_BOOL) { a = convert(a, ta, ct); b = convert(b, tb, ct); }
        sp = base;
        int d = reg();
        emit(BC_CMP, d, a, b, (c << 4) | ct);
        return d;
      }
    }
    static const char* maths[] = {"+", "-", "*", "/", "%"};
    for (int m = 0; m < 5; m++) {
      if (op == maths[m]) {
        Ty ta, tb;
        int a = node(e["a"], &ta), b = node(e["b"], &tb);
        a = convert(a, ta, et); b = convert(b, tb, et);
        sp = base;
        int d = reg();
        emit(BC_MATH, d, a, b, (m << 4) | et);
        return d;
      }
    }
    throw CompileError("expression op '" + op + "' has no device lowering");
  }

  void compile(const J& e) {
    Ty t;
    int r = node(e, &t);
    emit(BC_RET, 0, r, 0, 0);
  }
};

// Compile a conjunction of filters (FilterProcessor chain) into one predicate program.
inline void compile_filters(Prog& p, const J& filters, std::function<int(int, int)> sm,
                            std::function<int(const std::string&)> intern) {
  p = Prog();
  if (filters.size() == 0) return;
  Compiler c{p, sm, intern};
  if (filters.size() == 1) { c.compile(filters[0]); return; }
  Ty t;
  int acc = c.node(filters[0], &t);
  for (size_t i = 1; i < filters.size(); i++) {
    int r = c.node(filters[i], &t);
    c.sp = acc;   // acc is register 0 and stays below r: AND(acc, r) -> acc
    int d = c.reg();
    c.emit(BC_AND, d, acc, r, 0);
    acc = d;
  }
  c.emit(BC_RET, 0, acc, 0, 0);
}

inline void compile_expr(Prog& p, const J& e, std::function<int(int, int)> sm,
                         std::function<int(const std::string&)> intern) {
  p = Prog();
  Compiler c{p, sm, intern};
  c.compile(e);
}

}  // namespace sg
