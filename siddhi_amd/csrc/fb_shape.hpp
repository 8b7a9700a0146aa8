// fb_shape.hpp — shape recognition shared by the followed-by paths (plain and keyed).
//
// The atom fast path covers `every e1=S[f1] -> e2=S[f2]` with f2 = `e2.x OP e1.y` (one compare of one
// type, either operand order), f1 absent or one `e1.c OP const` atom, and a select list of plain
// e1/e2 attributes.  Everything else runs through the bytecode interpreter.
#pragma once
#include <vector>

#include "runtime.hpp"

namespace sg {

constexpr int FB_MAXP = 8;

template <int OP, class V>
__device__ __forceinline__ bool cmpv(V x, V y) {
  if constexpr (OP == C_GT) return x > y;
  else if constexpr (OP == C_LT) return x < y;
  else if constexpr (OP == C_GE) return x >= y;
  else if constexpr (OP == C_LE) return x <= y;
  else if constexpr (OP == C_EQ) return x == y;
  else return x != y;
}


struct FastPath {
  bool ok = false;
  int op = 0;          // f2: e2.x OP e1.y
  Ty t = T_FLOAT;
  int xcol = -1, ycol = -1;
  int f1kind = 0;      // 0 none, 1 atom, 2 generic (flags pre-pass: not built; falls back)
  int f1op = 0, f1col = -1;
  Ty f1t = T_INT;
  int64_t f1c = 0;
  bool plain_proj = false;
  std::vector<int> pslot, pcol;
};

inline bool is_own_var(const J& e, int slot) {
  return e["op"].s == "var" && e["slot"].as_int() == slot && (e["chain"].as_int() == -1 || e["chain"].as_int() == 0);
}

inline int flip(int op) {
  switch (op) { case C_GT: return C_LT; case C_LT: return C_GT; case C_GE: return C_LE; case C_LE: return C_GE; default: return op; }
}

inline int cmp_code(const std::string& s) {
  static const char* c[] = {">", "<", ">=", "<=", "==", "!="};
  for (int k = 0; k < 6; k++) if (s == c[k]) return k;
  return -1;
}

inline FastPath recognise(App& app, int sA, int sB, const J& e1, const J& e2, const J& sel) {
  FastPath fp;
  if (sA != sB) return fp;
  const auto& types = app.streams[sA].types;
  // f2: exactly one filter, `e2.x OP e1.y` (either order) of one type, no conversion
  if (e2["filters"].size() != 1) return fp;
  const J& f = e2["filters"][0];
  int op = cmp_code(f["op"].s);
  if (op < 0) return fp;
  const J *l = &f["a"], *r = &f["b"];
  if (is_own_var(*l, 0) && is_own_var(*r, 1)) { std::swap(l, r); op = flip(op); }
  if (!is_own_var(*l, 1) || !is_own_var(*r, 0)) return fp;
  Ty ct = ty_of(f["ct"].s);
  int xc = (int)(*l)["attr"].as_int(), yc = (int)(*r)["attr"].as_int();
  if (types[xc] != ct || types[yc] != ct) return fp;
  if (ct == T_STRING || ct == T_BOOL) { if (op != C_EQ && op != C_NE) return fp; ct = T_INT; }
  fp.op = op; fp.t = ct; fp.xcol = xc; fp.ycol = yc;
  // f1: none, or one `e1.c OP const` atom (constant folded to the compare type)
  if (e1["filters"].size() == 0) fp.f1kind = 0;
  else if (e1["filters"].size() == 1) {
    const J& g = e1["filters"][0];
    int op1 = cmp_code(g["op"].s);
    const J *gl = &g["a"], *gr = &g["b"];
    if (op1 >= 0 && gl->has("op") && (*gl)["op"].s == "const" && is_own_var(*gr, 0)) { std::swap(gl, gr); op1 = flip(op1); }
    if (op1 < 0 || !is_own_var(*gl, 0) || (*gr)["op"].s != "const") return fp;
    Ty ct1 = ty_of(g["ct"].s);
    int c1 = (int)(*gl)["attr"].as_int();
    if (types[c1] != ct1 || ct1 == T_OBJECT) return fp;
    Ty kt = ty_of((*gr)["t"].s);
    const J& v = (*gr)["v"];
    int64_t raw;
    switch (kt) {
      case T_INT: raw = (int32_t)v.as_int(); break;
      case T_LONG: raw = v.as_int(); break;
      case T_FLOAT: raw = f_bits((float)v.n); break;
      case T_DOUBLE: raw = d_bits(v.n); break;
      case T_STRING: raw = app.intern(v.s); break;
      case T_BOOL: raw = v.b ? 1 : 0; break;
      default: return fp;
    }
    if (ct1 != T_STRING && ct1 != T_BOOL) raw = cvt(raw, kt, ct1);
    fp.f1kind = 1; fp.f1op = op1; fp.f1t = ct1; fp.f1col = c1; fp.f1c = raw;
  } else {
    return fp;
  }
  // projection: plain variables of e1 / e2
  fp.plain_proj = true;
  for (size_t k = 0; k < sel["attrs"].size(); k++) {
    const J& e = sel["attrs"][k]["e"];
    if (!(is_own_var(e, 0) || is_own_var(e, 1)) || k >= (size_t)FB_MAXP) { fp.plain_proj = false; break; }
    fp.pslot.push_back((int)e["slot"].as_int());
    fp.pcol.push_back((int)e["attr"].as_int());
  }
  if (!fp.plain_proj) { fp.pslot.clear(); fp.pcol.clear(); }
  fp.ok = true;
  return fp;
}

}  // namespace sg
