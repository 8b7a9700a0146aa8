// expr.hpp — predicate / projection bytecode for the gfx950 kernels.
//
// Siddhi evaluates filters and selectors through a tree of boxed ExpressionExecutors
// (CORE/executor/condition/compare/**, CORE/executor/math/**, VariableExpressionExecutor).  On the
// device the same tree is lowered once on the host to a short register bytecode.  The program is
// identical for every lane, so the interpreter's dispatch is wave-uniform (scalar branches, no
// divergence); only operand values differ per lane.  Java semantics are fixed at compile time:
//   * binary numeric promotion (JLS §5.6.2) becomes explicit CVT ops, so each CMP/MATH op is typed;
//   * a null operand makes a compare FALSE (CompareConditionExpressionExecutor.execute :38-41);
//   * int/long arithmetic wraps, x/0 and x%0 yield null (DivideExpressionExecutorInt etc.);
//   * AND/OR treat null as false (AndConditionExpressionExecutor / OrConditionExpressionExecutor).
// Values live in 64-bit registers as raw bits: int32 sign-extended, float32 bits, float64 bits,
// bool 0/1, string dictionary id.
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#define SG_HD
#else
#define SG_HD __host__ __device__
#endif

namespace sg {

enum Ty : uint8_t { T_STRING = 0, T_INT = 1, T_LONG = 2, T_FLOAT = 3, T_DOUBLE = 4, T_BOOL = 5, T_OBJECT = 6 };

enum BcOp : uint8_t {
  BC_LD,       // dst <- attr `imm` of slot `a` (chain index resolved at compile time)
  BC_CONST,    // dst <- consts[imm]; b = 1 -> null constant
  BC_NULL,     // dst <- null
  BC_CVT,      // dst <- convert(a) ; imm = (from << 4) | to
  BC_CMP,      // dst <- a OP b ; imm = (op << 4) | type
  BC_MATH,     // dst <- a OP b ; imm = (op << 4) | type
  BC_AND,      // dst <- a && b (null -> false)
  BC_OR,       // dst <- a || b
  BC_NOT,      // dst <- !a (null -> true, Siddhi NotConditionExpressionExecutor)
  BC_ISNULL,   // dst <- a == null
  BC_RET,      // result <- a
};

enum CmpOp : uint8_t { C_GT = 0, C_LT, C_GE, C_LE, C_EQ, C_NE };
enum MathOp : uint8_t { M_ADD = 0, M_SUB, M_MUL, M_DIV, M_MOD };

struct Ins {
  uint8_t op, dst, a, b;
  int32_t imm;
};

constexpr int MAX_INS = 48;
constexpr int MAX_CONST = 16;
constexpr int MAX_REG = 16;

struct Prog {
  int32_t n = 0;
  int32_t nreg = 0;
  Ins ins[MAX_INS];
  int64_t consts[MAX_CONST];
};

SG_HD inline float bits_f(int64_t r) { union { uint32_t u; float f; } x; x.u = (uint32_t)r; return x.f; }
SG_HD inline double bits_d(int64_t r) { union { int64_t i; double d; } x; x.i = r; return x.d; }
SG_HD inline int64_t f_bits(float f) { union { uint32_t u; float f; } x; x.f = f; return (int64_t)x.u; }
SG_HD inline int64_t d_bits(double d) { union { int64_t i; double d; } x; x.d = d; return x.i; }

SG_HD inline int64_t cvt(int64_t v, int from, int to) {
  switch (from) {
    case T_INT:
      if (to == T_LONG) return (int64_t)(int32_t)v;
      if (to == T_FLOAT) return f_bits((float)(int32_t)v);
      if (to == T_DOUBLE) return d_bits((double)(int32_t)v);
      return v;
    case T_LONG:
      if (to == T_FLOAT) return f_bits((float)v);
      if (to == T_DOUBLE) return d_bits((double)v);
      return v;
    case T_FLOAT:
      if (to == T_DOUBLE) return d_bits((double)bits_f(v));
      return v;
    default:
      return v;
  }
}

SG_HD inline bool cmp(int op, int t, int64_t a, int64_t b) {
  switch (t) {
    case T_INT: case T_STRING: case T_BOOL: {
      int32_t x = (int32_t)a, y = (int32_t)b;
      switch (op) { case C_GT: return x > y; case C_LT: return x < y; case C_GE: return x >= y;
                    case C_LE: return x <= y; case C_EQ: return x == y; default: return x != y; }
    }
    case T_LONG: {
      switch (op) { case C_GT: return a > b; case C_LT: return a < b; case C_GE: return a >= b;
                    case C_LE: return a <= b; case C_EQ: return a == b; default: return a != b; }
    }
    case T_FLOAT: {
      float x = bits_f(a), y = bits_f(b);
      switch (op) { case C_GT: return x > y; case C_LT: return x < y; case C_GE: return x >= y;
                    case C_LE: return x <= y; case C_EQ: return x == y; default: return x != y; }
    }
    default: {
      double x = bits_d(a), y = bits_d(b);
      switch (op) { case C_GT: return x > y; case C_LT: return x < y; case C_GE: return x >= y;
                    case C_LE: return x <= y; case C_EQ: return x == y; default: return x != y; }
    }
  }
}

// returns false when the result is null
SG_HD inline bool math(int op, int t, int64_t a, int64_t b, int64_t& out) {
  switch (t) {
    case T_INT: {
      uint32_t x = (uint32_t)a, y = (uint32_t)b;
      int32_t ix = (int32_t)x, iy = (int32_t)y;
      switch (op) {
        case M_ADD: out = (int32_t)(x + y); return true;
        case M_SUB: out = (int32_t)(x - y); return true;
        case M_MUL: out = (int32_t)(x * y); return true;
        case M_DIV: if (iy == 0) return false; out = (ix == INT32_MIN && iy == -1) ? (int64_t)INT32_MIN : (int64_t)(ix / iy); return true;
        default: if (iy == 0) return false; out = (iy == -1) ? 0 : (int64_t)(ix % iy); return true;
      }
    }
    case T_LONG: {
      uint64_t x = (uint64_t)a, y = (uint64_t)b;
      switch (op) {
        case M_ADD: out = (int64_t)(x + y); return true;
        case M_SUB: out = (int64_t)(x - y); return true;
        case M_MUL: out = (int64_t)(x * y); return true;
        case M_DIV: if (b == 0) return false; out = (a == INT64_MIN && b == -1) ? INT64_MIN : a / b; return true;
        default: if (b == 0) return false; out = (b == -1) ? 0 : a % b; return true;
      }
    }
    case T_FLOAT: {
      float x = bits_f(a), y = bits_f(b);
      switch (op) {
        case M_ADD: out = f_bits(x + y); return true;
        case M_SUB: out = f_bits(x - y); return true;
        case M_MUL: out = f_bits(x * y); return true;
        case M_DIV: if (y == 0.0f) return false; out = f_bits(x / y); return true;
        default: if (y == 0.0f) return false; out = f_bits(__builtin_fmodf(x, y)); return true;
      }
    }
    default: {
      double x = bits_d(a), y = bits_d(b);
      switch (op) {
        case M_ADD: out = d_bits(x + y); return true;
        case M_SUB: out = d_bits(x - y); return true;
        case M_MUL: out = d_bits(x * y); return true;
        case M_DIV: if (y == 0.0) return false; out = d_bits(x / y); return true;
        default: if (y == 0.0) return false; out = d_bits(__builtin_fmod(x, y)); return true;
      }
    }
  }
}

// Interpreter.  `Loader` provides: bool load(int slot, int attr, int64_t& v) (false -> null).
// The register file is caller-provided (`rf`, register k at rf[k * stride]): on the device it lives
// in LDS with stride = block size so that runtime register indices never spill to scratch memory.
template <class Loader, class PR = Prog, class RFP = int64_t*>
SG_HD inline bool run(const PR& p, Loader& ld, int64_t& result, bool& isnull, RFP rf, int stride) {
#define r_(k) rf[(k) * stride]
  uint32_t nul = 0;
  for (int pc = 0; pc < p.n; pc++) {
    const auto& in = p.ins[pc];
    switch (in.op) {
      case BC_LD: {
        int64_t v = 0;
        bool ok = ld.load(in.a, in.imm, v);
        r_(in.dst) = v;
        if (ok) nul &= ~(1u << in.dst); else nul |= (1u << in.dst);
        break;
      }
      case BC_CONST:
        r_(in.dst) = p.consts[in.imm];
        if (in.b) nul |= (1u << in.dst); else nul &= ~(1u << in.dst);
        break;
      case BC_NULL:
        r_(in.dst) = 0; nul |= (1u << in.dst);
        break;
      case BC_CVT:
        r_(in.dst) = cvt(r_(in.a), (in.imm >> 4) & 15, in.imm & 15);
        if (nul & (1u << in.a)) nul |= (1u << in.dst); else nul &= ~(1u << in.dst);
        break;
      case BC_CMP: {
        bool n = (nul >> in.a & 1) | (nul >> in.b & 1);
        r_(in.dst) = n ? 0 : (int64_t)cmp((in.imm >> 4) & 15, in.imm & 15, r_(in.a), r_(in.b));
        nul &= ~(1u << in.dst);
        break;
      }
      case BC_MATH: {
        bool n = (nul >> in.a & 1) | (nul >> in.b & 1);
        int64_t o = 0;
        if (!n) n = !math((in.imm >> 4) & 15, in.imm & 15, r_(in.a), r_(in.b), o);
        r_(in.dst) = o;
        if (n) nul |= (1u << in.dst); else nul &= ~(1u << in.dst);
        break;
      }
      case BC_AND: {
        bool x = !(nul >> in.a & 1) && r_(in.a) != 0, y = !(nul >> in.b & 1) && r_(in.b) != 0;
        r_(in.dst) = x && y; nul &= ~(1u << in.dst);
        break;
      }
      case BC_OR: {
        bool x = !(nul >> in.a & 1) && r_(in.a) != 0, y = !(nul >> in.b & 1) && r_(in.b) != 0;
        r_(in.dst) = x || y; nul &= ~(1u << in.dst);
        break;
      }
      case BC_NOT: {
        bool x = (nul >> in.a & 1) ? true : (r_(in.a) == 0);
        r_(in.dst) = x; nul &= ~(1u << in.dst);
        break;
      }
      case BC_ISNULL:
        r_(in.dst) = (nul >> in.a) & 1; nul &= ~(1u << in.dst);
        break;
      case BC_RET:
        result = r_(in.a);
        isnull = (nul >> in.a) & 1;
        return true;
    }
  }
  return false;
#undef r_
}

template <class Loader, class PR = Prog, class RFP = int64_t*>
SG_HD inline bool run_pred(const PR& p, Loader& ld, RFP rf, int stride) {
  if (p.n == 0) return true;   // no filter
  int64_t v; bool n;
  run(p, ld, v, n, rf, stride);
  return !n && v != 0;
}

}  // namespace sg
