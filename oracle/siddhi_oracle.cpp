// siddhi_oracle.cpp — CPU restatement of siddhi-core's per-event semantics for the pattern /
// window hot path.
//
// *** TEST INFRASTRUCTURE ONLY. ***  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load this library, and only as the checker / timed CPU baseline.
// The product path (siddhi_amd/, libsiddhi_gfx.so) never links or calls it.
//
// It restates, object for object, the Java data flow of Siddhi 5.1.20-SNAPSHOT:
//   CORE = /root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/
//   * StateInputStreamParser.parse            CORE/util/parser/StateInputStreamParser.java:148-408
//   * StreamPre/PostStateProcessor            CORE/query/input/stream/state/StreamPreStateProcessor.java:46-500,
//                                             StreamPostStateProcessor.java:31-163
//   * Count / Logical / Absent processors     CountPreStateProcessor.java:34-221, CountPostStateProcessor.java:29-90,
//                                             LogicalPreStateProcessor.java:33-202, LogicalPostStateProcessor.java:29-130,
//                                             AbsentStreamPreStateProcessor.java:35-343, AbsentStreamPostStateProcessor.java:28-58
//   * inner runtimes (init/reset/update)      CORE/query/input/stream/state/runtime/*.java
//   * receivers                               CORE/query/input/MultiProcessStreamReceiver.java:216-241,
//                                             SingleProcessStreamReceiver.java:48-73, receiver/*.java
//   * StateEvent chains / cloners             CORE/event/state/StateEvent.java:138-236, StateEventCloner.java:48-60
//   * expression executors                    CORE/executor/condition/compare/**, executor/math/**
//   * QuerySelector batching                  CORE/query/selector/QuerySelector.java:76-374
//   * aggregators                             CORE/query/selector/attribute/aggregator/{Sum,Avg,Count,Min,Max}*.java
//   * windows                                 CORE/query/processor/stream/window/{Length,Time,LengthBatch}WindowProcessor.java
//   * partitions                              CORE/partition/PartitionStreamReceiver.java:82-282
//   * output                                  CORE/query/output/ratelimit/OutputRateLimiter.java:64-110,
//                                             callback/QueryCallback.java:61-91, InsertIntoStreamCallback.java:44-58
//   * time / timers                           CORE/util/Scheduler.java:64-212, util/timestamp/TimestampGeneratorImpl.java:78-122
//
// Pinned by the known-answer fixtures in tests/golden/ (transcribed from the reference's TestNG
// suites: TEST/query/{pattern,sequence,window,partition}/...).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

// the descriptor JSON reader is shared with the C ABI (one copy: siddhi_amd/csrc/json.hpp)
#include "../siddhi_amd/csrc/json.hpp"

using sgjson::J;

namespace orc {

// ------------------------------------------------------------------------------------------------
// Values (Java boxed types restated)
// ------------------------------------------------------------------------------------------------
enum Ty : uint8_t { T_STRING = 0, T_INT, T_LONG, T_FLOAT, T_DOUBLE, T_BOOL, T_OBJECT };

static Ty ty_of(const std::string& s) {
  if (s == "STRING") return T_STRING;
  if (s == "INT") return T_INT;
  if (s == "LONG") return T_LONG;
  if (s == "FLOAT") return T_FLOAT;
  if (s == "DOUBLE") return T_DOUBLE;
  if (s == "BOOL") return T_BOOL;
  return T_OBJECT;
}

struct Val {
  Ty t = T_OBJECT;
  bool null = true;
  union {
    int32_t i;
    int64_t l;
    float f;
    double d;
    int32_t s;  // interned string id
    bool b;
  };
  Val() : l(0) {}
  static Val I(int32_t v) { Val x; x.t = T_INT; x.null = false; x.l = 0; x.i = v; return x; }
  static Val L(int64_t v) { Val x; x.t = T_LONG; x.null = false; x.l = v; return x; }
  static Val F(float v) { Val x; x.t = T_FLOAT; x.null = false; x.l = 0; x.f = v; return x; }
  static Val D(double v) { Val x; x.t = T_DOUBLE; x.null = false; x.d = v; return x; }
  static Val B(bool v) { Val x; x.t = T_BOOL; x.null = false; x.l = 0; x.b = v; return x; }
  static Val S(int32_t v) { Val x; x.t = T_STRING; x.null = false; x.l = 0; x.s = v; return x; }
  static Val N(Ty t) { Val x; x.t = t; x.null = true; x.l = 0; return x; }
  // raw 8-byte slot used across the C ABI
  int64_t raw() const {
    int64_t r = 0;
    switch (t) {
      case T_INT: r = (int64_t)i; break;
      case T_LONG: r = l; break;
      case T_FLOAT: { uint32_t u; std::memcpy(&u, &f, 4); r = (int64_t)u; break; }
      case T_DOUBLE: std::memcpy(&r, &d, 8); break;
      case T_BOOL: r = b ? 1 : 0; break;
      case T_STRING: r = s; break;
      default: r = 0;
    }
    return r;
  }
  static Val from_raw(Ty t, int64_t r, bool isnull) {
    if (isnull) return N(t);
    switch (t) {
      case T_INT: return I((int32_t)r);
      case T_LONG: return L(r);
      case T_FLOAT: { uint32_t u = (uint32_t)r; float f; std::memcpy(&f, &u, 4); return F(f); }
      case T_DOUBLE: { double d; std::memcpy(&d, &r, 8); return D(d); }
      case T_BOOL: return B(r != 0);
      case T_STRING: return S((int32_t)r);
      default: return N(t);
    }
  }
  // key for hashing / toString-equivalence (Java toString is injective on these values)
  std::pair<int, int64_t> key() const { return {null ? -1 : (int)t, null ? 0 : raw()}; }
};

// Number.xxxValue() conversions
static inline float as_float(const Val& v) {
  switch (v.t) {
    case T_INT: return (float)v.i;
    case T_LONG: return (float)v.l;
    case T_FLOAT: return v.f;
    case T_DOUBLE: return (float)v.d;
    default: return 0;
  }
}
static inline double as_double(const Val& v) {
  switch (v.t) {
    case T_INT: return (double)v.i;
    case T_LONG: return (double)v.l;
    case T_FLOAT: return (double)v.f;
    case T_DOUBLE: return v.d;
    default: return 0;
  }
}
static inline int64_t as_long(const Val& v) {
  switch (v.t) {
    case T_INT: return (int64_t)v.i;
    case T_LONG: return v.l;
    case T_FLOAT: return (int64_t)v.f;   // not reached for compare/math of integral types
    case T_DOUBLE: return (int64_t)v.d;
    default: return 0;
  }
}
static inline int32_t as_int(const Val& v) { return (int32_t)as_long(v); }

// Java's Double.equals / Float.equals (used by Deque.removeFirstOccurrence)
static bool boxed_equals(const Val& a, const Val& b) {
  if (a.null || b.null) return a.null && b.null;
  if (a.t != b.t) return false;
  if (a.t == T_DOUBLE) {
    double x = a.d, y = b.d;
    if (std::isnan(x) && std::isnan(y)) return true;
    uint64_t ux, uy; std::memcpy(&ux, &x, 8); std::memcpy(&uy, &y, 8);
    return ux == uy;
  }
  if (a.t == T_FLOAT) {
    float x = a.f, y = b.f;
    if (std::isnan(x) && std::isnan(y)) return true;
    uint32_t ux, uy; std::memcpy(&ux, &x, 4); std::memcpy(&uy, &y, 4);
    return ux == uy;
  }
  return a.raw() == b.raw();
}

// ------------------------------------------------------------------------------------------------
// Events (CORE/event/stream/StreamEvent.java, CORE/event/state/StateEvent.java)
// ------------------------------------------------------------------------------------------------
enum EvType : uint8_t { CURRENT = 0, EXPIRED = 1, TIMER = 2, RESET = 3 };

struct StreamEvent {
  int64_t ts = 0;
  const Val* data = nullptr;  // immutable attribute data shared by clones
  StreamEvent* next = nullptr;
  EvType type = CURRENT;
  Val* out = nullptr;         // outputData for single-stream selectors
};

struct StateEvent {
  std::vector<StreamEvent*> slots;
  int64_t ts = -1;
  EvType type = CURRENT;
  std::vector<Val> out;
  StateEvent* next = nullptr;
};

struct Pool {
  std::vector<StreamEvent*> free_se;
  std::deque<std::vector<Val>> rows;
  std::vector<std::unique_ptr<StreamEvent[]>> blocks;
  size_t used = 4096;
  StreamEvent* se() {
    if (!free_se.empty()) { auto* e = free_se.back(); free_se.pop_back(); *e = StreamEvent(); return e; }
    if (used == 4096) { blocks.emplace_back(new StreamEvent[4096]); used = 0; }
    auto* e = &blocks.back()[used++];
    *e = StreamEvent();
    return e;
  }
  void release(StreamEvent* e) { free_se.push_back(e); }
  // StreamEventCloner.copyStreamEvent: new event, same data, same ts/type, next = null
  StreamEvent* copy(const StreamEvent* src) {
    auto* e = se();
    e->ts = src->ts; e->data = src->data; e->type = src->type;
    return e;
  }
};

// ------------------------------------------------------------------------------------------------
// Expressions
// ------------------------------------------------------------------------------------------------
enum Op {
  O_CONST, O_VAR, O_OUTVAR, O_AND, O_OR, O_NOT, O_ISNULL,
  O_GT, O_LT, O_GE, O_LE, O_EQ, O_NE, O_ADD, O_SUB, O_MUL, O_DIV, O_MOD, O_AGG, O_MULTIVAR
};

enum AggK { A_SUM, A_AVG, A_COUNT, A_MIN, A_MAX };

struct Ex {
  Op op;
  Ty t = T_OBJECT;   // result type
  Ty ct = T_OBJECT;  // compare type
  Val c;
  int slot = -1, chain = 0, attr = 0;
  std::unique_ptr<Ex> a, b;
  AggK agg = A_SUM;
  int agg_idx = -1;  // index into selector aggregator list
};

struct App;

// context for evaluating an expression
struct EvalCtx {
  const StateEvent* se = nullptr;
  const StreamEvent* ev = nullptr;  // single-stream
  const std::vector<Val>* out = nullptr;  // having / order-by context
  std::vector<Val>* aggvals = nullptr;    // precomputed aggregator outputs
};

// StateEvent.getStreamEvent(int[]) (StateEvent.java:138-182)
static const StreamEvent* chain_at(const StreamEvent* head, int idx) {
  if (!head) return nullptr;
  const StreamEvent* e = head;
  if (idx >= 0) {
    for (int i = 1; i <= idx; i++) { e = e->next; if (!e) return nullptr; }
    return e;
  }
  if (idx == -1) {  // CURRENT
    while (e->next) e = e->next;
    return e;
  }
  if (idx == -2) {  // LAST
    if (!e->next) return nullptr;
    while (e->next->next) e = e->next;
    return e;
  }
  std::vector<const StreamEvent*> lst;
  while (e) { lst.push_back(e); e = e->next; }
  long k = (long)lst.size() + idx;
  if (k < 0) return nullptr;
  return lst[k];
}

static Val eval(const Ex* x, const EvalCtx& c);

static bool cmp(Op op, Ty ct, const Val& l, const Val& r) {
  // CompareConditionExpressionExecutor.execute: null on either side -> false
  if (l.null || r.null) return false;
  switch (ct) {
    case T_INT: { int32_t a = as_int(l), b = as_int(r);
      switch (op) { case O_GT: return a > b; case O_LT: return a < b; case O_GE: return a >= b; case O_LE: return a <= b;
                    case O_EQ: return a == b; default: return a != b; } }
    case T_LONG: { int64_t a = as_long(l), b = as_long(r);
      switch (op) { case O_GT: return a > b; case O_LT: return a < b; case O_GE: return a >= b; case O_LE: return a <= b;
                    case O_EQ: return a == b; default: return a != b; } }
    case T_FLOAT: { float a = as_float(l), b = as_float(r);
      switch (op) { case O_GT: return a > b; case O_LT: return a < b; case O_GE: return a >= b; case O_LE: return a <= b;
                    case O_EQ: return a == b; default: return a != b; } }
    case T_DOUBLE: { double a = as_double(l), b = as_double(r);
      switch (op) { case O_GT: return a > b; case O_LT: return a < b; case O_GE: return a >= b; case O_LE: return a <= b;
                    case O_EQ: return a == b; default: return a != b; } }
    case T_STRING: { bool eq = l.s == r.s; return op == O_EQ ? eq : !eq; }
    case T_BOOL: { bool eq = l.b == r.b; return op == O_EQ ? eq : !eq; }
    default: return false;
  }
}

static Val math(Op op, Ty t, const Val& l, const Val& r) {
  if (l.null || r.null) return Val::N(t);
  switch (t) {
    case T_INT: {
      uint32_t a = (uint32_t)as_int(l), b = (uint32_t)as_int(r);
      int32_t ia = (int32_t)a, ib = (int32_t)b;
      switch (op) {
        case O_ADD: return Val::I((int32_t)(a + b));
        case O_SUB: return Val::I((int32_t)(a - b));
        case O_MUL: return Val::I((int32_t)(a * b));
        case O_DIV: if (ib == 0) return Val::N(t); if (ia == INT32_MIN && ib == -1) return Val::I(INT32_MIN); return Val::I(ia / ib);
        default: if (ib == 0) return Val::N(t); if (ib == -1) return Val::I(0); return Val::I(ia % ib);
      }
    }
    case T_LONG: {
      uint64_t a = (uint64_t)as_long(l), b = (uint64_t)as_long(r);
      int64_t ia = (int64_t)a, ib = (int64_t)b;
      switch (op) {
        case O_ADD: return Val::L((int64_t)(a + b));
        case O_SUB: return Val::L((int64_t)(a - b));
        case O_MUL: return Val::L((int64_t)(a * b));
        case O_DIV: if (ib == 0) return Val::N(t); if (ia == INT64_MIN && ib == -1) return Val::L(INT64_MIN); return Val::L(ia / ib);
        default: if (ib == 0) return Val::N(t); if (ib == -1) return Val::L(0); return Val::L(ia % ib);
      }
    }
    case T_FLOAT: {
      float a = as_float(l), b = as_float(r);
      switch (op) {
        case O_ADD: return Val::F(a + b);
        case O_SUB: return Val::F(a - b);
        case O_MUL: return Val::F(a * b);
        case O_DIV: if (b == 0.0f) return Val::N(t); return Val::F(a / b);
        default: if (b == 0.0f) return Val::N(t); return Val::F(std::fmod(a, b));
      }
    }
    default: {
      double a = as_double(l), b = as_double(r);
      switch (op) {
        case O_ADD: return Val::D(a + b);
        case O_SUB: return Val::D(a - b);
        case O_MUL: return Val::D(a * b);
        case O_DIV: if (b == 0.0) return Val::N(T_DOUBLE); return Val::D(a / b);
        default: if (b == 0.0) return Val::N(T_DOUBLE); return Val::D(std::fmod(a, b));
      }
    }
  }
}

static Val eval(const Ex* x, const EvalCtx& c) {
  switch (x->op) {
    case O_CONST: return x->c;
    case O_VAR: {
      const StreamEvent* e;
      if (x->slot < 0) e = c.ev;
      else e = chain_at(c.se->slots[x->slot], x->chain);
      // an absent slot filled with StreamEventFactory.newInstance() (AbsentLogicalPreStateProcessor
      // :192-203) carries no data: every attribute reads null
      if (!e || !e->data) return Val::N(x->t);
      return e->data[x->attr];
    }
    case O_OUTVAR: return (*c.out)[x->attr];
    case O_AND: { Val a = eval(x->a.get(), c); if (a.null || !a.b) return Val::B(false);
                  Val b = eval(x->b.get(), c); return Val::B(!b.null && b.b); }
    case O_OR: { Val a = eval(x->a.get(), c); if (!a.null && a.b) return Val::B(true);
                 Val b = eval(x->b.get(), c); return Val::B(!b.null && b.b); }
    case O_NOT: { Val a = eval(x->a.get(), c); return Val::B(a.null ? true : !a.b); }
    case O_ISNULL: { Val a = eval(x->a.get(), c); return Val::B(a.null); }
    case O_GT: case O_LT: case O_GE: case O_LE: case O_EQ: case O_NE:
      return Val::B(cmp(x->op, x->ct, eval(x->a.get(), c), eval(x->b.get(), c)));
    case O_ADD: case O_SUB: case O_MUL: case O_DIV: case O_MOD:
      return math(x->op, x->t, eval(x->a.get(), c), eval(x->b.get(), c));
    case O_AGG: return (*c.aggvals)[x->agg_idx];
    default: return Val::N(T_OBJECT);
  }
}

// ------------------------------------------------------------------------------------------------
// Aggregators (CORE/query/selector/attribute/aggregator/*)
// ------------------------------------------------------------------------------------------------
struct AggState {
  // sum/avg
  double dsum = 0.0; int64_t lsum = 0; int64_t count = 0;
  // min/max
  bool track = false;
  std::deque<Val> dq;
  Val mv;  // current min/max (null initially)
};

struct AggSpec {
  AggK k;
  Ty in_t = T_OBJECT;
  std::unique_ptr<Ex> arg;
  bool track = false;   // min/max trackFutureStates
};

static bool agg_can_destroy(const AggSpec& s, const AggState& st) {
  switch (s.k) {
    case A_SUM: return (s.in_t == T_INT || s.in_t == T_LONG) ? (st.count == 0 && st.lsum == 0) : (st.count == 0 && st.dsum == 0.0);
    case A_AVG: return st.dsum == 0.0 && st.count == 0;
    case A_COUNT: return st.count == 0;
    default: return (!st.track || st.dq.empty()) && st.mv.null;
  }
}

static bool lt(const Val& a, const Val& b) {  // a < b on same numeric type (boxed compare via primitives)
  switch (a.t) {
    case T_INT: return a.i < b.i;
    case T_LONG: return a.l < b.l;
    case T_FLOAT: return a.f < b.f;
    default: return a.d < b.d;
  }
}

static Val agg_apply(const AggSpec& s, AggState& st, EvType type, const Val& in) {
  Ty rt;
  switch (s.k) {
    case A_COUNT:
      if (type == CURRENT) { st.count++; return Val::L(st.count); }
      if (type == EXPIRED) { st.count--; return Val::L(st.count); }
      st.count = 0; return Val::L(0);
    case A_SUM: {
      bool integral = (s.in_t == T_INT || s.in_t == T_LONG);
      rt = integral ? T_LONG : T_DOUBLE;
      if (type == RESET) {
        st.dsum = 0; st.lsum = 0; st.count = 0;
        return integral ? Val::L(0) : Val::N(T_DOUBLE);
      }
      if (in.null) {  // SumAttributeAggregatorExecutor.processAdd/Remove(null) -> currentValue()
        if (st.count == 0) return Val::N(rt);
        return integral ? Val::L(st.lsum) : Val::D(st.dsum);
      }
      if (type == CURRENT) {
        if (integral) { st.lsum = (int64_t)((uint64_t)st.lsum + (uint64_t)as_long(in)); st.count++; return Val::L(st.lsum); }
        st.dsum += as_double(in); st.count++; return Val::D(st.dsum);
      } else {
        if (integral) {  // processRemove(double): sum = (long)(sum - (double)x)  (Sum...:283-291)
          double r = (double)st.lsum - (double)as_long(in);
          int64_t v;
          if (std::isnan(r)) v = 0;
          else if (r >= 9.2233720368547758e18) v = INT64_MAX;
          else if (r <= -9.2233720368547758e18) v = INT64_MIN;
          else v = (int64_t)r;
          st.lsum = v; st.count--;
          if (st.count == 0) return Val::N(T_LONG);
          return Val::L(st.lsum);
        }
        st.dsum -= as_double(in); st.count--;
        if (st.count == 0) return Val::N(T_DOUBLE);
        return Val::D(st.dsum);
      }
    }
    case A_AVG: {
      if (type == RESET) { st.dsum = 0; st.count = 0; return Val::N(T_DOUBLE); }
      if (in.null) { if (st.count == 0) return Val::N(T_DOUBLE); return Val::D(st.dsum / st.count); }
      if (type == CURRENT) { st.count++; st.dsum += as_double(in); }
      else { st.count--; st.dsum -= as_double(in); }
      if (st.count == 0) return Val::N(T_DOUBLE);
      return Val::D(st.dsum / (double)st.count);
    }
    case A_MIN: case A_MAX: {
      bool isMin = s.k == A_MIN;
      if (type == RESET) { st.dq.clear(); st.mv = Val::N(s.in_t); return Val::N(s.in_t); }
      if (in.null) return st.mv.null ? Val::N(s.in_t) : st.mv;
      Val v = in;
      if (type == CURRENT) {
        if (st.track) {
          while (!st.dq.empty()) {
            const Val& back = st.dq.back();
            bool drop = isMin ? lt(v, back) : lt(back, v);
            if (drop) st.dq.pop_back(); else break;
          }
          st.dq.push_back(v);
        }
        if (st.mv.null || (isMin ? lt(v, st.mv) : lt(st.mv, v))) st.mv = v;
        return st.mv;
      } else {
        if (st.track) {
          for (auto it = st.dq.begin(); it != st.dq.end(); ++it)
            if (boxed_equals(*it, v)) { st.dq.erase(it); break; }
          st.mv = st.dq.empty() ? Val::N(s.in_t) : st.dq.front();
        } else if (!st.mv.null && boxed_equals(st.mv, v)) {
          st.mv = Val::N(s.in_t);
        }
        return st.mv;
      }
    }
  }
  return Val::N(T_OBJECT);
}

// ------------------------------------------------------------------------------------------------
// Output
// ------------------------------------------------------------------------------------------------
struct OutEvent {
  int64_t ts;
  bool expired;
  std::vector<Val> data;
};
struct Callback {
  int kind;     // 0 = QueryCallback, 1 = StreamCallback
  int target;   // query index / stream index
  int64_t ts;
  int64_t seq = -1;   // arrival index of the sent event whose processing fired it (sharded-run merge key)
  std::vector<OutEvent> in, rm;
};

// ------------------------------------------------------------------------------------------------
// Selector (QuerySelector.java) — shared by state & single-stream queries
// ------------------------------------------------------------------------------------------------
struct SelEvent {   // a selector-level event (either a StateEvent or a StreamEvent)
  StateEvent* se = nullptr;
  StreamEvent* ev = nullptr;
  EvType type;
  int64_t ts;
  std::vector<Val> out;
  std::vector<Val> aggv;   // aggregator results of populate (a having aggregator reads its own)
};

struct Query;

struct Selector {
  std::vector<std::unique_ptr<Ex>> attrs;
  std::vector<Ty> out_types;
  std::vector<AggSpec> aggs;
  std::vector<std::unique_ptr<Ex>> group_by;
  std::unique_ptr<Ex> having;
  std::vector<std::pair<std::unique_ptr<Ex>, bool>> order_by;  // (expr over output, desc)
  int64_t limit = -1, offset = -1;
  bool currentOn = true, expiredOn = false;
  bool groupBy = false, containsAgg = false;
  bool partitioned = false;
  // aggregator states: key = group key (vector of values) -> states
  std::map<std::vector<std::pair<int, int64_t>>, std::vector<AggState>> agg_states;

  std::vector<AggState>& states_for(const std::vector<std::pair<int, int64_t>>& gk) {
    auto it = agg_states.find(gk);
    if (it != agg_states.end()) return it->second;
    auto& v = agg_states[gk];
    v.resize(aggs.size());
    for (size_t i = 0; i < aggs.size(); i++) { v[i].track = aggs[i].track; v[i].mv = Val::N(aggs[i].in_t); }
    return v;
  }

  std::vector<std::pair<int, int64_t>> group_key(const EvalCtx& c) {
    std::vector<std::pair<int, int64_t>> k;
    for (auto& g : group_by) k.push_back(eval(g.get(), c).key());
    return k;
  }

  // AttributeProcessor.process for every attribute (incl. aggregators), for one event
  void populate(SelEvent& e) {
    EvalCtx c; c.se = e.se; c.ev = e.ev;
    std::vector<Val> aggvals(aggs.size());
    if (!aggs.empty()) {
      auto gk = group_key(c);
      auto& st = states_for(gk);
      for (size_t i = 0; i < aggs.size(); i++) {
        Val in = aggs[i].arg ? eval(aggs[i].arg.get(), c) : Val::N(T_OBJECT);
        aggvals[i] = agg_apply(aggs[i], st[i], e.type, in);
      }
      // PartitionStateHolder.returnState: destroy when canDestroy (groupBy or partitioned holders)
      if (groupBy || partitioned) {
        bool all = true;
        for (size_t i = 0; i < aggs.size(); i++) {
          // each aggregator has its own holder; destroy independently
          if (agg_can_destroy(aggs[i], st[i])) { st[i] = AggState(); st[i].track = aggs[i].track; st[i].mv = Val::N(aggs[i].in_t); }
          else all = false;
        }
        (void)all;
      }
    }
    e.aggv = aggvals;
    c.aggvals = &e.aggv;
    e.out.resize(attrs.size());
    if (e.type == RESET) return;
    for (size_t i = 0; i < attrs.size(); i++) e.out[i] = eval(attrs[i].get(), c);
  }

  bool having_ok(const SelEvent& e) {
    if (!having) return true;
    EvalCtx c; c.se = e.se; c.ev = e.ev; c.out = &e.out;
    c.aggvals = const_cast<std::vector<Val>*>(&e.aggv);
    Val v = eval(having.get(), c);
    return !v.null && v.b;
  }

  bool type_on(const SelEvent& e) {
    return (e.type == CURRENT && currentOn) || (e.type == EXPIRED && expiredOn);
  }

  const std::vector<std::string>* strings = nullptr;
  // OrderByEventComparator.compare (CORE/query/selector/OrderByEventComparator.java:62-113): Comparable
  // compareTo per type (String lexicographic, Float/Double.compare total order, false < true); a null
  // sorts after a value whatever the direction
  int java_compare(const Val& a, const Val& b) const {
    switch (a.t) {
      case T_STRING: { int c = (*strings)[a.s].compare((*strings)[b.s]); return c < 0 ? -1 : (c > 0 ? 1 : 0); }
      case T_INT: return a.i < b.i ? -1 : (a.i > b.i ? 1 : 0);
      case T_LONG: return a.l < b.l ? -1 : (a.l > b.l ? 1 : 0);
      case T_BOOL: return (int)a.b - (int)b.b;
      case T_FLOAT: {
        if (a.f < b.f) return -1;
        if (a.f > b.f) return 1;
        int32_t x, y;
        float fa = a.f != a.f ? NAN : a.f, fb = b.f != b.f ? NAN : b.f;   // floatToIntBits: canonical NaN
        std::memcpy(&x, &fa, 4); std::memcpy(&y, &fb, 4);
        return x == y ? 0 : (x < y ? -1 : 1);
      }
      case T_DOUBLE: {
        if (a.d < b.d) return -1;
        if (a.d > b.d) return 1;
        int64_t x, y;
        double da = a.d != a.d ? (double)NAN : a.d, db = b.d != b.d ? (double)NAN : b.d;
        std::memcpy(&x, &da, 8); std::memcpy(&y, &db, 8);
        return x == y ? 0 : (x < y ? -1 : 1);
      }
      default: return 0;
    }
  }

  void order_limit(std::vector<SelEvent>& v) {
    if (!order_by.empty()) {
      std::stable_sort(v.begin(), v.end(), [&](const SelEvent& x, const SelEvent& y) {
        for (auto& ob : order_by) {
          EvalCtx cx; cx.out = &x.out; EvalCtx cy; cy.out = &y.out;
          Val a = eval(ob.first.get(), cx), b = eval(ob.first.get(), cy);
          if (!a.null && !b.null) {
            int r = java_compare(a, b);
            if (ob.second) r = -r;
            if (r != 0) return r < 0;
          } else if (!a.null) {
            return true;
          } else if (!b.null) {
            return false;
          }
        }
        return false;
      });
    }
    if (offset >= 0) {
      if ((size_t)offset >= v.size()) v.clear(); else v.erase(v.begin(), v.begin() + offset);
    }
    if (limit >= 0 && (size_t)limit < v.size()) v.resize(limit);
  }

  // QuerySelector.process (batch mode: ComplexEventChunk.isBatch() is always true)
  std::vector<SelEvent> process(std::vector<SelEvent>& chunk) {
    std::vector<SelEvent> out;
    if (groupBy) {   // processInBatchGroupBy
      std::vector<std::vector<std::pair<int, int64_t>>> order;
      std::map<std::vector<std::pair<int, int64_t>>, SelEvent> grouped;
      for (auto& e : chunk) {
        if (e.type == TIMER) continue;
        if (e.type == RESET) { populate(e); continue; }
        EvalCtx c; c.se = e.se; c.ev = e.ev;
        auto gk = group_key(c);
        populate(e);
        if (having_ok(e) && type_on(e)) {
          if (!grouped.count(gk)) order.push_back(gk);
          grouped[gk] = e;
        }
      }
      for (auto& k : order) out.push_back(grouped[k]);
      order_limit(out);
      return out;
    }
    if (containsAgg) {  // processInBatchNoGroupBy
      SelEvent* last = nullptr;
      for (auto& e : chunk) {
        if (e.type == TIMER) continue;
        populate(e);
        if (e.type == RESET) continue;
        if (having_ok(e) && type_on(e)) last = &e;
      }
      if (last && (offset <= 0) && (limit < 0 || limit > 0)) out.push_back(*last);
      return out;
    }
    // processNoGroupBy
    for (auto& e : chunk) {
      if (e.type == TIMER) continue;
      populate(e);
      if (e.type == RESET) continue;
      if (type_on(e) && having_ok(e)) out.push_back(e);
    }
    order_limit(out);
    return out;
  }
};

// ------------------------------------------------------------------------------------------------
// State processors
// ------------------------------------------------------------------------------------------------
struct Post;
struct QueryRT;

enum PreKind { K_STREAM, K_COUNT, K_LOGICAL, K_ABSENT };

struct Pre {
  PreKind kind = K_STREAM;
  QueryRT* rt = nullptr;
  int stateId = 0;
  bool isStartState = false;
  bool seq = false;
  int64_t withinTime = -1;
  std::vector<int> startStateIds;
  Pre* withinEveryPre = nullptr;
  Post* thisPost = nullptr;
  Post* thisLast = nullptr;
  std::vector<Ex*> filters;
  // state (StreamPreState)
  std::list<StateEvent*> pending, newEvery;
  bool stateChanged = false, initialized = false;
  // count
  int minCount = 0, maxCount = 0;
  bool successCondition = false, startStateReset = false;
  Post* countPost = nullptr;
  // logical
  bool isAnd = false;
  Pre* partner = nullptr;
  // absent
  int64_t waitingTime = -1;
  int64_t lastScheduledTime = 0;
  bool active = true, started = false;
  // logical absent (AbsentLogicalPreStateProcessor: kind K_LOGICAL with absentLogical set)
  bool absentLogical = false;
  int64_t lastArrivalTime = 0;

  virtual ~Pre() = default;
  void init();
  void addState(StateEvent* se);
  void addEveryState(StateEvent* se);
  void resetState();
  void updateState();
  void expireEvents(int64_t ts);
  bool isExpired(StateEvent* se, int64_t ts);
  std::vector<StateEvent*> processAndReturn(StreamEvent* ev);
  void processChain(StateEvent* se);  // StreamPreStateProcessor.process(StateEvent)
  // count
  void countStartStateReset();
  // absent
  void absentTimer(int64_t ts);
  void updateLastArrivalTime(int64_t ts);
  // logical absent
  void absentLogicalTimer(int64_t ts);
  bool partnerCanProceed(StateEvent* se);
  std::vector<StateEvent*> absentLogicalProcessAndReturn(StreamEvent* ev);
  void sendAbsentLogical(StateEvent* se);
};

enum PostKind { P_STREAM, P_COUNT, P_LOGICAL, P_ABSENT, P_ABSENT_LOGICAL };

struct Post {
  PostKind kind = P_STREAM;
  int stateId = 0;
  Pre* nextStatePre = nullptr;
  Pre* nextEveryStatePre = nullptr;
  Pre* thisPre = nullptr;
  Pre* callbackPre = nullptr;
  bool hasNext = false;   // nextProcessor (selector) != null
  bool isEventReturned = false;
  // count
  int minCount = 0, maxCount = 0;
  // logical
  bool isAnd = false;
  Pre* partnerPre = nullptr;
  Post* partnerPost = nullptr;

  void process(StateEvent* se);
  void streamProcess(StateEvent* se);  // StreamPostStateProcessor.process
  void processMinCountReached(StateEvent* se);
  void setNextStatePre(Pre* p);
  void setNextEveryStatePre(Pre* p);
};

struct Inner {  // InnerStateRuntime
  enum K { STREAM, NEXT, EVERY, LOGICAL, COUNT } k;
  Pre* first = nullptr;
  Post* last = nullptr;
  std::vector<std::string> streamsList;     // SingleStreamRuntime list (stream ids in order)
  std::vector<Pre*> streamFirstProcs;       // first processor of each single stream runtime
  std::unique_ptr<Inner> a, b;              // next: cur/nxt; logical: r1/r2; every/count: a
  void init() {
    switch (k) {
      case STREAM: case COUNT: first->init(); break;
      case NEXT: a->init(); b->init(); break;
      case EVERY: a->init(); break;
      case LOGICAL: b->init(); a->init(); break;
    }
  }
  void reset() {
    switch (k) {
      case STREAM: case COUNT: first->resetState(); break;
      case NEXT: b->reset(); a->reset(); break;
      case EVERY: first->resetState(); break;       // EveryInnerStateRuntime inherits Stream reset (firstProcessor)
      case LOGICAL: b->reset(); break;
    }
  }
  void update() {
    switch (k) {
      case STREAM: case COUNT: first->updateState(); break;
      case NEXT: a->update(); b->update(); break;
      case EVERY: first->updateState(); break;
      case LOGICAL: b->update(); break;
    }
  }
};

struct Receiver {   // ProcessStreamReceiver for one stream id
  int stream = -1;
  std::vector<Pre*> nexts;          // setNext order (setup order)
  std::vector<Pre*> forStream;      // stateProcessorsForStream
  bool multi = false;
};

struct Window {
  enum K { NONE, LENGTH, TIME, LENGTH_BATCH } k = NONE;
  int64_t param = 0;
  bool streamCurrent = false;
  // state
  std::deque<StreamEvent*> q;       // length/time expired queue
  int64_t count = 0;
  int64_t lastTimestamp = INT64_MIN;
  std::vector<StreamEvent*> cur, exq;
  StreamEvent* resetEvent = nullptr;
};

struct App;

struct QueryDef;  // immutable per-query definition

struct QueryRT {   // one instance per partition key (or one if unpartitioned)
  App* app = nullptr;
  const QueryDef* def = nullptr;
  Pool* pool = nullptr;
  int nslots = 0;
  bool seq = false;
  std::vector<std::unique_ptr<Pre>> pres;
  std::vector<std::unique_ptr<Post>> posts;
  std::vector<Pre*> allPre;   // preStateProcessors (expire order)
  std::vector<Pre*> startupPre;
  std::unique_ptr<Inner> inner;
  std::map<int, Receiver> receivers;
  Selector sel;
  // single stream
  std::vector<Ex*> sfilters;
  Window win;
  int64_t key_dummy = 0;
  int32_t key_hash = 0;   // String.hashCode of the partition key (toString of the key value)
  std::pair<int, int64_t> pkey{-1, 0};   // the partition key value (Val::key)

  // the ReturnEventHolder for the multi receiver currently processing (thread-local in Java)
  std::vector<SelEvent>* holder = nullptr;

  StateEvent* newStateEvent() {
    auto* s = new StateEvent();
    s->slots.assign(nslots, nullptr);
    return s;
  }
  StateEvent* cloneStateEvent(const StateEvent* o) {  // StateEventCloner.copyStateEvent (shallow)
    auto* s = new StateEvent();
    s->slots = o->slots; s->out = o->out; s->type = o->type; s->ts = o->ts;
    return s;
  }
  void selectAndEmit(StateEvent* se);            // QuerySelector.process for one StateEvent
  void emitChunk(std::vector<SelEvent>& out);    // OutputRateLimiter.sendToCallBacks
  void receive(int stream, int64_t ts, const Val* data);
  void receiveBatch(int stream, const std::vector<std::pair<int64_t, const Val*>>& evs);
  void receiveSingle(int stream, const std::vector<std::pair<int64_t, const Val*>>& evs, bool batch);
  void onTimer(int64_t ts);
  void deliverHolders(std::vector<std::vector<SelEvent>>& holders);
  void app_notify_at(Pre* p, int64_t t);   // Scheduler.notifyAt
};

// ---- Pre implementations ----
void Pre::init() {
  // StreamPreStateProcessor.init (:178-194); Absent start seeds via partitionCreated instead.
  if (isStartState && (!initialized || thisPost->nextEveryStatePre != nullptr ||
                       (seq && thisPost->nextStatePre && thisPost->nextStatePre->kind == K_ABSENT))) {
    StateEvent* se = rt->newStateEvent();
    addState(se);
    initialized = true;
  }
}

void Pre::addState(StateEvent* se) {
  switch (kind) {
    case K_LOGICAL:  // LogicalPreStateProcessor.addState (:43-62)
      if (absentLogical && !active) return;   // AbsentLogicalPreStateProcessor.addState (:78-99)
      if (isStartState || seq) {
        if (newEvery.empty()) newEvery.push_back(se);
        if (partner && partner->newEvery.empty()) partner->newEvery.push_back(se);
      } else {
        newEvery.push_back(se);
        if (partner) partner->newEvery.push_back(se);
      }
      if (absentLogical && !isStartState && waitingTime != -1) {
        rt->app_notify_at(this, se->ts + waitingTime);
        if (partner->absentLogical) rt->app_notify_at(partner, se->ts + partner->waitingTime);
      }
      return;
    case K_ABSENT:  // AbsentStreamPreStateProcessor.addState (:78-100)
      if (!active) return;
      if (seq) { newEvery.clear(); newEvery.push_back(se); }
      else newEvery.push_back(se);
      if (!isStartState) {
        lastScheduledTime = se->ts + waitingTime;
        rt->app_notify_at(this, lastScheduledTime);
      }
      return;
    default:
      if (seq) { if (newEvery.empty()) newEvery.push_back(se); }
      else newEvery.push_back(se);
      if (kind == K_COUNT && minCount == 0 && se->slots[stateId] == nullptr) {
        // CountPreStateProcessor.addState (:126-134)
        countPost->processMinCountReached(se);
      }
      return;
  }
}

void Pre::addEveryState(StateEvent* se) {
  StateEvent* c = rt->cloneStateEvent(se);
  c->type = CURRENT;
  if (absentLogical) {   // AbsentLogicalPreStateProcessor.addEveryState (:101-121): own + partner slot only
    if (c->slots[stateId]) c->ts = c->slots[stateId]->ts;
    c->slots[stateId] = nullptr;
    c->slots[partner->stateId] = nullptr;
    newEvery.push_back(c);
    partner->newEvery.push_back(c);
    return;
  }
  for (int i = stateId; i < (int)c->slots.size(); i++) c->slots[i] = nullptr;
  newEvery.push_back(c);
  if (kind == K_LOGICAL && partner) {  // LogicalPreStateProcessor.addEveryState (:65-84)
    c->slots[partner->stateId] = nullptr;
    partner->newEvery.push_back(c);
  }
  if (kind == K_ABSENT) {
    lastScheduledTime = se->ts + waitingTime;
    rt->app_notify_at(this, lastScheduledTime);
  }
}

void Pre::resetState() {
  if (kind == K_LOGICAL) {  // LogicalPreStateProcessor.resetState (:87-110)
    if (!isAnd || pending.size() == partner->pending.size()) {
      pending.clear();
      partner->pending.clear();
      if (isStartState && newEvery.empty()) {
        if (seq && thisPost->nextEveryStatePre == nullptr && thisPost->nextStatePre &&
            !thisPost->nextStatePre->pending.empty())
          return;
        init();
      }
    }
    return;
  }
  if (kind == K_ABSENT) {   // AbsentStreamPreStateProcessor.resetState
    pending.clear();
    if (isStartState) {
      if (seq && thisPost->nextEveryStatePre == nullptr && thisPost->nextStatePre &&
          !thisPost->nextStatePre->pending.empty())
        return;
      init();
    }
    return;
  }
  pending.clear();
  if (isStartState && newEvery.empty()) {
    if (seq && thisPost->nextEveryStatePre == nullptr && thisPost->nextStatePre &&
        !thisPost->nextStatePre->pending.empty())
      return;
    init();
  }
}

static void sort_by_ts(std::list<StateEvent*>& l) {
  // LinkedList.sort(eventTimeComparator) — stable, ts == -1 sorts last
  l.sort([](const StateEvent* a, const StateEvent* b) {
    if (a->ts == -1) return false;
    if (b->ts == -1) return true;
    return a->ts < b->ts;
  });
}

void Pre::updateState() {
  if (kind == K_COUNT && startStateReset) {  // CountPreStateProcessor.updateState (:183-193)
    startStateReset = false;
    init();
  }
  sort_by_ts(newEvery);
  pending.splice(pending.end(), newEvery);
  if (kind == K_LOGICAL && partner) {  // moveAllNewAndEveryStateEventListEventsToPendingStateEventList
    sort_by_ts(partner->newEvery);
    partner->pending.splice(partner->pending.end(), partner->newEvery);
  }
}

bool Pre::isExpired(StateEvent* se, int64_t ts) {
  if (withinTime == -1) return false;
  for (int s : startStateIds) {
    StreamEvent* e = se->slots[s];
    if (e != nullptr) {
      int64_t d = e->ts - ts;
      if (d < 0) d = -d;
      if (d > withinTime) return true;
    }
  }
  return false;
}

void Pre::expireEvents(int64_t ts) {   // StreamPreStateProcessor.expireEvents (:325-361)
  StateEvent* expired = nullptr;
  for (auto it = pending.begin(); it != pending.end();) {
    StateEvent* se = *it;
    if (isExpired(se, ts)) {
      it = pending.erase(it);
      if (se->type != EXPIRED) { se->type = EXPIRED; expired = se; }
    } else {
      break;
    }
  }
  for (auto it = newEvery.begin(); it != newEvery.end();) {
    StateEvent* se = *it;
    if (isExpired(se, ts)) {
      it = newEvery.erase(it);
      if (se->type != EXPIRED) { se->type = EXPIRED; expired = se; }
    } else {
      ++it;
    }
  }
  if (expired && withinEveryPre) {
    withinEveryPre->addEveryState(expired);
    withinEveryPre->updateState();
  }
}

void Pre::processChain(StateEvent* se) {
  stateChanged = false;
  EvalCtx c; c.se = se;
  for (Ex* f : filters) {
    Val v = eval(f, c);
    if (v.null || !v.b) return;  // FilterProcessor drops the event
  }
  thisPost->process(se);
}

std::vector<StateEvent*> Pre::processAndReturn(StreamEvent* ev) {
  if (absentLogical) return absentLogicalProcessAndReturn(ev);
  std::vector<StateEvent*> ret;
  Pool* pool = rt->pool;
  if (kind == K_ABSENT) {
    // AbsentStreamPreStateProcessor.processAndReturn: runs Stream logic, always returns empty
    if (!active) return ret;
  }
  if (kind == K_COUNT) {   // CountPreStateProcessor.processAndReturn (:53-95)
    for (auto it = pending.begin(); it != pending.end();) {
      StateEvent* se = *it;
      if ((int)se->slots.size() > stateId + 1 && se->slots[stateId + 1] != nullptr) { it = pending.erase(it); continue; }
      if ((int)se->slots.size() > stateId + 2 && se->slots[stateId + 2] != nullptr) { it = pending.erase(it); continue; }
      StreamEvent* clone = pool->copy(ev);
      // StateEvent.addEvent (:212-222)
      if (se->slots[stateId] == nullptr) se->slots[stateId] = clone;
      else { StreamEvent* t = se->slots[stateId]; while (t->next) t = t->next; t->next = clone; }
      successCondition = false;
      processChain(se);
      if (thisLast->isEventReturned) { thisLast->isEventReturned = false; ret.push_back(se); }
      bool removed = false;
      if (stateChanged) { it = pending.erase(it); removed = true; }
      if (!successCondition) {
        // StateEvent.removeLastEvent (:224-236)
        StreamEvent* h = se->slots[stateId];
        if (h) {
          StreamEvent* t = h;
          bool done = false;
          while (t->next) {
            if (t->next->next == nullptr) { t->next = nullptr; done = true; break; }
            t = t->next;
          }
          if (!done) se->slots[stateId] = nullptr;
        }
        if (seq && !removed) { it = pending.erase(it); removed = true; }
      }
      if (!removed) ++it;
    }
    return ret;
  }
  for (auto it = pending.begin(); it != pending.end();) {
    StateEvent* se = *it;
    if (kind == K_LOGICAL && !isAnd && se->slots[partner->stateId] != nullptr) {
      it = pending.erase(it);
      continue;
    }
    StreamEvent* clone = pool->copy(ev);
    se->slots[stateId] = clone;
    processChain(se);
    if (thisLast->isEventReturned) { thisLast->isEventReturned = false; ret.push_back(se); }
    if (stateChanged) {
      it = pending.erase(it);
    } else {
      se->slots[stateId] = nullptr;
      pool->release(clone);
      if (seq) {
        if (kind != K_ABSENT) { it = pending.erase(it); }   // removeOnNoStateChange (Absent: false)
        else ++it;
        if (kind == K_STREAM || kind == K_ABSENT) {
          if (thisPost->callbackPre) thisPost->callbackPre->countStartStateReset();
        }
      } else {
        ++it;
      }
    }
  }
  if (kind == K_ABSENT) ret.clear();
  return ret;
}

void Pre::countStartStateReset() {   // CountPreStateProcessor.startStateReset (:168-181)
  startStateReset = true;
  if (thisPost->callbackPre != nullptr) countPost->thisPre->countStartStateReset();
}

// ---- Post implementations ----
void Post::streamProcess(StateEvent* se) {   // StreamPostStateProcessor.process (:64-83)
  thisPre->stateChanged = true;
  se->ts = se->slots[stateId]->ts;
  if (hasNext) isEventReturned = true;
  if (nextStatePre) nextStatePre->addState(se);
  if (nextEveryStatePre) nextEveryStatePre->addEveryState(se);
  if (callbackPre) callbackPre->countStartStateReset();
}

void Post::processMinCountReached(StateEvent* se) {  // CountPostStateProcessor (:67-79)
  if (hasNext) { thisPre->stateChanged = true; isEventReturned = true; }
  if (nextStatePre) nextStatePre->addState(se);
  if (nextEveryStatePre) nextEveryStatePre->addEveryState(se);
}

void Post::process(StateEvent* se) {
  switch (kind) {
    case P_COUNT: {   // CountPostStateProcessor.process (:39-65)
      StreamEvent* e = se->slots[stateId];
      int n = 1;
      while (e->next) { n++; e = e->next; }
      thisPre->successCondition = true;
      se->ts = e->ts;
      if (n >= minCount) {
        if (thisPre->seq) {
          if (nextStatePre) nextStatePre->addState(se);
          if (n != maxCount) thisPre->addState(se);
        } else if (n == minCount) {
          processMinCountReached(se);
        }
        if (n == maxCount) thisPre->stateChanged = true;
      }
      return;
    }
    case P_LOGICAL: {  // LogicalPostStateProcessor.process (:59-87)
      if (isAnd) {
        bool go = false;
        if (partnerPre->absentLogical) go = partnerPre->partnerCanProceed(se);
        else if (se->slots[partnerPre->stateId] != nullptr) go = true;
        if (go) streamProcess(se);
        else thisPre->stateChanged = true;
      } else {
        streamProcess(se);
        if (partnerPost->hasNext && thisPre->thisLast == partnerPost) partnerPost->isEventReturned = true;
      }
      return;
    }
    case P_ABSENT_LOGICAL: {   // AbsentLogicalPostStateProcessor.process (:36-47)
      thisPre->stateChanged = true;
      isEventReturned = true;
      thisPre->lastArrivalTime = se->slots[stateId]->ts;   // updateLastArrivalTime (:66-75)
      return;
    }
    case P_ABSENT: {   // AbsentStreamPostStateProcessor.process (:36-56)
      thisPre->stateChanged = true;
      StreamEvent* e = se->slots[stateId];
      se->ts = e->ts;
      isEventReturned = true;
      if (thisPre->isStartState) {
        if (nextEveryStatePre != nullptr && nextEveryStatePre == thisPre) nextEveryStatePre->addEveryState(se);
      }
      thisPre->updateLastArrivalTime(e->ts);
      return;
    }
    default:
      streamProcess(se);
  }
}

void Post::setNextStatePre(Pre* p) {
  nextStatePre = p;
  if (kind == P_LOGICAL || kind == P_ABSENT_LOGICAL) partnerPost->nextStatePre = p;
  if (kind == P_COUNT) {  // CountPostStateProcessor.setNextStatePreProcessor (:81-89)
    if (thisPre->isStartState && thisPre->seq && minCount == 0) p->thisPost->callbackPre = thisPre;
  }
}

void Post::setNextEveryStatePre(Pre* p) {
  nextEveryStatePre = p;
  if (kind == P_LOGICAL || kind == P_ABSENT_LOGICAL) partnerPost->nextEveryStatePre = p;
}

}  // namespace orc

// ================================================================================================
// Part 2: query construction (StateInputStreamParser restated), app, junctions, time, C ABI
// ================================================================================================
namespace orc {

struct App;

struct Timer {     // one Scheduler state (per processor per partition instance)
  std::deque<int64_t> q;      // toNotifyQueue: a LinkedBlockingQueue, FIFO (Scheduler.java:332)
};

// java.util.HashMap<String, ...> restated for iteration order (JDK 8 HashMap.computeIfAbsent /
// remove / resize): a bin is a chain, computeIfAbsent inserts at the HEAD of its bin and resizes
// first when size > threshold; resize splits every bin into lo/hi preserving relative order; a bin
// reaching TREEIFY_THRESHOLD resizes while the table is < 64 (treeified bins are not restated).
// Used for the partition-keyed Scheduler state maps (PartitionStateHolder.states), whose iteration
// order picks the instance that fires when several share a deadline (Scheduler.java:74-104).
struct JMap {
  struct E { int32_t hash; QueryRT* rt; };
  std::vector<std::vector<E>> tab;   // bin -> chain (index 0 = head)
  size_t size = 0, thr = 0;
  static int32_t spread(int32_t h) { return h ^ (int32_t)((uint32_t)h >> 16); }
  void resize() {
    size_t oldCap = tab.size();
    if (oldCap == 0) { tab.assign(16, {}); thr = 12; return; }
    std::vector<std::vector<E>> nt(oldCap * 2);
    for (size_t b = 0; b < oldCap; b++)
      for (const E& e : tab[b]) nt[((uint32_t)e.hash & (uint32_t)oldCap) ? b + oldCap : b].push_back(e);
    tab.swap(nt);
    thr *= 2;
  }
  void compute_if_absent(int32_t h, QueryRT* rt) {
    if (size > thr || tab.empty()) resize();
    auto& bin = tab[(uint32_t)h & (uint32_t)(tab.size() - 1)];
    for (const E& e : bin) if (e.rt == rt) return;
    size_t binCount = bin.size();
    bin.insert(bin.begin(), E{h, rt});
    if (binCount >= 7) {   // treeifyBin
      if (tab.size() < 64) resize();
      else throw std::runtime_error("partition scheduler map bin treeified (not restated)");
    }
    size++;
  }
  void remove(QueryRT* rt, int32_t h) {
    if (tab.empty()) return;
    auto& bin = tab[(uint32_t)h & (uint32_t)(tab.size() - 1)];
    for (size_t i = 0; i < bin.size(); i++)
      if (bin[i].rt == rt) { bin.erase(bin.begin() + i); size--; return; }
  }
};

struct QueryDef {
  int index = 0;
  std::string name;
  J desc;                 // the query descriptor
  bool partitioned = false;
  std::map<int, int> partition_attr;   // stream idx -> attr idx
  int partition_id = -1;               // the `partition ... begin ... end` block
  bool purge = false;                  // @purge(enable='true', ...) on that block
  bool state = false;
  std::vector<Ty> out_types;
  int out_kind = 0;        // 0 = return, 1 = insert
  int out_stream = -1;
  bool currentOn = true, expiredOn = false;
  std::vector<int> input_streams;
};

struct SchedulerReg {   // Scheduler object identity = (query, processor index or window)
  int query = 0;
  int proc = -1;        // -1 = time window
  JMap states;          // partitioned: PartitionSyncStateHolder's key -> SchedulerState map
};

// @purge of one partition block (PartitionRuntimeImpl.java:79-81, 120-147, 346-402).  initPartition
// (once per key chunk sent into the partition, PartitionStreamReceiver.send :261-272) records the key's
// last-seen time and schedules a purge task every `interval` from that moment (a new task per call);
// a task at time c removes every key with lastSeen + idle < c and cleans all of the partition's query
// states for it (PartitionStateHolder.cleanGroupByStates), so the key's next chunk re-initialises it.
// Restated on the app clock (the reference's tasks run on the wall clock even in playback).  Removal is
// observable only when the key is touched again (an event, a timer, a broadcast), so it is applied there:
// a key is purged by time T iff some task time c lies in (lastSeen + idle, T].
struct PurgeState {
  int64_t interval = 300000, idle = 0;
  std::map<int64_t, int64_t> first;            // task-time residue mod interval -> earliest call time
  int64_t t0 = INT64_MAX;                       // earliest initPartition call
  std::map<std::pair<int, int64_t>, int64_t> last;   // partitionKeys: key -> last initPartition time
  static int64_t mod(int64_t a, int64_t m) { int64_t r = a % m; return r < 0 ? r + m : r; }
  void note(int64_t t) {
    auto it = first.find(mod(t, interval));
    if (it == first.end()) first[mod(t, interval)] = t;
    else it->second = std::min(it->second, t);
    t0 = std::min(t0, t);
  }
  // does a task fire in (A, T]?  Tasks of a call at time f fire at f + k*interval, k >= 1
  bool task_in(int64_t A, int64_t T) const {
    if (T <= A || first.empty() || T < t0 + interval) return false;
    if (T - A >= interval) return true;               // the earliest call's task fires in any such span
    const int64_t ra = mod(A + 1, interval), rb = mod(T, interval);
    auto hit = [&](int64_t r) {                       // the one time c == r (mod interval) in (A, T]
      const int64_t c = A + 1 + mod(r - (A + 1), interval);
      auto it = first.find(r);
      return c <= T && c >= it->second + interval;
    };
    if (ra <= rb) {
      for (auto it = first.lower_bound(ra); it != first.end() && it->first <= rb; ++it) if (hit(it->first)) return true;
    } else {
      for (auto it = first.lower_bound(ra); it != first.end(); ++it) if (hit(it->first)) return true;
      for (auto it = first.begin(); it != first.end() && it->first <= rb; ++it) if (hit(it->first)) return true;
    }
    return false;
  }
  bool purged(const std::pair<int, int64_t>& key, int64_t T) const {
    auto it = last.find(key);
    return it != last.end() && task_in(it->second + idle, T);
  }
};

struct App {
  J desc;
  bool playback = false;
  std::map<int, PurgeState> purges;                     // partition block -> its @purge state
  std::vector<std::unique_ptr<QueryRT>> purged_rts;     // cleaned instances (kept alive, never used)
  void purge_key(int part, const std::pair<int, int64_t>& key);
  bool purge_check(QueryRT* rt, int64_t T);             // a timer/broadcast touch: purge if due
  void init_partition_call(int qi, const std::pair<int, int64_t>& key);
  std::vector<std::string> stream_names;
  std::vector<std::vector<Ty>> stream_types;
  std::map<std::string, int> stream_idx;
  std::vector<std::string> strings;
  std::unordered_map<std::string, int> string_ids;
  std::vector<std::unique_ptr<QueryDef>> qdefs;
  Pool pool;
  // unpartitioned runtimes (one per query) / partitioned (per key)
  std::vector<std::unique_ptr<QueryRT>> single_rt;   // index by query (null when partitioned)
  std::vector<std::map<std::pair<int, int64_t>, std::unique_ptr<QueryRT>>> part_rt;
  std::vector<std::vector<QueryRT*>> part_order;       // creation order of partition instances
  std::vector<std::vector<std::string>> part_key_str;  // key.toString() per instance
  // junction subscriptions: stream -> list of query indices (subscription order)
  std::vector<std::vector<int>> subscribers;
  // callbacks
  std::vector<bool> query_cb;        // QueryCallback registered for query i
  std::vector<bool> stream_cb;       // StreamCallback registered for stream i
  std::vector<Callback> out;
  // time
  int64_t now = 0;                   // TimestampGenerator.currentTime()
  int64_t lastEventTimestamp = INT64_MIN;
  std::vector<SchedulerReg> schedulers;                 // creation order
  int64_t cur_seq = 0;                                  // arrival index of the event being sent
  int64_t nsent = 0;                                    // events sent so far
  std::map<std::pair<QueryRT*, int>, Timer> timers;     // (instance, proc or -1) -> queue
  std::map<std::pair<int, int>, int> reg_of;            // (query, proc) -> index in schedulers
  void notify_at(QueryRT* rt, int proc, int64_t t);     // Scheduler.notifyAt (:113-126)
  bool started = false;

  int intern(const std::string& s) {
    auto it = string_ids.find(s);
    if (it != string_ids.end()) return it->second;
    int id = (int)strings.size();
    strings.push_back(s);
    string_ids[s] = id;
    return id;
  }

  QueryRT* build(int qi);
  QueryRT* instance(int qi, const Val* data, int stream);
  void junction_send(int stream, const std::vector<std::pair<int64_t, const Val*>>& evs, bool batch);
  void send(int stream, const std::vector<std::pair<int64_t, const Val*>>& evs, bool batch);
  void set_time(int64_t t);
  void fire_timers(int64_t t);
  void start();
  std::vector<QueryRT*> java_hashset_order(int qi);
};

// --------------------------------------------------------------------------------------------
// Expression construction from the descriptor
// --------------------------------------------------------------------------------------------
static std::unique_ptr<Ex> build_ex(App& app, const J& j, Selector* sel) {
  auto x = std::make_unique<Ex>();
  const std::string& op = j["op"].s;
  x->t = ty_of(j["t"].s);
  if (op == "const") {
    x->op = O_CONST;
    const J& v = j["v"];
    switch (x->t) {
      case T_INT: x->c = Val::I((int32_t)v.as_int()); break;
      case T_LONG: x->c = Val::L(v.as_int()); break;
      case T_FLOAT: x->c = Val::F((float)v.n); break;
      case T_DOUBLE: x->c = Val::D(v.n); break;
      case T_BOOL: x->c = Val::B(v.b); break;
      case T_STRING: x->c = Val::S(app.intern(v.s)); break;
      default: x->c = Val::N(T_OBJECT);
    }
  } else if (op == "var") {
    x->op = O_VAR; x->slot = (int)j["slot"].as_int(); x->chain = (int)j["chain"].as_int(); x->attr = (int)j["attr"].as_int();
  } else if (op == "outvar") {
    x->op = O_OUTVAR; x->attr = (int)j["attr"].as_int();
  } else if (op == "and" || op == "or") {
    x->op = op == "and" ? O_AND : O_OR;
    x->a = build_ex(app, j["a"], sel); x->b = build_ex(app, j["b"], sel);
  } else if (op == "not" || op == "isnull") {
    x->op = op == "not" ? O_NOT : O_ISNULL;
    x->a = build_ex(app, j["a"], sel);
  } else if (op == ">" || op == "<" || op == ">=" || op == "<=" || op == "==" || op == "!=") {
    x->op = op == ">" ? O_GT : op == "<" ? O_LT : op == ">=" ? O_GE : op == "<=" ? O_LE : op == "==" ? O_EQ : O_NE;
    x->ct = ty_of(j["ct"].s);
    x->a = build_ex(app, j["a"], sel); x->b = build_ex(app, j["b"], sel);
  } else if (op == "+" || op == "-" || op == "*" || op == "/" || op == "%") {
    x->op = op == "+" ? O_ADD : op == "-" ? O_SUB : op == "*" ? O_MUL : op == "/" ? O_DIV : O_MOD;
    x->a = build_ex(app, j["a"], sel); x->b = build_ex(app, j["b"], sel);
  } else if (op == "agg") {
    if (!sel) throw std::runtime_error("aggregator outside selector");
    x->op = O_AGG;
    AggSpec s;
    const std::string& n = j["name"].s;
    if (n == "sum") s.k = A_SUM; else if (n == "avg") s.k = A_AVG; else if (n == "count") s.k = A_COUNT;
    else if (n == "min") s.k = A_MIN; else if (n == "max") s.k = A_MAX;
    else throw std::runtime_error("unsupported aggregator " + n);
    if (j["args"].size() > 0) { s.arg = build_ex(app, j["args"][0], nullptr); s.in_t = s.arg->t; }
    x->agg_idx = (int)sel->aggs.size();
    sel->aggs.push_back(std::move(s));
    sel->containsAgg = true;
  } else {
    throw std::runtime_error("unsupported expression op " + op);
  }
  return x;
}

// --------------------------------------------------------------------------------------------
// StateInputStreamParser.parse restated (CORE/util/parser/StateInputStreamParser.java:148-408)
// --------------------------------------------------------------------------------------------
struct Builder {
  App& app;
  QueryRT& rt;
  std::vector<std::unique_ptr<Ex>>& exprs;
  bool seq;

  std::unique_ptr<Inner> parse(const J& el, Pre* pre, Post* post, std::vector<Pre*>& preList, bool isStart) {
    const std::string& k = el["k"].s;
    if (k == "stream" || k == "absent") {
      int stateIndex = (int)el["slot"].as_int();
      int stream = app.stream_idx.at(el["stream"].s);
      if (!pre) {
        rt.pres.emplace_back(new Pre());
        pre = rt.pres.back().get();
        pre->kind = k == "absent" ? K_ABSENT : K_STREAM;
        if (k == "absent") { pre->waitingTime = el["wait"].as_int(); rt.startupPre.push_back(pre); }
        pre->rt = &rt; pre->seq = seq;
      }
      pre->stateId = stateIndex;
      pre->isStartState = isStart;
      for (size_t i = 0; i < el["filters"].size(); i++) {
        exprs.push_back(build_ex(app, el["filters"][i], nullptr));
        pre->filters.push_back(exprs.back().get());
      }
      if (!post) {
        rt.posts.emplace_back(new Post());
        post = rt.posts.back().get();
        post->kind = k == "absent" ? P_ABSENT : P_STREAM;
      }
      post->stateId = stateIndex;
      post->thisPre = pre;
      pre->thisPost = post;
      pre->thisLast = post;
      auto in = std::make_unique<Inner>();
      in->k = Inner::STREAM; in->first = pre; in->last = post;
      in->streamsList.push_back(el["stream"].s);
      in->streamFirstProcs.push_back(pre);
      (void)stream;
      preList.push_back(pre);
      return in;
    }
    if (k == "next") {
      auto cur = parse(el["a"], pre, post, preList, isStart);
      auto nxt = parse(el["b"], pre, post, preList, false);
      cur->last->setNextStatePre(nxt->first);
      auto in = std::make_unique<Inner>();
      in->k = Inner::NEXT; in->first = cur->first; in->last = nxt->last;
      for (auto& s : cur->streamsList) in->streamsList.push_back(s);
      for (auto* p : cur->streamFirstProcs) in->streamFirstProcs.push_back(p);
      for (auto& s : nxt->streamsList) in->streamsList.push_back(s);
      for (auto* p : nxt->streamFirstProcs) in->streamFirstProcs.push_back(p);
      in->a = std::move(cur); in->b = std::move(nxt);
      return in;
    }
    if (k == "every") {
      std::vector<Pre*> withinEvery;
      auto inner = parse(el["e"], pre, post, withinEvery, isStart);
      auto in = std::make_unique<Inner>();
      in->k = Inner::EVERY; in->first = inner->first; in->last = inner->last;
      in->streamsList = inner->streamsList; in->streamFirstProcs = inner->streamFirstProcs;
      in->last->setNextEveryStatePre(in->first);
      for (Pre* p : withinEvery) p->withinEveryPre = in->first;
      for (Pre* p : withinEvery) preList.push_back(p);
      in->a = std::move(inner);
      return in;
    }
    if (k == "logical") {
      bool isAnd = el["op"].s == "AND";
      auto mk = [&](const J& sub) {
        rt.pres.emplace_back(new Pre());
        Pre* p = rt.pres.back().get();
        p->kind = K_LOGICAL; p->isAnd = isAnd; p->rt = &rt; p->seq = seq;
        rt.posts.emplace_back(new Post());
        Post* q = rt.posts.back().get();
        q->kind = P_LOGICAL; q->isAnd = isAnd;
        if (sub["k"].s == "absent") {   // AbsentLogicalPreStateProcessor + AbsentLogicalPostStateProcessor (:289-335)
          p->absentLogical = true;
          p->waitingTime = sub["wait"].null() ? -1 : sub["wait"].as_int();
          rt.startupPre.push_back(p);
          q->kind = P_ABSENT_LOGICAL;
        }
        return std::make_pair(p, q);
      };
      auto [pre1, post1] = mk(el["a"]);
      auto [pre2, post2] = mk(el["b"]);
      post1->partnerPre = pre2; post2->partnerPre = pre1;
      post1->partnerPost = post2; post2->partnerPost = post1;
      pre1->partner = pre2; pre2->partner = pre1;
      auto r2 = parse(el["b"], pre2, post2, preList, isStart);
      auto r1 = parse(el["a"], pre1, post1, preList, isStart);
      auto in = std::make_unique<Inner>();
      in->k = Inner::LOGICAL; in->first = r1->first; in->last = r2->last;
      for (auto& s : r2->streamsList) in->streamsList.push_back(s);
      for (auto* p : r2->streamFirstProcs) in->streamFirstProcs.push_back(p);
      for (auto& s : r1->streamsList) in->streamsList.push_back(s);
      for (auto* p : r1->streamFirstProcs) in->streamFirstProcs.push_back(p);
      in->a = std::move(r1); in->b = std::move(r2);
      return in;
    }
    if (k == "count") {
      int mn = (int)el["min"].as_int(), mx = (int)el["max"].as_int();
      if (mn == -1) mn = 0;
      if (mx == -1) mx = INT32_MAX;
      rt.pres.emplace_back(new Pre());
      Pre* p = rt.pres.back().get();
      p->kind = K_COUNT; p->minCount = mn; p->maxCount = mx; p->rt = &rt; p->seq = seq;
      rt.posts.emplace_back(new Post());
      Post* q = rt.posts.back().get();
      q->kind = P_COUNT; q->minCount = mn; q->maxCount = mx;
      p->countPost = q;
      auto inner = parse(el["e"], p, q, preList, isStart);
      inner->k = Inner::COUNT;
      return inner;
    }
    throw std::runtime_error("unknown state element " + k);
  }
};

// setup(): receivers' setNext / addStatefulProcessorForStream in setup order
static void setup(App& app, QueryRT& rt, Inner* in) {
  switch (in->k) {
    case Inner::STREAM: case Inner::COUNT: {
      int s = app.stream_idx.at(in->streamsList[0]);
      Receiver& r = rt.receivers[s];
      r.stream = s;
      r.nexts.push_back(in->first);
      r.forStream.push_back(in->first);
      break;
    }
    case Inner::NEXT: setup(app, rt, in->a.get()); setup(app, rt, in->b.get()); break;
    case Inner::EVERY: setup(app, rt, in->a.get()); break;
    case Inner::LOGICAL: setup(app, rt, in->b.get()); setup(app, rt, in->a.get()); break;
  }
}

static void build_selector(App& app, QueryRT& rt, const QueryDef& qd, std::vector<std::unique_ptr<Ex>>& exprs) {
  const J& s = qd.desc["select"];
  Selector& sel = rt.sel;
  for (size_t i = 0; i < s["attrs"].size(); i++) sel.attrs.push_back(build_ex(app, s["attrs"][i]["e"], &sel));
  for (size_t i = 0; i < s["group_by"].size(); i++) sel.group_by.push_back(build_ex(app, s["group_by"][i], nullptr));
  sel.groupBy = !sel.group_by.empty();
  if (!s["having"].null()) sel.having = build_ex(app, s["having"], &sel);
  for (size_t i = 0; i < s["order_by"].size(); i++)
    sel.order_by.emplace_back(build_ex(app, s["order_by"][i][0], nullptr), s["order_by"][i][1].s == "desc");
  if (!s["limit"].null()) sel.limit = s["limit"].as_int();
  if (!s["offset"].null()) sel.offset = s["offset"].as_int();
  sel.currentOn = qd.currentOn; sel.expiredOn = qd.expiredOn;
  sel.strings = &app.strings;
  sel.partitioned = qd.partitioned;
  sel.out_types = qd.out_types;
  (void)exprs;
}

QueryRT* App::build(int qi) {
  const QueryDef& qd = *qdefs[qi];
  auto* rt = new QueryRT();
  rt->app = this; rt->def = &qd; rt->pool = &pool;
  static thread_local std::vector<std::unique_ptr<Ex>>* unused = nullptr; (void)unused;
  auto* exprs = new std::vector<std::unique_ptr<Ex>>();   // owned for the app lifetime
  const J& inp = qd.desc["input"];
  if (inp["kind"].s == "state") {
    rt->seq = inp["type"].s == "SEQUENCE";
    rt->nslots = (int)inp["slots"].size();
    Builder b{*this, *rt, *exprs, rt->seq};
    rt->inner = b.parse(inp["element"], nullptr, nullptr, rt->allPre, true);
    if (!inp["within"].null()) {
      std::vector<int> startIds;
      for (Pre* p : rt->allPre) if (p->isStartState) startIds.push_back(p->stateId);
      for (Pre* p : rt->allPre) { p->startStateIds = startIds; p->withinTime = inp["within"].as_int(); }
    }
    rt->inner->first->thisLast = rt->inner->last;
    // setCommonProcessor: setQuerySelector then setup
    std::function<void(Inner*)> setq = [&](Inner* in) {
      switch (in->k) {
        case Inner::STREAM: case Inner::COUNT: in->last->hasNext = true; break;
        case Inner::NEXT: setq(in->b.get()); break;
        case Inner::EVERY: setq(in->a.get()); break;
        case Inner::LOGICAL: setq(in->b.get()); setq(in->a.get()); break;
      }
    };
    setq(rt->inner.get());
    setup(*this, *rt, rt->inner.get());
    for (auto& kv : rt->receivers) kv.second.multi = kv.second.nexts.size() > 1;
  } else {
    for (size_t i = 0; i < inp["handlers"].size(); i++) {
      const J& h = inp["handlers"][i];
      if (h["k"].s == "filter") {
        exprs->push_back(build_ex(*this, h["e"], nullptr));
        rt->sfilters.push_back(exprs->back().get());
      } else {
        const std::string& n = h["name"].s;
        const J& p0 = h["params"][0];
        if (n == "length") rt->win.k = Window::LENGTH;
        else if (n == "time") rt->win.k = Window::TIME;
        else if (n == "lengthBatch") rt->win.k = Window::LENGTH_BATCH;
        else throw std::runtime_error("unsupported window " + n);
        rt->win.param = p0["v"].as_int();
        if (h["params"].size() > 1) rt->win.streamCurrent = h["params"][1]["v"].b;
        if (!rt->sfilters.empty() && i + 1 < inp["handlers"].size())
          ;  // post-window filters are applied after the window below
      }
    }
  }
  build_selector(*this, *rt, qd, *exprs);
  // min/max trackFutureStates = SLIDE processing mode || outputExpectsExpiredEvents
  bool slide = rt->win.k == Window::LENGTH || rt->win.k == Window::TIME;
  for (auto& a : rt->sel.aggs) a.track = slide || qd.expiredOn;
  return rt;
}

// StateStreamRuntime.initPartition: inner.init() then startup processors partitionCreated()
static void init_partition(App& app, QueryRT* rt) {
  if (!rt->inner) return;
  rt->inner->init();
  for (Pre* p : rt->startupPre) {   // partitionCreated (Absent :296-310, AbsentLogical :387-404)
    if (!p->started) {
      p->started = true;
      if (p->isStartState && p->waitingTime != -1 && p->active) {
        if (p->absentLogical) { rt->app_notify_at(p, app.now + p->waitingTime); continue; }
        p->lastScheduledTime = app.now + p->waitingTime;
        rt->app_notify_at(p, p->lastScheduledTime);
      }
    }
  }
}

// Java String.hashCode over the key's toString() (ASCII)
static int32_t java_string_hash(const std::string& s) {
  uint32_t h = 0;
  for (unsigned char c : s) h = 31u * h + c;
  return (int32_t)h;
}

void App::notify_at(QueryRT* rt, int proc, int64_t t) {
  timers[{rt, proc}].q.push_back(t);
  // PartitionSyncStateHolder.getState: states.computeIfAbsent(partitionKey) on this scheduler's map
  if (rt->def->partitioned) schedulers[reg_of.at({rt->def->index, proc})].states.compute_if_absent(rt->key_hash, rt);
}

QueryRT* App::instance(int qi, const Val* data, int stream) {
  const QueryDef& qd = *qdefs[qi];
  if (!qd.partitioned) return single_rt[qi].get();
  auto it = qd.partition_attr.find(stream);
  if (it == qd.partition_attr.end()) return nullptr;
  const Val& kv = data[it->second];
  if (kv.null) return nullptr;   // null key: event dropped
  auto key = kv.key();
  auto& m = part_rt[qi];
  auto f = m.find(key);
  if (f != m.end()) return f->second.get();
  QueryRT* rt = build(qi);
  rt->pkey = key;
  m[key].reset(rt);
  part_order[qi].push_back(rt);
  std::string ks;
  switch (kv.t) {
    case T_STRING: ks = strings[kv.s]; break;
    case T_INT: ks = std::to_string(kv.i); break;
    case T_LONG: ks = std::to_string(kv.l); break;
    case T_BOOL: ks = kv.b ? "true" : "false"; break;
    default: ks = std::to_string(part_order[qi].size());
  }
  part_key_str[qi].push_back(ks);
  rt->key_hash = JMap::spread(java_string_hash(ks));
  init_partition(*this, rt);
  return rt;
}

// the purge task's removal of `key`: partitionKeys.remove + cleanGroupByStates of every query state of
// the partition (its Scheduler states included)
void App::purge_key(int part, const std::pair<int, int64_t>& key) {
  purges[part].last.erase(key);
  for (size_t qi = 0; qi < qdefs.size(); qi++) {
    if (qdefs[qi]->partition_id != part || !qdefs[qi]->partitioned) continue;
    auto f = part_rt[qi].find(key);
    if (f == part_rt[qi].end()) continue;
    QueryRT* rt = f->second.get();
    for (auto it = timers.begin(); it != timers.end();) {
      if (it->first.first == rt) it = timers.erase(it); else ++it;
    }
    for (auto& reg : schedulers) if (reg.query == (int)qi) reg.states.remove(rt, rt->key_hash);
    auto& ord = part_order[qi];
    for (size_t i = 0; i < ord.size(); i++) {
      if (ord[i] != rt) continue;
      ord.erase(ord.begin() + i);
      part_key_str[qi].erase(part_key_str[qi].begin() + i);
      break;
    }
    purged_rts.push_back(std::move(f->second));
    part_rt[qi].erase(f);
  }
}

bool App::purge_check(QueryRT* rt, int64_t T) {
  const QueryDef& qd = *rt->def;
  if (!qd.partitioned || !qd.purge) return false;
  if (!purges[qd.partition_id].purged(rt->pkey, T)) return false;
  purge_key(qd.partition_id, rt->pkey);
  return true;
}

// PartitionRuntimeImpl.initPartition for one key chunk: tasks due by now ran first (a purged key is
// re-initialised by this call), then the key's last-seen time and this call's task schedule
void App::init_partition_call(int qi, const std::pair<int, int64_t>& key) {
  const QueryDef& qd = *qdefs[qi];
  if (!qd.purge) return;
  PurgeState& ps = purges[qd.partition_id];
  if (ps.purged(key, now)) purge_key(qd.partition_id, key);
  ps.note(now);
  ps.last[key] = now;
}

// --------------------------------------------------------------------------------------------
// Output (OutputRateLimiter.sendToCallBacks / QueryCallback / InsertIntoStreamCallback)
// --------------------------------------------------------------------------------------------
void QueryRT::emitChunk(std::vector<SelEvent>& outv) {
  if (outv.empty()) return;
  App& a = *app;
  const QueryDef& qd = *def;
  if (a.query_cb[qd.index]) {
    Callback cb; cb.kind = 0; cb.target = qd.index; cb.ts = -1; cb.seq = a.cur_seq;
    for (auto& e : outv) {
      OutEvent oe{e.ts, e.type == EXPIRED, e.out};
      if (e.type == EXPIRED) cb.rm.push_back(oe);
      else if (e.type == CURRENT) cb.in.push_back(oe);
      cb.ts = e.ts;
    }
    a.out.push_back(std::move(cb));
  }
  if (qd.out_kind == 1) {
    // InsertIntoStreamCallback: EXPIRED -> CURRENT, RESET removed, publish to the junction
    std::vector<std::pair<int64_t, const Val*>> evs;
    for (auto& e : outv) {
      if (e.type == RESET) continue;
      a.pool.rows.emplace_back(e.out);
      evs.emplace_back(e.ts, a.pool.rows.back().data());
    }
    if (!evs.empty()) a.junction_send(qd.out_stream, evs, true);
  }
}

void QueryRT::selectAndEmit(StateEvent* se) {
  std::vector<SelEvent> chunk(1);
  chunk[0].se = se; chunk[0].type = se->type; chunk[0].ts = se->ts;
  auto outv = sel.process(chunk);
  for (auto& o : outv) se->out = o.out;
  if (outv.empty()) return;
  if (holder) { for (auto& o : outv) holder->push_back(o); return; }
  emitChunk(outv);
}

void QueryRT::deliverHolders(std::vector<std::vector<SelEvent>>& holders) {
  for (auto& h : holders) emitChunk(h);
}

// PatternMulti/SequenceMulti receiver, one event (MultiProcessStreamReceiver.java:216-241)
void QueryRT::receive(int stream, int64_t ts, const Val* data) {
  std::vector<std::pair<int64_t, const Val*>> v{{ts, data}};
  receiveBatch(stream, v);
}

void QueryRT::receiveBatch(int stream, const std::vector<std::pair<int64_t, const Val*>>& evs) {
  auto it = receivers.find(stream);
  if (it == receivers.end()) return;
  Receiver& r = it->second;
  if (!r.multi) { receiveSingle(stream, evs, true); return; }
  std::vector<std::vector<SelEvent>> holders;
  for (auto& e : evs) {
    // stabilizeStates (PatternMultiProcessStreamReceiver :42-50 / SequenceMulti :45-50)
    for (Pre* p : allPre) p->expireEvents(e.first);
    if (seq) { inner->reset(); inner->update(); }
    else for (Pre* p : r.forStream) p->updateState();
    for (int k = (int)r.nexts.size() - 1; k >= 0; k--) {
      StreamEvent* ev = pool->se();
      ev->ts = e.first; ev->data = e.second;
      std::vector<SelEvent> h;
      holder = &h;
      auto ret = r.nexts[k]->processAndReturn(ev);
      for (StateEvent* se : ret) selectAndEmit(se);
      holder = nullptr;
      if (!h.empty()) holders.push_back(std::move(h));
    }
  }
  deliverHolders(holders);
}

// PatternSingle/SequenceSingle receiver (SingleProcessStreamReceiver.java:48-73)
void QueryRT::receiveSingle(int stream, const std::vector<std::pair<int64_t, const Val*>>& evs, bool) {
  Receiver& r = receivers[stream];
  std::vector<StateEvent*> ret;
  for (auto& e : evs) {
    for (Pre* p : allPre) p->expireEvents(e.first);
    if (seq) { inner->reset(); inner->update(); }
    else if (!r.forStream.empty()) r.forStream[0]->updateState();
    StreamEvent* ev = pool->se();
    ev->ts = e.first; ev->data = e.second;
    auto rr = r.nexts[0]->processAndReturn(ev);
    for (auto* s : rr) ret.push_back(s);
  }
  for (StateEvent* se : ret) selectAndEmit(se);
}

// ---- absent timers ----
void QueryRT::app_notify_at(Pre* p, int64_t t) {
  int idx = -1;
  for (size_t i = 0; i < pres.size(); i++) if (pres[i].get() == p) idx = (int)i;
  app->notify_at(this, idx, t);
}

void Pre::updateLastArrivalTime(int64_t ts) {
  lastScheduledTime = ts + waitingTime;
  rt->app_notify_at(this, lastScheduledTime);
}

// AbsentStreamPreStateProcessor.process(TIMER chunk) (:150-227)
void Pre::absentTimer(int64_t currentTime) {
  // In a partitioned query the pre-state is dropped whenever its lists are empty and it is not an
  // initialised start state (StreamPreState.canDestroy :444-448 via PartitionSyncStateHolder.returnState),
  // so a non-start absent state reads a fresh lastScheduledTime (0) here.
  if (rt->def->partitioned && !isStartState && pending.empty() && newEvery.empty()) lastScheduledTime = 0;
  if (!active) return;
  bool notProcessed = true;
  std::vector<StateEvent*> ret;
  bool initialize = isStartState && newEvery.empty() && pending.empty();
  if (initialize && seq && thisPost->nextEveryStatePre == nullptr && lastScheduledTime > 0) initialize = false;
  if (initialize) {
    StateEvent* se = rt->newStateEvent();
    addState(se);
  } else if (seq && !newEvery.empty()) {
    resetState();
  }
  updateState();
  for (auto it = pending.begin(); it != pending.end();) {
    StateEvent* e = *it;
    if (isExpired(e, currentTime)) {
      it = pending.erase(it);
      if (withinEveryPre != nullptr && thisPost->nextEveryStatePre != this)
        thisPost->nextEveryStatePre->addEveryState(e);
      continue;
    }
    if ((e->ts == -1 && currentTime >= lastScheduledTime) || (e->ts != -1 && currentTime >= e->ts + waitingTime)) {
      it = pending.erase(it);
      e->ts = currentTime;
      ret.push_back(e);
      continue;
    }
    ++it;
  }
  if (withinEveryPre != nullptr) withinEveryPre->updateState();
  notProcessed = ret.empty();
  for (StateEvent* se : ret) {   // sendEvent
    if (thisPost->hasNext) rt->selectAndEmit(se);
    if (thisPost->nextStatePre) thisPost->nextStatePre->addState(se);
    if (thisPost->nextEveryStatePre) thisPost->nextEveryStatePre->addEveryState(se);
    else if (isStartState) active = false;
    if (thisPost->callbackPre) thisPost->callbackPre->countStartStateReset();
  }
  int64_t actual = rt->app->now;
  if (actual > waitingTime + currentTime) lastScheduledTime = actual + waitingTime;
  if (notProcessed && lastScheduledTime < currentTime) {
    lastScheduledTime = currentTime + waitingTime;
    rt->app_notify_at(this, lastScheduledTime);
  }
}


// ---- logical absent (AbsentLogicalPreStateProcessor.java:38-422) ----
// processAndReturn (:313-369): an arrival that passes the filter only records lastArrivalTime (via
// AbsentLogicalPostStateProcessor) and drops the candidate; nothing is ever returned
std::vector<StateEvent*> Pre::absentLogicalProcessAndReturn(StreamEvent* ev) {
  std::vector<StateEvent*> ret;
  if (!active) return ret;
  for (auto it = pending.begin(); it != pending.end();) {
    StateEvent* se = *it;
    if (!isAnd && se->slots[partner->stateId] != nullptr) { it = pending.erase(it); continue; }
    StreamEvent* cur = se->slots[stateId];
    se->slots[stateId] = rt->pool->copy(ev);
    processChain(se);
    if (waitingTime != -1 || (seq && isAnd && thisPost->nextEveryStatePre != nullptr)) se->slots[stateId] = cur;
    bool removed = false;
    if (thisLast->isEventReturned) {
      thisLast->isEventReturned = false;
      it = pending.erase(it);
      removed = true;
      if (seq) {   // LinkedList.remove(Object): first occurrence, identity equality
        auto f = std::find(partner->pending.begin(), partner->pending.end(), se);
        if (f != partner->pending.end()) partner->pending.erase(f);
      }
    }
    if (!stateChanged) {
      se->slots[stateId] = cur;
      if (seq && !removed) { it = pending.erase(it); removed = true; }
    }
    if (!removed) ++it;
  }
  return ret;
}

// partnerCanProceed (:371-399), asked by the present partner's LogicalPostStateProcessor (AND)
bool Pre::partnerCanProceed(StateEvent* se) {
  if (seq && thisPost->nextEveryStatePre == nullptr && lastArrivalTime > 0) return false;
  if (waitingTime == -1) {
    if (thisPost->nextEveryStatePre == nullptr) return se->slots[stateId] == nullptr;
    if (lastArrivalTime > 0) { lastArrivalTime = 0; init(); return false; }
    return true;
  }
  return se->slots[stateId] != nullptr;
}

// sendEvent (:270-292)
void Pre::sendAbsentLogical(StateEvent* se) {
  if (thisPost->hasNext) rt->selectAndEmit(se);
  if (thisPost->nextStatePre) thisPost->nextStatePre->addState(se);
  if (thisPost->nextEveryStatePre) thisPost->nextEveryStatePre->addEveryState(se);
  else if (isStartState) {
    active = false;
    if (!isAnd && partner->absentLogical) partner->active = false;   // setActive(false)
  }
  if (thisPost->callbackPre) thisPost->callbackPre->countStartStateReset();
}

// process(TIMER chunk) (:124-227)
void Pre::absentLogicalTimer(int64_t currentTime) {
  if (!active) return;
  bool notProcessed = true;
  if (currentTime >= lastArrivalTime + waitingTime) {
    if (isStartState && seq && newEvery.empty() && pending.empty()) {
      addState(rt->newStateEvent());
    } else if (seq && !newEvery.empty()) {
      resetState();
    }
    updateState();
    StateEvent* expired = nullptr;
    std::vector<StateEvent*> ret;
    for (auto it = pending.begin(); it != pending.end();) {
      StateEvent* e = *it;
      if (isExpired(e, currentTime)) { expired = e; it = pending.erase(it); continue; }
      StreamEvent* own = e->slots[stateId];
      bool passed = own == nullptr ? currentTime >= e->ts + waitingTime : currentTime >= own->ts + waitingTime;
      if (passed) {
        it = pending.erase(it);
        bool partnerSet = e->slots[partner->stateId] != nullptr;
        if (!isAnd && !partnerSet) {
          // StateEvent.addEvent(stateId, streamEventFactory.newInstance()): an empty event (ts -1)
          StreamEvent* d = rt->pool->se(); d->ts = -1; d->data = nullptr;
          if (!e->slots[stateId]) e->slots[stateId] = d;
          else { StreamEvent* t = e->slots[stateId]; while (t->next) t = t->next; t->next = d; }
          ret.push_back(e);
        } else if (isAnd && partnerSet) {
          ret.push_back(e);
        } else if (isAnd && !partnerSet) {
          StreamEvent* d = rt->pool->se(); d->ts = -1; d->data = nullptr;
          if (!e->slots[stateId]) e->slots[stateId] = d;
          else { StreamEvent* t = e->slots[stateId]; while (t->next) t = t->next; t->next = d; }
        }
        continue;
      }
      ++it;
    }
    if (expired && withinEveryPre) { withinEveryPre->addEveryState(expired); withinEveryPre->updateState(); }
    notProcessed = ret.empty();
    for (StateEvent* se : ret) { se->ts = currentTime; sendAbsentLogical(se); }
    lastArrivalTime = 0;
  }
  if (thisPost->nextEveryStatePre != nullptr || (notProcessed && isStartState)) {
    int64_t nextBreak = lastArrivalTime == 0 ? rt->app->now + waitingTime : lastArrivalTime + waitingTime;
    rt->app_notify_at(this, nextBreak);
  }
}

// ---- single-stream query (filter / window / selector) ----
static void window_process(QueryRT& rt, std::vector<SelEvent>& chunk, int64_t currentTime, std::vector<std::vector<SelEvent>>& outChunks);

void QueryRT::onTimer(int64_t ts) {
  // TIMER into the time window (TimeWindowProcessor.process)
  std::vector<SelEvent> chunk(1);
  chunk[0].type = TIMER; chunk[0].ts = ts; chunk[0].ev = nullptr;
  std::vector<std::vector<SelEvent>> outs;
  window_process(*this, chunk, app->now, outs);
  for (auto& c : outs) {
    auto o = sel.process(c);
    emitChunk(o);
  }
}

static SelEvent mk_sel(StreamEvent* e) {
  SelEvent s; s.ev = e; s.type = e->type; s.ts = e->ts; return s;
}

static void window_process(QueryRT& rt, std::vector<SelEvent>& chunk, int64_t currentTime, std::vector<std::vector<SelEvent>>& outChunks) {
  Window& w = rt.win;
  Pool& pool = *rt.pool;
  if (w.k == Window::NONE) { outChunks.push_back(chunk); return; }
  if (w.k == Window::LENGTH) {   // LengthWindowProcessor.process (:106-141)
    std::vector<SelEvent> out;
    for (auto& e : chunk) {
      StreamEvent* clone = pool.copy(e.ev);
      clone->type = EXPIRED;
      if (w.count < w.param) {
        w.count++;
        w.q.push_back(clone);
        out.push_back(e);
      } else {
        if (!w.q.empty()) {
          StreamEvent* first = w.q.front(); w.q.pop_front();
          first->ts = currentTime;
          out.push_back(mk_sel(first));
          out.push_back(e);
          w.q.push_back(clone);
        } else {
          StreamEvent* reset = pool.copy(e.ev); reset->type = RESET;
          out.push_back(e);
          out.push_back(mk_sel(clone));
          out.push_back(mk_sel(reset));
        }
      }
    }
    outChunks.push_back(out);
    return;
  }
  if (w.k == Window::TIME) {   // TimeWindowProcessor.process (:133-169)
    std::vector<SelEvent> out;
    for (auto& e : chunk) {
      int64_t now = rt.app->now;
      while (!w.q.empty()) {
        StreamEvent* ex = w.q.front();
        int64_t diff = ex->ts - now + w.param;
        if (diff <= 0) { w.q.pop_front(); ex->ts = now; out.push_back(mk_sel(ex)); }
        else break;
      }
      if (e.type == CURRENT) {
        StreamEvent* clone = pool.copy(e.ev); clone->type = EXPIRED;
        w.q.push_back(clone);
        if (w.lastTimestamp < clone->ts) {
          rt.app->notify_at(&rt, -1, clone->ts + w.param);
          w.lastTimestamp = clone->ts;
        }
        out.push_back(e);
      }
    }
    outChunks.push_back(out);
    return;
  }
  // LENGTH_BATCH (LengthBatchWindowProcessor.process :154-351)
  bool outputExpectsExpired = rt.def->expiredOn;
  for (auto& e : chunk) {
    std::vector<SelEvent> out;
    StreamEvent* ev = e.ev;
    if (w.param == 0) {
      out.push_back(e);
      if (outputExpectsExpired) { StreamEvent* x = pool.copy(ev); x->type = EXPIRED; x->ts = currentTime; out.push_back(mk_sel(x)); }
      StreamEvent* r = pool.copy(ev); r->type = RESET; r->ts = currentTime; out.push_back(mk_sel(r));
    } else {
      if (!w.resetEvent) { w.resetEvent = pool.copy(ev); w.resetEvent->type = RESET; }
      if (w.streamCurrent) {
        w.count++;
        if (w.count == w.param + 1) {
          if (outputExpectsExpired && !w.exq.empty()) {
            for (auto* x : w.exq) { x->ts = currentTime; out.push_back(mk_sel(x)); }
            w.exq.clear();
          }
          if (w.resetEvent) { w.resetEvent->ts = currentTime; out.push_back(mk_sel(w.resetEvent)); w.resetEvent = nullptr; }
          w.count = 1;
        }
        out.push_back(e);
        if (outputExpectsExpired) { StreamEvent* c = pool.copy(ev); c->type = EXPIRED; w.exq.push_back(c); }
      } else {
        StreamEvent* c = pool.copy(ev);
        w.cur.push_back(c);
        w.count++;
        if (w.count == w.param) {
          if (outputExpectsExpired && !w.exq.empty()) {
            for (auto* x : w.exq) { x->ts = currentTime; out.push_back(mk_sel(x)); }
            w.exq.clear();
          }
          if (w.resetEvent) { w.resetEvent->ts = currentTime; out.push_back(mk_sel(w.resetEvent)); w.resetEvent = nullptr; }
          if (!w.cur.empty()) {
            if (outputExpectsExpired) {
              for (auto* x : w.cur) { StreamEvent* t = pool.copy(x); t->type = EXPIRED; w.exq.push_back(t); }
            }
            for (auto* x : w.cur) out.push_back(mk_sel(x));
            w.cur.clear();
          }
          w.count = 0;
        }
      }
    }
    if (!out.empty()) outChunks.push_back(out);
  }
}

static void single_process(QueryRT& rt, const std::vector<std::pair<int64_t, const Val*>>& evs) {
  std::vector<SelEvent> chunk;
  for (auto& e : evs) {
    StreamEvent* ev = rt.pool->se();
    ev->ts = e.first; ev->data = e.second;
    // filters (FilterProcessor.process)
    EvalCtx c; c.ev = ev;
    bool ok = true;
    for (Ex* f : rt.sfilters) { Val v = eval(f, c); if (v.null || !v.b) { ok = false; break; } }
    if (!ok) continue;
    chunk.push_back(mk_sel(ev));
  }
  if (chunk.empty()) return;
  std::vector<std::vector<SelEvent>> outs;
  window_process(rt, chunk, rt.app->now, outs);
  for (auto& c : outs) {
    auto o = rt.sel.process(c);
    rt.emitChunk(o);
  }
}

// --------------------------------------------------------------------------------------------
// Junctions, partitions, time
// --------------------------------------------------------------------------------------------
void App::junction_send(int stream, const std::vector<std::pair<int64_t, const Val*>>& evs, bool batch) {
  if (stream_cb[stream]) {
    Callback cb; cb.kind = 1; cb.target = stream; cb.ts = evs.back().first; cb.seq = cur_seq;
    for (auto& e : evs) cb.in.push_back(OutEvent{e.first, false, std::vector<Val>(e.second, e.second + stream_types[stream].size())});
    out.push_back(std::move(cb));
  }
  for (int qi : subscribers[stream]) {
    QueryDef& qd = *qdefs[qi];
    if (!qd.partitioned) {
      QueryRT* rt = single_rt[qi].get();
      if (qd.state) rt->receiveBatch(stream, evs);
      else single_process(*rt, evs);
    } else {
      if (!qd.partition_attr.count(stream)) {
        // stream not named in `partition with`: PartitionStreamReceiver.send(event) delivers to every
        // existing partition key, iterating PartitionRuntimeImpl.getPartitionKeys() (a HashSet<String>)
        for (QueryRT* rt : java_hashset_order(qi)) {
          if (purge_check(rt, now)) continue;   // no longer in partitionKeys
          if (qd.state) rt->receiveBatch(stream, evs);
          else single_process(*rt, evs);
        }
        continue;
      }
      // PartitionStreamReceiver: consecutive same-key events form one chunk
      size_t i = 0;
      while (i < evs.size()) {
        const Val& kv0 = evs[i].second[qd.partition_attr.at(stream)];
        if (!kv0.null) init_partition_call(qi, kv0.key());
        QueryRT* rt = instance(qi, evs[i].second, stream);
        size_t j = i + 1;
        if (batch) {
          while (j < evs.size()) {
            QueryRT* r2 = instance(qi, evs[j].second, stream);
            if (r2 != rt) break;
            j++;
          }
        }
        std::vector<std::pair<int64_t, const Val*>> sub(evs.begin() + i, evs.begin() + j);
        if (rt) {
          if (qd.state) rt->receiveBatch(stream, sub);
          else single_process(*rt, sub);
        }
        i = j;
      }
    }
  }
}


std::vector<QueryRT*> App::java_hashset_order(int qi) {
  auto& order = part_order[qi];
  size_t n = order.size();
  size_t want = std::max<size_t>((size_t)((float)n / .75f) + 1, 16);
  size_t cap = 1;
  while (cap < want) cap <<= 1;
  std::vector<std::pair<uint32_t, size_t>> keyed;
  for (size_t i = 0; i < n; i++) {
    const std::string& ks = part_key_str[qi][i];
    uint32_t h = (uint32_t)java_string_hash(ks);
    h ^= (h >> 16);
    keyed.emplace_back(h & (uint32_t)(cap - 1), i);
  }
  std::stable_sort(keyed.begin(), keyed.end(), [](auto& a, auto& b) { return a.first < b.first; });
  std::vector<QueryRT*> out;
  for (auto& k : keyed) out.push_back(order[k.second]);
  return out;
}

void App::fire_timers(int64_t t) {
  // Scheduler.onTimeChange for each scheduler (creation order); TreeMultimap keeps ONE state per
  // distinct first deadline (SchedulerState.compareTo == 0, Scheduler.java:364-366).
  for (auto& reg : schedulers) {
    std::vector<std::pair<int64_t, QueryRT*>> due;
    auto consider = [&](QueryRT* rt) {
      auto it = timers.find({rt, reg.proc});
      if (it == timers.end() || it->second.q.empty()) return;
      int64_t first = it->second.q.front();
      if (first <= t) due.emplace_back(first, rt);
    };
    const bool part = qdefs[reg.query]->partitioned;
    if (part && qdefs[reg.query]->purge) {   // states of keys purged by now are gone from the map
      std::vector<QueryRT*> live;
      for (auto& bin : reg.states.tab) for (auto& e : bin) live.push_back(e.rt);
      for (QueryRT* rt : live) purge_check(rt, t);
    }
    // getAllStates(): the key -> state map in HashMap iteration order (bin, then chain order)
    if (part) { for (auto& bin : reg.states.tab) for (auto& e : bin) consider(e.rt); }
    else consider(single_rt[reg.query].get());
    // TreeMultimap<Long, SchedulerState>: keys ascending, ONE value per key (compareTo == 0)
    std::stable_sort(due.begin(), due.end(), [](auto& a, auto& b) { return a.first < b.first; });
    std::set<int64_t> seen;
    for (auto& d : due) {
      if (seen.count(d.first)) continue;
      seen.insert(d.first);
      QueryRT* rt = d.second;
      auto& q = timers[{rt, reg.proc}].q;
      while (!q.empty() && q.front() - now <= 0) {   // sendTimerEvents: FIFO head only
        int64_t tt = q.front();
        q.pop_front();
        if (reg.proc < 0) rt->onTimer(tt);
        else if (rt->pres[reg.proc]->absentLogical) rt->pres[reg.proc]->absentLogicalTimer(tt);
        else rt->pres[reg.proc]->absentTimer(tt);
      }
    }
    if (part) {   // returnAllStates: drop the states whose queue is empty (SchedulerState.canDestroy)
      std::vector<QueryRT*> gone;
      for (auto& bin : reg.states.tab)
        for (auto& e : bin) if (timers[{e.rt, reg.proc}].q.empty()) gone.push_back(e.rt);
      for (QueryRT* rt : gone) reg.states.remove(rt, rt->key_hash);
    }
  }
}

void App::set_time(int64_t t) {
  if (t >= now) now = t;
  fire_timers(now);
}

void App::send(int stream, const std::vector<std::pair<int64_t, const Val*>>& evs, bool batch) {
  if (playback) {
    // InputHandler.send -> TimestampGeneratorImpl.setCurrentTimestamp (fires due timers first)
    int64_t ts = evs.back().first;
    if (ts >= lastEventTimestamp) { lastEventTimestamp = ts; now = ts; fire_timers(now); }
  }
  junction_send(stream, evs, batch);
}

void App::start() {
  if (started) return;
  started = true;
  for (size_t qi = 0; qi < qdefs.size(); qi++)
    if (!qdefs[qi]->partitioned) init_partition(*this, single_rt[qi].get());
}

static App* create_app(const std::string& json) {
  auto* app = new App();
  app->desc = sgjson::parse(json);
  const J& d = app->desc;
  app->playback = d["playback"].b;
  for (auto& kv : d["streams"].o) {
    app->stream_idx[kv.first] = (int)app->stream_names.size();
    app->stream_names.push_back(kv.first);
    std::vector<Ty> ts;
    for (auto& a : kv.second.a) ts.push_back(ty_of(a[1].s));
    app->stream_types.push_back(ts);
  }
  app->subscribers.resize(app->stream_names.size());
  app->stream_cb.assign(app->stream_names.size(), false);
  const J& qs = d["queries"];
  for (size_t i = 0; i < qs.size(); i++) {
    auto qd = std::make_unique<QueryDef>();
    qd->index = (int)i;
    qd->desc = qs[i];
    qd->name = qs[i]["name"].s;
    qd->state = qs[i]["input"]["kind"].s == "state";
    for (auto& a : qs[i]["out_attrs"].a) qd->out_types.push_back(ty_of(a[1].s));
    const J& o = qs[i]["output"];
    qd->out_kind = o["kind"].s == "insert" ? 1 : 0;
    if (qd->out_kind == 1) qd->out_stream = app->stream_idx.at(o["stream"].s);
    const std::string& ev = o["events"].s;
    qd->currentOn = ev == "current" || ev == "all" || ev.empty();
    qd->expiredOn = ev == "expired" || ev == "all";
    if (qs[i].has("partition")) {
      qd->partitioned = true;
      for (auto& kv : qs[i]["partition"].o) qd->partition_attr[app->stream_idx.at(kv.first)] = (int)kv.second.as_int();
      qd->partition_id = qs[i].has("partition_id") ? (int)qs[i]["partition_id"].as_int() : -1;
      if (qs[i].has("purge")) {
        qd->purge = true;
        PurgeState& ps = app->purges[qd->partition_id];
        ps.interval = qs[i]["purge"]["interval"].as_int();
        ps.idle = qs[i]["purge"]["idle"].as_int();
        if (ps.interval <= 0) throw std::runtime_error("@purge interval must be positive");
      }
    }
    // subscriptions (SiddhiAppRuntimeBuilder.addQuery): one receiver per distinct input stream
    std::vector<int> ins;
    if (qd->state) {
      for (auto& s : qs[i]["input"]["slots"].a) {
        int si = app->stream_idx.at(s["stream"].s);
        if (std::find(ins.begin(), ins.end(), si) == ins.end()) ins.push_back(si);
      }
    } else {
      ins.push_back(app->stream_idx.at(qs[i]["input"]["stream"].s));
    }
    qd->input_streams = ins;
    for (int s : ins) app->subscribers[s].push_back((int)i);
    app->qdefs.push_back(std::move(qd));
  }
  app->single_rt.resize(app->qdefs.size());
  app->part_rt.resize(app->qdefs.size());
  app->part_order.resize(app->qdefs.size());
  app->part_key_str.resize(app->qdefs.size());
  app->query_cb.assign(app->qdefs.size(), false);
  for (size_t qi = 0; qi < app->qdefs.size(); qi++) {
    QueryDef& qd = *app->qdefs[qi];
    // scheduler registrations in creation order: absent processors (parse order), time window
    QueryRT* probe = app->build((int)qi);
    for (size_t p = 0; p < probe->pres.size(); p++)
      if (probe->pres[p]->kind == K_ABSENT || probe->pres[p]->absentLogical) {
        app->reg_of[{(int)qi, (int)p}] = (int)app->schedulers.size();
        app->schedulers.push_back({(int)qi, (int)p, {}});
      }
    if (probe->win.k == Window::TIME) {
      app->reg_of[{(int)qi, -1}] = (int)app->schedulers.size();
      app->schedulers.push_back({(int)qi, -1, {}});
    }
    if (!qd.partitioned) app->single_rt[qi].reset(probe);
    else delete probe;
  }
  return app;
}

}  // namespace orc

// ================================================================================================
// C ABI (test infrastructure)
// ================================================================================================
using namespace orc;

static thread_local std::string g_err;

extern "C" {

const char* or_last_error() { return g_err.c_str(); }

void* or_create(const char* desc_json) {
  try {
    return create_app(desc_json);
  } catch (std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}

void or_destroy(void* h) { delete (App*)h; }

int or_stream_index(void* h, const char* name) {
  App* a = (App*)h;
  auto it = a->stream_idx.find(name);
  return it == a->stream_idx.end() ? -1 : it->second;
}

int or_query_index(void* h, const char* name) {
  App* a = (App*)h;
  for (auto& q : a->qdefs) if (q->name == name) return q->index;
  return -1;
}

int or_intern(void* h, const char* s) { return ((App*)h)->intern(s); }
// intern "<prefix>0" .. "<prefix>{k-1}" in order (bulk form of the test harness's symbol setup)
void or_intern_range(void* h, const char* prefix, int k) {
  App* a = (App*)h;
  std::string p(prefix);
  for (int i = 0; i < k; i++) a->intern(p + std::to_string(i));
}
const char* or_string(void* h, int id) { return ((App*)h)->strings.at(id).c_str(); }

void or_add_query_callback(void* h, int q) { ((App*)h)->query_cb.at(q) = true; }
void or_add_stream_callback(void* h, int s) { ((App*)h)->stream_cb.at(s) = true; }
void or_start(void* h) { ((App*)h)->start(); }

// wall-clock emulation (non-playback): advance System.currentTimeMillis and fire due timers
void or_set_time(void* h, int64_t now) {
  App* a = (App*)h;
  a->cur_seq = a->nsent;
  try { a->set_time(now); } catch (std::exception& e) { g_err = e.what(); }
}

// InputHandler.send(long ts, Object[] data) for n events (batch=0) or send(Event[]) (batch=1).
// raw: n * nattrs 8-byte slots (see Val::raw), nulls: n * nattrs bytes (may be NULL).
int or_send(void* h, int stream, int64_t n, const int64_t* ts, const int64_t* raw, const uint8_t* nulls, int batch) {
  App* a = (App*)h;
  try {
    a->start();
    const auto& types = a->stream_types.at(stream);
    size_t na = types.size();
    std::vector<std::pair<int64_t, const Val*>> evs;
    for (int64_t i = 0; i < n; i++) {
      if (!batch || i == 0) a->cur_seq = a->nsent + i;
      a->pool.rows.emplace_back(na);
      auto& row = a->pool.rows.back();
      for (size_t k = 0; k < na; k++) row[k] = Val::from_raw(types[k], raw[i * na + k], nulls && nulls[i * na + k]);
      evs.emplace_back(ts[i], row.data());
      if (!batch) {
        if (!a->playback && ts[i] > a->now) a->set_time(ts[i]);
        a->send(stream, evs, false);
        evs.clear();
      }
    }
    if (batch && !evs.empty()) {
      if (!a->playback && ts[n - 1] > a->now) a->set_time(ts[n - 1]);
      a->send(stream, evs, true);
    }
    a->nsent += n;
    return 0;
  } catch (std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// send(Event[]) of each chunk [starts[c], starts[c+1]) in turn (starts[nchunks] == n); callbacks fired
// by chunk c carry seqs[c] as their arrival index (key-sharded runs: one chunk per key run of the
// unsharded stream, so each shard sees exactly the chunks PartitionStreamReceiver would form)
int or_send_chunks(void* h, int stream, int64_t n, const int64_t* ts, const int64_t* raw, const uint8_t* nulls,
                   int64_t nchunks, const int64_t* starts, const int64_t* seqs) {
  App* a = (App*)h;
  try {
    a->start();
    const auto& types = a->stream_types.at(stream);
    size_t na = types.size();
    for (int64_t c = 0; c < nchunks; c++) {
      std::vector<std::pair<int64_t, const Val*>> evs;
      for (int64_t i = starts[c]; i < starts[c + 1]; i++) {
        a->pool.rows.emplace_back(na);
        auto& row = a->pool.rows.back();
        for (size_t k = 0; k < na; k++) row[k] = Val::from_raw(types[k], raw[i * na + k], nulls && nulls[i * na + k]);
        evs.emplace_back(ts[i], row.data());
      }
      if (evs.empty()) continue;
      a->cur_seq = seqs[c];
      if (!a->playback && evs.back().first > a->now) a->set_time(evs.back().first);
      a->send(stream, evs, true);
    }
    a->nsent += n;
    return 0;
  } catch (std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// diagnostics: [max pending, max newAndEvery, max Scheduler queue, partition instances] over all live state
void or_debug_stats(void* h, int64_t* out) {
  App* a = (App*)h;
  int64_t mp = 0, mn = 0, mq = 0, ni = 0;
  auto scan = [&](QueryRT* rt) {
    ni++;
    for (auto& p : rt->pres) { mp = std::max<int64_t>(mp, p->pending.size()); mn = std::max<int64_t>(mn, p->newEvery.size()); }
  };
  for (auto& r : a->single_rt) if (r) scan(r.get());
  for (auto& m : a->part_rt) for (auto& kv : m) scan(kv.second.get());
  for (auto& kv : a->timers) if (kv.first.second >= 0) mq = std::max<int64_t>(mq, kv.second.q.size());
  out[0] = mp; out[1] = mn; out[2] = mq; out[3] = ni;
}

// StreamPreStateProcessor.StreamPreState.snapshot (:450-469) of every instance (creation order) and pre-state
// processor (preStateProcessors order) of query q, in the JSON shape of sg_query_state_json (siddhi_gfx.h): the
// restatement's side of the device state check (tests/test_gpu_nfa_state.py)
int64_t or_query_state_json(void* h, int q, char* buf, int64_t cap) {
  App* a = (App*)h;
  if (q < 0 || q >= (int)a->qdefs.size()) { g_err = "bad query index"; return -1; }
  const QueryDef& d = *a->qdefs[q];
  if (!d.state) { g_err = "not a pattern query"; return -1; }
  std::vector<QueryRT*> rts;
  if (d.partitioned) rts = a->part_order[q];
  else if (a->single_rt[q]) rts.push_back(a->single_rt[q].get());
  std::vector<int> slot_arity;
  for (auto& sl : d.desc["input"]["slots"].a) slot_arity.push_back((int)a->stream_types[a->stream_idx.at(sl["stream"].s)].size());
  std::string o;
  auto num = [&](int64_t v) { o += std::to_string(v); };
  auto stev = [&](const StateEvent* se) {
    o += "{\"ts\":"; num(se->ts);
    o += ",\"type\":"; num((int)se->type);
    o += ",\"slots\":[";
    for (size_t k = 0; k < se->slots.size(); k++) {
      if (k) o += ',';
      o += '[';
      bool first = true;
      for (const StreamEvent* e = se->slots[k]; e; e = e->next, first = false) {
        if (!first) o += ',';
        o += '[';
        num(e->ts);
        if (e->data)
          for (int x = 0; x < slot_arity[k]; x++) {
            o += ',';
            if (e->data[x].null) o += "null"; else num(e->data[x].raw());
          }
        o += ']';
      }
      o += ']';
    }
    o += "]}";
  };
  auto list = [&](const std::list<StateEvent*>& l) {
    o += '[';
    bool first = true;
    for (const StateEvent* se : l) { if (!first) o += ','; stev(se); first = false; }
    o += ']';
  };
  o = "{\"instances\":[";
  for (size_t r = 0; r < rts.size(); r++) {
    QueryRT* rt = rts[r];
    if (r) o += ',';
    o += "{\"key\":";
    if (d.partitioned) num(rt->pkey.second); else o += "null";
    o += ",\"processors\":[";
    for (size_t k = 0; k < rt->allPre.size(); k++) {
      const Pre* p = rt->allPre[k];
      if (k) o += ',';
      o += "{\"initialized\":"; o += p->initialized ? "true" : "false";
      o += ",\"pending\":"; list(p->pending);
      o += ",\"new_and_every\":"; list(p->newEvery);
      if (p->kind == K_ABSENT) { o += ",\"last_scheduled\":"; num(p->lastScheduledTime); }
      o += '}';
    }
    o += "]}";
  }
  o += "]}";
  if (buf && cap > 0) std::memcpy(buf, o.data(), (size_t)std::min<int64_t>(cap, (int64_t)o.size()));
  return (int64_t)o.size();
}

// ---- outputs ----
int64_t or_out_ncb(void* h) { return (int64_t)((App*)h)->out.size(); }

// per callback: kind, target, ts, n_in, n_rm
void or_out_cbs(void* h, int32_t* kind, int32_t* target, int64_t* ts, int32_t* n_in, int32_t* n_rm) {
  App* a = (App*)h;
  for (size_t i = 0; i < a->out.size(); i++) {
    kind[i] = a->out[i].kind; target[i] = a->out[i].target; ts[i] = a->out[i].ts;
    n_in[i] = (int32_t)a->out[i].in.size(); n_rm[i] = (int32_t)a->out[i].rm.size();
  }
}

// rows in callback order, in-events then removed-events; each row `width` slots
int64_t or_out_nrows(void* h) {
  App* a = (App*)h;
  int64_t n = 0;
  for (auto& c : a->out) n += c.in.size() + c.rm.size();
  return n;
}

void or_out_rows(void* h, int width, int64_t* ts, int64_t* raw, uint8_t* nulls) {
  App* a = (App*)h;
  int64_t r = 0;
  for (auto& c : a->out) {
    for (int part = 0; part < 2; part++) {
      auto& v = part == 0 ? c.in : c.rm;
      for (auto& e : v) {
        ts[r] = e.ts;
        for (int k = 0; k < width; k++) {
          if (k < (int)e.data.size()) { raw[r * width + k] = e.data[k].raw(); nulls[r * width + k] = e.data[k].null; }
          else { raw[r * width + k] = 0; nulls[r * width + k] = 1; }
        }
        r++;
      }
    }
  }
}

void or_out_clear(void* h) { ((App*)h)->out.clear(); }

// per callback: arrival index (events sent before it, over all streams) of the send that fired it
void or_out_cb_seq(void* h, int64_t* seq) {
  App* a = (App*)h;
  for (size_t i = 0; i < a->out.size(); i++) seq[i] = a->out[i].seq;
}

}  // extern "C"
