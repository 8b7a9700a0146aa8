// selector.hpp — QuerySelector over a query's pre-selector event stream (host side of the library).
//
// The device paths project, per output event, the values the selector reads: plain output attributes
// (select expressions without aggregators), aggregator arguments and group-by keys.  This stage then
// runs the reference selector on them, chunk by chunk (CORE/query/selector/QuerySelector.java:76-374):
//   * aggregators with the reference's add / remove / reset arithmetic and per-(partition key, group
//     key) state, dropped when it can be destroyed (SumAttributeAggregatorExecutor :69-355,
//     Avg :64-390, Count :67-146, Min :69-495, Max :69-475; PartitionSyncStateHolder :33-90),
//   * group-by batching: last event per group per chunk, in first-appearance order
//     (processInBatchGroupBy :315-374), aggregators without group-by: last event of the chunk
//     (processInBatchNoGroupBy :271-313), plain projection otherwise (processNoGroupBy :161-205),
//   * having over the output attributes, order by, offset and limit per chunk.
// It is O(events) scalar bookkeeping after the match; the matching itself stays on the device.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "compile.hpp"
#include "snapshot.hpp"

namespace sg {

enum SelAggK { SA_SUM = 0, SA_AVG, SA_COUNT, SA_MIN, SA_MAX };
enum SelEvType { SE_CURRENT = 0, SE_EXPIRED = 1, SE_RESET = 3 };

struct SelAgg {
  int k = SA_SUM;
  Ty in_t = T_OBJECT;   // argument type
  Ty out_t = T_OBJECT;
  int arg = -1;         // pre-selector value index of the argument (-1: count())
  bool track = false;   // min/max trackFutureStates (sliding windows or expired output)
};

struct SelSpec {
  std::vector<int> akind;   // per output attribute: 0 plain (value index aidx), 2 host program aidx
  std::vector<int> aidx;
  std::vector<Prog> host;   // output expressions with aggregators: loader slot 253 = pre-selector value,
                            // 254 = aggregator result
  std::vector<Ty> out_t;
  std::vector<SelAgg> aggs;
  std::vector<int> group;   // pre-selector value indices of the group-by keys
  bool has_having = false;
  Prog having;              // over the output attributes (loader slot 255)
  std::vector<std::pair<int, bool>> order;   // (output attribute, descending)
  int64_t limit = -1, offset = -1;
  bool current_on = true, expired_on = false;
  bool partitioned = false;
  bool active = false;      // the query needs this stage (aggregators, group-by, having, order, limit)
};

// one pre-selector event
struct SelIn {
  int type;                 // SelEvType
  int64_t ts;
  const int64_t* v;         // pre-selector values (raw slots)
  const uint8_t* nul;
  int64_t part;             // partition instance (lane) for per-key aggregator state
};

struct SelOut {
  int64_t ts;
  bool expired;
  std::vector<int64_t> raw;
  std::vector<uint8_t> nul;
};

// One aggregator's state and its add / remove / reset arithmetic (AttributeAggregatorExecutor.execute,
// :59-67, and the Sum/Avg/Count/Min/Max executors' processAdd / processRemove / reset / canDestroy):
// shared by SelectorStage and the aggregator extension ABI (ext.hip, sg_agg_*).
struct AggSt {
  double dsum = 0.0;
  int64_t lsum = 0, count = 0;
  std::deque<int64_t> dq;
  bool mv_null = true;
  int64_t mv = 0;
};

struct AggOps {
  static double as_d(Ty t, int64_t r) {
    switch (t) {
      case T_INT: return (double)(int32_t)r;
      case T_LONG: return (double)r;
      case T_FLOAT: return (double)bits_f(r);
      default: return bits_d(r);
    }
  }
  static int64_t as_l(Ty t, int64_t r) { return t == T_INT ? (int64_t)(int32_t)r : r; }
  static bool lt(Ty t, int64_t a, int64_t b) {
    switch (t) {
      case T_INT: return (int32_t)a < (int32_t)b;
      case T_LONG: return a < b;
      case T_FLOAT: return bits_f(a) < bits_f(b);
      default: return bits_d(a) < bits_d(b);
    }
  }
  // Float/Double.equals: bit equality of the canonical NaN form (deque removeFirstOccurrence)
  static bool boxed_eq(Ty t, int64_t a, int64_t b) {
    if (t == T_FLOAT) {
      float x = bits_f(a), y = bits_f(b);
      if (x != x && y != y) return true;
      return (uint32_t)a == (uint32_t)b;
    }
    if (t == T_DOUBLE) {
      double x = bits_d(a), y = bits_d(b);
      if (x != x && y != y) return true;
      return a == b;
    }
    return as_l(t, a) == as_l(t, b);
  }

  // AttributeAggregatorExecutor.execute for one event; returns (value, null)
  static std::pair<int64_t, bool> apply(const SelAgg& A, AggSt& s, int type, int64_t in, bool in_null) {
    switch (A.k) {
      case SA_COUNT:
        if (type == SE_CURRENT) s.count++;
        else if (type == SE_EXPIRED) s.count--;
        else s.count = 0;
        return {s.count, false};
      case SA_SUM: {
        const bool integral = A.in_t == T_INT || A.in_t == T_LONG;
        if (type == SE_RESET) { s.dsum = 0; s.lsum = 0; s.count = 0; return {0, !integral}; }
        if (in_null) {
          if (s.count == 0) return {0, true};
          return {integral ? s.lsum : d_bits(s.dsum), false};
        }
        if (type == SE_CURRENT) {
          if (integral) { s.lsum = (int64_t)((uint64_t)s.lsum + (uint64_t)as_l(A.in_t, in)); s.count++; return {s.lsum, false}; }
          s.dsum += as_d(A.in_t, in); s.count++;
          return {d_bits(s.dsum), false};
        }
        if (integral) {   // processRemove(double): sum = (long) (sum - (double) x)
          const double r = (double)s.lsum - (double)as_l(A.in_t, in);
          int64_t v;
          if (std::isnan(r)) v = 0;
          else if (r >= 9.2233720368547758e18) v = INT64_MAX;
          else if (r <= -9.2233720368547758e18) v = INT64_MIN;
          else v = (int64_t)r;
          s.lsum = v; s.count--;
          if (s.count == 0) return {0, true};
          return {s.lsum, false};
        }
        s.dsum -= as_d(A.in_t, in); s.count--;
        if (s.count == 0) return {0, true};
        return {d_bits(s.dsum), false};
      }
      case SA_AVG: {
        if (type == SE_RESET) { s.dsum = 0; s.count = 0; return {0, true}; }
        if (in_null) {
          if (s.count == 0) return {0, true};
          return {d_bits(s.dsum / (double)s.count), false};
        }
        if (type == SE_CURRENT) { s.count++; s.dsum += as_d(A.in_t, in); }
        else { s.count--; s.dsum -= as_d(A.in_t, in); }
        if (s.count == 0) return {0, true};
        return {d_bits(s.dsum / (double)s.count), false};
      }
      default: {   // min / max
        const bool mn = A.k == SA_MIN;
        if (type == SE_RESET) { s.dq.clear(); s.mv_null = true; return {0, true}; }
        if (in_null) return {s.mv, s.mv_null};
        if (type == SE_CURRENT) {
          if (A.track) {
            while (!s.dq.empty() && (mn ? lt(A.in_t, in, s.dq.back()) : lt(A.in_t, s.dq.back(), in))) s.dq.pop_back();
            s.dq.push_back(in);
          }
          if (s.mv_null || (mn ? lt(A.in_t, in, s.mv) : lt(A.in_t, s.mv, in))) { s.mv = in; s.mv_null = false; }
          return {s.mv, s.mv_null};
        }
        if (A.track) {
          for (auto it = s.dq.begin(); it != s.dq.end(); ++it)
            if (boxed_eq(A.in_t, *it, in)) { s.dq.erase(it); break; }
          s.mv_null = s.dq.empty();
          if (!s.mv_null) s.mv = s.dq.front();
        } else if (!s.mv_null && boxed_eq(A.in_t, s.mv, in)) {
          s.mv_null = true;
        }
        return {s.mv, s.mv_null};
      }
    }
  }

  static bool can_destroy(const SelAgg& A, const AggSt& s) {
    switch (A.k) {
      case SA_SUM: return (A.in_t == T_INT || A.in_t == T_LONG) ? (s.count == 0 && s.lsum == 0) : (s.count == 0 && s.dsum == 0.0);
      case SA_AVG: return s.dsum == 0.0 && s.count == 0;
      case SA_COUNT: return s.count == 0;
      default: return (!A.track || s.dq.empty()) && s.mv_null;
    }
  }

};

class SelectorStage {
 public:
  SelectorStage(const SelSpec& s, const std::vector<std::string>* strs) : sp(s), strings(strs) {}
  void clear() { states.clear(); }

  // aggregator states per (group key, partition instance) (AttributeAggregatorExecutor state maps)
  void snapshot(SnapWriter& w) const {
    w.pod<uint64_t>(states.size());
    for (auto& kv : states) {
      w.vec(kv.first);
      w.pod<uint64_t>(kv.second.size());
      for (const St& x : kv.second) {
        w.pod(x.dsum); w.pod(x.lsum); w.pod(x.count); w.deq(x.dq); w.pod(x.mv_null); w.pod(x.mv);
      }
    }
  }
  void restore(SnapReader& r) {
    states.clear();
    const uint64_t ns = r.pod<uint64_t>();
    for (uint64_t i = 0; i < ns; i++) {
      GKey k;
      r.vec(k);
      std::vector<St> v(r.pod<uint64_t>());
      if (v.size() != sp.aggs.size()) throw Error(-1, "snapshot selector state does not match the query");
      for (St& x : v) {
        x.dsum = r.pod<double>(); x.lsum = r.pod<int64_t>(); x.count = r.pod<int64_t>(); r.deq(x.dq);
        x.mv_null = r.pod<bool>(); x.mv = r.pod<int64_t>();
      }
      states.emplace(std::move(k), std::move(v));
    }
  }

  // the carried aggregator states by key (the device window path, window_gen.hip, reads and writes them
  // per flush so host and device share one state store)
  using GKey = std::vector<int64_t>;
  const std::vector<AggSt>* state_find(const GKey& k) const {
    auto it = states.find(k);
    return it == states.end() ? nullptr : &it->second;
  }
  void state_put(const GKey& k, std::vector<AggSt>&& v) { states[k] = std::move(v); }
  void state_erase(const GKey& k) { states.erase(k); }
  bool destroyable(const std::vector<AggSt>& v) const {
    for (size_t i = 0; i < sp.aggs.size(); i++) if (!can_destroy(sp.aggs[i], v[i])) return false;
    return true;
  }
  // order by / offset / limit of one output chunk (processNoGroupBy and the group-by batch)
  void finish_chunk(std::vector<SelOut>& v) const { order_limit(v); }

  // QuerySelector.process on one chunk (ComplexEventChunk.isBatch() is always true)
  std::vector<SelOut> process(const std::vector<SelIn>& chunk) {
    std::vector<SelOut> out;
    const bool gb = !sp.group.empty();
    const bool agg = !sp.aggs.empty();
    if (gb) {
      std::vector<GKey> order;
      std::map<GKey, SelOut> grouped;
      for (const SelIn& e : chunk) {
        SelOut o = populate(e);
        if (e.type == SE_RESET) continue;
        if (having_ok(o) && type_on(e)) {
          GKey k = gkey(e);
          if (!grouped.count(k)) order.push_back(k);
          grouped[k] = std::move(o);
        }
      }
      for (auto& k : order) out.push_back(std::move(grouped[k]));
      order_limit(out);
      return out;
    }
    if (agg) {
      int last = -1;
      std::vector<SelOut> all;
      all.reserve(chunk.size());
      for (size_t i = 0; i < chunk.size(); i++) {
        all.push_back(populate(chunk[i]));
        if (chunk[i].type == SE_RESET) continue;
        if (having_ok(all.back()) && type_on(chunk[i])) last = (int)i;
      }
      if (last >= 0 && sp.offset <= 0 && sp.limit != 0) out.push_back(std::move(all[last]));
      return out;
    }
    for (const SelIn& e : chunk) {
      SelOut o = populate(e);
      if (e.type == SE_RESET) continue;
      if (type_on(e) && having_ok(o)) out.push_back(std::move(o));
    }
    order_limit(out);
    return out;
  }

 private:
  using St = AggSt;
  static std::pair<int64_t, bool> apply(const SelAgg& A, St& st, int type, int64_t in, bool in_null) {
    return AggOps::apply(A, st, type, in, in_null);
  }
  static bool can_destroy(const SelAgg& A, const St& st) { return AggOps::can_destroy(A, st); }
  static bool lt(Ty t, int64_t a, int64_t b) { return AggOps::lt(t, a, b); }
  // (partition instance, group-by key values) -> aggregator states
  const SelSpec& sp;
  const std::vector<std::string>* strings;   // dictionary (order by on strings compares the text)
  std::map<GKey, std::vector<St>> states;

  GKey gkey(const SelIn& e) const {
    GKey k;
    for (int g : sp.group) { k.push_back(e.nul[g] ? INT64_MIN : e.v[g]); k.push_back(e.nul[g]); }
    return k;
  }
  bool type_on(const SelIn& e) const {
    return (e.type == SE_CURRENT && sp.current_on) || (e.type == SE_EXPIRED && sp.expired_on);
  }

  SelOut populate(const SelIn& e) {
    cur_in = &e;
    SelOut o;
    o.ts = e.ts;
    o.expired = e.type == SE_EXPIRED;
    std::vector<int64_t>& av = av_;
    std::vector<uint8_t>& an = an_;
    av.assign(sp.aggs.size(), 0);
    an.assign(sp.aggs.size(), 1);
    if (!sp.aggs.empty()) {
      GKey k = gkey(e);
      if (sp.partitioned) k.push_back(e.part);
      auto it = states.find(k);
      if (it == states.end()) it = states.emplace(k, std::vector<St>(sp.aggs.size())).first;
      auto& st = it->second;
      bool all = true;
      for (size_t i = 0; i < sp.aggs.size(); i++) {
        const SelAgg& A = sp.aggs[i];
        const bool inn = A.arg < 0 ? false : e.nul[A.arg] != 0;
        const int64_t in = A.arg < 0 ? 0 : e.v[A.arg];
        auto r = apply(A, st[i], e.type, in, inn);
        av[i] = r.first;
        an[i] = r.second;
        // each aggregator's state holder drops a destroyable state (group-by / partitioned holders)
        if ((!sp.group.empty() || sp.partitioned) && can_destroy(A, st[i])) st[i] = St();
        else all = false;
      }
      if (all && (!sp.group.empty() || sp.partitioned)) states.erase(it);
    }
    if (e.type == SE_RESET) return o;
    cur_av = &av; cur_an = &an;
    for (size_t a = 0; a < sp.akind.size(); a++) {
      if (sp.akind[a] == 0) { o.raw.push_back(e.v[sp.aidx[a]]); o.nul.push_back(e.nul[sp.aidx[a]]); continue; }
      int64_t rf[MAX_REG], v = 0;
      bool isnull = true;
      InLoader ld{this, nullptr};
      run(sp.host[sp.aidx[a]], ld, v, isnull, rf, 1);
      o.raw.push_back(v);
      o.nul.push_back(isnull);
    }
    return o;
  }

  // loader of the host programs: 253 pre-selector value, 254 aggregator result, 255 output attribute
  std::vector<int64_t> av_;
  std::vector<uint8_t> an_;
  const std::vector<int64_t>* cur_av = nullptr;
  const std::vector<uint8_t>* cur_an = nullptr;
  const SelIn* cur_in = nullptr;
  struct InLoader {
    const SelectorStage* st;
    const SelOut* o;
    bool load(int slot, int attr, int64_t& v) const {
      if (slot == 255) {
        if (!o || attr < 0 || attr >= (int)o->raw.size() || o->nul[attr]) return false;
        v = o->raw[attr];
        return true;
      }
      if (slot == 254) {
        if ((*st->cur_an)[attr]) return false;
        v = (*st->cur_av)[attr];
        return true;
      }
      if (st->cur_in->nul[attr]) return false;
      v = st->cur_in->v[attr];
      return true;
    }
  };

  // having runs right after populate on the same event (cur_* still point at its values)
  bool having_ok(const SelOut& o) const {
    if (!sp.has_having) return true;
    int64_t rf[MAX_REG];
    InLoader ld{this, &o};
    return run_pred(sp.having, ld, rf, 1);
  }

  // Comparable.compareTo of the attribute's type (OrderByEventComparator.java:62-113): String
  // lexicographic, Float/Double.compare (total order: -0.0 < 0.0, NaN last and equal to itself)
  int java_compare(Ty t, int64_t a, int64_t b) const {
    switch (t) {
      case T_STRING: {
        const int c = (*strings)[(size_t)(int32_t)a].compare((*strings)[(size_t)(int32_t)b]);
        return c < 0 ? -1 : (c > 0 ? 1 : 0);
      }
      case T_INT: return (int32_t)a < (int32_t)b ? -1 : ((int32_t)a > (int32_t)b ? 1 : 0);
      case T_LONG: return a < b ? -1 : (a > b ? 1 : 0);
      case T_BOOL: return (int)(a != 0) - (int)(b != 0);
      case T_FLOAT: {
        const float x = bits_f(a), y = bits_f(b);
        if (x < y) return -1;
        if (x > y) return 1;
        const int32_t bx = x != x ? 0x7fc00000 : (int32_t)(uint32_t)a, by = y != y ? 0x7fc00000 : (int32_t)(uint32_t)b;
        return bx == by ? 0 : (bx < by ? -1 : 1);
      }
      case T_DOUBLE: {
        const double x = bits_d(a), y = bits_d(b);
        if (x < y) return -1;
        if (x > y) return 1;
        const int64_t bx = x != x ? 0x7ff8000000000000ll : a, by = y != y ? 0x7ff8000000000000ll : b;
        return bx == by ? 0 : (bx < by ? -1 : 1);
      }
      default: return 0;
    }
  }

  void order_limit(std::vector<SelOut>& v) const {
    if (!sp.order.empty()) {
      std::stable_sort(v.begin(), v.end(), [&](const SelOut& x, const SelOut& y) {
        for (auto& ob : sp.order) {
          const int a = ob.first;
          if (!x.nul[a] && !y.nul[a]) {
            int r = java_compare(sp.out_t[a], x.raw[a], y.raw[a]);
            if (ob.second) r = -r;
            if (r != 0) return r < 0;
          } else if (!x.nul[a]) {
            return true;              // a value sorts before a null, in either direction
          } else if (!y.nul[a]) {
            return false;
          }
        }
        return false;
      });
    }
    if (sp.offset >= 0) {
      if ((size_t)sp.offset >= v.size()) v.clear();
      else v.erase(v.begin(), v.begin() + sp.offset);
    }
    if (sp.limit >= 0 && (size_t)sp.limit < v.size()) v.resize(sp.limit);
  }
};

inline bool has_agg(const J& e) {
  if (e["op"].s == "agg" || e["op"].s == "multivar") return true;
  for (const char* c : {"a", "b"})
    if (e.has(c) && has_agg(e[c])) return true;
  return false;
}

// SelectorParser restated for the host selector stage (CORE/util/parser/SelectorParser.java:64-260):
// plain select expressions are projected on the device; with aggregators, group-by, having, order by,
// limit or offset (`active`) the device projects the pre-selector values (aggregator arguments, group-by keys, the
// variables an aggregated expression or having reads) and SelectorStage does the rest.
inline bool build_selector(const J& s, const J& q, bool slide, SelSpec& sp, std::vector<const J*>& dev,
                           const std::function<int(const std::string&)>& intern, std::string& why) {
  bool agg = false;
  for (size_t k = 0; k < s["attrs"].size(); k++) agg = agg || has_agg(s["attrs"][k]["e"]);
  sp.active = agg || s["group_by"].size() || !s["having"].null() || s["order_by"].size() ||
              !s["limit"].null() || !s["offset"].null();
  const std::string& evs = q["output"]["events"].s;
  sp.current_on = evs == "current" || evs == "all" || evs.empty();
  sp.expired_on = evs == "expired" || evs == "all";
  auto leaf = [&](const J& e, int& slot, int& attr) -> bool {
    const std::string& op = e["op"].s;
    if (op == "var") { slot = 253; attr = (int)dev.size(); dev.push_back(&e); return true; }
    if (op == "multivar") throw CompileError("multi-value variable in a selector");
    if (op != "agg") return false;
    SelAgg A;
    const std::string& n = e["name"].s;
    if (n == "sum") A.k = SA_SUM;
    else if (n == "avg") A.k = SA_AVG;
    else if (n == "count") A.k = SA_COUNT;
    else if (n == "min") A.k = SA_MIN;
    else if (n == "max") A.k = SA_MAX;
    else throw CompileError("aggregator " + n + " is not lowered");
    A.out_t = ty_of(e["t"].s);
    if (e["args"].size() > 0) {
      if (has_agg(e["args"][0])) throw CompileError("nested aggregator");
      A.arg = (int)dev.size();
      dev.push_back(&e["args"][0]);
      A.in_t = ty_of(e["args"][0]["t"].s);
    }
    A.track = slide || sp.expired_on;   // trackFutureStates: SLIDE processing mode or expired output
    slot = 254;
    attr = (int)sp.aggs.size();
    sp.aggs.push_back(A);
    return true;
  };
  auto none = [](int, int) { return -1; };
  for (size_t k = 0; k < s["attrs"].size(); k++) {
    const J& e = s["attrs"][k]["e"];
    sp.out_t.push_back(ty_of(e["t"].s));
    if (!has_agg(e)) {
      sp.akind.push_back(0);
      sp.aidx.push_back((int)dev.size());
      dev.push_back(&e);
    } else {
      sp.akind.push_back(2);
      sp.aidx.push_back((int)sp.host.size());
      sp.host.emplace_back();
      Compiler c{sp.host.back(), none, intern, leaf};
      c.compile(e);
    }
  }
  for (size_t g = 0; g < s["group_by"].size(); g++) {
    if (has_agg(s["group_by"][g])) throw CompileError("aggregator in group by");
    sp.group.push_back((int)dev.size());
    dev.push_back(&s["group_by"][g]);
  }
  if (!s["having"].null()) {
    sp.has_having = true;
    Compiler c{sp.having, none, intern, leaf};
    c.compile(s["having"]);
  }
  for (size_t o = 0; o < s["order_by"].size(); o++) {
    const J& ob = s["order_by"][o];
    if (ob[0]["op"].s != "outvar") { why = "order by on a value that is not an output attribute"; return false; }
    sp.order.push_back({(int)ob[0]["attr"].as_int(), ob[1].s == "desc"});
  }
  if (!s["limit"].null()) sp.limit = s["limit"].as_int();
  if (!s["offset"].null()) sp.offset = s["offset"].as_int();
  return true;
}

}  // namespace sg
