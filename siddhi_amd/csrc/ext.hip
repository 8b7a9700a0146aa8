// ext.hip — the window / aggregator extension ABI (include/siddhi_gfx_ext.h).
//
// The Java extension classes (java/src/main/java/io/siddhi/gpu/ext/) registered with
// SiddhiManager.setExtension call these per chunk (windows) or per selector pass (aggregators).  They run
// the same restatements the query paths use: the window processors of window_proc.hpp (general window
// path) and AggOps of selector.hpp (every selector stage).  A window holds the ids of the events it
// retains; the shim keeps the StreamEvent clones and emits them in the order returned here.
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/siddhi_gfx.h"
#include "../../include/siddhi_gfx_ext.h"
#include "selector.hpp"
#include "snapshot.hpp"
#include "window_proc.hpp"

namespace sg {
int set_error(int code, const std::string& m);
}
using namespace sg;

struct sg_window {
  WinSpec spec;
  WinState<int64_t> st;                      // payload: the shim's event id
  std::vector<int64_t> out_id, out_ts, chunk_end;
  std::vector<int32_t> out_type;
  std::vector<int64_t> fresh_dl;             // notifyAt deadlines queued since the shim last took them
  void emit(const std::vector<WinItem<int64_t>>& o) {
    if (o.empty()) return;                   // QuerySelector sees no chunk (window_gen select())
    for (const auto& x : o) {
      out_id.push_back(x.val);
      out_type.push_back(x.type);
      out_ts.push_back(x.ts);
    }
    chunk_end.push_back((int64_t)out_id.size());
  }
};

struct sg_aggregator {
  SelAgg spec;
  AggSt st;
};

template <class F>
static int ext_try(F&& f) {
  try {
    return f();
  } catch (::sg::Error& e) {
    return set_error(e.code, e.what());
  } catch (std::exception& e) {
    return set_error(SG_E_INVALID, e.what());
  }
}

extern "C" {

int sg_window_create(int kind, int64_t param, int stream_current, int expired_on, sg_window** out) {
  if (!out) return set_error(SG_E_INVALID, "null output pointer");
  if (kind != SG_WIN_LENGTH && kind != SG_WIN_TIME && kind != SG_WIN_LENGTH_BATCH)
    return set_error(SG_E_INVALID, "unknown window kind");
  if (param < 0) return set_error(SG_E_INVALID, "negative window parameter");
  if (stream_current && kind != SG_WIN_LENGTH_BATCH)
    return set_error(SG_E_INVALID, "streamCurrentEvents is a lengthBatch parameter");
  auto* w = new sg_window();
  w->spec.kind = kind == SG_WIN_LENGTH ? WK_LENGTH : kind == SG_WIN_TIME ? WK_TIME : WK_BATCH;
  w->spec.L = param;
  w->spec.stream_current = stream_current != 0;
  w->spec.expired_on = expired_on != 0;
  *out = w;
  return SG_OK;
}

void sg_window_destroy(sg_window* w) { delete w; }

int sg_window_process(sg_window* w, int64_t n, const int64_t* ids, const int64_t* ts, int64_t now) {
  if (!w || n < 0 || (n > 0 && (!ids || !ts))) return set_error(SG_E_INVALID, "bad window chunk");
  return ext_try([&]() -> int {
    std::vector<WinItem<int64_t>> evs((size_t)n);
    for (int64_t k = 0; k < n; k++) evs[(size_t)k] = WinItem<int64_t>{WE_CURRENT, ts[k], ids[k]};
    // TimeWindowProcessor.process calls Scheduler.notifyAt(ts + T) once per new timestamp (:158-160):
    // every deadline the window queues is handed to the shim, which forwards each to its Scheduler
    win_process(w->spec, w->st, evs, now, [&](std::vector<WinItem<int64_t>>& o) { w->emit(o); },
                [&]() { w->fresh_dl.push_back(w->st.timers.back()); });
    return SG_OK;
  });
}

int sg_window_on_time(sg_window* w, int64_t now) {
  if (!w) return set_error(SG_E_INVALID, "null window");
  return ext_try([&]() -> int {
    win_drain(w->spec, w->st, now, [&](std::vector<WinItem<int64_t>>& o) { w->emit(o); });
    return SG_OK;
  });
}

int64_t sg_window_next_deadline(const sg_window* w) {
  return (!w || w->st.timers.empty()) ? INT64_MIN : w->st.timers.front();
}

int64_t sg_window_take_deadlines(sg_window* w, int64_t* out, int64_t cap) {
  if (!w || cap < 0) return set_error(SG_E_INVALID, "bad deadline buffer");
  const int64_t n = (int64_t)w->fresh_dl.size();
  if (!out) return n;                        // size query
  if (cap < n) return set_error(SG_E_INVALID, "deadline buffer too small");
  if (n) std::memcpy(out, w->fresh_dl.data(), (size_t)n * 8);
  w->fresh_dl.clear();
  return n;
}

int sg_window_out_sizes(const sg_window* w, int64_t* n_items, int64_t* n_chunks) {
  if (!w || !n_items || !n_chunks) return set_error(SG_E_INVALID, "null argument");
  *n_items = (int64_t)w->out_id.size();
  *n_chunks = (int64_t)w->chunk_end.size();
  return SG_OK;
}

int sg_window_out_copy(sg_window* w, int64_t* ids, int32_t* types, int64_t* ts, int64_t* chunk_end) {
  if (!w) return set_error(SG_E_INVALID, "null window");
  const size_t n = w->out_id.size();
  if (n && (!ids || !types || !ts)) return set_error(SG_E_INVALID, "null output array");
  if (!w->chunk_end.empty() && !chunk_end) return set_error(SG_E_INVALID, "null chunk_end");
  if (n) {
    std::memcpy(ids, w->out_id.data(), n * 8);
    std::memcpy(types, w->out_type.data(), n * 4);
    std::memcpy(ts, w->out_ts.data(), n * 8);
  }
  if (!w->chunk_end.empty()) std::memcpy(chunk_end, w->chunk_end.data(), w->chunk_end.size() * 8);
  w->out_id.clear(); w->out_type.clear(); w->out_ts.clear(); w->chunk_end.clear();
  return SG_OK;
}

static constexpr uint64_t SG_WIN_MAGIC = 0x316e6977677366ull;   // "fsgwin1"

int sg_window_snapshot(sg_window* w, uint8_t** buf, int64_t* len) {
  if (!w || !buf || !len) return set_error(SG_E_INVALID, "null argument");
  return ext_try([&]() -> int {
    SnapWriter o;
    o.pod(SG_WIN_MAGIC);
    o.pod(w->spec.kind); o.pod(w->spec.L); o.pod(w->spec.stream_current); o.pod(w->spec.expired_on);
    auto items = [&](const auto& c) {
      o.pod<uint64_t>(c.size());
      for (const auto& x : c) { o.pod(x.type); o.pod(x.ts); o.pod(x.val); }
    };
    items(w->st.q); items(w->st.cur); items(w->st.exq);
    o.pod(w->st.count); o.pod(w->st.last_ts); o.deq(w->st.timers);
    o.pod(w->st.has_reset); o.pod(w->st.reset.type); o.pod(w->st.reset.ts); o.pod(w->st.reset.val);
    *buf = (uint8_t*)malloc(o.b.size());
    if (!*buf) return set_error(SG_E_INVALID, "out of host memory");
    std::memcpy(*buf, o.b.data(), o.b.size());
    *len = (int64_t)o.b.size();
    return SG_OK;
  });
}

int sg_window_restore(sg_window* w, const uint8_t* buf, int64_t len) {
  if (!w || !buf || len < 0) return set_error(SG_E_INVALID, "bad snapshot buffer");
  return ext_try([&]() -> int {
    SnapReader r(buf, (size_t)len);
    if (r.pod<uint64_t>() != SG_WIN_MAGIC) return set_error(SG_E_INVALID, "not a window snapshot");
    WinSpec sp;
    sp.kind = r.pod<int>(); sp.L = r.pod<int64_t>(); sp.stream_current = r.pod<bool>(); sp.expired_on = r.pod<bool>();
    if (sp.kind != w->spec.kind || sp.L != w->spec.L || sp.stream_current != w->spec.stream_current ||
        sp.expired_on != w->spec.expired_on)
      return set_error(SG_E_INVALID, "snapshot of another window");
    WinState<int64_t> st;
    auto item = [&]() {
      WinItem<int64_t> x;
      x.type = r.pod<int>(); x.ts = r.pod<int64_t>(); x.val = r.pod<int64_t>();
      return x;
    };
    for (uint64_t k = r.pod<uint64_t>(); k > 0; k--) st.q.push_back(item());
    for (uint64_t k = r.pod<uint64_t>(); k > 0; k--) st.cur.push_back(item());
    for (uint64_t k = r.pod<uint64_t>(); k > 0; k--) st.exq.push_back(item());
    st.count = r.pod<int64_t>(); st.last_ts = r.pod<int64_t>(); r.deq(st.timers);
    st.has_reset = r.pod<bool>();
    st.reset = item();
    if (r.at != r.n) return set_error(SG_E_INVALID, "trailing bytes in window snapshot");
    w->st = std::move(st);
    w->fresh_dl.clear();
    return SG_OK;
  });
}

int sg_agg_create(int kind, int in_type, int track, sg_aggregator** out) {
  if (!out) return set_error(SG_E_INVALID, "null output pointer");
  if (kind < SG_AGG_SUM || kind > SG_AGG_MAX) return set_error(SG_E_INVALID, "unknown aggregator");
  const bool numeric = in_type == SG_T_INT || in_type == SG_T_LONG || in_type == SG_T_FLOAT || in_type == SG_T_DOUBLE;
  if (kind != SG_AGG_COUNT && !numeric)
    return set_error(SG_E_INVALID, "sum/avg/min/max take INT, LONG, FLOAT or DOUBLE");
  auto* a = new sg_aggregator();
  a->spec.k = kind;   // SG_AGG_* == SelAggK
  a->spec.in_t = numeric ? (Ty)in_type : T_LONG;
  a->spec.track = track != 0;
  a->spec.arg = kind == SG_AGG_COUNT ? -1 : 0;
  switch (kind) {
    case SG_AGG_SUM: a->spec.out_t = (in_type == SG_T_INT || in_type == SG_T_LONG) ? T_LONG : T_DOUBLE; break;
    case SG_AGG_AVG: a->spec.out_t = T_DOUBLE; break;
    case SG_AGG_COUNT: a->spec.out_t = T_LONG; break;
    default: a->spec.out_t = (Ty)in_type; break;
  }
  *out = a;
  return SG_OK;
}

void sg_agg_destroy(sg_aggregator* a) { delete a; }

int sg_agg_out_type(const sg_aggregator* a) { return a ? (int)a->spec.out_t : set_error(SG_E_INVALID, "null aggregator"); }

int sg_agg_process(sg_aggregator* a, int64_t n, const int32_t* types, const int64_t* in, const uint8_t* in_null,
                   int64_t* out, uint8_t* out_null) {
  if (!a || n < 0 || (n > 0 && (!types || !out || !out_null))) return set_error(SG_E_INVALID, "bad aggregator batch");
  if (n > 0 && a->spec.arg >= 0 && !in) return set_error(SG_E_INVALID, "null argument values");
  for (int64_t k = 0; k < n; k++)
    if (types[k] != SG_EV_CURRENT && types[k] != SG_EV_EXPIRED && types[k] != SG_EV_RESET)
      return set_error(SG_E_INVALID, "event type must be SG_EV_CURRENT, SG_EV_EXPIRED or SG_EV_RESET");
  return ext_try([&]() -> int {
    for (int64_t k = 0; k < n; k++) {
      const bool inn = a->spec.arg >= 0 && in_null && in_null[k];
      const auto r = AggOps::apply(a->spec, a->st, types[k], a->spec.arg >= 0 ? in[k] : 0, inn);
      out[k] = r.first;
      out_null[k] = r.second ? 1 : 0;
    }
    return SG_OK;
  });
}

int sg_agg_can_destroy(const sg_aggregator* a) {
  if (!a) return set_error(SG_E_INVALID, "null aggregator");
  return AggOps::can_destroy(a->spec, a->st) ? 1 : 0;
}

static constexpr uint64_t SG_AGG_MAGIC = 0x31676761677366ull;   // "fsgagg1"

// the executors' State.snapshot maps (SumAttributeAggregatorExecutor.AggregatorState :321-354, the Avg /
// Count / Min / Max states likewise): running sums, count, the min/max deque and its current value
int sg_agg_snapshot(sg_aggregator* a, uint8_t** buf, int64_t* len) {
  if (!a || !buf || !len) return set_error(SG_E_INVALID, "null argument");
  return ext_try([&]() -> int {
    SnapWriter o;
    o.pod(SG_AGG_MAGIC);
    o.pod(a->spec.k); o.pod((int)a->spec.in_t); o.pod(a->spec.track);
    o.pod(a->st.dsum); o.pod(a->st.lsum); o.pod(a->st.count); o.deq(a->st.dq); o.pod(a->st.mv_null); o.pod(a->st.mv);
    *buf = (uint8_t*)malloc(o.b.size());
    if (!*buf) return set_error(SG_E_INVALID, "out of host memory");
    std::memcpy(*buf, o.b.data(), o.b.size());
    *len = (int64_t)o.b.size();
    return SG_OK;
  });
}

int sg_agg_restore(sg_aggregator* a, const uint8_t* buf, int64_t len) {
  if (!a || !buf || len < 0) return set_error(SG_E_INVALID, "bad snapshot buffer");
  return ext_try([&]() -> int {
    SnapReader r(buf, (size_t)len);
    if (r.pod<uint64_t>() != SG_AGG_MAGIC) return set_error(SG_E_INVALID, "not an aggregator snapshot");
    const int k = r.pod<int>(), in_t = r.pod<int>();
    const bool track = r.pod<bool>();
    if (k != a->spec.k || in_t != (int)a->spec.in_t || track != a->spec.track)
      return set_error(SG_E_INVALID, "snapshot of another aggregator");
    AggSt st;
    st.dsum = r.pod<double>(); st.lsum = r.pod<int64_t>(); st.count = r.pod<int64_t>(); r.deq(st.dq);
    st.mv_null = r.pod<bool>(); st.mv = r.pod<int64_t>();
    if (r.at != r.n) return set_error(SG_E_INVALID, "trailing bytes in aggregator snapshot");
    a->st = std::move(st);   // validated in full before the live state changes
    return SG_OK;
  });
}

}  // extern "C"
