// api.hip — the C ABI of include/siddhi_gfx.h over the host runtime (runtime.hpp).
//
// sg_app_create lowers every query of the descriptor to one execution path, trying the
// specialised kernels first (followed-by, window+aggregate) and the general per-partition NFA
// interpreter last.  A query no path accepts makes creation fail with SG_E_UNSUPPORTED and the
// reasons each path gave — the caller keeps the reference engine for it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <unordered_set>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>

#include "../../include/siddhi_gfx.h"
#include "runtime.hpp"
#include "snapshot.hpp"

using namespace sg;

struct sg_app {
  App a;
};

// A query no device path lowers: creation still succeeds, sg_query_path reports SG_E_UNSUPPORTED and
// sg_query_unsupported_reason says why; the host keeps the reference runtime for it (and pushes its
// inserted events, if device queries read them, like any input stream).
struct UnsupportedExec : Exec {
  std::string reason;
  void push(const HostBatch&) override {}
  void flush(std::vector<Callback>&, bool, hipStream_t) override {}
  void reset() override {}
};

// The HIP device and stream are bound at the first call that needs them, so a descriptor can be
// validated and lowered (sg_app_create, sg_query_path, ...) on a host without a GPU.
static void ensure_device(App& app) {
  if (app.stream) { SG_HIP(hipSetDevice(app.device)); return; }
  int ndev = 0;
  SG_HIP(hipGetDeviceCount(&ndev));
  if (ndev <= 0) throw Error(SG_E_DEVICE, "no HIP device visible");
  SG_HIP(hipSetDevice(app.device));
  SG_HIP(hipStreamCreateWithFlags(&app.stream, hipStreamNonBlocking));
}

static thread_local std::string g_err;

static int fail(int code, const std::string& m) {
  g_err = m;
  return code;
}

namespace sg {
int set_error(int code, const std::string& m) { return fail(code, m); }   // for ext.hip (sg_last_error)
}

#define SG_TRY(body)                                  \
  try {                                               \
    body;                                             \
  } catch (::sg::Error & e) {                         \
    return fail(e.code, e.what());                    \
  } catch (std::exception & e) {                      \
    return fail(SG_E_INVALID, e.what());              \
  }

extern "C" {

const char* sg_last_error(void) { return g_err.c_str(); }

int sg_app_create(const char* descriptor_json, const sg_options* opts, sg_app** out) {
  if (!descriptor_json || !out) return fail(SG_E_INVALID, "null argument");
  auto* h = new sg_app();
  App& app = h->a;
  try {
    app.desc = sgjson::parse(descriptor_json);
    app.device = opts ? opts->device : 0;
    // descriptor schema: include/siddhi_gfx_descriptor.schema.json
    if (!app.desc.has("version") || app.desc["version"].as_int() != SG_DESCRIPTOR_VERSION)
      throw Error(SG_E_INVALID, "descriptor version must be " + std::to_string(SG_DESCRIPTOR_VERSION));
    app.playback = app.desc["playback"].b;
    for (auto& kv : app.desc["streams"].o) {
      app.stream_idx[kv.first] = (int)app.streams.size();
      StreamDef sd;
      sd.name = kv.first;
      for (auto& at : kv.second.a) sd.types.push_back(ty_of(at[1].s));
      app.streams.push_back(sd);
    }
    app.subscribers.resize(app.streams.size());
    app.stream_cb.assign(app.streams.size(), false);
    const J& qs = app.desc["queries"];
    std::vector<int> produced(app.streams.size(), 0);
    for (size_t qi = 0; qi < qs.size(); qi++) {
      const J& q = qs[qi];
      app.qnames.push_back(q["name"].s);
      std::vector<Ty> ot;
      for (auto& a : q["out_attrs"].a) ot.push_back(ty_of(a[1].s));
      app.qout_types.push_back(ot);
      int os = -1;
      if (q["output"]["kind"].s == "insert") {
        os = app.stream_idx.at(q["output"]["stream"].s);
        produced[os] = 1;
      }
      app.qout_stream.push_back(os);
    }
    std::string reasons;
    for (size_t qi = 0; qi < qs.size(); qi++) {
      const J& q = qs[qi];
      std::string why1, why2, why3, why4, why5;
      // SG_PATHS (test/bring-up hook): comma list of enabled paths, default all
      const char* en = getenv("SG_PATHS");
      auto on = [&](const char* p) { return !en || std::strstr(en, p) != nullptr; };
      std::unique_ptr<Exec> ex;
      if (on("followed_by")) ex = make_followed_by(app, (int)qi, q, why1); else why1 = "disabled";
      if (!ex) { if (on("keyed")) ex = make_keyed_followed_by(app, (int)qi, q, why4); else why4 = "disabled"; }
      if (!ex) { if (on("window_agg")) ex = make_window_agg(app, (int)qi, q, why2); else why2 = "disabled"; }
      if (!ex) { if (on("nfa")) ex = make_nfa(app, (int)qi, q, why3); else why3 = "disabled"; }
      if (!ex) { if (on("window_gen")) ex = make_window_gen(app, (int)qi, q, why5); else why5 = "disabled"; }
      if (!ex) {
        auto ux = std::make_unique<UnsupportedExec>();
        ux->reason = "followed-by: " + why1 + "; keyed followed-by: " + why4 + "; window-agg: " + why2 + "; nfa: " + why3 +
                     "; window: " + why5;
        ux->path = SG_E_UNSUPPORTED;
        ux->name = q["name"].s;
        ux->app = &app;
        ux->qi = (int)qi;
        app.execs.push_back(std::move(ux));
        continue;
      }
      for (int s : ex->in_streams) {
        // a query reading another query's output (InsertIntoStreamCallback -> StreamJunction,
        // InsertIntoStreamCallback.java:44-58): single-stream consumers keep arrival order by
        // construction, the NFA places inputs by arrival seq; multi-stream scans do not
        if (produced[s] && ex->in_streams.size() > 1 && ex->path != SG_PATH_NFA)
          throw Error(SG_E_UNSUPPORTED, "query '" + q["name"].s + "' reads another query's output together with "
                                        "other streams on a scan path (only the NFA path orders chained inputs)");
        app.subscribers[s].push_back((int)qi);
      }
      ex->name = q["name"].s;
      app.execs.push_back(std::move(ex));
    }
    (void)reasons;
    app.query_cb.assign(app.execs.size(), false);
    app.feeds.assign(app.execs.size(), false);
    for (size_t qi = 0; qi < app.execs.size(); qi++) {
      const int os = app.qout_stream[qi];
      if (os < 0 || app.subscribers[os].empty() || app.execs[qi]->path == SG_E_UNSUPPORTED) continue;
      if (qs[qi]["output"]["events"].s == "expired" || qs[qi]["output"]["events"].s == "all")
        throw Error(SG_E_UNSUPPORTED, "query '" + qs[qi]["name"].s + "' inserts expired events into a stream other "
                                      "device queries read (timer-driven chained output is not lowered)");
      app.feeds[qi] = true;
    }
  } catch (Error& e) {
    delete h;
    return fail(e.code, e.what());
  } catch (std::exception& e) {
    delete h;
    return fail(SG_E_INVALID, e.what());
  }
  *out = h;
  return SG_OK;
}

void sg_app_destroy(sg_app* h) {
  if (!h) return;
  hipStream_t s = h->a.stream;
  h->a.execs.clear();
  if (s) (void)hipStreamDestroy(s);
  delete h;
}

int sg_stream_index(sg_app* h, const char* name) {
  auto it = h->a.stream_idx.find(name);
  return it == h->a.stream_idx.end() ? fail(SG_E_INVALID, std::string("no stream ") + name) : it->second;
}

int sg_query_index(sg_app* h, const char* name) {
  for (size_t i = 0; i < h->a.qnames.size(); i++)
    if (h->a.qnames[i] == name) return (int)i;
  return fail(SG_E_INVALID, std::string("no query ") + name);
}

int sg_stream_arity(sg_app* h, int s) {
  if (!h || s < 0 || s >= (int)h->a.streams.size()) return fail(SG_E_INVALID, "bad stream index");
  return (int)h->a.streams[s].types.size();
}
int sg_stream_attr_type(sg_app* h, int s, int k) {
  if (!h || s < 0 || s >= (int)h->a.streams.size()) return fail(SG_E_INVALID, "bad stream index");
  if (k < 0 || k >= (int)h->a.streams[s].types.size()) return fail(SG_E_INVALID, "bad attribute index");
  return (int)h->a.streams[s].types[k];
}
int sg_query_path(sg_app* h, int q) {
  if (!h || q < 0 || q >= (int)h->a.execs.size()) return fail(SG_E_INVALID, "bad query index");
  return h->a.execs[q]->path;
}
const char* sg_query_unsupported_reason(sg_app* h, int q) {
  if (!h || q < 0 || q >= (int)h->a.execs.size()) return nullptr;
  auto* u = dynamic_cast<UnsupportedExec*>(h->a.execs[q].get());
  return u ? u->reason.c_str() : nullptr;
}
int sg_query_count(sg_app* h) { return h ? (int)h->a.execs.size() : fail(SG_E_INVALID, "null app"); }
int sg_stream_count(sg_app* h) { return h ? (int)h->a.streams.size() : fail(SG_E_INVALID, "null app"); }

int sg_intern(sg_app* h, const char* s) { return h->a.intern(s); }
const char* sg_string(sg_app* h, int id) {
  if (id < 0 || id >= (int)h->a.strings.size()) return nullptr;
  return h->a.strings[id].c_str();
}

int sg_add_query_callback(sg_app* h, int q) {
  if (q < 0 || q >= (int)h->a.query_cb.size()) return fail(SG_E_INVALID, "bad query index");
  h->a.query_cb[q] = true;
  return SG_OK;
}

int sg_add_stream_callback(sg_app* h, int s) {
  if (s < 0 || s >= (int)h->a.stream_cb.size()) return fail(SG_E_INVALID, "bad stream index");
  h->a.stream_cb[s] = true;
  return SG_OK;
}

int sg_start(sg_app* h) {
  SG_TRY({
    ensure_device(h->a);
    if (!h->a.started)
      for (auto& e : h->a.execs) e->start(h->a.now);   // App.start -> initPartition of unpartitioned queries
    h->a.started = true;
    return SG_OK;
  })
}

}  // extern "C"
// A restarted runtime: every query's state dropped, the playback clock starting over (TimestampGeneratorImpl is
// recreated), the @purge schedules cleared, and the start-time state of a started app armed again (App.start ->
// initPartition of unpartitioned queries).  sg_reset, and sg_restore when a query's state fails to load.
static void reset_app(App& a) {
  for (auto& e : a.execs) e->reset();
  a.out.clear();
  a.early.clear();
  a.blocks.clear();
  a.seq = 0;
  a.now = 0;
  a.last_event_ts = INT64_MIN;
  for (auto& pc : a.purges) { pc.second.first.clear(); pc.second.t0 = INT64_MAX; }
  if (a.started)
    for (auto& e : a.execs) e->start(a.now);
}
extern "C" {

int sg_reset(sg_app* h) {
  SG_TRY({
    ensure_device(h->a);
    reset_app(h->a);
    return SG_OK;
  })
}

// StreamJunction.sendEvent restated for the device queries of one push: every subscriber in
// subscription order (StreamJunction.java:254-272); a query whose output another device query reads
// runs at once and its chunks go through the output stream's junction before the next subscriber
// (OutputRateLimiter.sendToCallBacks -> InsertIntoStreamCallback.send, OutputRateLimiter.java:64-110).
static bool host_timing() { static const bool on = getenv("SG_HOST_TIMING") != nullptr; return on; }
struct HostTimer {
  const char* what;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit HostTimer(const char* w) : what(w) {}
  ~HostTimer() {
    if (host_timing())
      fprintf(stderr, "[sg host] %s %.1f ms\n", what,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  }
};

static void dispatch(App& app, int stream, const HostBatch& hb) {
  for (int q : app.subscribers[stream]) {
    {
      HostTimer ht("push");
      app.execs[q]->push(hb);
    }
    if (!app.feeds[q]) continue;
    const int os = app.qout_stream[q];
    const StreamDef& sd = app.streams[os];
    const int na = (int)sd.types.size();
    // the upstream query runs now; its output chunks become the inserted stream's input
    ChainOut co;
    co.ts = app.take64();
    co.seq = app.take64();
    std::vector<Callback> cbs;
    const bool own_cb = app.query_cb[q] || app.stream_cb[os];
    // the export may stay in HBM (DevChain) when every consumer takes device columns whole (NFA queries that feed
    // nothing further, one partition attribute among them); the exporter decides whether its rows qualify
    DevChain dc;
    bool dev = !own_cb && !app.subscribers[os].empty() && !getenv("SG_HOST_CHAIN");
    for (int c : app.subscribers[os]) {
      const int a = app.execs[c]->chain_key_attr(os);
      if (a == -2 || app.feeds[c] || app.execs[c]->chunk_sensitive() || (c != app.subscribers[os][0] && a != dc.key_attr))
        dev = false;
      dc.key_attr = a;
    }
    if (dev) {
      for (int k = 0; k < na; k++) dc.widths.push_back(tsize(sd.types[k]));
      app.execs[q]->set_chain_request(&dc);
    }
    {
      HostTimer ht("upstream flush + materialise");
      bool exported = false;
      try {
        exported = !own_cb && app.execs[q]->flush_export(co, app.stream);
      } catch (...) {
        app.execs[q]->set_chain_request(nullptr);
        throw;
      }
      app.execs[q]->set_chain_request(nullptr);
      if (dc.done) {
        HostTimer ht2("downstream device push");
        for (int c : app.subscribers[os]) app.execs[c]->push_device_chain(os, dc, hb.now, app.stream);
        app.give64(std::move(co.ts));
        app.give64(std::move(co.seq));
        continue;
      }
      if (!exported) {
        app.execs[q]->flush(cbs, true, app.stream);
        co = ChainOut();
        co.raw.assign(na, {});
        for (auto& c : cbs) {
          if (c.blk) {                                   // columnar callbacks: each one is a chunk
            const OutBlock& b = *c.blk;
            for (int64_t k = 0; k < b.ncb(); k++) {
              for (int64_t r = b.cb_row[k]; r < b.cb_row[k + 1]; r++) {
                co.ts.push_back(b.ts[r]);
                co.seq.push_back(b.cb_seq[k]);
                for (int x = 0; x < na; x++) co.raw[x].push_back(x < b.width ? b.raw[r * b.width + x] : 0);
              }
              co.chunk_end.push_back((int64_t)co.ts.size());
            }
            continue;
          }
          for (auto& e : c.ev) {
            co.ts.push_back(e.ts);
            co.seq.push_back(c.seq);
            for (int k = 0; k < na; k++) {
              co.raw[k].push_back(k < (int)e.raw.size() ? e.raw[k] : 0);
              co.nulls = co.nulls || (k < (int)e.nul.size() && e.nul[k]);
            }
          }
          co.chunk_end.push_back((int64_t)co.ts.size());
        }
      }
    }
    HostTimer ht2("chain convert + downstream");
    if (co.nulls) throw Error(SG_E_UNSUPPORTED, "null attribute values in a chained stream are not lowered");
    if ((int)co.raw.size() != na) throw Error(SG_E_INVALID, "chained output arity differs from the inserted stream");
    // app clock of each source send (playback: the clock at that send; else the push's clock)
    auto now_of = [&](int64_t sq) -> int64_t {
      if (hb.seqs.empty()) {
        const int64_t k = sq - hb.seq0;
        return (k >= 0 && k < hb.n) ? hb.now_ev[k] : app.now;
      }
      auto it = std::lower_bound(hb.seqs.begin(), hb.seqs.end(), sq);
      return (it != hb.seqs.end() && *it == sq) ? hb.now_ev[it - hb.seqs.begin()] : app.now;
    };
    // NFA consumers take the whole derived stream at once; chunk-sensitive ones one chunk at a time
    bool per_chunk = false;
    for (int c : app.subscribers[os]) per_chunk = per_chunk || app.execs[c]->chunk_sensitive();
    int64_t r0 = 0;
    const size_t nchunks = co.nchunks();
    for (size_t ci = 0; ci < nchunks; ci++) {
      const int64_t r1 = co.chunk_end_at(ci);
      if (per_chunk || ci + 1 == nchunks) {
        HostBatch d;
        d.stream = os; d.n = r1 - r0; d.seq0 = 0; d.batch = true; d.now = hb.now;
        if (r0 == 0 && r1 == (int64_t)co.ts.size()) {   // the whole export in one push: take it over
          d.own_ts = std::move(co.ts);
          d.own_seqs = std::move(co.seq);
        } else {
          d.own_ts.assign(co.ts.begin() + r0, co.ts.begin() + r1);
          d.own_seqs.assign(co.seq.begin() + r0, co.seq.begin() + r1);
        }
        d.ts = HSpan<int64_t>(d.own_ts);
        d.seqs = HSpan<int64_t>(d.own_seqs);
        d.own_now = app.take64();
        d.own_now.resize(d.n);
        d.own_cols.assign(na, {});
        d.cols.resize(na);
        for (int k = 0; k < na; k++) {
          if (tsize(sd.types[k]) == 8) {   // 8-byte attributes: the exported column as it is
            d.cols[k] = HSpan<uint8_t>((const uint8_t*)(co.raw[k].data() + r0), (size_t)d.n * 8);
          } else {
            d.own_cols[k] = app.take8();           // recycled: no first-touch page faults per push
            d.own_cols[k].resize((size_t)d.n * 4);
            d.cols[k] = HSpan<uint8_t>(d.own_cols[k]);
          }
        }
        const int nth = host_threads(d.n);
        host_parallel(nth, [&](int t) {
          const int64_t a0 = d.n * t / nth, a1 = d.n * (t + 1) / nth;
          if (hb.seqs.empty() || a0 >= a1) {
            for (int64_t r = a0; r < a1; r++) d.own_now[r] = now_of(d.own_seqs[r]);
          } else {   // rows come in seq order: one search, then a sweep over the source seqs
            const int64_t* sb = hb.seqs.begin(), *se = hb.seqs.end();
            const int64_t* it = std::lower_bound(sb, se, d.own_seqs[a0]);
            for (int64_t r = a0; r < a1; r++) {
              const int64_t sq = d.own_seqs[r];
              if (r > a0 && sq < d.own_seqs[r - 1]) it = std::lower_bound(sb, se, sq);
              while (it != se && *it < sq) ++it;
              d.own_now[r] = (it != se && *it == sq) ? hb.now_ev[it - sb] : app.now;
            }
          }
          for (int k = 0; k < na; k++) {
            if (tsize(sd.types[k]) == 8) continue;
            const int64_t* src = co.raw[k].data() + r0;
            int32_t* dst = (int32_t*)d.own_cols[k].data();
            for (int64_t r = a0; r < a1; r++) dst[r] = (int32_t)src[r];
          }
        });
        d.now_ev = HSpan<int64_t>(d.own_now);
        if (d.n) dispatch(app, os, d);
        app.give64(std::move(d.own_ts));
        app.give64(std::move(d.own_seqs));
        app.give64(std::move(d.own_now));
        for (auto& c : d.own_cols) app.give8(std::move(c));
        r0 = r1;
      }
    }
    app.give64(std::move(co.ts));
    app.give64(std::move(co.seq));
    for (auto& c : co.raw) app.give64(std::move(c));
    for (auto& c : cbs) app.early.push_back(std::move(c));
  }
}

// A pushed batch read on the device by two or more queries (config 5: StockStream into the window query and the
// pattern) crosses PCIe once: staged in HBM here, each query's push copies device to device (HostBatch::d_*)
// (two calls: the timestamps and columns before the push's clock is computed -- the copies from the caller's pinned
// buffers run meanwhile -- and the per-event clock after it)
static void stage_batch(App& app, HostBatch& hb, bool clock) {
  int takers = 0;
  for (int q : app.subscribers[hb.stream]) takers += app.execs[q]->takes_device_batch() ? 1 : 0;
  if (takers < 2 || hb.n <= 0 || getenv("SG_NO_STAGE")) return;
  hipStream_t s = app.stream;
  if (clock) {
    if (!hb.now_uniform && !hb.now_ev.empty()) {
      app.stage_now.reserve((size_t)hb.n);
      SG_HIP(hipMemcpyAsync(app.stage_now.p, hb.now_ev.data(), (size_t)hb.n * 8, hipMemcpyHostToDevice, s));
      hb.d_now = app.stage_now.p;
    }
    return;
  }
  app.stage_ts.reserve((size_t)hb.n);
  SG_HIP(hipMemcpyAsync(app.stage_ts.p, hb.ts.data(), (size_t)hb.n * 8, hipMemcpyHostToDevice, s));
  hb.d_ts = app.stage_ts.p;
  hb.d_cols.assign(hb.cols.size(), nullptr);
  for (size_t k = 0; k < hb.cols.size(); k++) {
    DBuf<uint8_t>& c = app.stage_cols[(int)k];
    c.reserve(std::max<size_t>(hb.cols[k].size(), 1));
    SG_HIP(hipMemcpyAsync(c.p, hb.cols[k].data(), hb.cols[k].size(), hipMemcpyHostToDevice, s));
    hb.d_cols[k] = c.p;
  }
}

// The playback/wall-clock advance of a per-event push over thread ranges (the sequential loops in sg_push and
// sg_push_shard restated): the clock is a running maximum of the send timestamps T[0, N) (playback: from
// last_event_ts, a send at or above it ticks; else from the clock, a send above it ticks), so each range starts
// from the maxima of the ranges before it; ticks are counted, then written in place.  Send g's tick carries seq
// tseq[g] (or sq0 + g).  loc_seq null: every send is an event of the push (now_out[g], tick position g); else the
// push holds the sends with the increasing seqs loc_seq[0, nloc) (a rank's share of a global send: now_out[k],
// tick position = the local events before the send).
static void clock_ranges(App& app, const int64_t* T, int64_t N, const int64_t* tseq, int64_t sq0,
                         const int64_t* loc_seq, int64_t nloc, int64_t* now_out, TickBuf& tk) {
  const int nth = host_threads(N);
  const bool pb = app.playback;
  const int64_t m0 = pb ? app.last_event_ts : app.now, now0 = app.now;
  std::vector<int64_t> cmax(nth, INT64_MIN), cnt(nth + 1, 0);
  host_parallel(nth, [&](int t) {
    int64_t m = INT64_MIN;
    for (int64_t g = N * t / nth, e = N * (t + 1) / nth; g < e; g++) m = std::max(m, T[g]);
    cmax[t] = m;
  });
  std::vector<int64_t> start(nth);
  std::vector<uint8_t> ticked0(nth);
  int64_t run = m0, tmax = INT64_MIN;
  for (int t = 0; t < nth; t++) {
    start[t] = run;
    ticked0[t] = pb && tmax >= m0;    // (playback: the clock moved once any earlier send reached m0)
    run = std::max(run, cmax[t]);
    tmax = std::max(tmax, cmax[t]);
  }
  auto sweep = [&](int t, bool write) {
    const int64_t g0 = N * t / nth, g1 = N * (t + 1) / nth;
    int64_t m = start[t], c = 0, at = cnt[t];
    int64_t k = loc_seq ? std::lower_bound(loc_seq, loc_seq + nloc, sq0 + g0) - loc_seq : 0;
    bool any = ticked0[t];
    for (int64_t g = g0; g < g1; g++) {
      const int64_t x = T[g];
      if (pb ? x >= m : x > m) {
        m = x; any = true;
        if (write) {
          tk.now[at] = x;
          tk.seq[at] = tseq ? tseq[g] : sq0 + g;
          tk.k[at] = loc_seq ? k : g;
          at++;
        } else c++;
      }
      if (!write) {
        const int64_t now = pb ? (any ? m : now0) : m;
        if (!loc_seq) now_out[g] = now;
        else if (k < nloc && loc_seq[k] == sq0 + g) now_out[k++] = now;
      } else if (loc_seq && k < nloc && loc_seq[k] == sq0 + g) k++;
    }
    if (!write) cnt[t + 1] = c;
  };
  host_parallel(nth, [&](int t) { sweep(t, false); });
  for (int t = 0; t < nth; t++) cnt[t + 1] += cnt[t];
  tk.now.resize(cnt[nth]); tk.seq.resize(cnt[nth]); tk.k.resize(cnt[nth]);
  host_parallel(nth, [&](int t) { sweep(t, true); });
  if (cnt[nth] > 0) {
    if (pb) app.last_event_ts = run;
    app.now = pb ? run : std::max(now0, run);
  }
}

int sg_push(sg_app* h, int stream, const sg_batch* b) {
  App& app = h->a;
  SG_TRY({
    if (stream < 0 || stream >= (int)app.streams.size()) return fail(SG_E_INVALID, "bad stream index");
    if (!b || b->n < 0) return fail(SG_E_INVALID, "bad batch");
    if (b->n == 0) return SG_OK;
    ensure_device(app);
    const StreamDef& sd = app.streams[stream];
    int na = (int)sd.types.size();
    HostBatch hb;
    if (b->nulls) {
      bool any = false;
      for (int64_t i = 0; i < b->n * na && !any; i++) any = b->nulls[i] != 0;
      if (any) {
        // the NFA and general single-stream paths load nulls (CompareConditionExpressionExecutor: null
        // compares false); the scan paths have no null lanes and refuse rather than differ
        for (int q : app.subscribers[stream])
          if (!app.execs[q]->supports_nulls())
            return fail(SG_E_UNSUPPORTED, "query '" + app.qnames[q] + "' runs on a path without null attribute values");
        hb.nulls = HSpan<uint8_t>(b->nulls, (size_t)(b->n * na));
      }
    }
    hb.stream = stream;
    hb.n = b->n;
    hb.seq0 = app.seq;
    hb.batch = b->batch != 0;
    hb.now = app.now;
    hb.ts = HSpan<int64_t>(b->ts, (size_t)b->n);
    if (b->seq) {
      hb.seqs = HSpan<int64_t>(b->seq, (size_t)b->n);
      for (int64_t k = 1; k < b->n; k++)
        if (hb.seqs[k] <= hb.seqs[k - 1]) return fail(SG_E_INVALID, "batch seq must be increasing");
    }
    hb.cols.resize(na);
    hb.own_cols.resize(na);
    for (int k = 0; k < na; k++) {
      Ty t = sd.types[k];
      int w = tsize(t);
      if (t == T_BOOL) {             // the API's bool column is one byte per event; the lanes read 4
        hb.own_cols[k].resize((size_t)b->n * w);
        const uint8_t* src = (const uint8_t*)b->cols[k];
        int32_t* dst = (int32_t*)hb.own_cols[k].data();
        for (int64_t i = 0; i < b->n; i++) dst[i] = src[i] ? 1 : 0;
        hb.cols[k] = HSpan<uint8_t>(hb.own_cols[k]);
      } else {
        hb.cols[k] = HSpan<uint8_t>((const uint8_t*)b->cols[k], (size_t)b->n * w);
      }
    }
    stage_batch(app, hb, false);
    // the clock each event is processed at: playback advances it from event timestamps before the
    // chunk is dispatched (InputHandler.send -> setCurrentTimestamp, once per send call), otherwise
    // it is the wall clock at push
    // (a buffer the app keeps: its pages stay mapped from one push to the next)
    app.push_now.reserve((size_t)b->n);
    int64_t* now_ev = app.push_now.p;
    // each advance also fires the due timers of every scheduler (App::send -> fire_timers).  Playback:
    // the clock follows event timestamps (TimestampGeneratorImpl.setCurrentTimestamp); otherwise the
    // shim's wall clock, which an event stamped later than it moves forward before the send
    TickBuf& tk = app.push_ticks;
    tk.clear();
    auto adv = [&](int64_t t, int64_t k) {
      if (app.playback ? t >= app.last_event_ts : t > app.now) {
        if (app.playback) app.last_event_ts = t;
        app.now = t;
        // the tick carries the arrival seq of the send it precedes (a routed batch: the event's own seq)
        tk.add(app.now, b->seq ? b->seq[k] : app.seq + k, k);
      }
    };
    {
      HostTimer ht("push clock");
      if (hb.batch) {
        adv(b->ts[b->n - 1], 0);
        std::fill(now_ev, now_ev + b->n, app.now);
        hb.now_uniform = true;
      } else if (host_threads(b->n) == 1) {
        for (int64_t k = 0; k < b->n; k++) { adv(b->ts[k], k); now_ev[k] = app.now; }
      } else {
        clock_ranges(app, b->ts, b->n, b->seq, app.seq, nullptr, 0, now_ev, tk);
      }
    }
    if (!tk.now.empty()) {
      HostTimer ht("push scheduler ticks");
      for (auto& e : app.execs) e->on_ticks(tk, stream);
    }
    hb.now_ev = HSpan<int64_t>(now_ev, (size_t)b->n);
    stage_batch(app, hb, true);
    hb.now = app.now;
    app.seq += b->n;
    dispatch(app, stream, hb);
    return SG_OK;
  })
}

// pred(k) for every k in [0, n), over thread ranges for large n
extern "C++" {
template <class P>
static bool ranged_ok(int64_t n, P pred) {
  const int nth = host_threads(n);
  std::vector<uint8_t> ok(nth, 1);
  host_parallel(nth, [&](int t) {
    for (int64_t k = n * t / nth, e = n * (t + 1) / nth; k < e; k++)
      if (!pred(k)) { ok[t] = 0; return; }
  });
  return std::all_of(ok.begin(), ok.end(), [](uint8_t x) { return x != 0; });
}
}

int sg_push_shard(sg_app* h, int stream, const sg_batch* b, int64_t n_global, const int64_t* global_ts, int64_t seq0) {
  App& app = h->a;
  SG_TRY({
    if (stream < 0 || stream >= (int)app.streams.size()) return fail(SG_E_INVALID, "bad stream index");
    if (!b || b->n < 0 || n_global < b->n || (n_global > 0 && !global_ts)) return fail(SG_E_INVALID, "bad shard batch");
    if (b->n > 0 && !b->seq) return fail(SG_E_INVALID, "a shard batch needs the global seq of each event");
    if (!ranged_ok(b->n, [&](int64_t k) { return b->seq[k] >= seq0 && b->seq[k] < seq0 + n_global && (!k || b->seq[k] > b->seq[k - 1]); }))
      return fail(SG_E_INVALID, "shard batch seqs must increase inside the global send");
    if (app.playback && !ranged_ok(n_global, [&](int64_t k) { return !k || global_ts[k] >= global_ts[k - 1]; }))
      return fail(SG_E_INVALID, "global timestamps go backwards");
    ensure_device(app);
    // the playback clock of the single runtime: InputHandler.send -> setCurrentTimestamp once per send
    // (TimestampGeneratorImpl.java:105-122) -- every global send ticks every rank's Schedulers, local
    // events or not; each local event is processed at the clock of its own send
    hvec<int64_t> now_loc((size_t)b->n);
    TickBuf& tk = app.push_ticks;
    tk.clear();
    // (a tick before the k-th local event is placed there: on_tick's position is local)
    auto tick = [&](int64_t t, int64_t sq, int64_t kloc) {
      if (app.playback ? t >= app.last_event_ts : t > app.now) {
        if (app.playback) app.last_event_ts = t;
        app.now = t;
        tk.add(app.now, sq, kloc);
      }
    };
    if (b->batch) {
      if (n_global > 0) tick(global_ts[n_global - 1], seq0, 0);
      std::fill(now_loc.begin(), now_loc.end(), app.now);
    } else if (host_threads(n_global) > 1) {
      clock_ranges(app, global_ts, n_global, nullptr, seq0, b->seq, b->n, now_loc.data(), tk);
    } else {
      int64_t k = 0;
      for (int64_t g = 0; g < n_global; g++) {
        tick(global_ts[g], seq0 + g, k);
        if (k < b->n && b->seq[k] == seq0 + g) now_loc[(size_t)k++] = app.now;
      }
    }
    if (!tk.now.empty())
      for (auto& e : app.execs) e->on_ticks(tk, stream);
    app.seq = seq0 + n_global;
    if (b->n == 0) return SG_OK;
    const StreamDef& sd = app.streams[stream];
    const int na = (int)sd.types.size();
    HostBatch hb;
    if (b->nulls) {
      bool any = false;
      for (int64_t i = 0; i < b->n * na && !any; i++) any = b->nulls[i] != 0;
      if (any) {
        for (int q : app.subscribers[stream])
          if (!app.execs[q]->supports_nulls())
            return fail(SG_E_UNSUPPORTED, "query '" + app.qnames[q] + "' runs on a path without null attribute values");
        hb.nulls = HSpan<uint8_t>(b->nulls, (size_t)(b->n * na));
      }
    }
    hb.stream = stream;
    hb.n = b->n;
    hb.seq0 = b->seq[0];
    hb.seqs = HSpan<int64_t>(b->seq, (size_t)b->n);
    hb.batch = b->batch != 0;
    hb.ts = HSpan<int64_t>(b->ts, (size_t)b->n);
    hb.cols.resize(na);
    hb.own_cols.resize(na);
    for (int k = 0; k < na; k++) {
      const Ty t = sd.types[k];
      if (t == T_BOOL) {
        hb.own_cols[k].resize((size_t)b->n * 4);
        const uint8_t* src = (const uint8_t*)b->cols[k];
        int32_t* dst = (int32_t*)hb.own_cols[k].data();
        for (int64_t i = 0; i < b->n; i++) dst[i] = src[i] ? 1 : 0;
        hb.cols[k] = HSpan<uint8_t>(hb.own_cols[k]);
      } else {
        hb.cols[k] = HSpan<uint8_t>((const uint8_t*)b->cols[k], (size_t)b->n * tsize(t));
      }
    }
    hb.own_now = std::move(now_loc);
    hb.now_ev = HSpan<int64_t>(hb.own_now);
    hb.now_uniform = b->batch != 0;
    hb.now = app.now;
    stage_batch(app, hb, false);
    stage_batch(app, hb, true);
    dispatch(app, stream, hb);
    return SG_OK;
  })
}

int sg_push_device(sg_app* h, int stream, int64_t n, const int64_t* d_ts, const void* const* d_cols, int batch,
                   void* hip_stream) {
  App& app = h->a;
  SG_TRY({
    if (stream < 0 || stream >= (int)app.streams.size()) return fail(SG_E_INVALID, "bad stream index");
    if (n < 0 || (n > 0 && !d_ts)) return fail(SG_E_INVALID, "bad batch");
    ensure_device(app);
    for (int q : app.subscribers[stream])
      app.execs[q]->push_device(stream, n, d_ts, d_cols, batch, hip_stream ? (hipStream_t)hip_stream : app.stream);
    app.seq += n;
    return SG_OK;
  })
}

int sg_push_device_seq(sg_app* h, int stream, int64_t n, const int64_t* d_ts, const void* const* d_cols,
                       const int64_t* d_seq, int batch, void* hip_stream) {
  const int rc = sg_push_device(h, stream, n, d_ts, d_cols, batch, hip_stream);
  if (rc != SG_OK) return rc;
  App& app = h->a;
  SG_TRY({
    for (int q : app.subscribers[stream]) app.execs[q]->set_device_seq(d_seq);
    return SG_OK;
  })
}

int sg_set_halo(sg_app* h, int stream, int64_t n_halo) {
  App& app = h->a;
  SG_TRY({
    if (stream < 0 || stream >= (int)app.streams.size() || n_halo < 0) return fail(SG_E_INVALID, "bad halo");
    for (int q : app.subscribers[stream]) app.execs[q]->set_halo(stream, n_halo);
    return SG_OK;
  })
}

int sg_advance_time(sg_app* h, int64_t now_ms) {
  App& app = h->a;
  SG_TRY({
    ensure_device(app);
    if (now_ms > app.now) app.now = now_ms;
    for (auto& e : app.execs) e->advance_time(app.now);
    for (auto& e : app.execs) e->on_tick(app.now, app.seq, -1, 0);   // App.set_time -> fire_timers
    return SG_OK;
  })
}

static int flush_impl(sg_app* h, bool materialise, hipStream_t s) {
  App& app = h->a;
  HostTimer ht("flush");
  SG_TRY({
    ensure_device(app);
    std::vector<Callback> cbs;
    if (app.early.empty()) {         // (an emptied vector's capacity: no first touch of ~80 B per callback)
      cbs.swap(app.cb_spare);
      cbs.clear();
    } else {
      cbs.swap(app.early);
    }
    for (auto& e : app.execs) e->flush(cbs, materialise, s);
    if (!materialise) { cbs.clear(); if (app.cb_spare.capacity() < cbs.capacity()) app.cb_spare.swap(cbs); return SG_OK; }
    // a bulk entry (columnar callbacks of one query) stays one entry when it is the flush's only output and goes
    // to one kind of callback; otherwise it is expanded so that the merge below orders every callback
    const bool bulk_alone = cbs.size() == 1 && cbs[0].blk && !(app.qout_stream[cbs[0].target] >= 0 &&
                             app.stream_cb[app.qout_stream[cbs[0].target]] && app.query_cb[cbs[0].target]);
    if (!bulk_alone && std::any_of(cbs.begin(), cbs.end(), [](const Callback& c) { return c.blk != nullptr; })) {
      std::vector<Callback> ex;
      for (auto& c : cbs) {
        if (!c.blk) { ex.push_back(std::move(c)); continue; }
        const OutBlock& b = *c.blk;
        for (int64_t k = 0; k < b.ncb(); k++) {
          Callback x;
          x.seq = b.cb_seq[k]; x.order = c.order; x.kind = c.kind; x.target = c.target; x.ts = b.cb_ts[k];
          for (int64_t r = b.cb_row[k]; r < b.cb_row[k + 1]; r++) {
            OutEvent e;
            e.ts = b.ts[r];
            for (int w = 0; w < b.width; w++) { e.raw.push_back(b.raw[r * b.width + w]); e.nul.push_back(0); }
            x.ev.push_back(std::move(e));
          }
          ex.push_back(std::move(x));
        }
      }
      cbs.swap(ex);
    }
    auto before = [](const Callback& x, const Callback& y) {
      if (x.seq != y.seq) return x.seq < y.seq;
      return x.order < y.order;
    };
    if (!std::is_sorted(cbs.begin(), cbs.end(), before)) std::stable_sort(cbs.begin(), cbs.end(), before);
    // every callback to its query's callback and none to a stream callback, nothing queued: the vector is the output
    if (app.out.empty() && std::all_of(cbs.begin(), cbs.end(), [&](const Callback& c) {
          const int os = app.qout_stream[c.target];
          return !(os >= 0 && app.stream_cb[os]) && app.query_cb[c.target];
        })) {
      app.out.clear();
      app.out.swap(cbs);               // (the emptied output vector's capacity goes back to the spare)
      if (app.cb_spare.capacity() < cbs.capacity()) app.cb_spare.swap(cbs);
      return SG_OK;
    }
    app.out.reserve(app.out.size() + cbs.size());
    for (auto& c : cbs) {
      int q = c.target;
      int os = app.qout_stream[q];
      const bool to_stream = os >= 0 && app.stream_cb[os];
      if (to_stream) {
        // InsertIntoStreamCallback: EXPIRED -> CURRENT, one StreamCallback call per chunk
        Callback sc = c;
        sc.kind = 1;
        sc.target = os;
        for (auto& e : sc.ev) e.expired = false;
        if (app.query_cb[q]) app.out.push_back(std::move(c));
        app.out.push_back(std::move(sc));
      } else if (app.query_cb[q]) {
        app.out.push_back(std::move(c));
      }
    }
    return SG_OK;
  })
}

int sg_flush(sg_app* h) {
  SG_TRY(ensure_device(h->a));
  return flush_impl(h, true, h->a.stream);
}

int sg_flush_device(sg_app* h, void* hip_stream) {
  SG_TRY(ensure_device(h->a));
  return flush_impl(h, false, hip_stream ? (hipStream_t)hip_stream : h->a.stream);
}

// ---- persistence (SiddhiAppRuntime.snapshot() / restore(byte[])) ----
static constexpr uint64_t SG_SNAP_MAGIC = 0x3170616e73677366ull;   // "fsgsnap1"

int sg_snapshot(sg_app* h, uint8_t** out, int64_t* len) {
  App& app = h->a;
  if (!out || !len) return fail(SG_E_INVALID, "null output pointer");
  *out = nullptr;
  *len = 0;
  int rc = flush_impl(h, true, app.stream);   // the state is taken between flushes; its callbacks stay queued
  if (rc != SG_OK) return rc;
  SG_TRY({
    for (size_t q = 0; q < app.execs.size(); q++)
      if (app.execs[q]->path != SG_E_UNSUPPORTED && !app.execs[q]->can_snapshot())
        return fail(SG_E_UNSUPPORTED, "query '" + app.qnames[q] + "' runs on a path without snapshot support");
    SnapWriter w;
    w.pod(SG_SNAP_MAGIC);
    w.pod<uint64_t>(app.execs.size());
    for (size_t q = 0; q < app.execs.size(); q++) { w.str(app.qnames[q]); w.pod(app.execs[q]->path); }
    w.pod(app.seq); w.pod(app.now); w.pod(app.last_event_ts); w.pod(app.started);
    w.pod<uint64_t>(app.strings.size());
    for (auto& str : app.strings) w.str(str);
    w.pod<uint64_t>(app.purges.size());   // @purge task schedules (PartitionRuntimeImpl.initPartition)
    for (auto& pc : app.purges) {
      w.pod(pc.first); w.pod(pc.second.t0);
      PurgeFirst f(pc.second.first.begin(), pc.second.first.end());
      w.vec(f);
    }
    for (auto& e : app.execs)
      if (e->path != SG_E_UNSUPPORTED) e->snapshot(w, app.stream);
    *out = (uint8_t*)malloc(w.b.size());
    if (!*out) return fail(SG_E_INVALID, "out of host memory");
    std::memcpy(*out, w.b.data(), w.b.size());
    *len = (int64_t)w.b.size();
    return SG_OK;
  })
}

}  // extern "C"
struct PurgeRestore {   // one @purge partition's schedule, parsed before sg_restore applies it
  int64_t t0;
  PurgeFirst first;
};
extern "C" {

int sg_restore(sg_app* h, const uint8_t* buf, int64_t len) {
  App& app = h->a;
  if (!buf || len < 0) return fail(SG_E_INVALID, "bad snapshot buffer");
  SG_TRY({
    ensure_device(app);
    SnapReader r(buf, (size_t)len);
    if (r.pod<uint64_t>() != SG_SNAP_MAGIC) return fail(SG_E_INVALID, "not a siddhi_gfx snapshot");
    if (r.pod<uint64_t>() != app.execs.size()) return fail(SG_E_INVALID, "snapshot of another app (query count)");
    for (size_t q = 0; q < app.execs.size(); q++) {
      if (r.str() != app.qnames[q] || r.pod<int>() != app.execs[q]->path)
        return fail(SG_E_INVALID, "snapshot of another app (query '" + app.qnames[q] + "')");
    }
    // parse and check the header before anything changes; the execs' restores follow, and one that fails
    // leaves every query reset (a restarted runtime), never half-restored
    const int64_t seq = r.pod<int64_t>();
    const int64_t now = r.pod<int64_t>();
    const int64_t last_ts = r.pod<int64_t>();
    const bool started = r.pod<bool>();
    // the dictionary: string ids inside the state stay valid (ids interned since are appended after)
    const uint64_t ns = r.pod<uint64_t>();
    std::vector<std::string> strs(ns);
    for (auto& str : strs) str = r.str();
    for (size_t i = 0; i < std::min<size_t>(ns, app.strings.size()); i++)
      if (app.strings[i] != strs[i]) return fail(SG_E_INVALID, "snapshot dictionary conflicts with strings interned here");
    const uint64_t np = r.pod<uint64_t>();
    if (np != app.purges.size()) return fail(SG_E_INVALID, "snapshot of another app (@purge partitions)");
    std::vector<PurgeRestore> pst;
    std::vector<decltype(app.purges.begin())> pit;
    for (uint64_t k = 0; k < np; k++) {
      const int part = r.pod<int>();
      auto it = app.purges.find(part);
      if (it == app.purges.end()) return fail(SG_E_INVALID, "snapshot of another app (@purge partitions)");
      const int64_t t0 = r.pod<int64_t>();
      PurgeFirst f;
      r.vec(f);
      pit.push_back(it);
      pst.push_back(PurgeRestore{t0, std::move(f)});
    }
    for (size_t i = app.strings.size(); i < ns; i++) app.intern(strs[i]);   // append-only: harmless on failure
    try {
      for (auto& e : app.execs)
        if (e->path != SG_E_UNSUPPORTED) e->restore(r, app.stream);
      if (r.at != r.n) throw Error(SG_E_INVALID, "trailing bytes in snapshot");
    } catch (...) {
      reset_app(app);   // never half-restored: the app is left as sg_reset leaves it
      throw;
    }
    app.seq = seq; app.now = now; app.last_event_ts = last_ts;
    for (size_t k = 0; k < pit.size(); k++) {
      pit[k]->second.t0 = pst[k].t0;
      pit[k]->second.first.clear();
      pit[k]->second.first.insert(pst[k].first.begin(), pst[k].first.end());
    }
    app.out.clear();
    app.early.clear();
    app.blocks.clear();
    app.started = app.started || started;
    return SG_OK;
  })
}

void sg_free_buffer(void* p) { free(p); }

int64_t sg_out_ncallbacks(sg_app* h) {
  int64_t n = 0;
  for (auto& c : h->a.out) n += c.blk ? c.blk->ncb() : 1;
  return n;
}

// the queued callbacks hold no bulk entry: callback i is output i (the copies below then run over thread ranges)
static bool out_flat(const std::vector<Callback>& out) {
  return std::none_of(out.begin(), out.end(), [](const Callback& c) { return c.blk != nullptr; });
}

int sg_out_callbacks(sg_app* h, int32_t* kind, int32_t* target, int64_t* ts, int32_t* n_in, int32_t* n_rm) {
  auto& out = h->a.out;
  const int nth = host_threads((int64_t)out.size() * 4);
  if (nth > 1 && out_flat(out)) {
    host_parallel(nth, [&](int t) {
      for (size_t i = out.size() * t / nth, e = out.size() * (t + 1) / nth; i < e; i++) {
        kind[i] = out[i].kind;
        target[i] = out[i].target;
        ts[i] = out[i].ts;
        int ni = 0, nr = 0;
        for (auto& x : out[i].ev) (x.expired ? nr : ni)++;
        n_in[i] = ni;
        n_rm[i] = nr;
      }
    });
    return SG_OK;
  }
  size_t o = 0;
  for (size_t i = 0; i < out.size(); i++) {
    if (out[i].blk) {                                   // a bulk entry: its callbacks' columns
      const OutBlock& b = *out[i].blk;
      const int64_t m = b.ncb();
      std::fill(kind + o, kind + o + m, out[i].kind);
      std::fill(target + o, target + o + m, out[i].target);
      std::memcpy(ts + o, b.cb_ts.data(), (size_t)m * 8);
      for (int64_t k = 0; k < m; k++) n_in[o + (size_t)k] = (int32_t)(b.cb_row[k + 1] - b.cb_row[k]);
      std::fill(n_rm + o, n_rm + o + m, 0);
      o += (size_t)m;
      continue;
    }
    kind[o] = out[i].kind;
    target[o] = out[i].target;
    ts[o] = out[i].ts;
    int ni = 0, nr = 0;
    for (auto& e : out[i].ev) (e.expired ? nr : ni)++;
    n_in[o] = ni;
    n_rm[o] = nr;
    o++;
  }
  return SG_OK;
}

int64_t sg_out_nrows(sg_app* h) {
  int64_t n = 0;
  for (auto& c : h->a.out) n += c.blk ? (int64_t)c.blk->ts.size() : (int64_t)c.ev.size();
  return n;
}

// one callback's rows (current events first, then expired: the order sg_out_callbacks counts them in) at row r
static int64_t out_cb_rows(const Callback& c, int width, int64_t r, int64_t* ts, int64_t* raw, uint8_t* nulls) {
  for (int part = 0; part < 2; part++) {
    for (auto& e : c.ev) {
      if (e.expired != (part == 1)) continue;
      ts[r] = e.ts;
      for (int k = 0; k < width; k++) {
        bool have = k < (int)e.raw.size();
        raw[r * width + k] = have ? e.raw[k] : 0;
        nulls[r * width + k] = have ? e.nul[k] : 1;
      }
      r++;
    }
  }
  return r;
}

int sg_out_rows(sg_app* h, int width, int64_t* ts, int64_t* raw, uint8_t* nulls) {
  auto& out = h->a.out;
  const int nth = host_threads((int64_t)out.size() * 4);
  if (nth > 1 && out_flat(out)) {
    std::vector<int64_t> r0(out.size() + 1, 0);
    for (size_t i = 0; i < out.size(); i++) r0[i + 1] = r0[i] + (int64_t)out[i].ev.size();
    host_parallel(nth, [&](int t) {
      for (size_t i = out.size() * t / nth, e = out.size() * (t + 1) / nth; i < e; i++)
        out_cb_rows(out[i], width, r0[i], ts, raw, nulls);
    });
    return SG_OK;
  }
  int64_t r = 0;
  for (auto& c : out) {
    if (c.blk) {
      const OutBlock& b = *c.blk;
      const int64_t m = (int64_t)b.ts.size();
      // a bulk block's rows, widened to the caller's width; split over host threads (memory-bound copies)
      sg::par_rows(m, [&](int64_t x0, int64_t x1) {
        std::memcpy(ts + r + x0, b.ts.data() + x0, (size_t)(x1 - x0) * 8);
        if (width == b.width) {
          std::memcpy(raw + (r + x0) * width, b.raw.data() + x0 * width, (size_t)((x1 - x0) * width) * 8);
          std::memset(nulls + (r + x0) * width, 0, (size_t)((x1 - x0) * width));
        } else {
          for (int64_t x = x0; x < x1; x++)
            for (int k = 0; k < width; k++) {
              const bool have = k < b.width;
              raw[(r + x) * width + k] = have ? b.raw[x * b.width + k] : 0;
              nulls[(r + x) * width + k] = have ? 0 : 1;
            }
        }
      });
      r += m;
      continue;
    }
    r = out_cb_rows(c, width, r, ts, raw, nulls);
  }
  return SG_OK;
}

int sg_out_callback_seq(sg_app* h, int64_t* seq) {
  auto& out = h->a.out;
  size_t o = 0;
  for (size_t i = 0; i < out.size(); i++) {
    if (out[i].blk) {
      std::memcpy(seq + o, out[i].blk->cb_seq.data(), (size_t)out[i].blk->ncb() * 8);
      o += (size_t)out[i].blk->ncb();
    } else {
      seq[o++] = out[i].seq;
    }
  }
  return SG_OK;
}

int sg_out_callback_tick(sg_app* h, int32_t* sched, int64_t* deadline) {
  auto& out = h->a.out;
  size_t o = 0;
  for (size_t i = 0; i < out.size(); i++) {
    const int64_t m = out[i].blk ? out[i].blk->ncb() : 1;
    for (int64_t k = 0; k < m; k++, o++) {
      sched[o] = out[i].tsched;
      deadline[o] = out[i].tdl;
    }
  }
  return SG_OK;
}

int sg_out_clear(sg_app* h) {
  auto& out = h->a.out;
  const int nth = host_threads((int64_t)out.size() * 4);
  if (nth > 1)                     // (the callbacks' row vectors freed over thread ranges)
    host_parallel(nth, [&](int t) {
      for (size_t i = out.size() * t / nth, e = out.size() * (t + 1) / nth; i < e; i++) std::vector<OutEvent>().swap(out[i].ev);
    });
  out.clear();
  // free every OutBlock (and return its pinned memory to the pool) that no queued upstream callback (`early`)
  // still references; the referenced ones stay until the flush that drains them
  auto& blocks = h->a.blocks;
  if (h->a.early.empty()) {
    blocks.clear();
  } else {
    std::unordered_set<const OutBlock*> live;
    for (const auto& c : h->a.early) if (c.blk) live.insert(c.blk);
    blocks.erase(std::remove_if(blocks.begin(), blocks.end(),
                                [&](const std::unique_ptr<OutBlock>& b) { return !live.count(b.get()); }),
                 blocks.end());
  }
  return SG_OK;
}

int64_t sg_last_match_count(sg_app* h, int q) {
  if (!h || q < 0 || q >= (int)h->a.execs.size()) return fail(SG_E_INVALID, "bad query index");
  return h->a.execs[q]->last_matches;
}

int64_t sg_query_kernel_source(sg_app* h, int q, char* buf, int64_t cap) {
  if (!h || q < 0 || q >= (int)h->a.execs.size() || cap < 0) return fail(SG_E_INVALID, "bad query index");
  std::string src;
  SG_TRY({
    if (!h->a.execs[q]->kernel_source(src)) return fail(SG_E_UNSUPPORTED, "the query's path has no compiled kernel");
  });
  if (buf && cap > 0) {
    const size_t m = std::min<size_t>(src.size(), (size_t)cap - 1);
    memcpy(buf, src.data(), m);
    buf[m] = 0;
  }
  return (int64_t)src.size();
}

int sg_query_compile(sg_app* h, int q, double* compile_ms, int* from_cache) {
  if (!h || q < 0 || q >= (int)h->a.execs.size()) return fail(SG_E_INVALID, "bad query index");
  double ms = 0;
  bool disk = false;
  std::string err;
  SG_TRY({
    if (!h->a.execs[q]->compile_kernel(ms, disk, err)) {
      if (err.empty()) return fail(SG_E_UNSUPPORTED, "the query's path has no compiled kernel");
      return fail(SG_E_DEVICE, "compiling the query's kernel: " + err);
    }
  });
  if (compile_ms) *compile_ms = ms;
  if (from_cache) *from_cache = disk ? 1 : 0;
  return SG_OK;
}

int64_t sg_query_buffered(sg_app* h, int q) {
  if (!h || q < 0 || q >= (int)h->a.execs.size()) return fail(SG_E_INVALID, "bad query index");
  return h->a.execs[q]->buffered();
}

int sg_query_shard_mode(sg_app* h, int q, int mode) {
  if (!h || q < 0 || q >= (int)h->a.execs.size() || mode < 0 || mode > 2) return fail(SG_E_INVALID, "bad query index or mode");
  SG_TRY({
    if (!h->a.execs[q]->shard_mode(mode))
      return fail(SG_E_UNSUPPORTED, "shard mode needs a partitioned pattern query with absent states");
  });
  return SG_OK;
}

int64_t sg_query_sched_fires(sg_app* h, int q, sg_sched_fire* out, int64_t cap) {
  if (!h || q < 0 || q >= (int)h->a.execs.size() || cap < 0) return fail(SG_E_INVALID, "bad query index");
  const int64_t c = h->a.execs[q]->sched_fires(out, out ? cap : 0);
  return c < 0 ? fail(SG_E_UNSUPPORTED, "query is not in shard mode") : c;
}

int64_t sg_query_sched_clock(sg_app* h, int q, int64_t* now, int64_t cap, int64_t* min_wait) {
  if (!h || q < 0 || q >= (int)h->a.execs.size() || cap < 0) return fail(SG_E_INVALID, "bad query index");
  const int64_t c = h->a.execs[q]->sched_clock(now, now ? cap : 0, min_wait);
  return c < 0 ? fail(SG_E_UNSUPPORTED, "not a partitioned query with absent states") : c;
}

int64_t sg_query_sched_ops(sg_app* h, int q, sg_sched_op* out, int64_t cap) {
  if (!h || q < 0 || q >= (int)h->a.execs.size() || cap < 0) return fail(SG_E_INVALID, "bad query index");
  const int64_t c = h->a.execs[q]->sched_ops(out, out ? cap : 0);
  return c < 0 ? fail(SG_E_UNSUPPORTED, "query is not in shard mode 2") : c;
}

int64_t sg_query_state_json(sg_app* h, int q, char* buf, int64_t cap) {
  if (!h || q < 0 || q >= (int)h->a.execs.size() || cap < 0) return fail(SG_E_INVALID, "bad query index");
  SG_TRY({
    ensure_device(h->a);
    std::string js;
    if (!h->a.execs[q]->state_json(js, h->a.stream)) return fail(SG_E_UNSUPPORTED, "not a pattern query path");
    if (buf && cap > 0) std::memcpy(buf, js.data(), (size_t)std::min<int64_t>(cap, (int64_t)js.size()));
    return (int64_t)js.size();
  })
}

int sg_query_shard_resolver(sg_app* h, int q, sg_shard_resolver_fn resolve, void* user) {
  if (!h || q < 0 || q >= (int)h->a.execs.size() || !resolve) return fail(SG_E_INVALID, "bad query index or resolver");
  SG_TRY({
    if (!h->a.execs[q]->shard_resolver(resolve, user))
      return fail(SG_E_UNSUPPORTED, "shard mode needs a partitioned pattern query with absent states");
  });
  return SG_OK;
}

int sg_query_sched_defer(sg_app* h, int q, int64_t key, int32_t tick, int32_t sched) {
  if (!h || q < 0 || q >= (int)h->a.execs.size() || tick < 0 || sched < 0 || sched > 127)
    return fail(SG_E_INVALID, "bad query index, tick or scheduler");
  if (!h->a.execs[q]->sched_defer(key, tick, sched))
    return fail(SG_E_INVALID, "no instance of that key in shard mode");
  return SG_OK;
}

double sg_last_kernel_ms(sg_app* h, const char* kernel) {
  for (auto& e : h->a.execs) {
    auto it = e->kernel_ms.find(kernel);
    if (it != e->kernel_ms.end()) return it->second;
  }
  return -1.0;
}

}  // extern "C"
