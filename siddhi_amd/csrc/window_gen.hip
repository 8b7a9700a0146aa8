// window_gen.hip — execution path SG_PATH_WINDOW: single-stream queries in full generality.
//
// Query shape:  [partition with (a of S) begin]
//               from S[f]* [#window.length(L) | #window.time(T) | #window.lengthBatch(L[, streamCurrent])]
//               select <expressions, aggregators> [group by ...] [having ...] [order by ...] [limit / offset]
//               insert [current | expired | all] events into ...
//
// WindowAggExec (window_agg.hip) keeps the throughput shapes (current events, one group-by attribute, plain
// aggregators); this path takes every other single-stream query and restates the reference per chunk:
//   * the device evaluates, for every pushed event, the filter conjunction and the pre-selector values
//     the selector reads (k_gw_eval: plain select expressions, aggregator arguments, group-by keys,
//     having variables -- SelectorParser, build_selector in selector.hpp);
//   * the window processors run over the filtered events of each chunk with the reference's queue
//     discipline and emit the selector chunk of CURRENT / EXPIRED / RESET events:
//       LengthWindowProcessor.process (CORE/query/processor/stream/window/LengthWindowProcessor.java:106-141),
//       TimeWindowProcessor.process (TimeWindowProcessor.java:133-169) with its Scheduler timer
//         (notifyAt(ts + T) per new timestamp, Scheduler.java:57-140: every due deadline fires one TIMER
//         chunk when the app clock moves -- TimestampGeneratorImpl / sg_advance_time),
//       LengthBatchWindowProcessor.process (LengthBatchWindowProcessor.java:154-351, both modes);
//   * QuerySelector runs on each chunk (SelectorStage): aggregators with their add / remove / reset
//     arithmetic per group key, having, group-by batching, order by, offset, limit;
//   * `partition with (a of S)`: one window + selector state per key value, created on the key's first
//     event; a batch send is split into runs of consecutive same-key events (PartitionStreamReceiver
//     .java:82-282), each run one chunk of its instance.
// Partitioned time windows keep one Scheduler state per instance in the Scheduler's key -> state
// HashMap; onTimeChange collects the due states in its iteration order and keeps ONE per distinct first
// deadline (SchedulerState.compareTo == 0, Scheduler.java:77-97, 364-366): instances sharing a deadline
// fire at later ticks.  Restated with the JDK 8 HashMap order (SchedMap).  Streams a partition does not
// key (broadcast) are not lowered; an event whose partition key is null is dropped (PartitionStreamReceiver).

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <deque>
#include <memory>
#include <unordered_map>

#include "runtime.hpp"
#include "selector.hpp"
#include "snapshot.hpp"
#include "siddhi_gfx.h"
#include "selector_dev.hpp"
#include "window_dev.hpp"
#include "window_proc.hpp"

namespace sg {

constexpr int GW_MAXA = 16;   // stream attributes
constexpr int GW_B = 256;

struct GwCols {
  const uint8_t* c[GW_MAXA];
  int32_t w[GW_MAXA];
  const uint8_t* nul;   // [event * na + attr] null flags (nullptr: no null pushed yet)
  int32_t na;
};

struct GwLoader {
  const GwCols* cols;
  int64_t e;
  __device__ bool load(int slot, int attr, int64_t& v) const {
    (void)slot;
    if (cols->nul && cols->nul[e * cols->na + attr]) return false;
    v = cols->w[attr] == 8 ? ((const int64_t*)cols->c[attr])[e] : (int64_t)((const int32_t*)cols->c[attr])[e];
    return true;
  }
};

// one thread per event: filter conjunction, then the pre-selector values of the events that pass
__global__ void __launch_bounds__(GW_B) k_gw_eval(int64_t lo, int64_t n, GwCols cols, const Prog* __restrict__ progs,
                                                   int has_filter, int nv, uint8_t* __restrict__ flags,
                                                   int64_t* __restrict__ pv, uint8_t* __restrict__ pn, int64_t pitch) {
  __shared__ int64_t rf[MAX_REG * GW_B];
  const int64_t e = lo + (int64_t)blockIdx.x * GW_B + threadIdx.x;
  if (e >= n) return;
  GwLoader ld{&cols, e};
  const bool ok = has_filter ? run_pred(progs[0], ld, rf + threadIdx.x, GW_B) : true;
  flags[e - lo] = (uint8_t)ok;
  if (!ok) return;
  for (int k = 0; k < nv; k++) {
    int64_t v = 0;
    bool isnull = false;
    run(progs[1 + k], ld, v, isnull, rf + threadIdx.x, GW_B);
    pv[(int64_t)k * pitch + (e - lo)] = v;
    pn[(int64_t)k * pitch + (e - lo)] = (uint8_t)isnull;
  }
}

enum GwWin { GW_NONE = WK_NONE, GW_LENGTH = WK_LENGTH, GW_TIME = WK_TIME, GW_BATCH = WK_BATCH };

// java.util.HashMap<partition key, SchedulerState> iteration order (JDK 8: bins by the spread hash, a new
// key at the head of its bin, order-preserving resize splits; a treeified bin is refused)
struct SchedMap {
  std::vector<std::vector<std::pair<int32_t, int>>> tab;   // bin -> chain of (hash, instance)
  size_t size = 0, thr = 0;
  void resize() {
    const size_t old = tab.size();
    if (old == 0) { tab.assign(16, {}); thr = 12; return; }
    std::vector<std::vector<std::pair<int32_t, int>>> nt(old * 2);
    for (size_t b = 0; b < old; b++)
      for (auto& e : tab[b]) nt[((uint32_t)e.first & (uint32_t)old) ? b + old : b].push_back(e);
    tab.swap(nt);
    thr *= 2;
  }
  void touch(int32_t h, int id) {   // computeIfAbsent
    if (size > thr || tab.empty()) resize();
    auto& bin = tab[(uint32_t)h & (uint32_t)(tab.size() - 1)];
    for (auto& e : bin) if (e.second == id) return;
    const size_t cnt = bin.size();
    bin.insert(bin.begin(), {h, id});
    if (cnt >= 7) {
      if (tab.size() < 64) resize();
      else throw Error(-2, "partition Scheduler map bin would be treeified (not lowered)");
    }
    size++;
  }
  void remove(int32_t h, int id) {
    if (tab.empty()) return;
    auto& bin = tab[(uint32_t)h & (uint32_t)(tab.size() - 1)];
    for (size_t i = 0; i < bin.size(); i++)
      if (bin[i].second == id) { bin.erase(bin.begin() + i); size--; return; }
  }
  void clear() { tab.clear(); size = thr = 0; }
};

struct GenWindowExec : Exec {
  int st = -1;
  int wkind = GW_NONE;
  int64_t L = 0;                 // length / batch count, or time span (ms)
  bool stream_current = false;   // lengthBatch(L, true)
  bool has_filter = false;
  std::vector<Prog> progs;       // [filter] + pre-selector value programs
  int nv = 0;
  SelSpec sp;
  std::unique_ptr<SelectorStage> sel;
  bool partitioned = false;
  int pattr = -1;
  Ty key_ty = T_STRING;

  // events pushed and not yet planned (device columns hold [0, n); planned up to `done`)
  std::vector<DCol> cols;
  DBuf<uint8_t> nulcol;            // null flags [event][attr], from the first null on
  bool has_nul = false;
  bool supports_nulls() const override { return true; }
  int64_t n = 0, done = 0;
  std::vector<int64_t> h_ts, h_now, h_seq, h_cseq, h_key;   // per event: ts, clock, seq, chunk seq, key
  std::vector<uint8_t> h_knull;                              // partition key is null (event dropped)
  SchedMap smap;                                             // partitioned time window: Scheduler states
  std::vector<int64_t> h_chunk;                              // send-call id per event
  int64_t chunk_ctr = 0;
  struct Tick { int64_t now, seq, pos; };
  std::vector<Tick> ticks;                                   // Scheduler ticks before event `pos`
  DBuf<Prog> d_progs;
  DBuf<uint8_t> d_flags, d_pn;
  DBuf<int64_t> d_pv;
  hipEvent_t e0 = nullptr, e1 = nullptr;

  // a retained event: the pre-selector values of one filtered event (window queues hold clones)
  struct Val { std::vector<int64_t> v; std::vector<uint8_t> nul; };
  using Item = WinItem<std::shared_ptr<const Val>>;
  struct Inst : WinState<std::shared_ptr<const Val>> {   // the window processor's state (window_proc.hpp)
    int id = 0;
    int32_t khash = 0;                   // partitioned time window: spread hash of the key string
    int64_t key = 0;                     // partition key value
    int64_t seen = INT64_MIN;            // @purge: the key's last initPartition time
  };
  WinSpec wspec() const {
    WinSpec w;
    w.kind = wkind; w.L = L; w.stream_current = stream_current; w.expired_on = sp.expired_on;
    return w;
  }
  std::unordered_map<int64_t, std::unique_ptr<Inst>> inst;
  std::unique_ptr<Inst> single;
  PurgeClock* purge = nullptr;                  // @purge of the partition (runtime.hpp)
  std::vector<std::unique_ptr<Inst>> purged;    // cleaned instances (ids stay unique)

  // the purge task's cleanGroupByStates for one key: window, Scheduler state and selector state (a new
  // instance id) are gone; the key's next chunk creates a fresh instance
  void purge_inst(Inst* I) {
    if (wkind == GW_TIME) smap.remove(I->khash, I->id);
    auto it = inst.find(I->key);
    purged.push_back(std::move(it->second));
    inst.erase(it);
  }

  ~GenWindowExec() override {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
  }

  void push(const HostBatch& b) override {
    if (b.stream != st) return;
    hipStream_t s = app->stream;
    for (size_t k = 0; k < cols.size(); k++) {
      cols[k].b.reserve((n + b.n) * cols[k].w, true, s, n * cols[k].w);
      SG_HIP(hipMemcpyAsync(cols[k].b.p + n * cols[k].w, b.cols[k].data(), b.n * cols[k].w, hipMemcpyHostToDevice, s));
    }
    const size_t na = cols.size();
    if (!b.nulls.empty() && !has_nul) {
      has_nul = true;
      nulcol.reserve(std::max<size_t>((n + b.n) * na, 1));
      SG_HIP(hipMemsetAsync(nulcol.p, 0, std::max<size_t>(n * na, 1), s));
    }
    if (has_nul) {
      nulcol.reserve((n + b.n) * na, true, s, n * na);
      if (b.nulls.empty()) SG_HIP(hipMemsetAsync(nulcol.p + n * na, 0, b.n * na, s));
      else SG_HIP(hipMemcpyAsync(nulcol.p + n * na, b.nulls.data(), b.n * na, hipMemcpyHostToDevice, s));
    }
    const int64_t first_seq = b.seqs.empty() ? b.seq0 : b.seqs[0];
    for (int64_t k = 0; k < b.n; k++) {
      const int64_t sq = b.seqs.empty() ? b.seq0 + k : b.seqs[k];
      h_ts.push_back(b.ts[k]);
      h_now.push_back(b.now_ev.empty() ? b.now : b.now_ev[k]);
      h_seq.push_back(sq);
      h_cseq.push_back(b.batch ? first_seq : sq);   // InputHandler.send(Event[]): one arrival index
      h_chunk.push_back(b.batch ? chunk_ctr : chunk_ctr + k);
      if (partitioned) {
        const int w = tsize(app->streams[st].types[pattr]);
        int64_t key;
        if (w == 8) std::memcpy(&key, b.cols[pattr].data() + (size_t)k * 8, 8);
        else { int32_t x; std::memcpy(&x, b.cols[pattr].data() + (size_t)k * 4, 4); key = x; }
        h_key.push_back(key);
        h_knull.push_back(!b.nulls.empty() && b.nulls[(size_t)k * na + pattr]);
      }
    }
    chunk_ctr += b.batch ? 1 : b.n;
    n += b.n;
    SG_HIP(hipStreamSynchronize(s));
  }

  void on_tick(int64_t now, int64_t seq, int stream, int64_t k) override {
    if (wkind != GW_TIME) return;
    ticks.push_back({now, seq, n + (stream == st ? k : 0)});
  }
  void on_ticks(const TickBuf& t, int stream) override {
    if (wkind != GW_TIME) return;
    const size_t m = t.now.size();
    ticks.reserve(ticks.size() + m);
    for (size_t i = 0; i < m; i++) ticks.push_back({t.now[i], t.seq[i], n + (stream == st ? t.k[i] : 0)});
  }

  void reset() override {
    n = done = 0; chunk_ctr = 0; has_nul = false;
    h_ts.clear(); h_now.clear(); h_seq.clear(); h_cseq.clear(); h_chunk.clear(); h_key.clear(); h_knull.clear();
    ticks.clear();
    inst.clear();
    by_id.clear();
    smap.clear();
    purged.clear();
    single = std::make_unique<Inst>();
    sel->clear();
  }

  std::vector<Inst*> by_id;   // instances in creation order
  Inst& instance(int64_t e) {
    if (!partitioned) return *single;
    const int64_t now_e = h_now[e];
    if (purge) {   // PartitionRuntimeImpl.initPartition: a purge task since the key's last chunk cleaned it
      auto f = inst.find(h_key[e]);
      if (f != inst.end() && purge->task_in(f->second->seen + purge->idle, now_e)) purge_inst(f->second.get());
    }
    auto& p = inst[h_key[e]];
    if (!p) {
      p = std::make_unique<Inst>();
      p->id = (int)by_id.size();
      p->key = h_key[e];
      if (wkind == GW_TIME) p->khash = java_key_hash(*app, key_ty, h_key[e]);
      by_id.push_back(p.get());
    }
    if (purge) { purge->note(now_e); p->seen = now_e; }
    return *p;
  }

  // QuerySelector on one window output chunk; appends the callback (if any output)
  void select(Inst& I, const std::vector<Item>& chunk, int64_t seq, std::vector<Callback>& out) {
    if (chunk.empty()) return;
    std::vector<SelIn> in(chunk.size());
    for (size_t i = 0; i < chunk.size(); i++)
      in[i] = SelIn{chunk[i].type, chunk[i].ts, chunk[i].val->v.data(), chunk[i].val->nul.data(), (int64_t)I.id};
    std::vector<SelOut> so = sel->process(in);
    if (so.empty()) return;
    Callback cb;
    cb.seq = seq; cb.order = qi; cb.kind = 0; cb.target = qi;
    for (auto& o : so) {
      OutEvent oe;
      oe.ts = o.ts;
      oe.expired = o.expired;
      oe.raw = std::move(o.raw);
      oe.nul = std::move(o.nul);
      cb.ev.push_back(std::move(oe));
    }
    cb.ts = cb.ev.back().ts;
    last_matches += (int64_t)cb.ev.size();
    out.push_back(std::move(cb));
  }

  // the window processor on the filtered events of one chunk (clock `now`), QuerySelector per output chunk
  void window(Inst& I, const std::vector<Item>& evs, int64_t now, int64_t seq, std::vector<Callback>& out) {
    win_process(wspec(), I, evs, now, [&](std::vector<Item>& o) { select(I, o, seq, out); },
                [&]() { if (partitioned) smap.touch(I.khash, I.id); });
  }

  // Scheduler.onTimeChange: each due deadline of a firing state is one TIMER chunk
  void drain(Inst& I, const Tick& t, std::vector<Callback>& out) {
    win_drain(wspec(), I, t.now, [&](std::vector<Item>& o) { select(I, o, t.seq, out); });
  }
  void tick(const Tick& t, std::vector<Callback>& out) {
    if (!partitioned) { drain(*single, t, out); return; }
    if (purge) {   // keys cleaned by a purge task by now have no Scheduler state left
      std::vector<Inst*> gone;
      for (auto& bin : smap.tab)
        for (auto& e : bin) {
          Inst* I = by_id[e.second];
          if (purge->task_in(I->seen + purge->idle, t.now)) gone.push_back(I);
        }
      for (Inst* I : gone) purge_inst(I);
    }
    // the states in map order; ONE per distinct first deadline (the TreeMultimap key), earliest first
    std::vector<std::pair<int64_t, int>> due;
    for (auto& bin : smap.tab)
      for (auto& e : bin) {
        Inst& I = *by_id[e.second];
        if (!I.timers.empty() && I.timers.front() <= t.now) due.push_back({I.timers.front(), e.second});
      }
    std::stable_sort(due.begin(), due.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    for (size_t k = 0; k < due.size(); k++) {
      if (k > 0 && due[k].first == due[k - 1].first) continue;
      drain(*by_id[due[k].second], t, out);
    }
    // returnAllStates: a state whose queue drained is removed (re-inserted at its bin head later)
    std::vector<std::pair<int32_t, int>> gone;
    for (auto& bin : smap.tab)
      for (auto& e : bin) if (by_id[e.second]->timers.empty()) gone.push_back(e);
    for (auto& g : gone) smap.remove(g.first, g.second);
  }

  // ---- device window path (window_dev.hpp) ----
  bool dev = false;               // shape lowered to the device window path (make_window_gen)
  int64_t dev_flushes = 0, host_flushes = 0;
  struct GwdBufs {
    DBuf<int32_t> ev_lid, ev_ord, fidx, f_lid, f_ord, cnt, st, byinst, skey, rank, nit, ioff, iota, nF;
    DBuf<int64_t> ev_ts, ev_now, f_ts, f_now, c_ts, vt, tk_pos, tk_now, cp_now;
    DBuf<int32_t> tk_ord, cp_ev, cp_ord, f_cp, x, cnt_exp, e_off, hflag, hpos, nH, c_lid;
    DBuf<uint8_t> vn, tmp, held;
    DBuf<GwdInst> inst;
    DBuf<uint8_t> it_type;
    DBuf<int64_t> it_ts;
    DBuf<int32_t> it_row, it_lid, it_ord;
    DBuf<int64_t> hrow;
    DBuf<uint8_t> hnul;
    DBuf<int32_t> hlid;
  } gd;
  DevSelector dsel;                 // QuerySelector on the device (selector_dev.hpp)
  template <class T>
  void h2d(DBuf<T>& d, const T* h, size_t n, hipStream_t s) {
    d.reserve(std::max<size_t>(n, 1), false);
    if (n) SG_HIP(hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, s));
  }
  template <class T>
  void d2h(T* h, const T* d, size_t n, hipStream_t s) {
    if (n) SG_HIP(hipMemcpyAsync(h, d, n * sizeof(T), hipMemcpyDeviceToHost, s));
  }
  void cub_tmp(size_t b) { gd.tmp.reserve(std::max<size_t>(b, 1), false); }
  static unsigned gdim(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + GWD_B - 1) / GWD_B); }
  template <class T>
  void excl_sum(const T* in, T* out, int64_t n, hipStream_t s) {
    size_t tb = 0;
    SG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, (int)n, s));
    cub_tmp(tb);
    SG_HIP(hipcub::DeviceScan::ExclusiveSum(gd.tmp.p, tb, in, out, (int)n, s));
  }
  template <class T>
  void incl_sum(const T* in, T* out, int64_t n, hipStream_t s) {
    size_t tb = 0;
    SG_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, in, out, (int)n, s));
    cub_tmp(tb);
    SG_HIP(hipcub::DeviceScan::InclusiveSum(gd.tmp.p, tb, in, out, (int)n, s));
  }
  template <class K, class T>
  void incl_sum_by_key(const K* keys, const T* in, T* out, int64_t n, hipStream_t s) {
    size_t tb = 0;
    SG_HIP(hipcub::DeviceScan::InclusiveSumByKey(nullptr, tb, keys, in, out, (int)n, hipcub::Equality(), s));
    cub_tmp(tb);
    SG_HIP(hipcub::DeviceScan::InclusiveSumByKey(gd.tmp.p, tb, keys, in, out, (int)n, hipcub::Equality(), s));
  }
  // positions in [0, n) whose flag is set, in order -> out; returns the count
  int64_t select_flagged(const uint8_t* flags, int32_t* out, DBuf<int32_t>& cnt, int64_t n, hipStream_t s) {
    if (n <= 0) return 0;
    hipcub::CountingInputIterator<int32_t> idx(0);
    size_t tb = 0;
    cnt.reserve(1, false);
    SG_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb, idx, flags, out, cnt.p, (int)n, s));
    cub_tmp(tb);
    SG_HIP(hipcub::DeviceSelect::Flagged(gd.tmp.p, tb, idx, flags, out, cnt.p, (int)n, s));
    int32_t m = 0;
    d2h(&m, cnt.p, 1, s);
    SG_HIP(hipStreamSynchronize(s));
    return m;
  }

  // One flush on the device (window_dev.hpp).  Returns false -- before any window or aggregator state has
  // changed -- when this flush needs the host path: a time window whose timestamps or clocks go backwards
  // (the queue's FIFO discipline then differs from the closed form), an inexact double sum, a group-key
  // hash collision.
  bool flush_device(std::vector<Callback>& out, hipStream_t s, int64_t nn) {
    if (n >= (int64_t)INT32_MAX / 4) return false;
    const bool time_w = wkind == GW_TIME, batch_w = wkind == GW_BATCH;
    // time windows: timestamps and clocks non-decreasing (events and ticks in arrival order)
    if (time_w) {
      int64_t lt = single->q.empty() ? INT64_MIN : single->q.back().ts, lc = INT64_MIN;
      size_t ti = 0;
      for (int64_t e = 0; e <= n; e++) {
        for (; ti < ticks.size() && ticks[ti].pos <= e; ti++) {
          if (ticks[ti].now < lc) return false;
          lc = ticks[ti].now;
        }
        if (e == n) break;
        if (h_ts[e] < lt || h_now[e] < lc) return false;   // (a chunk's clock is its first event's: also monotone)
        lt = h_ts[e]; lc = h_now[e];
      }
    }
    hipEvent_t d0 = e0;
    SG_HIP(hipEventRecord(d0, s));
    // per event: instance (partition key -> instance, created on first sight), selector chunk ordinal
    std::vector<int32_t> ev_lid((size_t)nn), ev_ord((size_t)nn);
    std::vector<int64_t> ev_now((size_t)nn);      // the clock of each event's chunk (its first event's)
    std::vector<int64_t> ord_seq;
    std::vector<Inst*> touched;
    std::vector<int64_t> tk_pos, tk_now;
    std::vector<int32_t> tk_ord;
    std::unordered_map<int, int32_t> lid_of;
    int32_t o = -1;
    size_t ti = 0;
    auto take_ticks = [&](int64_t pos) {
      for (; ti < ticks.size() && ticks[ti].pos <= pos; ti++) {
        ord_seq.push_back(ticks[ti].seq);
        tk_pos.push_back(pos); tk_now.push_back(ticks[ti].now); tk_ord.push_back(++o);
      }
    };
    if (!partitioned) touched.push_back(single.get());
    int32_t cur_lid = -1;
    int64_t cur_now = 0;
    for (int64_t e = 0; e < nn; e++) {
      const bool new_run = e == 0 || batch_w || h_chunk[e] != h_chunk[e - 1] ||
                           (partitioned && (h_key[e] != h_key[e - 1] || h_knull[e] != h_knull[e - 1]));
      if (new_run) {
        if (time_w) take_ticks(e);                 // due ticks fire before a chunk (never inside one)
        ord_seq.push_back(h_cseq[e]);
        ++o;
        cur_now = h_now[e];
        if (partitioned) {
          if (h_knull[e]) cur_lid = -1;
          else {
            Inst& I = instance(e);
            auto it = lid_of.find(I.id);
            if (it == lid_of.end()) { it = lid_of.emplace(I.id, (int32_t)touched.size()).first; touched.push_back(&I); }
            cur_lid = it->second;
          }
        } else cur_lid = 0;
      }
      ev_lid[(size_t)e] = cur_lid;
      ev_ord[(size_t)e] = o;
      ev_now[(size_t)e] = cur_now;
    }
    if (time_w) take_ticks(nn);
    const int64_t NL = (int64_t)touched.size();
    if (time_w && partitioned) {               // each instance's held rows are older than its new events
      std::vector<int64_t> first_ts((size_t)NL, INT64_MAX);
      for (int64_t e = nn - 1; e >= 0; e--) if (ev_lid[(size_t)e] >= 0) first_ts[(size_t)ev_lid[(size_t)e]] = h_ts[e];
      for (int64_t l = 0; l < NL; l++)
        if (!touched[(size_t)l]->q.empty() && touched[(size_t)l]->q.back().ts > first_ts[(size_t)l]) return false;
    }
    const int nvv = std::max(nv, 1);
    // filtered events in arrival order
    h2d(gd.ev_lid, ev_lid.data(), (size_t)nn, s);
    h2d(gd.ev_ord, ev_ord.data(), (size_t)nn, s);
    h2d(gd.ev_ts, h_ts.data(), (size_t)nn, s);
    h2d(gd.ev_now, ev_now.data(), (size_t)nn, s);
    if (partitioned && nn > 0) hipLaunchKernelGGL(k_gwd_mask, dim3(gdim(nn)), dim3(GWD_B), 0, s, nn, d_flags.p, gd.ev_lid.p);
    gd.fidx.reserve(std::max<int64_t>(nn, 1), false);
    const int64_t F = select_flagged(d_flags.p, gd.fidx.p, gd.nF, nn, s);
    // what the windows carried in: rows [0, C) of the value table
    std::vector<GwdInst> hin((size_t)NL);
    std::vector<std::vector<int64_t>> cv((size_t)nvv);
    std::vector<std::vector<uint8_t>> cn((size_t)nvv);
    std::vector<int64_t> cts;
    std::vector<int32_t> c_lid;                  // instance of each carried row
    int32_t cur_l = 0;
    auto push_row = [&](const Item& x) -> int32_t {
      for (int k = 0; k < nv; k++) { cv[(size_t)k].push_back(x.val->v[(size_t)k]); cn[(size_t)k].push_back(x.val->nul[(size_t)k]); }
      cts.push_back(x.ts);
      c_lid.push_back(cur_l);
      return (int32_t)(cts.size() - 1);
    };
    for (int64_t l = 0; l < NL; l++) {
      cur_l = (int32_t)l;
      Inst& I = *touched[(size_t)l];
      GwdInst& g = hin[(size_t)l];
      g.count = I.count; g.cc = 0; g.co = (int32_t)cts.size(); g.cx = 0; g.cxo = 0; g.h0 = 0; g.r0 = -1;
      if (wkind == GW_LENGTH || time_w) {
        for (auto& x : I.q) push_row(x);
        g.cc = (int32_t)I.q.size();
      } else if (batch_w) {
        if (!stream_current) {
          for (auto& x : I.cur) push_row(x);
          g.cc = (int32_t)I.cur.size();
          g.cxo = (int32_t)cts.size();
          for (auto& x : I.exq) push_row(x);
          g.cx = (int32_t)I.exq.size();
        } else if (sp.expired_on) {
          for (auto& x : I.exq) push_row(x);
          g.cc = (int32_t)I.exq.size();
        }
        g.h0 = I.has_reset;
        if (I.has_reset) g.r0 = push_row(I.reset);
      }
    }
    const int64_t C = (int64_t)cts.size(), R = C + F;
    gd.vt.reserve((size_t)nvv * std::max<int64_t>(R, 1), false);
    gd.vn.reserve((size_t)nvv * std::max<int64_t>(R, 1), false);
    for (int k = 0; k < nv; k++) {
      if (C) SG_HIP(hipMemcpyAsync(gd.vt.p + (size_t)k * R, cv[(size_t)k].data(), (size_t)C * 8, hipMemcpyHostToDevice, s));
      if (C) SG_HIP(hipMemcpyAsync(gd.vn.p + (size_t)k * R, cn[(size_t)k].data(), (size_t)C, hipMemcpyHostToDevice, s));
    }
    h2d(gd.c_ts, cts.data(), (size_t)C, s);
    h2d(gd.inst, hin.data(), (size_t)NL, s);
    gd.f_lid.reserve(std::max<int64_t>(F, 1), false); gd.f_ord.reserve(std::max<int64_t>(F, 1), false);
    gd.f_ts.reserve(std::max<int64_t>(F, 1), false); gd.f_now.reserve(std::max<int64_t>(F, 1), false);
    gd.cnt.reserve(std::max<int64_t>(NL, 1), false);
    if (partitioned) SG_HIP(hipMemsetAsync(gd.cnt.p, 0, (size_t)NL * 4, s));
    if (F > 0) {
      GwdGatherArgs ga;
      ga.F = F; ga.C = C; ga.R = R; ga.fidx = gd.fidx.p; ga.nv = nv; ga.pv = d_pv.p; ga.pn = d_pn.p; ga.pitch = nn;
      ga.vt = gd.vt.p; ga.vn = gd.vn.p; ga.ev_lid = gd.ev_lid.p; ga.ev_ts = gd.ev_ts.p; ga.ev_now = gd.ev_now.p;
      ga.ev_ord = gd.ev_ord.p; ga.f_lid = gd.f_lid.p; ga.f_ts = gd.f_ts.p; ga.f_now = gd.f_now.p; ga.f_ord = gd.f_ord.p;
      ga.cnt = partitioned ? gd.cnt.p : nullptr;
      hipLaunchKernelGGL(k_gwd_gather, dim3(gdim(F)), dim3(GWD_B), 0, s, ga);
      SG_HIP(hipGetLastError());
    }
    // ranks inside the instances
    gd.iota.reserve(std::max<int64_t>(std::max(F, NL), 1), false);
    {
      std::vector<int32_t> io((size_t)std::max(F, NL));
      for (size_t k = 0; k < io.size(); k++) io[k] = (int32_t)k;
      h2d(gd.iota, io.data(), io.size(), s);
    }
    gd.byinst.reserve(std::max<int64_t>(F, 1), false);
    gd.rank.reserve(std::max<int64_t>(F, 1), false);
    gd.st.reserve(std::max<int64_t>(NL, 1), false);
    std::vector<int32_t> hcnt((size_t)NL, 0);
    if (partitioned) {
      if (NL > 0) excl_sum(gd.cnt.p, gd.st.p, NL, s);
      if (F > 0) {
        gd.skey.reserve((size_t)F, false);
        int bits = 1;
        while ((int64_t(1) << bits) < NL) bits++;
        size_t tb = 0;
        SG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, gd.f_lid.p, gd.skey.p, gd.iota.p, gd.byinst.p, (int)F, 0, bits, s));
        cub_tmp(tb);
        SG_HIP(hipcub::DeviceRadixSort::SortPairs(gd.tmp.p, tb, gd.f_lid.p, gd.skey.p, gd.iota.p, gd.byinst.p, (int)F, 0, bits, s));
        hipLaunchKernelGGL(k_gwd_rank, dim3(gdim(F)), dim3(GWD_B), 0, s, F, gd.byinst.p, gd.f_lid.p, gd.st.p, gd.rank.p);
      }
      d2h(hcnt.data(), gd.cnt.p, (size_t)NL, s);
      SG_HIP(hipStreamSynchronize(s));
    } else {
      if (F > 0) {
        SG_HIP(hipMemcpyAsync(gd.byinst.p, gd.iota.p, (size_t)F * 4, hipMemcpyDeviceToDevice, s));
        SG_HIP(hipMemcpyAsync(gd.rank.p, gd.iota.p, (size_t)F * 4, hipMemcpyDeviceToDevice, s));
      }
      SG_HIP(hipMemsetAsync(gd.st.p, 0, 4, s));
      hcnt[0] = (int32_t)F;
      h2d(gd.cnt, hcnt.data(), 1, s);
    }
    // ---- the window processor: items of every output chunk ----
    int64_t M = 0, NT = (int64_t)tk_pos.size(), NC = F + NT;
    GwdItems it;
    auto reserve_items = [&](int64_t m) {
      const size_t c = (size_t)std::max<int64_t>(m, 1);
      gd.it_type.reserve(c, false); gd.it_ts.reserve(c, false); gd.it_row.reserve(c, false);
      gd.it_lid.reserve(c, false); gd.it_ord.reserve(c, false);
      it = GwdItems{gd.it_type.p, gd.it_ts.p, gd.it_row.p, gd.it_lid.p, gd.it_ord.p, m};
    };
    if (!time_w) {
      GwdPlanArgs pa;
      pa.F = F; pa.C = C; pa.L = wkind == GW_NONE ? -1 : L; pa.expired_on = sp.expired_on; pa.stream_current = stream_current;
      pa.byinst = gd.byinst.p; pa.st = gd.st.p; pa.cnt = gd.cnt.p; pa.f_lid = gd.f_lid.p; pa.rank = gd.rank.p;
      pa.f_ts = gd.f_ts.p; pa.f_now = gd.f_now.p; pa.f_ord = gd.f_ord.p; pa.c_ts = gd.c_ts.p; pa.inst = gd.inst.p;
      gd.nit.reserve((size_t)F + 1, false); gd.ioff.reserve((size_t)F + 1, false);
      SG_HIP(hipMemsetAsync(gd.nit.p, 0, ((size_t)F + 1) * 4, s));
      pa.nit = gd.nit.p; pa.ioff = gd.ioff.p;
      if (F > 0) {
        if (batch_w) hipLaunchKernelGGL(k_gwd_batch<false>, dim3(gdim(F)), dim3(GWD_B), 0, s, pa);
        else hipLaunchKernelGGL(k_gwd_len<false>, dim3(gdim(F)), dim3(GWD_B), 0, s, pa);
      }
      excl_sum(gd.nit.p, gd.ioff.p, F + 1, s);
      int32_t m32 = 0;
      d2h(&m32, gd.ioff.p + F, 1, s);
      SG_HIP(hipStreamSynchronize(s));
      M = m32;
      reserve_items(M);
      pa.it = it;
      if (F > 0 && M > 0) {
        if (batch_w) hipLaunchKernelGGL(k_gwd_batch<true>, dim3(gdim(F)), dim3(GWD_B), 0, s, pa);
        else hipLaunchKernelGGL(k_gwd_len<true>, dim3(gdim(F)), dim3(GWD_B), 0, s, pa);
      }
    } else if (partitioned) {                  // time window per instance, current-events output
      gd.x.reserve(std::max<int64_t>(C + F, 1), false);
      gd.cnt_exp.reserve((size_t)F + 1, false); gd.e_off.reserve((size_t)F + 1, false); gd.cp_ev.reserve((size_t)F + 1, false);
      gd.nit.reserve((size_t)F + 1, false); gd.ioff.reserve((size_t)F + 1, false);
      SG_HIP(hipMemsetAsync(gd.cnt_exp.p, 0, ((size_t)F + 1) * 4, s));
      SG_HIP(hipMemsetAsync(gd.nit.p, 0, ((size_t)F + 1) * 4, s));
      SG_HIP(hipMemsetAsync(gd.cp_ev.p, 0, ((size_t)F + 1) * 4, s));
      h2d(gd.c_lid, c_lid.data(), c_lid.size(), s);
      GwdPTimeArgs pt;
      pt.F = F; pt.C = C; pt.T = L; pt.byinst = gd.byinst.p; pt.st = gd.st.p; pt.cnt = gd.cnt.p; pt.f_lid = gd.f_lid.p;
      pt.rank = gd.rank.p; pt.f_ts = gd.f_ts.p; pt.f_now = gd.f_now.p; pt.f_ord = gd.f_ord.p; pt.c_ts = gd.c_ts.p;
      pt.c_lid = gd.c_lid.p; pt.inst = gd.inst.p; pt.x = gd.x.p; pt.cnt_exp = gd.cnt_exp.p; pt.es = gd.e_off.p;
      pt.nit = gd.nit.p; pt.ioff = gd.ioff.p;
      if (C + F > 0) hipLaunchKernelGGL(k_gwd_ptime_exp, dim3(gdim(C + F)), dim3(GWD_B), 0, s, pt);
      if (F > 0) hipLaunchKernelGGL(k_gwd_ptime_nit, dim3(gdim(F)), dim3(GWD_B), 0, s, pt, gd.cp_ev.p);
      excl_sum(gd.cp_ev.p, gd.e_off.p, F + 1, s);
      excl_sum(gd.nit.p, gd.ioff.p, F + 1, s);
      int32_t m32 = 0;
      d2h(&m32, gd.ioff.p + F, 1, s);
      SG_HIP(hipStreamSynchronize(s));
      M = m32;
      reserve_items(M);
      pt.it = it;
      if (M > 0) hipLaunchKernelGGL(k_gwd_ptime_fill, dim3(gdim(C + F)), dim3(GWD_B), 0, s, pt);
    } else {
      h2d(gd.tk_pos, tk_pos.data(), (size_t)NT, s);
      h2d(gd.tk_now, tk_now.data(), (size_t)NT, s);
      h2d(gd.tk_ord, tk_ord.data(), (size_t)NT, s);
      const size_t nc1 = (size_t)NC + 1;
      gd.cp_now.reserve(nc1, false); gd.cp_ev.reserve(nc1, false); gd.cp_ord.reserve(nc1, false);
      gd.f_cp.reserve(std::max<int64_t>(F, 1), false); gd.x.reserve(std::max<int64_t>(C + F, 1), false);
      gd.cnt_exp.reserve(nc1, false); gd.e_off.reserve(nc1, false); gd.nit.reserve(nc1, false); gd.ioff.reserve(nc1, false);
      SG_HIP(hipMemsetAsync(gd.cnt_exp.p, 0, nc1 * 4, s));
      SG_HIP(hipMemsetAsync(gd.nit.p, 0, nc1 * 4, s));
      GwdTimeArgs ta;
      ta.F = F; ta.C = C; ta.NT = NT; ta.NC = NC; ta.T = L; ta.fidx = gd.fidx.p; ta.tk_pos = gd.tk_pos.p;
      ta.tk_now = gd.tk_now.p; ta.tk_ord = gd.tk_ord.p; ta.f_ts = gd.f_ts.p; ta.f_now = gd.f_now.p; ta.f_ord = gd.f_ord.p;
      ta.c_ts = gd.c_ts.p; ta.cp_now = gd.cp_now.p; ta.cp_ev = gd.cp_ev.p; ta.cp_ord = gd.cp_ord.p; ta.f_cp = gd.f_cp.p;
      ta.x = gd.x.p; ta.cnt_exp = gd.cnt_exp.p; ta.e_off = gd.e_off.p; ta.nit = gd.nit.p; ta.ioff = gd.ioff.p;
      if (NC > 0) hipLaunchKernelGGL(k_gwd_time_cp, dim3(gdim(NC)), dim3(GWD_B), 0, s, ta);
      if (C + F > 0) hipLaunchKernelGGL(k_gwd_time_exp, dim3(gdim(C + F)), dim3(GWD_B), 0, s, ta);
      if (NC > 0) hipLaunchKernelGGL(k_gwd_time_nit, dim3(gdim(NC)), dim3(GWD_B), 0, s, ta);
      excl_sum(gd.cnt_exp.p, gd.e_off.p, NC + 1, s);
      excl_sum(gd.nit.p, gd.ioff.p, NC + 1, s);
      int32_t m32 = 0;
      d2h(&m32, gd.ioff.p + NC, 1, s);
      SG_HIP(hipStreamSynchronize(s));
      M = m32;
      reserve_items(M);
      ta.it = it;
      if (M > 0) hipLaunchKernelGGL(k_gwd_time_fill, dim3(gdim(std::max(C + F, NC))), dim3(GWD_B), 0, s, ta);
    }
    SG_HIP(hipGetLastError());
    // ---- QuerySelector (selector_dev.hpp) ----
    DevSelRows rows;
    const GwdVals vals{gd.vt.p, gd.vn.p, R, 1};
    if (!dsel.run(sp, *sel, partitioned, M, it, vals, R,
                  [&](int32_t l) { return (int64_t)touched[(size_t)l]->id; }, s, rows))
      return false;                                          // nothing has changed: the host path runs
    // callbacks: QuerySelector's batching of each output chunk
    std::vector<SelOut> so;
    for (int64_t q = 0; q < rows.P;) {
      const int32_t ord = rows.ord(q);
      int64_t qe = q;
      while (qe < rows.P && rows.ord(qe) == ord) qe++;
      DevSelector::batch(sp, *sel, rows, q, qe, so);
      if (!so.empty()) {
        Callback cb;
        cb.seq = ord_seq[(size_t)ord]; cb.order = qi; cb.kind = 0; cb.target = qi;
        for (auto& x : so) {
          OutEvent oe;
          oe.ts = x.ts; oe.expired = x.expired; oe.raw = std::move(x.raw); oe.nul = std::move(x.nul);
          cb.ev.push_back(std::move(oe));
        }
        cb.ts = cb.ev.back().ts;
        last_matches += (int64_t)cb.ev.size();
        out.push_back(std::move(cb));
      }
      q = qe;
    }
    // ---- the window state the next flush starts from (held rows back to the host structures) ----
    std::vector<int32_t> hold((size_t)NL, 0);
    std::vector<int32_t> xc;   // time: expiry clock points of the carried rows
    for (int64_t l = 0; l < NL; l++) {
      const Inst& I = *touched[(size_t)l];
      const int64_t ni = hcnt[(size_t)l];
      int64_t keep_new = 0;
      if (wkind == GW_LENGTH && L > 0) keep_new = std::min<int64_t>(ni, std::min<int64_t>(I.count + ni, L));
      else if (batch_w && L > 0) {
        if (!stream_current) {
          const int64_t b0 = I.count, tot = b0 + ni, K = tot / L;
          const int64_t idx0 = (sp.expired_on && K >= 1) ? (K - 1) * L : K * L;
          keep_new = ni - std::max<int64_t>(0, std::min(ni, idx0 - b0));
        } else {
          const int64_t cnt2 = ni > 0 ? ((I.count + ni - 1) % L) + 1 : I.count;
          keep_new = std::min(ni, cnt2);
        }
      }
      hold[(size_t)l] = (int32_t)(ni - keep_new);
    }
    int64_t H = 0;
    std::vector<int64_t> hrow;
    std::vector<uint8_t> hnul;
    std::vector<int32_t> hlid;
    if (F > 0 && wkind != GW_NONE) {
      gd.hflag.reserve(NL, false);
      h2d(gd.hflag, hold.data(), (size_t)NL, s);
      gd.held.reserve((size_t)F, false); gd.hpos.reserve((size_t)F, false);
      hipLaunchKernelGGL(k_gwd_held, dim3(gdim(F)), dim3(GWD_B), 0, s, F, gd.byinst.p, gd.f_lid.p, gd.rank.p, gd.hflag.p,
                         time_w ? gd.x.p : nullptr, C, (time_w && partitioned) ? (int64_t)-1 : NC, gd.held.p);
      H = select_flagged(gd.held.p, gd.hpos.p, gd.nH, F, s);
      if (H > 0) {
        gd.hrow.reserve((size_t)H * (nv + 1), false); gd.hnul.reserve((size_t)H * nvv, false); gd.hlid.reserve((size_t)H, false);
        hipLaunchKernelGGL(k_gwd_pack_held, dim3(gdim(H)), dim3(GWD_B), 0, s, H, gd.hpos.p, gd.byinst.p, C, R, nv, gd.vt.p,
                           gd.vn.p, gd.f_ts.p, gd.f_lid.p, gd.hrow.p, gd.hnul.p, gd.hlid.p);
        hrow.resize((size_t)H * (nv + 1)); hnul.resize((size_t)H * nvv); hlid.resize((size_t)H);
        d2h(hrow.data(), gd.hrow.p, hrow.size(), s);
        d2h(hnul.data(), gd.hnul.p, (size_t)H * nv, s);
        d2h(hlid.data(), gd.hlid.p, hlid.size(), s);
      }
    }
    if (time_w && C > 0) {
      xc.resize((size_t)C);
      d2h(xc.data(), gd.x.p, (size_t)C, s);
    }
    SG_HIP(hipStreamSynchronize(s));
    // new held rows per instance, in rank order
    std::vector<std::vector<Item>> nh((size_t)NL);
    for (int64_t h = 0; h < H; h++) {
      auto v = std::make_shared<Val>();
      v->v.assign(hrow.begin() + h * (nv + 1) + 1, hrow.begin() + (h + 1) * (nv + 1));
      v->nul.assign(hnul.begin() + h * nv, hnul.begin() + (h + 1) * nv);
      nh[(size_t)hlid[(size_t)h]].push_back(Item{SE_CURRENT, hrow[(size_t)(h * (nv + 1))], std::move(v)});
    }
    for (int64_t l = 0; l < NL; l++) {
      Inst& I = *touched[(size_t)l];
      const int64_t ni = hcnt[(size_t)l];
      std::vector<Item>& nw = nh[(size_t)l];     // the last nw.size() new events of the instance
      const int64_t first_new = ni - (int64_t)nw.size();   // rank of nw[0]
      auto as_exp = [](Item x) { x.type = SE_EXPIRED; return x; };
      auto as_reset = [](Item x) { x.type = SE_RESET; return x; };
      if (wkind == GW_LENGTH && L > 0) {
        const int64_t keep = std::min<int64_t>(I.count + ni, L);
        while ((int64_t)I.q.size() + (int64_t)nw.size() > keep) I.q.pop_front();
        for (auto& x : nw) I.q.push_back(as_exp(x));
        I.count = keep;
      } else if (time_w) {
        // the carried rows that expired (a prefix of the instance's queue), then the new rows still held
        const GwdInst& gi = hin[(size_t)l];
        const int64_t lim = partitioned ? ni : NC;
        int64_t drop = 0;
        while (drop < gi.cc && xc[(size_t)(gi.co + drop)] < lim) drop++;
        for (int64_t k = 0; k < drop; k++) I.q.pop_front();
        for (auto& x : nw) I.q.push_back(as_exp(x));
        if (partitioned) {
          if (!I.q.empty()) I.last_ts = std::max(I.last_ts, I.q.back().ts);
        } else if (F > 0) {
          int64_t lts = 0;
          d2h(&lts, gd.f_ts.p + F - 1, 1, s);
          SG_HIP(hipStreamSynchronize(s));
          I.last_ts = std::max(I.last_ts, lts);
        }
        I.timers.clear();                             // notifyAt deadlines of the held rows (stale ones fire nothing)
        for (auto& x : I.q) if (I.timers.empty() || I.timers.back() != x.ts + L) I.timers.push_back(x.ts + L);
      } else if (batch_w && L > 0) {
        // FIFO item of index idx (carried head, then the new events; nw covers ranks >= first_new)
        const int64_t b0 = I.count;
        if (!stream_current) {
          std::vector<Item> fifo(I.cur.begin(), I.cur.end());   // FIFO indices [0, b0)
          const int64_t tot = b0 + ni, K = tot / L;
          auto at = [&](int64_t idx) -> Item { return idx < b0 ? fifo[(size_t)idx] : nw[(size_t)(idx - b0 - first_new)]; };
          std::vector<Item> cur2, exq2;
          for (int64_t idx = K * L; idx < tot; idx++) cur2.push_back(at(idx));
          if (sp.expired_on) {
            if (K >= 1) for (int64_t idx = (K - 1) * L; idx < K * L; idx++) exq2.push_back(as_exp(at(idx)));
            else exq2 = I.exq;
          }
          if (K == 0) {
            if (!I.has_reset && ni > 0) { I.reset = as_reset(at(0)); I.has_reset = true; }
          } else {
            I.has_reset = tot % L > 0;
            if (I.has_reset) I.reset = as_reset(at(K * L));
          }
          I.cur = std::move(cur2);
          I.exq = std::move(exq2);
          I.count = tot % L;
        } else {
          std::vector<Item> fifo(I.exq.begin(), I.exq.end());   // carried current batch (expired output)
          const int64_t cc = (int64_t)fifo.size();
          auto at_new = [&](int64_t r) -> Item { return nw[(size_t)(r - first_new)]; };
          int64_t rf = -1;                                       // the last flush among the new events
          for (int64_t r = ni - 1; r >= 0 && rf < 0; r--) {
            const int64_t t = b0 + r;
            if (t >= L && t % L == 0) rf = r;
            if (ni - 1 - r > L) break;
          }
          const int64_t cnt2 = ni > 0 ? ((b0 + ni - 1) % L) + 1 : b0;
          if (sp.expired_on) {
            std::vector<Item> exq2;
            const int64_t tot = cc + ni;
            for (int64_t idx = tot - cnt2; idx < tot; idx++)
              exq2.push_back(as_exp(idx < cc ? fifo[(size_t)idx] : at_new(idx - cc)));
            I.exq = std::move(exq2);
          }
          if (rf >= 0) {
            I.has_reset = ni - 1 > rf;
            if (I.has_reset) I.reset = as_reset(at_new(rf + 1));
          } else if (!I.has_reset && ni > 0) {
            I.reset = as_reset(at_new(0));
            I.has_reset = true;
          }
          I.count = cnt2;
        }
      }
    }
    // the planned events leave the host staging, as on the host path
    ticks.erase(ticks.begin(), ticks.begin() + (ptrdiff_t)ti);
    for (auto& t : ticks) t.pos -= n;
    h_ts.clear(); h_now.clear(); h_seq.clear(); h_cseq.clear(); h_chunk.clear(); h_key.clear(); h_knull.clear();
    n = done = 0;
    has_nul = false;
    SG_HIP(hipEventRecord(e1, s));
    SG_HIP(hipEventSynchronize(e1));
    float ms = 0;
    SG_HIP(hipEventElapsedTime(&ms, d0, e1));
    kernel_ms["k_gwd_flush"] = ms;
    kernel_ms["gwd_items"] = (double)M;
    kernel_ms["gw_device"] = 1;
    return true;
  }

  void flush(std::vector<Callback>& out, bool materialise, hipStream_t s) override {
    (void)materialise;
    last_matches = 0;
    kernel_ms.clear();
    const int64_t nn = n - done;
    std::vector<uint8_t> flags;
    std::vector<int64_t> pv;
    std::vector<uint8_t> pn;
    if (nn > 0) {
      if (!e0) { SG_HIP(hipEventCreate(&e0)); SG_HIP(hipEventCreate(&e1)); }
      GwCols gc;
      std::memset(&gc, 0, sizeof(gc));
      for (size_t k = 0; k < cols.size(); k++) { gc.c[k] = cols[k].b.p; gc.w[k] = cols[k].w; }
      gc.nul = has_nul ? nulcol.p : nullptr;
      gc.na = (int32_t)cols.size();
      d_progs.reserve(progs.size());
      SG_HIP(hipMemcpyAsync(d_progs.p, progs.data(), progs.size() * sizeof(Prog), hipMemcpyHostToDevice, s));
      d_flags.reserve(nn);
      d_pv.reserve((size_t)std::max(nv, 1) * nn);
      d_pn.reserve((size_t)std::max(nv, 1) * nn);
      SG_HIP(hipEventRecord(e0, s));
      hipLaunchKernelGGL(k_gw_eval, dim3((unsigned)((nn + GW_B - 1) / GW_B)), dim3(GW_B), 0, s, done, n, gc, d_progs.p,
                         has_filter ? 1 : 0, nv, d_flags.p, d_pv.p, d_pn.p, nn);
      SG_HIP(hipGetLastError());
      SG_HIP(hipEventRecord(e1, s));
      SG_HIP(hipEventSynchronize(e1));
      float ms0 = 0;
      SG_HIP(hipEventElapsedTime(&ms0, e0, e1));
      kernel_ms["k_gw_eval"] = ms0;
    }
    if (dev && (nn > 0 || !ticks.empty()) && flush_device(out, s, nn)) { dev_flushes++; return; }
    if (nn > 0) {
      flags.resize(nn);
      pv.resize((size_t)nv * nn);
      pn.resize((size_t)nv * nn);
      SG_HIP(hipMemcpyAsync(flags.data(), d_flags.p, nn, hipMemcpyDeviceToHost, s));
      if (nv) {
        SG_HIP(hipMemcpyAsync(pv.data(), d_pv.p, pv.size() * 8, hipMemcpyDeviceToHost, s));
        SG_HIP(hipMemcpyAsync(pn.data(), d_pn.p, pn.size(), hipMemcpyDeviceToHost, s));
      }
      SG_HIP(hipStreamSynchronize(s));
    }
    host_flushes++;
    kernel_ms["gw_device"] = 0;
    // plan: ticks and chunks in arrival order
    size_t ti = 0;
    auto ticks_before = [&](int64_t pos) {
      while (ti < ticks.size() && ticks[ti].pos <= pos) tick(ticks[ti++], out);
    };
    int64_t e = done;
    std::vector<Item> evs;
    while (e < n) {
      ticks_before(e);
      // one chunk: the events of one send call (batch) and, partitioned, one run of a single key
      int64_t f = e + 1;
      while (f < n && h_chunk[f] == h_chunk[e] &&
             (!partitioned || (h_key[f] == h_key[e] && h_knull[f] == h_knull[e]))) f++;
      if (partitioned && h_knull[e]) { e = f; continue; }   // null partition key: no instance
      Inst& I = instance(e);
      evs.clear();
      for (int64_t k = e; k < f; k++) {
        const int64_t r = k - done;
        if (!flags[r]) continue;
        auto v = std::make_shared<Val>();
        v->v.resize(nv);
        v->nul.resize(nv);
        for (int a = 0; a < nv; a++) { v->v[a] = pv[(size_t)a * nn + r]; v->nul[a] = pn[(size_t)a * nn + r]; }
        evs.push_back(Item{SE_CURRENT, h_ts[k], std::move(v)});
      }
      if (!evs.empty()) window(I, evs, h_now[e], h_cseq[e], out);
      e = f;
    }
    ticks_before(n);
    ticks.erase(ticks.begin(), ticks.begin() + ti);
    // the planned events leave the host staging (device columns are rebuilt from the next push)
    for (auto& t : ticks) t.pos -= n;
    h_ts.clear(); h_now.clear(); h_seq.clear(); h_cseq.clear(); h_chunk.clear(); h_key.clear(); h_knull.clear();
    n = done = 0;
    has_nul = false;
  }

  // Snapshot (after a flush): per instance the window's queues (LengthWindowProcessor / TimeWindowProcessor
  // expiredEventQueue, LengthBatchWindowProcessor currentEventQueue / expiredEventQueue / resetEvent,
  // count, lastTimestamp, the Scheduler deadlines) and the selector's aggregator states.
  bool can_snapshot() const override { return true; }
  static void put_item(SnapWriter& w, const Item& x) {
    w.pod(x.type); w.pod(x.ts); w.vec(x.val->v); w.vec(x.val->nul);
  }
  static Item get_item(SnapReader& r) {
    Item x;
    x.type = r.pod<int>(); x.ts = r.pod<int64_t>();
    auto v = std::make_shared<Val>();
    r.vec(v->v); r.vec(v->nul);
    x.val = std::move(v);
    return x;
  }
  static void put_inst(SnapWriter& w, const Inst& I) {
    w.pod(I.id); w.pod(I.count); w.pod(I.last_ts); w.pod(I.khash); w.pod(I.seen); w.deq(I.timers);
    w.pod<uint64_t>(I.q.size()); for (auto& x : I.q) put_item(w, x);
    w.pod<uint64_t>(I.cur.size()); for (auto& x : I.cur) put_item(w, x);
    w.pod<uint64_t>(I.exq.size()); for (auto& x : I.exq) put_item(w, x);
    w.pod(I.has_reset);
    if (I.has_reset) put_item(w, I.reset);
  }
  static void get_inst(SnapReader& r, Inst& I) {
    I.id = r.pod<int>(); I.count = r.pod<int64_t>(); I.last_ts = r.pod<int64_t>(); I.khash = r.pod<int32_t>();
    I.seen = r.pod<int64_t>();
    r.deq(I.timers);
    I.q.clear(); for (uint64_t k = r.pod<uint64_t>(); k > 0; k--) I.q.push_back(get_item(r));
    I.cur.clear(); for (uint64_t k = r.pod<uint64_t>(); k > 0; k--) I.cur.push_back(get_item(r));
    I.exq.clear(); for (uint64_t k = r.pod<uint64_t>(); k > 0; k--) I.exq.push_back(get_item(r));
    I.has_reset = r.pod<bool>();
    if (I.has_reset) I.reset = get_item(r);
  }
  void snapshot(SnapWriter& w, hipStream_t s) override {
    (void)s;
    w.pod(chunk_ctr);
    put_inst(w, *single);
    w.pod<uint64_t>(inst.size());
    for (auto& kv : inst) { w.pod(kv.first); put_inst(w, *kv.second); }
    w.pod<uint64_t>(smap.tab.size()); w.pod<uint64_t>(smap.size); w.pod<uint64_t>(smap.thr);
    for (auto& bin : smap.tab) w.vec(bin);
    sel->snapshot(w);
  }
  void restore(SnapReader& r, hipStream_t s) override {
    (void)s;
    reset();
    chunk_ctr = r.pod<int64_t>();
    get_inst(r, *single);
    for (uint64_t k = r.pod<uint64_t>(); k > 0; k--) {
      const int64_t key = r.pod<int64_t>();
      auto& p = inst[key];
      p = std::make_unique<Inst>();
      get_inst(r, *p);
    }
    int maxid = -1;
    for (auto& kv : inst) maxid = std::max(maxid, kv.second->id);
    by_id.assign((size_t)(maxid + 1), nullptr);
    for (auto& kv : inst) {
      if (kv.second->id < 0) throw Error(-1, "snapshot instance ids");
      kv.second->key = kv.first;
      by_id[kv.second->id] = kv.second.get();
    }
    for (auto& bin : smap.tab)
      for (auto& e : bin)
        if (e.second < 0 || e.second >= (int)by_id.size() || !by_id[e.second]) throw Error(-1, "snapshot instance ids");
    smap.tab.resize(r.pod<uint64_t>()); smap.size = r.pod<uint64_t>(); smap.thr = r.pod<uint64_t>();
    for (auto& bin : smap.tab) r.vec(bin);
    sel->restore(r);
  }

  bool flush_export(ChainOut& co, hipStream_t s) override {
    std::vector<Callback> cbs;
    flush(cbs, true, s);
    co.raw.assign(sp.akind.size(), {});
    for (auto& cb : cbs) {
      for (auto& ev : cb.ev) {
        co.ts.push_back(ev.ts);
        co.seq.push_back(cb.seq);
        for (size_t a = 0; a < ev.raw.size(); a++) {
          co.raw[a].push_back(ev.raw[a]);
          co.nulls = co.nulls || ev.nul[a];
        }
      }
      co.chunk_end.push_back((int64_t)co.ts.size());
    }
    return true;
  }
};

std::unique_ptr<Exec> make_window_gen(App& app, int qi, const J& q, std::string& why) {
  const J& in = q["input"];
  if (in["kind"].s != "single") { why = "not a single-stream query"; return nullptr; }
  auto ex = std::make_unique<GenWindowExec>();
  ex->app = &app; ex->qi = qi; ex->path = SG_PATH_WINDOW;
  ex->st = app.stream_idx.at(in["stream"].s);
  const auto& types = app.streams[ex->st].types;
  if (types.size() > (size_t)GW_MAXA) { why = "too many attributes"; return nullptr; }
  const J& hs = in["handlers"];
  std::vector<const J*> filt;
  int win = -1;
  for (size_t k = 0; k < hs.size(); k++) {
    if (hs[k]["k"].s == "filter") {
      if (win >= 0) { why = "filter after the window"; return nullptr; }
      filt.push_back(&hs[k]["e"]);
    } else {
      if (win >= 0) { why = "two windows"; return nullptr; }
      win = (int)k;
    }
  }
  if (win >= 0) {
    const J& w = hs[win];
    const std::string& wn = w["name"].s;
    if (wn == "length") ex->wkind = GW_LENGTH;
    else if (wn == "time") ex->wkind = GW_TIME;
    else if (wn == "lengthBatch") ex->wkind = GW_BATCH;
    else { why = "window." + wn + " is not lowered yet"; return nullptr; }
    if (w["params"].size() < 1 || w["params"][0]["op"].s != "const") { why = "window parameter"; return nullptr; }
    ex->L = w["params"][0]["v"].as_int();
    if (ex->L < 0) { why = "negative window parameter"; return nullptr; }
    if (w["params"].size() > 1) {
      if (ex->wkind != GW_BATCH || w["params"][1]["op"].s != "const") { why = "window parameter"; return nullptr; }
      ex->stream_current = w["params"][1]["v"].b;
    }
  }
  if (q.has("partition")) {
    ex->partitioned = true;
    const J& pm = q["partition"];
    if (!pm.has(in["stream"].s)) { why = "stream not named in `partition with` (broadcast)"; return nullptr; }
    ex->pattr = (int)pm[in["stream"].s].as_int();
    ex->key_ty = types.at(ex->pattr);
    if (ex->wkind == GW_TIME && (ex->key_ty == T_FLOAT || ex->key_ty == T_DOUBLE)) {
      why = "float partition key of a time window (Scheduler map order of Float.toString)";
      return nullptr;
    }
    std::string pw;
    ex->purge = purge_of(app, q, pw);
    if (!pw.empty()) { why = pw; return nullptr; }
    if (ex->purge && pm.o.size() != 1) { why = "@purge with a partition stream the query does not read"; return nullptr; }
  }
  auto intern = [&](const std::string& str) { return app.intern(str); };
  auto sm = [](int slot, int chain) -> int { (void)slot; (void)chain; return 0; };
  try {
    ex->progs.emplace_back();
    if (!filt.empty()) {
      J arr;
      arr.k = J::ARR;
      for (auto* f : filt) arr.a.push_back(*f);
      compile_filters(ex->progs[0], arr, sm, intern);
      ex->has_filter = true;
    }
    std::vector<const J*> dev;
    const bool slide = ex->wkind == GW_LENGTH || ex->wkind == GW_TIME;
    if (!build_selector(q["select"], q, slide, ex->sp, dev, intern, why)) return nullptr;
    for (const J* e : dev) {
      ex->progs.emplace_back();
      compile_expr(ex->progs.back(), *e, sm, intern);
    }
    ex->nv = (int)dev.size();
  } catch (CompileError& e) {
    why = e.what();
    return nullptr;
  }
  ex->sp.partitioned = ex->partitioned;
  ex->sp.active = true;
  // the device window path (window_dev.hpp): sum / count / avg / min / max selectors, every window but a partitioned
  // time window with expired output (the Scheduler map order of its TIMER chunks stays with the host path), no @purge
  {
    bool ok = !getenv("SG_GW_HOST") && !ex->purge && !(ex->wkind == GW_TIME && ex->partitioned && ex->sp.expired_on) &&
              ex->sp.aggs.size() <= (size_t)GWD_MAXAGG && ex->sp.group.size() <= (size_t)GWD_MAXG &&
              ex->sp.akind.size() <= (size_t)GWD_MAXOUT;
    for (auto& A : ex->sp.aggs) ok = ok && A.k >= SA_SUM && A.k <= SA_MAX;
    ex->dev = ok;
  }
  ex->sel = std::make_unique<SelectorStage>(ex->sp, &app.strings);
  ex->single = std::make_unique<GenWindowExec::Inst>();
  for (Ty t : types) { ex->cols.emplace_back(); ex->cols.back().w = tsize(t); }
  ex->in_streams = {ex->st};
  return ex;
}

}  // namespace sg
