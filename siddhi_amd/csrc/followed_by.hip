// followed_by.hip — execution path SG_PATH_FOLLOWED_BY.
//
// Query shape:  from every e1=A[f1] -> e2=B[f2(e1,e2)] (within W)?  select <projection of e1/e2>
//
// Reference semantics (restated, see oracle/siddhi_oracle.cpp for the object-level version):
//   * e1's pre-processor always holds one empty partial (every re-seeds it through
//     StreamPostStateProcessor.process -> addEveryState, StreamPreStateProcessor.java:229-247),
//     so a partial is created for event i iff i is an A event and f1(i) holds.
//   * the partial becomes visible to e2 at the next arrival (newAndEvery -> pending in
//     updateState, :307-323); e2 is processed before e1 for the same event (reverse order,
//     PatternMultiProcessStreamReceiver.java:29-39), so candidates are j > i.
//   * before each arrival j the partial expires iff |ts_i - ts_j| > W (isExpired :118-129, strict);
//     with non-decreasing timestamps the head-`break` in expireEvents (:340-341) removes exactly
//     the expired prefix, so expiry is the closed form  ts_j - ts_i > W.
//   * the first B event j with f2(i, j) completes the match and removes the partial (stateChanged).
//   => m(i) = min{ j > i : j in B, ts_j - ts_i <= W, f2(i,j) }, emitted at j, and all matches
//      completing at the same j are emitted in pending-list order = ascending i.
//   * callback grouping: when A == B the stream has a PatternMultiProcessStreamReceiver and every
//     (event, processor) pair gets one ReturnEventHolder -> one QueryCallback per distinct j
//     (MultiProcessStreamReceiver.java:216-241); when A != B, B's receiver is a
//     PatternSingleProcessStreamReceiver and every match is its own callback (:48-73).
//
// Kernels (gfx950):
//   k_fb_scan     one lane per start; bounded forward scan over the event columns, predicates by the
//                 wave-uniform bytecode interpreter; match records (j<<32|i) appended.
//   radix sort    match records sorted by (j, i) -> reference emission order.
//   k_fb_project  select-list evaluation per record straight into output columns in HBM.
// Non-decreasing timestamps are required (checked at push); otherwise SG_E_UNSUPPORTED.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>

#include "runtime.hpp"

namespace sg {

constexpr int FB_MAXC = 12;

struct FBCols {
  const uint8_t* a[FB_MAXC];
  const uint8_t* b[FB_MAXC];
  int32_t aw[FB_MAXC];
  int32_t bw[FB_MAXC];
};

struct FBLoader {
  const FBCols* c;
  int64_t i, j;
  __device__ __forceinline__ bool load(int slot, int attr, int64_t& v) const {
    const uint8_t* col = slot == 0 ? c->a[attr] : c->b[attr];
    int w = slot == 0 ? c->aw[attr] : c->bw[attr];
    int64_t idx = slot == 0 ? i : j;
    if (w == 8) v = ((const int64_t*)col)[idx];
    else v = (int64_t)((const int32_t*)col)[idx];
    return true;
  }
};

struct FBScanArgs {
  const int64_t* ts;
  const uint8_t* tag;     // bit0 = A event, bit1 = B event (nullptr: every event is both)
  int64_t n;
  int64_t within;         // -1: no within
  int64_t new_lo;         // first start index not yet examined
  int32_t n_pend;
  const int32_t* pend_i;
  const int32_t* pend_j;
  uint64_t* keys;
  uint32_t* nkeys;
  int32_t* npend_i;
  int32_t* npend_j;
  uint32_t* nnpend;
};

__global__ void __launch_bounds__(256) k_fb_scan(FBScanArgs a, const FBCols* __restrict__ cols,
                                                  const Prog* __restrict__ progs) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t i, j0;
  FBLoader ld{cols, 0, 0};
  if (t < a.n_pend) {
    i = a.pend_i[t];
    j0 = a.pend_j[t];
  } else {
    i = a.new_lo + (t - a.n_pend);
    if (i >= a.n) return;
    if (a.tag && !(a.tag[i] & 1)) return;
    ld.i = i;
    if (!run_pred(progs[0], ld)) return;
    j0 = i + 1;
  }
  ld.i = i;
  const int64_t tsi = a.ts[i];
  for (int64_t j = j0; j < a.n; j++) {
    if (a.within >= 0 && a.ts[j] - tsi > a.within) return;   // expired before j
    if (a.tag && !(a.tag[j] & 2)) continue;
    ld.j = j;
    if (run_pred(progs[1], ld)) {
      uint32_t k = atomicAdd(a.nkeys, 1u);
      a.keys[k] = ((uint64_t)j << 32) | (uint64_t)i;
      return;
    }
  }
  uint32_t k = atomicAdd(a.nnpend, 1u);
  a.npend_i[k] = (int32_t)i;
  a.npend_j[k] = (int32_t)a.n;
}

struct FBProjArgs {
  const uint64_t* keys;
  int64_t m;
  const int64_t* ts;
  int32_t nout;
  int64_t* out_raw;     // m * nout
  uint8_t* out_null;    // m * nout
  int64_t* out_ts;
  int32_t* out_j;
};

__global__ void __launch_bounds__(256) k_fb_project(FBProjArgs a, const FBCols* __restrict__ cols,
                                                     const Prog* __restrict__ sel) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.m) return;
  uint64_t key = a.keys[k];
  int64_t j = (int64_t)(key >> 32), i = (int64_t)(key & 0xffffffffu);
  FBLoader ld{cols, i, j};
  for (int c = 0; c < a.nout; c++) {
    int64_t v = 0;
    bool isnull = false;
    run(sel[c], ld, v, isnull);
    a.out_raw[k * a.nout + c] = v;
    a.out_null[k * a.nout + c] = isnull;
  }
  a.out_ts[k] = a.ts[j];
  a.out_j[k] = (int32_t)j;
}

// ------------------------------------------------------------------------------------------------
struct FollowedByExec : Exec {
  int sA = -1, sB = -1;
  bool same = false;
  int64_t within = -1;
  Prog progs[2];
  std::vector<Prog> sel;
  std::vector<Ty> out_types;
  // event buffer (device)
  int64_t n = 0;
  DBuf<int64_t> ts;
  DBuf<uint8_t> tag;
  std::vector<DCol> colA, colB;
  const int64_t* ext_ts = nullptr;               // adopted device input (push_device)
  std::vector<const void*> ext_cols;
  std::vector<int64_t> h_seq, h_ts;              // host mirror: arrival seq + ts per buffered event
  int64_t last_ts = INT64_MIN;
  int64_t examined = 0;                          // starts [0, examined) already scanned
  DBuf<int32_t> pend_i, pend_j, npend_i, npend_j;
  int32_t n_pend = 0;
  DBuf<uint64_t> keys, keys_sorted;
  DBuf<uint32_t> counters;
  DBuf<uint8_t> sort_tmp;
  DBuf<FBCols> d_cols;
  DBuf<Prog> d_progs, d_sel;
  DBuf<int64_t> out_raw, out_ts;
  DBuf<uint8_t> out_null;
  DBuf<int32_t> out_j;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;

  ~FollowedByExec() override {
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
  }

  int arity(int s) const;
  void ensure_cap(int64_t need, hipStream_t s);
  void append_host(const HostBatch& b, uint8_t tagv, hipStream_t s);

  void push(const HostBatch& b) override {
    if (b.stream != sA && b.stream != sB) return;
    for (int64_t k = 0; k < b.n; k++) {
      if (b.ts[k] < last_ts)
        throw Error(-2, "followed-by path needs non-decreasing event timestamps (got " + std::to_string(b.ts[k]) +
                            " after " + std::to_string(last_ts) + ")");
      last_ts = b.ts[k];
    }
    uint8_t tv = (b.stream == sA ? 1 : 0) | (b.stream == sB ? 2 : 0);
    append_host(b, tv, app->stream);
  }

  void push_device(int stream, int64_t cnt, const int64_t* d_ts, const void* const* d_cols, int batch,
                   hipStream_t s) override {
    (void)batch; (void)s;
    if (!same || stream != sA) throw Error(-2, "device ingest supports single-stream followed-by queries");
    if (n != 0 || ext_ts) throw Error(-2, "device ingest adopts one resident batch per runtime");
    ext_ts = d_ts;
    ext_cols.assign(d_cols, d_cols + arity(sA));
    n = cnt;
    h_seq.clear();
    last_ts = INT64_MIN;   // caller guarantees monotone ts for device-resident input
  }

  void flush(std::vector<Callback>& out, bool materialise, hipStream_t s) override;
  void reset() override {
    n = 0; examined = 0; n_pend = 0; ext_ts = nullptr; ext_cols.clear();
    h_seq.clear(); h_ts.clear(); last_ts = INT64_MIN; last_matches = 0;
  }
};

int FollowedByExec::arity(int s) const { return (int)app->streams[s].types.size(); }

void FollowedByExec::ensure_cap(int64_t need, hipStream_t s) {
  if (ext_ts) throw Error(-2, "cannot append host events after device-resident ingest");
  ts.reserve(need, true, s, n);
  if (!same) tag.reserve(need, true, s, n);
  for (auto& c : colA) { size_t used = n * c.w; c.b.reserve(need * c.w, true, s, used); }
  for (auto& c : colB) { size_t used = n * c.w; c.b.reserve(need * c.w, true, s, used); }
}

void FollowedByExec::append_host(const HostBatch& b, uint8_t tagv, hipStream_t s) {
  ensure_cap(n + b.n, s);
  SG_HIP(hipMemcpyAsync(ts.p + n, b.ts.data(), b.n * 8, hipMemcpyHostToDevice, s));
  if (!same) {
    std::vector<uint8_t> tv(b.n, tagv);
    SG_HIP(hipMemcpyAsync(tag.p + n, tv.data(), b.n, hipMemcpyHostToDevice, s));
    SG_HIP(hipStreamSynchronize(s));
  }
  std::vector<DCol>& cols = (b.stream == sA) ? colA : colB;
  for (size_t k = 0; k < cols.size(); k++) {
    SG_HIP(hipMemcpyAsync(cols[k].b.p + n * cols[k].w, b.cols[k].data(), b.n * cols[k].w,
                          hipMemcpyHostToDevice, s));
  }
  SG_HIP(hipStreamSynchronize(s));
  for (int64_t k = 0; k < b.n; k++) { h_seq.push_back(b.seq0 + k); h_ts.push_back(b.ts[k]); }
  n += b.n;
}

void FollowedByExec::flush(std::vector<Callback>& out, bool materialise, hipStream_t s) {
  int64_t new_starts = n - examined;
  int64_t work = new_starts + n_pend;
  last_matches = 0;
  if (work <= 0) return;
  if (n >= (int64_t)INT32_MAX) throw Error(-2, "followed-by buffer exceeds 2^31 events");
  // column table
  FBCols hc;
  std::memset(&hc, 0, sizeof(hc));
  int na = arity(sA), nb = arity(sB);
  for (int k = 0; k < na; k++) {
    hc.a[k] = ext_ts ? (const uint8_t*)ext_cols[k] : colA[k].b.p;
    hc.aw[k] = tsize(app->streams[sA].types[k]);
  }
  for (int k = 0; k < nb; k++) {
    const std::vector<DCol>& cb = same ? colA : colB;
    hc.b[k] = ext_ts ? (const uint8_t*)ext_cols[k] : cb[k].b.p;
    hc.bw[k] = tsize(app->streams[sB].types[k]);
  }
  d_cols.reserve(1);
  SG_HIP(hipMemcpyAsync(d_cols.p, &hc, sizeof(hc), hipMemcpyHostToDevice, s));
  d_progs.reserve(2);
  SG_HIP(hipMemcpyAsync(d_progs.p, progs, sizeof(progs), hipMemcpyHostToDevice, s));
  if (!sel.empty()) {
    d_sel.reserve(sel.size());
    SG_HIP(hipMemcpyAsync(d_sel.p, sel.data(), sel.size() * sizeof(Prog), hipMemcpyHostToDevice, s));
  }
  keys.reserve(work);
  npend_i.reserve(work);
  npend_j.reserve(work);
  counters.reserve(2);
  SG_HIP(hipMemsetAsync(counters.p, 0, 2 * sizeof(uint32_t), s));
  FBScanArgs a;
  a.ts = ext_ts ? ext_ts : ts.p;
  a.tag = same ? nullptr : tag.p;
  a.n = n;
  a.within = within;
  a.new_lo = examined;
  a.n_pend = n_pend;
  a.pend_i = pend_i.p;
  a.pend_j = pend_j.p;
  a.keys = keys.p;
  a.nkeys = counters.p;
  a.npend_i = npend_i.p;
  a.npend_j = npend_j.p;
  a.nnpend = counters.p + 1;
  if (!ev0) { SG_HIP(hipEventCreate(&ev0)); SG_HIP(hipEventCreate(&ev1)); }
  SG_HIP(hipEventRecord(ev0, s));
  int64_t blocks = (work + 255) / 256;
  hipLaunchKernelGGL(k_fb_scan, dim3((unsigned)blocks), dim3(256), 0, s, a, d_cols.p, d_progs.p);
  SG_HIP(hipGetLastError());
  SG_HIP(hipEventRecord(ev1, s));
  uint32_t hcnt[2];
  SG_HIP(hipMemcpyAsync(hcnt, counters.p, sizeof(hcnt), hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  float ms = 0;
  SG_HIP(hipEventElapsedTime(&ms, ev0, ev1));
  kernel_ms["k_fb_scan"] = ms;
  int64_t m = hcnt[0];
  last_matches = m;
  // pending for next flush
  std::swap(pend_i.p, npend_i.p); std::swap(pend_i.cap, npend_i.cap);
  std::swap(pend_j.p, npend_j.p); std::swap(pend_j.cap, npend_j.cap);
  n_pend = (int32_t)hcnt[1];
  examined = n;
  if (m == 0) return;
  // sort match records by (j, i)
  keys_sorted.reserve(m);
  int end_bit = 32;
  while (end_bit < 64 && (1ull << (end_bit - 32)) <= (uint64_t)n) end_bit++;
  size_t tmp = 0;
  SG_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, keys.p, keys_sorted.p, (int)m, 0, end_bit, s));
  sort_tmp.reserve(tmp);
  SG_HIP(hipEventRecord(ev0, s));
  SG_HIP(hipcub::DeviceRadixSort::SortKeys(sort_tmp.p, tmp, keys.p, keys_sorted.p, (int)m, 0, end_bit, s));
  SG_HIP(hipEventRecord(ev1, s));
  int nout = (int)sel.size();
  out_raw.reserve((size_t)m * std::max(nout, 1));
  out_null.reserve((size_t)m * std::max(nout, 1));
  out_ts.reserve(m);
  out_j.reserve(m);
  FBProjArgs pa{keys_sorted.p, m, ext_ts ? ext_ts : ts.p, nout, out_raw.p, out_null.p, out_ts.p, out_j.p};
  hipLaunchKernelGGL(k_fb_project, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, pa, d_cols.p, d_sel.p);
  SG_HIP(hipGetLastError());
  SG_HIP(hipStreamSynchronize(s));
  SG_HIP(hipEventElapsedTime(&ms, ev0, ev1));
  kernel_ms["sort"] = ms;
  if (!materialise) return;
  std::vector<int64_t> hraw((size_t)m * nout), hts(m);
  std::vector<uint8_t> hnul((size_t)m * nout);
  std::vector<int32_t> hj(m);
  if (nout) {
    SG_HIP(hipMemcpyAsync(hraw.data(), out_raw.p, (size_t)m * nout * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(hnul.data(), out_null.p, (size_t)m * nout, hipMemcpyDeviceToHost, s));
  }
  SG_HIP(hipMemcpyAsync(hts.data(), out_ts.p, m * 8, hipMemcpyDeviceToHost, s));
  SG_HIP(hipMemcpyAsync(hj.data(), out_j.p, m * 4, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  Callback* cur = nullptr;
  int32_t curj = -1;
  for (int64_t k = 0; k < m; k++) {
    if (!same || cur == nullptr || hj[k] != curj) {
      out.emplace_back();
      cur = &out.back();
      cur->seq = h_seq.empty() ? hj[k] : h_seq[hj[k]];
      cur->order = qi;
      cur->kind = 0;
      cur->target = qi;
      curj = hj[k];
    }
    OutEvent e;
    e.ts = hts[k];
    e.raw.assign(hraw.begin() + k * nout, hraw.begin() + (k + 1) * nout);
    e.nul.assign(hnul.begin() + k * nout, hnul.begin() + (k + 1) * nout);
    cur->ts = e.ts;
    cur->ev.push_back(std::move(e));
  }
}

// ------------------------------------------------------------------------------------------------
// Shape recognition: next(every(stream A [f1]), stream B [f2]), PATTERN, projection-only selector.
std::unique_ptr<Exec> make_followed_by(App& app, int qi, const J& q, std::string& why) {
  const J& in = q["input"];
  if (in["kind"].s != "state") { why = "not a state query"; return nullptr; }
  if (in["type"].s != "PATTERN") { why = "sequence"; return nullptr; }
  if (q.has("partition")) { why = "partitioned"; return nullptr; }
  const J& el = in["element"];
  if (el["k"].s != "next" || el["a"]["k"].s != "every" || el["a"]["e"]["k"].s != "stream" || el["b"]["k"].s != "stream") {
    why = "not `every e1 -> e2`";
    return nullptr;
  }
  const J& e1 = el["a"]["e"];
  const J& e2 = el["b"];
  if (e1["slot"].as_int() != 0 || e2["slot"].as_int() != 1) { why = "slot layout"; return nullptr; }
  const J& s = q["select"];
  if (s["group_by"].size() || !s["having"].null() || s["order_by"].size() || !s["limit"].null() || !s["offset"].null()) {
    why = "selector features";
    return nullptr;
  }
  const J& out = q["output"];
  if (out["events"].s != "current" && !out["events"].s.empty()) { why = "expired events output"; return nullptr; }
  for (size_t k = 0; k < s["attrs"].size(); k++) {
    std::string dump;
    std::function<bool(const J&)> has_agg = [&](const J& e) -> bool {
      if (e["op"].s == "agg" || e["op"].s == "multivar") return true;
      for (const char* c : {"a", "b"}) if (e.has(c) && has_agg(e[c])) return true;
      return false;
    };
    if (has_agg(s["attrs"][k]["e"])) { why = "aggregator in select"; return nullptr; }
  }
  auto ex = std::make_unique<FollowedByExec>();
  ex->app = &app;
  ex->qi = qi;
  ex->path = 1;
  ex->sA = app.stream_idx.at(e1["stream"].s);
  ex->sB = app.stream_idx.at(e2["stream"].s);
  ex->same = ex->sA == ex->sB;
  ex->within = in["within"].null() ? -1 : in["within"].as_int();
  auto intern = [&](const std::string& str) { return app.intern(str); };
  // chain index -1 (CURRENT) and 0 resolve to the slot's single event; anything else is null
  auto sm = [&](int slot, int chain) -> int {
    if (slot != 0 && slot != 1) return -1;
    if (chain != -1 && chain != 0) return -1;
    return slot;
  };
  // e1's own filter cannot see e2 (null) — map slot 1 to null there
  auto sm1 = [&](int slot, int chain) -> int { return slot == 0 ? sm(slot, chain) : -1; };
  try {
    compile_filters(ex->progs[0], e1["filters"], sm1, intern);
    compile_filters(ex->progs[1], e2["filters"], sm, intern);
    for (size_t k = 0; k < s["attrs"].size(); k++) {
      Prog p;
      compile_expr(p, s["attrs"][k]["e"], sm, intern);
      ex->sel.push_back(p);
    }
  } catch (CompileError& e) {
    why = e.what();
    return nullptr;
  }
  if (app.streams[ex->sA].types.size() > FB_MAXC || app.streams[ex->sB].types.size() > FB_MAXC) {
    why = "too many attributes";
    return nullptr;
  }
  for (Ty t : app.streams[ex->sA].types) { ex->colA.emplace_back(); ex->colA.back().w = tsize(t); }
  if (!ex->same)
    for (Ty t : app.streams[ex->sB].types) { ex->colB.emplace_back(); ex->colB.back().w = tsize(t); }
  ex->in_streams = {ex->sA};
  if (!ex->same) ex->in_streams.push_back(ex->sB);
  return ex;
}

}  // namespace sg
