// ext.hip — the window / aggregator extension ABI (include/siddhi_gfx_ext.h).
//
// The Java extension classes (java/src/main/java/io/siddhi/gpu/ext/) registered with
// SiddhiManager.setExtension call these per chunk (windows) or per selector pass (aggregators).  They run
// the same restatements the query paths use: the window processors of window_proc.hpp (general window
// path) and AggOps of selector.hpp (every selector stage).  A window holds the ids of the events it
// retains; the shim keeps the StreamEvent clones and emits them in the order returned here.
//
// Batched chunks run on the device (SG_EXT_DEVICE_MIN events or more, default 4096; SG_EXT_DEVICE=0 keeps the host,
// =1 sends every chunk to the device):
//   k_ext_len      the length window as index arithmetic over the held queue followed by the chunk: event k of a
//                  chunk is the k-th arrival after the window holds c0 events, so once c0 + k >= L it expires
//                  element k - (L - c0) of (queue ++ chunk) and its output pair sits at (L - c0) + 2 (k - (L - c0))
//                  (LengthWindowProcessor.process :106-141, one EXPIRED before each CURRENT once full);
//   k_ext_agg_*    count / sum / avg as a segmented inclusive scan of (count, sum) deltas, restarted at RESET
//                  events (AttributeAggregatorExecutor.execute :59-67 with processAdd / processRemove / reset):
//                  exact in int64 when the inputs are integral, or -- FLOAT / DOUBLE -- when every value and the held
//                  sum are multiples of 2^-S with every partial sum below 2^52 in units of 2^-S; the reference's
//                  sequential double arithmetic then never rounds, so the result is bit-identical.  Otherwise, and
//                  for min / max (the deque's value-equality removal is sequential), the host restatement runs.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/siddhi_gfx.h"
#include "../../include/siddhi_gfx_ext.h"
#include "runtime.hpp"
#include "selector.hpp"
#include "snapshot.hpp"
#include "window_proc.hpp"

namespace sg {
int set_error(int code, const std::string& m);

// a chunk of n events goes to the device when it is at least this long (and a GPU is present)
static bool ext_on_device(int64_t n) {
  static const int64_t lim = [] {
    const char* e = getenv("SG_EXT_DEVICE");
    if (e && atoi(e) == 0) return INT64_MAX;
    if (e && atoi(e) == 1) return (int64_t)1;
    const char* m = getenv("SG_EXT_DEVICE_MIN");
    return m ? (int64_t)atoll(m) : (int64_t)4096;
  }();
  static const bool gpu = [] {
    int c = 0;
    return hipGetDeviceCount(&c) == hipSuccess && c > 0;
  }();
  return gpu && n >= lim;
}

constexpr int EXT_B = 256;
static std::atomic<int64_t> ext_dev_chunks{0};

__global__ void __launch_bounds__(EXT_B) k_ext_len(int64_t n, int64_t k0, int64_t q, const int64_t* __restrict__ qid,
                                                   const int64_t* __restrict__ ids, const int64_t* __restrict__ ts,
                                                   int64_t now, int64_t* __restrict__ oid, int32_t* __restrict__ otype,
                                                   int64_t* __restrict__ ots) {
  const int64_t k = (int64_t)blockIdx.x * EXT_B + threadIdx.x;
  if (k >= n) return;
  if (k < k0) {                              // the window is filling: the event passes as CURRENT
    oid[k] = ids[k]; otype[k] = WE_CURRENT; ots[k] = ts[k];
    return;
  }
  const int64_t j = k - k0, pos = k0 + 2 * j;
  oid[pos] = j < q ? qid[j] : ids[j - q];    // the oldest held event, re-stamped with the chunk's clock
  otype[pos] = WE_EXPIRED;
  ots[pos] = now;
  oid[pos + 1] = ids[k]; otype[pos + 1] = WE_CURRENT; ots[pos + 1] = ts[k];
}

// one event's (count, sum) delta; `reset` restarts the running state
struct ExtSeg {
  int64_t dc, ds;
  int32_t reset;
};
struct ExtSegOp {
  __host__ __device__ ExtSeg operator()(const ExtSeg& a, const ExtSeg& b) const {
    return b.reset ? b : ExtSeg{a.dc + b.dc, a.ds + b.ds, a.reset};
  }
};

// the argument as a double (AggOps::as_d) and as an integer (AggOps::as_l)
__device__ __forceinline__ double ext_as_d(int t, int64_t r) {
  switch (t) {
    case T_INT: return (double)(int32_t)r;
    case T_LONG: return (double)r;
    case T_FLOAT: return (double)bits_f(r);
    default: return bits_d(r);
  }
}

// exactness check: the largest 2^-S grid any argument needs (-1: NaN / infinity), and the sum of |argument|
__global__ void __launch_bounds__(EXT_B) k_ext_agg_check(int64_t n, int t, const int32_t* __restrict__ types,
                                                         const int64_t* __restrict__ in, const uint8_t* __restrict__ nul,
                                                         int* __restrict__ need, double* __restrict__ mag) {
  __shared__ int sn[EXT_B / 64];
  __shared__ double sm[EXT_B / 64];
  const int64_t k = (int64_t)blockIdx.x * EXT_B + threadIdx.x;
  int nd = 0;
  double m = 0;
  if (k < n && types[k] != WE_RESET && !(nul && nul[k])) {
    const double v = ext_as_d(t, in[k]);
    if (!isfinite(v)) nd = 4096;
    else if (v != 0) {
      int e;
      const double fr = frexp(v, &e);                  // v = fr * 2^e, |fr| in [0.5, 1)
      const int64_t mant = (int64_t)ldexp(fabs(fr), 53);
      const int tz = __builtin_ctzll((uint64_t)mant);
      nd = max(0, 53 - tz - e);                        // the least significant set bit is 2^(e - 53 + tz)
      m = fabs(v);
    }
  }
  for (int d = 32; d >= 1; d >>= 1) {
    nd = max(nd, __shfl_xor(nd, d, 64));
    m += __shfl_xor(m, d, 64);
  }
  if ((threadIdx.x & 63) == 0) { sn[threadIdx.x >> 6] = nd; sm[threadIdx.x >> 6] = m; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int a = 0;
    double b = 0;
    for (int w = 0; w < EXT_B / 64; w++) { a = max(a, sn[w]); b += sm[w]; }
    atomicMax(need, a);
    atomicAdd(mag, b);
  }
}

// deltas: COUNT counts every CURRENT / EXPIRED event; SUM / AVG only non-null arguments, in units of 2^-S
__global__ void __launch_bounds__(EXT_B) k_ext_agg_delta(int64_t n, int kind, int t, int S,
                                                         const int32_t* __restrict__ types, const int64_t* __restrict__ in,
                                                         const uint8_t* __restrict__ nul, ExtSeg* __restrict__ d) {
  const int64_t k = (int64_t)blockIdx.x * EXT_B + threadIdx.x;
  if (k >= n) return;
  const int ty = types[k];
  ExtSeg x{0, 0, ty == WE_RESET};
  if (ty != WE_RESET && (kind == SA_COUNT || !(nul && nul[k]))) {
    const int64_t sgn = ty == WE_CURRENT ? 1 : -1;
    x.dc = sgn;
    if (kind != SA_COUNT) {
      const int64_t v = (t == T_INT || t == T_LONG) ? (t == T_INT ? (int64_t)(int32_t)in[k] : in[k])
                                                    : (int64_t)ldexp(ext_as_d(t, in[k]), S);
      x.ds = sgn * v;
    }
  }
  d[k] = x;
}

// outputs after each event (AggOps::apply's value and null rules) from the held state and the scanned deltas
__global__ void __launch_bounds__(EXT_B) k_ext_agg_out(int64_t n, int kind, int t, int S, int64_t c0, int64_t s0,
                                                       const int32_t* __restrict__ types, const uint8_t* __restrict__ nul,
                                                       const ExtSeg* __restrict__ p, int64_t* __restrict__ out,
                                                       uint8_t* __restrict__ onul) {
  const int64_t k = (int64_t)blockIdx.x * EXT_B + threadIdx.x;
  if (k >= n) return;
  const ExtSeg x = p[k];
  const int64_t c = x.reset ? x.dc : c0 + x.dc, sv = x.reset ? x.ds : s0 + x.ds;
  const int ty = types[k];
  const bool inn = kind != SA_COUNT && nul && nul[k];
  const bool integral = t == T_INT || t == T_LONG;
  int64_t v = 0;
  bool isnull = false;
  if (kind == SA_COUNT) {
    v = c;
  } else if (ty == WE_RESET) {
    isnull = !(kind == SA_SUM && integral);
  } else if (c == 0 && (inn || ty == WE_EXPIRED)) {
    isnull = true;
  } else if (kind == SA_SUM) {
    v = integral ? sv : d_bits(ldexp((double)sv, -S));
  } else if (c == 0) {                                 // AVG over nothing
    isnull = true;
  } else {                                             // AVG: the running double sum over the count
    v = d_bits(ldexp((double)sv, -S) / (double)c);
  }
  out[k] = v;
  onul[k] = (uint8_t)isnull;
}

struct ExtDev {                                        // device buffers of one handle, reused across chunks
  DBuf<int64_t> a, b, c, d, e;
  DBuf<int32_t> ty;
  DBuf<uint8_t> nul, onul, tmp;
  DBuf<ExtSeg> seg, pre;
  DBuf<int> need;
  DBuf<double> mag;
};
}  // namespace sg
using namespace sg;

struct sg_window {
  WinSpec spec;
  WinState<int64_t> st;                      // payload: the shim's event id
  std::vector<int64_t> out_id, out_ts, chunk_end;
  std::vector<int32_t> out_type;
  std::vector<int64_t> fresh_dl;             // notifyAt deadlines queued since the shim last took them
  ExtDev dev;
  // the length window over one chunk on the device (k_ext_len); false: the host restatement takes it
  bool process_device(int64_t n, const int64_t* ids, const int64_t* ts, int64_t now) {
    if (spec.kind != WK_LENGTH || spec.L <= 0 || !ext_on_device(n)) return false;
    const int64_t c0 = st.count, q = (int64_t)st.q.size();
    if (c0 != q || c0 > spec.L) return false;
    const int64_t k0 = std::min<int64_t>(n, spec.L - c0), nexp = n - k0, tot = n + nexp;
    const int64_t qn = std::min<int64_t>(q, nexp);                  // held events that expire in this chunk
    std::vector<int64_t> qid((size_t)std::max<int64_t>(qn, 1));
    for (int64_t j = 0; j < qn; j++) qid[(size_t)j] = st.q[(size_t)j].val;
    hipStream_t s = nullptr;
    dev.a.reserve(std::max<int64_t>(qn, 1)); dev.b.reserve(n); dev.c.reserve(n);
    dev.d.reserve(tot); dev.e.reserve(tot); dev.ty.reserve(tot);
    SG_HIP(hipMemcpyAsync(dev.a.p, qid.data(), (size_t)std::max<int64_t>(qn, 1) * 8, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(dev.b.p, ids, (size_t)n * 8, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(dev.c.p, ts, (size_t)n * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_ext_len, dim3((unsigned)((n + EXT_B - 1) / EXT_B)), dim3(EXT_B), 0, s, n, k0, qn, dev.a.p,
                       dev.b.p, dev.c.p, now, dev.d.p, dev.ty.p, dev.e.p);
    SG_HIP(hipGetLastError());
    const size_t o = out_id.size();
    out_id.resize(o + (size_t)tot); out_type.resize(o + (size_t)tot); out_ts.resize(o + (size_t)tot);
    SG_HIP(hipMemcpyAsync(out_id.data() + o, dev.d.p, (size_t)tot * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(out_type.data() + o, dev.ty.p, (size_t)tot * 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(out_ts.data() + o, dev.e.p, (size_t)tot * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    if (tot) chunk_end.push_back((int64_t)out_id.size());
    // the held queue: the last L of (queue ++ chunk), as expired copies with their own timestamps
    for (int64_t j = 0; j < qn; j++) st.q.pop_front();
    const int64_t from = std::max<int64_t>(0, n - spec.L);
    for (int64_t k = from; k < n; k++) {
      st.q.push_back(WinItem<int64_t>{WE_EXPIRED, ts[k], ids[k]});
      if ((int64_t)st.q.size() > spec.L) st.q.pop_front();
    }
    st.count = std::min<int64_t>(spec.L, c0 + n);
    ext_dev_chunks++;
    return true;
  }
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
  ExtDev dev;
  // count / sum / avg over one batch on the device (segmented scan of exact deltas); false: the host takes it
  bool process_device(int64_t n, const int32_t* types, const int64_t* in, const uint8_t* in_null, int64_t* out,
                      uint8_t* out_null) {
    if (spec.k == SA_MIN || spec.k == SA_MAX || !ext_on_device(n)) return false;
    const bool integral = spec.in_t == T_INT || spec.in_t == T_LONG;
    hipStream_t s = nullptr;
    dev.ty.reserve(n); dev.a.reserve(n); dev.b.reserve(n); dev.seg.reserve(n); dev.pre.reserve(n);
    dev.nul.reserve(n); dev.onul.reserve(n); dev.need.reserve(1); dev.mag.reserve(1);
    SG_HIP(hipMemcpyAsync(dev.ty.p, types, (size_t)n * 4, hipMemcpyHostToDevice, s));
    const bool arg = spec.arg >= 0;
    if (arg) SG_HIP(hipMemcpyAsync(dev.a.p, in, (size_t)n * 8, hipMemcpyHostToDevice, s));
    if (arg && in_null) SG_HIP(hipMemcpyAsync(dev.nul.p, in_null, (size_t)n, hipMemcpyHostToDevice, s));
    const uint8_t* dn = arg && in_null ? dev.nul.p : nullptr;
    const unsigned g = (unsigned)((n + EXT_B - 1) / EXT_B);
    int S = 0;
    int64_t s0 = 0;
    if (spec.k != SA_COUNT) {
      SG_HIP(hipMemsetAsync(dev.need.p, 0, sizeof(int), s));
      SG_HIP(hipMemsetAsync(dev.mag.p, 0, sizeof(double), s));
      hipLaunchKernelGGL(k_ext_agg_check, dim3(g), dim3(EXT_B), 0, s, n, (int)spec.in_t, dev.ty.p, dev.a.p, dn,
                         dev.need.p, dev.mag.p);
      SG_HIP(hipGetLastError());
      int need = 0;
      double mag = 0;
      SG_HIP(hipMemcpyAsync(&need, dev.need.p, sizeof(int), hipMemcpyDeviceToHost, s));
      SG_HIP(hipMemcpyAsync(&mag, dev.mag.p, sizeof(double), hipMemcpyDeviceToHost, s));
      SG_HIP(hipStreamSynchronize(s));
      // the held sum: the running long (SUM of INT / LONG) or double, on the same grid
      const double held = (spec.k == SA_SUM && integral) ? (double)st.lsum : st.dsum;
      if (spec.k == SA_SUM && integral) {
        S = 0;
        if (std::fabs((double)st.lsum) + mag >= 4503599627370496.0) return false;   // 2^52: no rounding, no wrap
        s0 = st.lsum;
      } else {
        if (!std::isfinite(held)) return false;
        int hneed = 0;
        if (held != 0) {
          int e;
          const double fr = std::frexp(held, &e);
          const int64_t mant = (int64_t)std::ldexp(std::fabs(fr), 53);
          hneed = std::max(0, 53 - __builtin_ctzll((uint64_t)mant) - e);
        }
        S = std::max(need, hneed);                     // (0 for integral arguments and an integral held sum)
        if (S > 1000 || std::ldexp(std::fabs(held) + mag, S) >= 4503599627370496.0) return false;
        s0 = (int64_t)std::ldexp(held, S);
      }
    }
    hipLaunchKernelGGL(k_ext_agg_delta, dim3(g), dim3(EXT_B), 0, s, n, (int)spec.k, (int)spec.in_t, S, dev.ty.p,
                       dev.a.p, dn, dev.seg.p);
    SG_HIP(hipGetLastError());
    size_t tb = 0;
    SG_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, tb, dev.seg.p, dev.pre.p, ExtSegOp(), (int)n, s));
    dev.tmp.reserve(tb);
    SG_HIP(hipcub::DeviceScan::InclusiveScan(dev.tmp.p, tb, dev.seg.p, dev.pre.p, ExtSegOp(), (int)n, s));
    const int64_t c0 = st.count;
    hipLaunchKernelGGL(k_ext_agg_out, dim3(g), dim3(EXT_B), 0, s, n, (int)spec.k, (int)spec.in_t, S, c0, s0, dev.ty.p,
                       dn, dev.pre.p, dev.b.p, dev.onul.p);
    SG_HIP(hipGetLastError());
    SG_HIP(hipMemcpyAsync(out, dev.b.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(out_null, dev.onul.p, (size_t)n, hipMemcpyDeviceToHost, s));
    ExtSeg last;
    SG_HIP(hipMemcpyAsync(&last, dev.pre.p + (n - 1), sizeof(ExtSeg), hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    // the state after the batch
    const int64_t c = last.reset ? last.dc : c0 + last.dc, sv = last.reset ? last.ds : s0 + last.ds;
    st.count = c;
    if (spec.k == SA_SUM && integral) st.lsum = sv;
    else if (spec.k != SA_COUNT) st.dsum = std::ldexp((double)sv, -S);
    ext_dev_chunks++;
    return true;
  }
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

int64_t sg_ext_device_chunks(void) { return ext_dev_chunks.load(); }

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
    if (w->process_device(n, ids, ts, now)) return SG_OK;
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
    if (n > 0 && a->process_device(n, types, in, in_null, out, out_null)) return SG_OK;
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
