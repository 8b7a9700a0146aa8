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
//                  sequential double arithmetic then never rounds, so the result is bit-identical.  Otherwise the
//                  host restatement runs;
//   k_ext_time_*   the time window as index arithmetic (one clock per chunk: the front after event k's expiry is
//                  min(h, q + k)) plus a running-maximum scan for the notifyAt deadlines (TimeWindowProcessor :133-169);
//   k_ext_batch_*  lengthBatch in both modes as closed-form batch layouts (LengthBatchWindowProcessor :154-351);
//   k_ext_minmax   min / max replayed by one lane (the deque's value-equality removal is sequential): only with
//                  SG_EXT_DEVICE=1, since for one aggregator instance the host replay is faster.
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
  const int64_t lim = [] {                   // (read per call: a caller may switch it between chunks)
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

// ---- time window (TimeWindowProcessor.process :133-169) over one chunk at clock `now` ----
// S = the held queue ++ the chunk (expired copies with their own timestamps).  Before each event the queue's front
// expires while ts - now + T <= 0; one clock serves the whole chunk, so after event k's expiry the front is
// f_k = min(h, q + k) with h the first position of S whose ts > now - T (the walk stops at the first item that
// does not expire, :141-149).  Event k therefore emits S[f_{k-1}, f_k) EXPIRED, stamped `now`, at output positions
// [f_{k-1} + k, f_k + k), then itself CURRENT at f_k + k.
__global__ void __launch_bounds__(EXT_B) k_ext_time_first(int64_t n, const int64_t* __restrict__ ts, int64_t cut,
                                                          unsigned long long* __restrict__ first) {
  const int64_t k = (int64_t)blockIdx.x * EXT_B + threadIdx.x;
  if (k < n && ts[k] > cut) atomicMin(first, (unsigned long long)k);
}
__global__ void __launch_bounds__(EXT_B) k_ext_time_out(int64_t n, int64_t q, int64_t h, int64_t F, int64_t now,
                                                        const int64_t* __restrict__ qid, const int64_t* __restrict__ ids,
                                                        const int64_t* __restrict__ ts, int64_t* __restrict__ oid,
                                                        int32_t* __restrict__ otype, int64_t* __restrict__ ots) {
  const int64_t x = (int64_t)blockIdx.x * EXT_B + threadIdx.x;
  if (x >= F + n) return;
  if (x < F) {                                    // S[x] expires before event max(0, x - q + 1)
    const int64_t pos = x + max<int64_t>(0, x - q + 1);
    oid[pos] = x < q ? qid[x] : ids[x - q];
    otype[pos] = WE_EXPIRED;
    ots[pos] = now;
  } else {
    const int64_t k = x - F, pos = min(h, q + k) + k;
    oid[pos] = ids[k];
    otype[pos] = WE_CURRENT;
    ots[pos] = ts[k];
  }
}
// Scheduler.notifyAt(ts + T) for each event whose timestamp exceeds every earlier one (lastTimestamp, :158-160):
// flags over the chunk's running maximum
__global__ void __launch_bounds__(EXT_B) k_ext_time_notify(int64_t n, const int64_t* __restrict__ ts,
                                                           const int64_t* __restrict__ runmax, int64_t last, int64_t T,
                                                           int64_t* __restrict__ dl, uint8_t* __restrict__ flag) {
  const int64_t k = (int64_t)blockIdx.x * EXT_B + threadIdx.x;
  if (k >= n) return;
  const int64_t before = k ? max(last, runmax[k - 1]) : last;
  flag[k] = ts[k] > before;
  dl[k] = ts[k] + T;
}

// ---- lengthBatch(L) (LengthBatchWindowProcessor.process :154-351), L > 0, over one chunk ----
// C = the current batch (c0 held events) ++ the chunk.  Default mode: batch m = C[mL, (m + 1)L) completes at its
// last event and emits one chunk [the previous batch EXPIRED (held exq for m = 0) if expired output is on, the
// RESET copy of the batch's first event, the batch CURRENT]; expired and reset items are stamped `now`.  Chunk m
// starts at s0 = 0, then S0 + (m - 1) S1 (every chunk after the first has the same size).
struct ExtBatch {
  int64_t n, c0, x0, L, now, S0, S1, E0, E1;
  int32_t has_reset;
  int64_t reset_id;
  const int64_t* cid;        // C's ids [c0 + n]
  const int64_t* cts;        // C's timestamps
  const int64_t* xid;        // the held expired batch [x0]
};
__device__ __forceinline__ void ext_put(int64_t* oid, int32_t* otype, int64_t* ots, int64_t pos, int64_t id, int ty,
                                        int64_t t) {
  oid[pos] = id; otype[pos] = ty; ots[pos] = t;
}
__global__ void __launch_bounds__(EXT_B) k_ext_batch_out(ExtBatch b, int64_t total, int64_t* __restrict__ oid,
                                                         int32_t* __restrict__ otype, int64_t* __restrict__ ots) {
  const int64_t x = (int64_t)blockIdx.x * EXT_B + threadIdx.x;
  if (x >= total) return;
  const int64_t m = x < b.S0 ? 0 : 1 + (x - b.S0) / b.S1;
  const int64_t o = x < b.S0 ? x : (x - b.S0) % b.S1;
  const int64_t E = m == 0 ? b.E0 : b.E1;
  if (o < E) {
    const int64_t id = m == 0 ? b.xid[o] : b.cid[(m - 1) * b.L + o];
    ext_put(oid, otype, ots, x, id, WE_EXPIRED, b.now);
  } else if (o == E) {
    const int64_t id = (m == 0 && b.has_reset) ? b.reset_id : b.cid[m * b.L];
    ext_put(oid, otype, ots, x, id, WE_RESET, b.now);
  } else {
    const int64_t j = m * b.L + (o - E - 1);
    ext_put(oid, otype, ots, x, b.cid[j], WE_CURRENT, b.cts[j]);
  }
}
// lengthBatch(L, true) (streamCurrentEvents): every event is its own chunk; the (L+1)-th event since the last flush
// first flushes [the events since the previous flush EXPIRED (the held exq, then the chunk's, for the first flush),
// the RESET copy of the first event after the previous flush], both stamped `now`, then passes itself CURRENT.
// Flushes happen at events k1 + jL; event k's chunk starts at k + (the flush items of the flushes before it).
struct ExtBatchS {
  int64_t n, L, now, k1, X0, X1;   // first flush event (n: none), expired items of the first / later flushes
  int32_t has_reset;
  int64_t reset_id;
  int64_t x0;                      // held exq
  const int64_t* ids;
  const int64_t* ts;
  const int64_t* xid;
  int64_t* chunk_end;              // [n]
};
__global__ void __launch_bounds__(EXT_B) k_ext_batch_stream_out(ExtBatchS b, int64_t* __restrict__ oid,
                                                                int32_t* __restrict__ otype, int64_t* __restrict__ ots) {
  const int64_t k = (int64_t)blockIdx.x * EXT_B + threadIdx.x;
  if (k >= b.n) return;
  const int64_t nf = k <= b.k1 ? 0 : 1 + (k - 1 - b.k1) / b.L;    // flushes at events before k
  int64_t pos = k + (nf > 0 ? (b.X0 + 1) + (nf - 1) * (b.X1 + 1) : 0);
  const bool flush = k >= b.k1 && (k - b.k1) % b.L == 0;
  if (flush) {
    const bool first = k == b.k1;
    const int64_t X = first ? b.X0 : b.X1;
    for (int64_t o = 0; o < X; o++) {
      int64_t id;
      if (first) id = o < b.x0 ? b.xid[o] : b.ids[o - b.x0];
      else id = b.ids[k - b.L + o];
      ext_put(oid, otype, ots, pos++, id, WE_EXPIRED, b.now);
    }
    const int64_t rid = first ? (b.has_reset ? b.reset_id : b.ids[0]) : b.ids[k - b.L + 1];
    ext_put(oid, otype, ots, pos++, rid, WE_RESET, b.now);
  }
  ext_put(oid, otype, ots, pos++, b.ids[k], WE_CURRENT, b.ts[k]);
  b.chunk_end[k] = pos;
}

// ---- min / max (MinAttributeAggregatorExecutor.processAdd / processRemove :175-203, Max likewise) ----
// One instance replays its batch in order: the monotone deque with removeFirstOccurrence by value equality
// (Float/Double.equals) under trackFutureStates, else the running extreme cleared by an equal EXPIRED value.  The
// deque is sequential by nature (a removal depends on every earlier add and removal), so this is one lane; it runs
// only when device chunks are forced (SG_EXT_DEVICE=1): for one aggregator instance the host replay is faster.
__device__ __forceinline__ bool ext_lt(int t, int64_t a, int64_t b) {
  switch (t) {
    case T_INT: return (int32_t)a < (int32_t)b;
    case T_LONG: return a < b;
    case T_FLOAT: return bits_f(a) < bits_f(b);
    default: return bits_d(a) < bits_d(b);
  }
}
__device__ __forceinline__ bool ext_boxed_eq(int t, int64_t a, int64_t b) {
  if (t == T_FLOAT) { const float x = bits_f(a), y = bits_f(b); if (x != x && y != y) return true; return (uint32_t)a == (uint32_t)b; }
  if (t == T_DOUBLE) { const double x = bits_d(a), y = bits_d(b); if (x != x && y != y) return true; return a == b; }
  if (t == T_INT) return (int32_t)a == (int32_t)b;
  return a == b;
}
struct ExtMinMax {
  int64_t n;
  int32_t t, is_min, track;
  const int32_t* types;
  const int64_t* in;
  const uint8_t* nul;
  int64_t* out;
  uint8_t* onul;
  int64_t* dq;               // the deque, held part first [dq_n], room for n more
  int64_t dq_n;
  int64_t* state;            // [0] mv, [1] mv_null, [2] head, [3] tail (in / out)
};
__global__ void __launch_bounds__(64) k_ext_minmax(ExtMinMax a) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int64_t mv = a.state[0];
  bool mvn = a.state[1] != 0;
  int64_t h = 0, tl = a.dq_n;
  for (int64_t k = 0; k < a.n; k++) {
    const int ty = a.types[k];
    if (ty == WE_RESET) { h = tl = 0; mvn = true; a.out[k] = 0; a.onul[k] = 1; continue; }
    if (a.nul && a.nul[k]) { a.out[k] = mv; a.onul[k] = mvn; continue; }
    const int64_t v = a.in[k];
    if (ty == WE_CURRENT) {
      if (a.track) {
        while (tl > h && (a.is_min ? ext_lt(a.t, v, a.dq[tl - 1]) : ext_lt(a.t, a.dq[tl - 1], v))) tl--;
        a.dq[tl++] = v;
      }
      if (mvn || (a.is_min ? ext_lt(a.t, v, mv) : ext_lt(a.t, mv, v))) { mv = v; mvn = false; }
    } else if (a.track) {
      for (int64_t x = h; x < tl; x++)
        if (ext_boxed_eq(a.t, a.dq[x], v)) {      // erase: the front part moves up by one
          for (int64_t y = x; y > h; y--) a.dq[y] = a.dq[y - 1];
          h++;
          break;
        }
      mvn = h == tl;
      if (!mvn) mv = a.dq[h];
    } else if (!mvn && ext_boxed_eq(a.t, mv, v)) {
      mvn = true;
    }
    a.out[k] = mv;
    a.onul[k] = mvn;
  }
  a.state[0] = mv; a.state[1] = mvn; a.state[2] = h; a.state[3] = tl;
}

static bool ext_forced() {
  const char* e = getenv("SG_EXT_DEVICE");
  return e && atoi(e) == 1;
}

struct ExtDev {                                        // device buffers of one handle, reused across chunks
  DBuf<int64_t> a, b, c, d, e, f, g, h;
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
  // one chunk on the device (length: k_ext_len, time: k_ext_time_*, lengthBatch: k_ext_batch_*); false: the host
  // restatement takes it
  bool process_device(int64_t n, const int64_t* ids, const int64_t* ts, int64_t now) {
    if (spec.L <= 0 || n <= 0 || !ext_on_device(n)) return false;
    if (spec.kind == WK_TIME) return time_device(n, ids, ts, now);
    if (spec.kind == WK_BATCH) return spec.stream_current ? batch_stream_device(n, ids, ts, now)
                                                          : batch_device(n, ids, ts, now);
    if (spec.kind != WK_LENGTH) return false;
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
  // the outputs of a device chunk: `tot` items from dev.d / dev.ty / dev.e, one chunk ending at each of `ends`
  void take_out(int64_t tot, const std::vector<int64_t>& ends, hipStream_t s) {
    const size_t o = out_id.size();
    out_id.resize(o + (size_t)tot); out_type.resize(o + (size_t)tot); out_ts.resize(o + (size_t)tot);
    if (tot) {
      SG_HIP(hipMemcpyAsync(out_id.data() + o, dev.d.p, (size_t)tot * 8, hipMemcpyDeviceToHost, s));
      SG_HIP(hipMemcpyAsync(out_type.data() + o, dev.ty.p, (size_t)tot * 4, hipMemcpyDeviceToHost, s));
      SG_HIP(hipMemcpyAsync(out_ts.data() + o, dev.e.p, (size_t)tot * 8, hipMemcpyDeviceToHost, s));
    }
    SG_HIP(hipStreamSynchronize(s));
    for (int64_t e : ends) chunk_end.push_back((int64_t)o + e);
  }

  // TimeWindowProcessor over one chunk (k_ext_time_*): the first non-expiring position h, the outputs, and the
  // notifyAt deadlines; the held queue becomes S[F, q + n)
  bool time_device(int64_t n, const int64_t* ids, const int64_t* ts, int64_t now) {
    hipStream_t s = nullptr;
    const int64_t T = spec.L, q = (int64_t)st.q.size(), cut = now - T;
    int64_t h = q;
    for (int64_t i = 0; i < q; i++)
      if (st.q[(size_t)i].ts > cut) { h = i; break; }
    std::vector<int64_t> qid((size_t)std::max<int64_t>(q, 1));
    for (int64_t i = 0; i < q; i++) qid[(size_t)i] = st.q[(size_t)i].val;
    const unsigned g = (unsigned)((n + EXT_B - 1) / EXT_B);
    dev.a.reserve(std::max<int64_t>(q, 1)); dev.b.reserve(n); dev.c.reserve(n); dev.need.reserve(2);
    SG_HIP(hipMemcpyAsync(dev.a.p, qid.data(), (size_t)std::max<int64_t>(q, 1) * 8, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(dev.b.p, ids, (size_t)n * 8, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(dev.c.p, ts, (size_t)n * 8, hipMemcpyHostToDevice, s));
    if (h == q) {                                        // every held item expires: the chunk's first survivor
      const unsigned long long none = (unsigned long long)n;
      SG_HIP(hipMemcpyAsync(dev.need.p, &none, 8, hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(k_ext_time_first, dim3(g), dim3(EXT_B), 0, s, n, dev.c.p, cut,
                         (unsigned long long*)dev.need.p);
      SG_HIP(hipGetLastError());
      unsigned long long f = 0;
      SG_HIP(hipMemcpyAsync(&f, dev.need.p, 8, hipMemcpyDeviceToHost, s));
      SG_HIP(hipStreamSynchronize(s));
      h = q + (int64_t)f;
    }
    const int64_t F = std::min(h, q + n - 1), tot = F + n;
    dev.d.reserve(tot); dev.e.reserve(tot); dev.ty.reserve(tot);
    hipLaunchKernelGGL(k_ext_time_out, dim3((unsigned)((tot + EXT_B - 1) / EXT_B)), dim3(EXT_B), 0, s, n, q, h, F, now,
                       dev.a.p, dev.b.p, dev.c.p, dev.d.p, dev.ty.p, dev.e.p);
    SG_HIP(hipGetLastError());
    // the notifyAt deadlines: events past the running maximum of the timestamps (lastTimestamp)
    size_t tb = 0, tb2 = 0;
    SG_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, tb, dev.c.p, dev.d.p, hipcub::Max(), (int)n, s));
    SG_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb2, dev.b.p, dev.nul.p, dev.b.p, dev.need.p, (int)n, s));
    dev.tmp.reserve(std::max(tb, tb2));
    dev.f.reserve(n); dev.g.reserve(n); dev.nul.reserve(n); dev.h.reserve(n);
    SG_HIP(hipcub::DeviceScan::InclusiveScan(dev.tmp.p, tb, dev.c.p, dev.f.p, hipcub::Max(), (int)n, s));
    hipLaunchKernelGGL(k_ext_time_notify, dim3(g), dim3(EXT_B), 0, s, n, dev.c.p, dev.f.p, st.last_ts, T, dev.g.p,
                       dev.nul.p);
    SG_HIP(hipGetLastError());
    SG_HIP(hipcub::DeviceSelect::Flagged(dev.tmp.p, tb2, dev.g.p, dev.nul.p, dev.h.p, (int*)dev.need.p, (int)n, s));
    int nd = 0;
    int64_t rmax = 0;
    SG_HIP(hipMemcpyAsync(&nd, dev.need.p, sizeof(int), hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(&rmax, dev.f.p + (n - 1), 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    std::vector<int64_t> dls((size_t)nd);
    if (nd) SG_HIP(hipMemcpy(dls.data(), dev.h.p, (size_t)nd * 8, hipMemcpyDeviceToHost));
    if (getenv("SG_EXT_DEBUG"))
      fprintf(stderr, "[ext time] n=%lld q=%lld h=%lld nd=%d rmax=%lld last=%lld tb=%zu tb2=%zu\n", (long long)n,
              (long long)q, (long long)h, nd, (long long)rmax, (long long)st.last_ts, tb, tb2);
    take_out(tot, {tot}, s);
    for (int64_t d : dls) { st.timers.push_back(d); fresh_dl.push_back(d); }
    if (rmax > st.last_ts) st.last_ts = rmax;
    // the held queue: S[F, q + n)
    for (int64_t i = 0; i < std::min(F, q); i++) st.q.pop_front();
    for (int64_t k = std::max<int64_t>(0, F - q); k < n; k++) st.q.push_back(WinItem<int64_t>{WE_EXPIRED, ts[k], ids[k]});
    ext_dev_chunks++;
    return true;
  }

  // LengthBatchWindowProcessor, default mode (k_ext_batch_out): one output chunk per completed batch
  bool batch_device(int64_t n, const int64_t* ids, const int64_t* ts, int64_t now) {
    hipStream_t s = nullptr;
    const int64_t L = spec.L, c0 = (int64_t)st.cur.size(), x0 = (int64_t)st.exq.size();
    if (c0 != st.count || c0 >= L) return false;
    const int64_t M = (c0 + n) / L, E0 = spec.expired_on ? x0 : 0, E1 = spec.expired_on ? L : 0;
    const int64_t S0 = E0 + 1 + L, S1 = E1 + 1 + L, tot = M ? S0 + (M - 1) * S1 : 0;
    std::vector<int64_t> cid((size_t)(c0 + n)), cts((size_t)(c0 + n)), xid((size_t)std::max<int64_t>(x0, 1));
    for (int64_t j = 0; j < c0; j++) { cid[(size_t)j] = st.cur[(size_t)j].val; cts[(size_t)j] = st.cur[(size_t)j].ts; }
    std::memcpy(cid.data() + c0, ids, (size_t)n * 8);
    std::memcpy(cts.data() + c0, ts, (size_t)n * 8);
    for (int64_t j = 0; j < x0; j++) xid[(size_t)j] = st.exq[(size_t)j].val;
    if (tot) {
      dev.a.reserve(c0 + n); dev.b.reserve(c0 + n); dev.c.reserve(std::max<int64_t>(x0, 1));
      SG_HIP(hipMemcpyAsync(dev.a.p, cid.data(), (size_t)(c0 + n) * 8, hipMemcpyHostToDevice, s));
      SG_HIP(hipMemcpyAsync(dev.b.p, cts.data(), (size_t)(c0 + n) * 8, hipMemcpyHostToDevice, s));
      SG_HIP(hipMemcpyAsync(dev.c.p, xid.data(), (size_t)std::max<int64_t>(x0, 1) * 8, hipMemcpyHostToDevice, s));
      ExtBatch b{n, c0, x0, L, now, S0, S1, E0, E1, st.has_reset ? 1 : 0, st.reset.val, dev.a.p, dev.b.p, dev.c.p};
      dev.d.reserve(tot); dev.e.reserve(tot); dev.ty.reserve(tot);
      hipLaunchKernelGGL(k_ext_batch_out, dim3((unsigned)((tot + EXT_B - 1) / EXT_B)), dim3(EXT_B), 0, s, b, tot,
                         dev.d.p, dev.ty.p, dev.e.p);
      SG_HIP(hipGetLastError());
    }
    std::vector<int64_t> ends((size_t)M);
    for (int64_t m = 0; m < M; m++) ends[(size_t)m] = S0 + m * S1;
    take_out(tot, ends, s);
    // the state after the chunk: the batch being filled, the last completed batch (expired copies), the reset event
    if (M > 0) {
      if (spec.expired_on) {
        st.exq.clear();
        for (int64_t j = (M - 1) * L; j < M * L; j++)
          st.exq.push_back(WinItem<int64_t>{WE_EXPIRED, cts[(size_t)j], cid[(size_t)j]});
      }
      st.has_reset = false;
    }
    st.cur.clear();
    for (int64_t j = M * L; j < c0 + n; j++) st.cur.push_back(WinItem<int64_t>{WE_CURRENT, cts[(size_t)j], cid[(size_t)j]});
    st.count = (int64_t)st.cur.size();
    if (!st.has_reset && !st.cur.empty()) {
      st.reset = st.cur.front();
      st.reset.type = WE_RESET;
      st.has_reset = true;
    }
    ext_dev_chunks++;
    return true;
  }

  // LengthBatchWindowProcessor, streamCurrentEvents mode (k_ext_batch_stream_out): one output chunk per event
  bool batch_stream_device(int64_t n, const int64_t* ids, const int64_t* ts, int64_t now) {
    hipStream_t s = nullptr;
    const int64_t L = spec.L, c0 = st.count, x0 = (int64_t)st.exq.size();
    if (c0 < 0 || c0 > L) return false;
    const int64_t k1 = L - c0 < n ? L - c0 : n;          // the first flush (n: none in this chunk)
    const int64_t nfl = k1 < n ? 1 + (n - 1 - k1) / L : 0;
    const int64_t X0 = spec.expired_on ? x0 + k1 : 0, X1 = spec.expired_on ? L : 0;
    const int64_t tot = n + (nfl ? (X0 + 1) + (nfl - 1) * (X1 + 1) : 0);
    std::vector<int64_t> xid((size_t)std::max<int64_t>(x0, 1));
    for (int64_t j = 0; j < x0; j++) xid[(size_t)j] = st.exq[(size_t)j].val;
    dev.a.reserve(n); dev.b.reserve(n); dev.c.reserve(std::max<int64_t>(x0, 1)); dev.f.reserve(n);
    SG_HIP(hipMemcpyAsync(dev.a.p, ids, (size_t)n * 8, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(dev.b.p, ts, (size_t)n * 8, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(dev.c.p, xid.data(), (size_t)std::max<int64_t>(x0, 1) * 8, hipMemcpyHostToDevice, s));
    ExtBatchS b{n, L, now, k1, X0, X1, st.has_reset ? 1 : 0, st.reset.val, x0, dev.a.p, dev.b.p, dev.c.p, dev.f.p};
    dev.d.reserve(tot); dev.e.reserve(tot); dev.ty.reserve(tot);
    hipLaunchKernelGGL(k_ext_batch_stream_out, dim3((unsigned)((n + EXT_B - 1) / EXT_B)), dim3(EXT_B), 0, s, b, dev.d.p,
                       dev.ty.p, dev.e.p);
    SG_HIP(hipGetLastError());
    std::vector<int64_t> ends((size_t)n);
    SG_HIP(hipMemcpyAsync(ends.data(), dev.f.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
    take_out(tot, ends, s);
    // the state after the chunk
    const int64_t klast = nfl ? k1 + (nfl - 1) * L : -1;   // the last flush event
    if (nfl) {
      st.count = 1 + (n - 1 - klast);
      // the reset event: the first event after the last flush (none yet when the flush was the chunk's last)
      st.has_reset = klast + 1 < n;
      if (st.has_reset) st.reset = WinItem<int64_t>{WE_RESET, ts[klast + 1], ids[klast + 1]};
      if (spec.expired_on) {
        st.exq.clear();
        for (int64_t k = klast; k < n; k++) st.exq.push_back(WinItem<int64_t>{WE_EXPIRED, ts[k], ids[k]});
      }
    } else {
      st.count = c0 + n;
      if (!st.has_reset) { st.reset = WinItem<int64_t>{WE_RESET, ts[0], ids[0]}; st.has_reset = true; }
      if (spec.expired_on)
        for (int64_t k = 0; k < n; k++) st.exq.push_back(WinItem<int64_t>{WE_EXPIRED, ts[k], ids[k]});
    }
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
  // min / max over one batch (k_ext_minmax): the held deque and extreme go up, the batch replays, they come back
  bool minmax_device(int64_t n, const int32_t* types, const int64_t* in, const uint8_t* in_null, int64_t* out,
                     uint8_t* out_null) {
    hipStream_t s = nullptr;
    const int64_t q = (int64_t)st.dq.size();
    std::vector<int64_t> dq(st.dq.begin(), st.dq.end());
    dev.ty.reserve(n); dev.a.reserve(n); dev.b.reserve(n); dev.nul.reserve(n); dev.onul.reserve(n);
    dev.c.reserve(q + n); dev.d.reserve(4);
    SG_HIP(hipMemcpyAsync(dev.ty.p, types, (size_t)n * 4, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(dev.a.p, in, (size_t)n * 8, hipMemcpyHostToDevice, s));
    if (in_null) SG_HIP(hipMemcpyAsync(dev.nul.p, in_null, (size_t)n, hipMemcpyHostToDevice, s));
    if (q) SG_HIP(hipMemcpyAsync(dev.c.p, dq.data(), (size_t)q * 8, hipMemcpyHostToDevice, s));
    int64_t sv[4] = {st.mv, st.mv_null ? 1 : 0, 0, q};
    SG_HIP(hipMemcpyAsync(dev.d.p, sv, sizeof(sv), hipMemcpyHostToDevice, s));
    ExtMinMax a{n, (int32_t)spec.in_t, spec.k == SA_MIN ? 1 : 0, spec.track ? 1 : 0, dev.ty.p, dev.a.p,
                in_null ? dev.nul.p : nullptr, dev.b.p, dev.onul.p, dev.c.p, q, dev.d.p};
    hipLaunchKernelGGL(k_ext_minmax, dim3(1), dim3(64), 0, s, a);
    SG_HIP(hipGetLastError());
    SG_HIP(hipMemcpyAsync(out, dev.b.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(out_null, dev.onul.p, (size_t)n, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(sv, dev.d.p, sizeof(sv), hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    const int64_t h = sv[2], t = sv[3];
    dq.resize((size_t)std::max<int64_t>(t, 0));
    if (t > h) SG_HIP(hipMemcpy(dq.data() + h, dev.c.p + h, (size_t)(t - h) * 8, hipMemcpyDeviceToHost));
    st.dq.assign(dq.begin() + h, dq.begin() + t);
    st.mv = sv[0];
    st.mv_null = sv[1] != 0;
    ext_dev_chunks++;
    return true;
  }
  // count / sum / avg over one batch on the device (segmented scan of exact deltas); false: the host takes it
  bool process_device(int64_t n, const int32_t* types, const int64_t* in, const uint8_t* in_null, int64_t* out,
                      uint8_t* out_null) {
    if (!ext_on_device(n)) return false;
    if (spec.k == SA_MIN || spec.k == SA_MAX) return ext_forced() && minmax_device(n, types, in, in_null, out, out_null);
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
