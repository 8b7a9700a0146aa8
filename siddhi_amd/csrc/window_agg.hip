// window_agg.hip — execution path SG_PATH_WINDOW_AGG.
//
// Query shape:  from S[f]*#window.length(L) | #window.time(T) | #window.lengthBatch(L)
//               select <S attrs>, sum/avg/count/min/max(...) [group by <one attribute>] insert into ...
//
// Reference semantics (restated; see oracle/siddhi_oracle.cpp window_process / Selector):
//   * FilterProcessor drops failing events before the window (FilterProcessor.java:48-61).
//   * LengthWindowProcessor (:106-141): once L events are held, each new event first emits the
//     oldest one as EXPIRED; the window is global (not per group) and runs over the filtered stream.
//   * TimeWindowProcessor (:133-169): before each event the queue expires every held event with
//     ts - now + T <= 0, now = the app clock of the event's chunk (playback: the chunk's last timestamp,
//     InputHandler.send -> setCurrentTimestamp; otherwise the wall clock the shim passes at push), and
//     the event is appended.  So filtered event p sees the window [ws(p), p] with ws(p) = min(p, first
//     filtered q with ts_q > now(p) - T) -- the length window is the case ws(p) = max(0, p - L + 1).
//     Timer chunks only move the same removals earlier; with current-event output they emit nothing.
//   * LengthBatchWindowProcessor (:154-351): every L filtered events form one output chunk [RESET,
//     e_1..e_L].  The RESET event is a copy of e_1, so with group-by it resets only e_1's group (the
//     other groups' aggregates run on across batches); the aggregators do not track expiries
//     (trackFutureStates is false), so min/max are plain running extremes since the last reset.
//   * Aggregators are per group (GroupByKeyGenerator key, PartitionStateHolder per group) and see,
//     in chunk order, `processRemove` for the expired event and `processAdd` for the current one
//     (Sum/Avg/Count/Min/MaxAttributeAggregatorExecutor).  So after filtered event p the state of
//     group g is the aggregate of the filtered events q in (p-L, p] with g(q) = g.
//   * QuerySelector batching (:315-374): per chunk (one send() call) the LAST current event of each
//     group is emitted, in order of the group's first current event in the chunk; without group-by
//     the last event of the chunk; without aggregators every current event.
//
// Kernels (gfx950):
//   k_wa_filter     filter bytecode per event -> flags; DeviceSelect compaction -> filtered index
//   k_wa_gather     group id + fixed-point values (+ timestamps) of the filtered events; exactness statistics
//   k_wa_wstart     window start ws(p) of every filtered event (time: binary search over the filtered
//                   timestamps for now(p) - T) and the widest window
//   k_wa_tile       exact fast path (sum/avg/count): a workgroup owns T filtered events and stages
//                   the preceding L as a halo in LDS; LDS counting sort by group, each group's
//                   bucket ordered by position, windowed sums as prefix differences in int64 fixed
//                   point.  Exactness check: every value is a multiple of 2^-S and (L+1)*max|x|*2^S
//                   < 2^53, so the reference's sequential double arithmetic never rounded and equals
//                   the integer result bit for bit.
//   k_wa_seq        general path (min/max deques, non-exact sums): one lane per group replays the
//                   group's add/remove sequence with the reference's exact double/long arithmetic
//                   and deque quirks (removeFirstOccurrence by value).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <unordered_map>

#include "runtime.hpp"
#include "snapshot.hpp"

namespace sg {

constexpr int WA_B = 512;
constexpr int WA_MAXK = 4096;      // dense group ids handled by the LDS fast path
constexpr int WA_MAXA = 6;         // aggregators
constexpr int WA_MAXV = 4;         // distinct aggregated value columns

enum AggK { A_SUM = 0, A_AVG, A_COUNT, A_MIN, A_MAX };

struct WaLoader {
  const uint8_t* const* cols;
  const int32_t* w;
  int64_t e;
  __device__ bool load(int slot, int attr, int64_t& v) const {
    (void)slot;
    v = w[attr] == 8 ? ((const int64_t*)cols[attr])[e] : (int64_t)((const int32_t*)cols[attr])[e];
    return true;
  }
};

struct WaCols {
  const uint8_t* c[12];
  int32_t w[12];
};

// Filter + compaction in two passes over WA_FT-event tiles: k_wa_filter evaluates the filter, writes one
// flag byte per event and the tile's pass count; an exclusive scan of the counts gives each tile's base;
// k_wa_place turns 16 flags per thread (one 16-B load) into the filtered event indices behind that base
// (block scan of the threads' counts), in event order.
constexpr int WA_FT = 4096;

__global__ void __launch_bounds__(256) k_wa_filter(int64_t lo, int64_t n, WaCols cols, const Prog* __restrict__ prog,
                                                    int has_filter, uint8_t* __restrict__ flags,
                                                    uint32_t* __restrict__ tcnt) {
  __shared__ int64_t rf[MAX_REG * 256];
  __shared__ uint32_t bc;
  if (threadIdx.x == 0) bc = 0;
  __syncthreads();
  const int64_t t0 = lo + (int64_t)blockIdx.x * WA_FT;
  uint32_t c = 0;
  for (int k = threadIdx.x; k < WA_FT; k += 256) {
    const int64_t e = t0 + k;
    if (e >= n) break;
    WaLoader ld{cols.c, cols.w, e};
    const bool f = has_filter ? run_pred(*prog, ld, rf + threadIdx.x, 256) : true;
    flags[e - lo] = (uint8_t)f;
    c += f;
  }
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(&bc, c);
  __syncthreads();
  if (threadIdx.x == 0) tcnt[blockIdx.x] = bc;
}

// a filter that is one `attr OP const` compare (the configs' `price > 20`): no interpreter, no LDS
// register file -- the constant already converted to the compare type, the column value converted on load
struct WaAtom {
  int32_t attr = -1, w = 4, cvt_from = -1, cvt_to = -1, op = 0, t = 0;
  int64_t c = 0;
  bool never = false;   // a compare with a null constant: no event passes
};

__global__ void __launch_bounds__(256) k_wa_filter_atom(int64_t lo, int64_t n, const uint8_t* __restrict__ col,
                                                         WaAtom at, uint8_t* __restrict__ flags,
                                                         uint32_t* __restrict__ tcnt) {
  __shared__ uint32_t bc;
  if (threadIdx.x == 0) bc = 0;
  __syncthreads();
  const int64_t t0 = lo + (int64_t)blockIdx.x * WA_FT;
  uint32_t c = 0;
  for (int k = threadIdx.x; k < WA_FT; k += 256) {
    const int64_t e = t0 + k;
    if (e >= n) break;
    int64_t v = at.w == 8 ? ((const int64_t*)col)[e] : (int64_t)((const int32_t*)col)[e];
    if (at.cvt_to >= 0) v = cvt(v, at.cvt_from, at.cvt_to);
    const bool f = !at.never && cmp(at.op, at.t, v, at.c);
    flags[e - lo] = (uint8_t)f;
    c += f;
  }
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(&bc, c);
  __syncthreads();
  if (threadIdx.x == 0) tcnt[blockIdx.x] = bc;
}

// the atom form of a compiled filter, if it is one: LD, CONST, at most one CVT per side, CMP, RET
static bool wa_atom_of(const Prog& p, WaAtom& at) {
  struct R { int kind = 0; int attr = -1; int64_t v = 0; bool nul = false; int cf = -1, ct = -1; };   // 1 attr, 2 const
  R r[MAX_REG];
  int cmp_reg = -1;
  WaAtom a;
  for (int pc = 0; pc < p.n; pc++) {
    const Ins& in = p.ins[pc];
    switch (in.op) {
      case BC_LD: r[in.dst] = R{1, in.imm, 0, false, -1, -1}; break;
      case BC_CONST: r[in.dst] = R{2, -1, p.consts[in.imm], in.b != 0, -1, -1}; break;
      case BC_CVT: {
        R x = r[in.a];
        const int from = (in.imm >> 4) & 15, to = in.imm & 15;
        if (x.kind == 2) { if (!x.nul) x.v = cvt(x.v, from, to); }
        else if (x.kind == 1 && x.ct < 0) { x.cf = from; x.ct = to; }
        else return false;
        r[in.dst] = x;
        break;
      }
      case BC_CMP: {
        const R &x = r[in.a], &y = r[in.b];
        int op = (in.imm >> 4) & 15;
        const R *attr, *cst;
        if (x.kind == 1 && y.kind == 2) { attr = &x; cst = &y; }
        else if (x.kind == 2 && y.kind == 1) {
          attr = &y; cst = &x;
          op = op == C_GT ? C_LT : op == C_LT ? C_GT : op == C_GE ? C_LE : op == C_LE ? C_GE : op;
        } else return false;
        if (cmp_reg >= 0) return false;
        a.attr = attr->attr; a.cvt_from = attr->cf; a.cvt_to = attr->ct;
        a.op = op; a.t = in.imm & 15; a.c = cst->v; a.never = cst->nul;
        cmp_reg = in.dst;
        r[in.dst] = R{3};
        break;
      }
      case BC_RET:
        if (in.a != cmp_reg || pc != p.n - 1) return false;
        at = a;
        return true;
      default:
        return false;
    }
  }
  return false;
}

__global__ void __launch_bounds__(256) k_wa_place(int64_t lo, int64_t nn, const uint8_t* __restrict__ flags,
                                                   const uint32_t* __restrict__ toff, const uint32_t* __restrict__ tcnt,
                                                   int64_t ntile, int32_t* __restrict__ out, int32_t* __restrict__ total) {
  __shared__ uint32_t wsum[4];
  const int64_t r0 = (int64_t)blockIdx.x * WA_FT + (int64_t)threadIdx.x * 16;   // 16 flags per thread
  uint8_t f[16];
  if (r0 + 16 <= nn) {
    const uint4 v = *(const uint4*)(flags + r0);
    __builtin_memcpy(f, &v, 16);
  } else {
    for (int k = 0; k < 16; k++) f[k] = r0 + k < nn ? flags[r0 + k] : 0;
  }
  uint32_t c = 0;
  for (int k = 0; k < 16; k++) c += f[k];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t inc = sg_wave_scan(c);
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t base = toff[blockIdx.x] + inc - c;
  for (int k = 0; k < w; k++) base += wsum[k];
  for (int k = 0; k < 16; k++)
    if (f[k]) out[base++] = (int32_t)(lo + r0 + k);
  if (blockIdx.x == ntile - 1 && threadIdx.x == 0) *total = (int32_t)(toff[ntile - 1] + tcnt[ntile - 1]);
}

// value column description for the gather
struct WaVal {
  int32_t col, t;      // source attribute and type
};

struct WaGatherArgs {
  const int32_t* fidx;     // filtered -> event index
  int64_t f0, nf;          // filtered positions [f0, f0+nf) (new)
  WaCols cols;
  int32_t gcol, gw;        // group-by attribute (-1: none)
  int32_t nv;
  WaVal v[WA_MAXV];
  int32_t* fg;             // group id per filtered position
  double* fx;              // [nv][cap] value as double
  int64_t* fx_raw;         // [nv][cap] raw bits (general path: exact long sums, boxed equality)
  int64_t cap;
  int32_t* stat_shift;     // [nv] max required fixed-point shift
  unsigned long long* stat_max;   // [nv] max |x| as double bits (monotone for non-negative)
  int32_t* stat_gmax;      // max group id
  int32_t* stat_gmin;      // min group id
  const int64_t* ts;       // event timestamps
  int64_t* fts;            // filtered timestamps
};

__device__ __forceinline__ int need_shift(double x) {
  if (x == 0.0 || !isfinite(x)) return x == 0.0 ? 0 : 4096;
  int e;
  double m = frexp(x, &e);                 // x = m * 2^e, 0.5 <= |m| < 1
  uint64_t bits = (uint64_t)__double_as_longlong(ldexp(fabs(m), 53));   // integer significand
  int tz = __ffsll((long long)bits) - 1;
  int lsb = e - 53 + tz;
  return lsb < 0 ? -lsb : 0;
}

__device__ __forceinline__ int wave_max_i(int v) {
  for (int d = 32; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, 64));
  return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
  for (int d = 32; d >= 1; d >>= 1) v = min(v, __shfl_xor(v, d, 64));
  return v;
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
  for (int d = 32; d >= 1; d >>= 1) {
    unsigned long long o = __shfl_xor(v, d, 64);
    v = o > v ? o : v;
  }
  return v;
}

// Grid-stride: each lane folds its elements' statistics locally, then one wave reduction and one atomic
// per wave and statistic (a single hot address would otherwise serialise millions of atomics).
__global__ void __launch_bounds__(256) k_wa_gather(WaGatherArgs a) {
  int gmx = INT32_MIN, gmn = INT32_MAX;
  int sh[WA_MAXV] = {0, 0, 0, 0};
  unsigned long long mx[WA_MAXV] = {0, 0, 0, 0};
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < a.nf; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = a.f0 + k;
    const int64_t e = a.fidx[p];
    int32_t g = 0;
    if (a.gcol >= 0) g = a.gw == 8 ? (int32_t)((const int64_t*)a.cols.c[a.gcol])[e] : ((const int32_t*)a.cols.c[a.gcol])[e];
    a.fg[p] = g;
    a.fts[p] = a.ts[e];
    gmx = max(gmx, g);
    gmn = min(gmn, g);
    for (int v = 0; v < a.nv; v++) {
      const uint8_t* col = a.cols.c[a.v[v].col];
      double x;
      int64_t r;
      switch (a.v[v].t) {
        case T_INT: r = ((const int32_t*)col)[e]; x = (double)r; break;
        case T_LONG: r = ((const int64_t*)col)[e]; x = (double)r; break;
        case T_FLOAT: { float f = ((const float*)col)[e]; r = f_bits(f); x = (double)f; break; }
        default: x = ((const double*)col)[e]; r = d_bits(x); break;
      }
      a.fx[(int64_t)v * a.cap + p] = x;
      if (a.fx_raw) a.fx_raw[(int64_t)v * a.cap + p] = r;
      sh[v] = max(sh[v], need_shift(x));
      const unsigned long long ax = (unsigned long long)__double_as_longlong(fabs(x));
      mx[v] = ax > mx[v] ? ax : mx[v];
    }
  }
  // one atomic per workgroup and statistic: device-scope atomics on one address serialise in L2, so
  // per-wave atomics over a 100M-event flush cost milliseconds
  __shared__ int s_i[2 + WA_MAXV][4];
  __shared__ unsigned long long s_m[WA_MAXV][4];
  const int w = threadIdx.x >> 6;
  const bool leader = (threadIdx.x & 63) == 0;
  gmx = wave_max_i(gmx);
  gmn = wave_min_i(gmn);
  if (leader) { s_i[0][w] = gmx; s_i[1][w] = gmn; }
  for (int v = 0; v < a.nv; v++) {
    const int s2 = wave_max_i(sh[v]);
    const unsigned long long m2 = wave_max_u64(mx[v]);
    if (leader) { s_i[2 + v][w] = s2; s_m[v][w] = m2; }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int bmx = s_i[0][0], bmn = s_i[1][0];
    for (int k = 1; k < 4; k++) { bmx = max(bmx, s_i[0][k]); bmn = min(bmn, s_i[1][k]); }
    atomicMax(a.stat_gmax, bmx);
    atomicMin(a.stat_gmin, bmn);
    for (int v = 0; v < a.nv; v++) {
      int s2 = s_i[2 + v][0];
      unsigned long long m2 = s_m[v][0];
      for (int k = 1; k < 4; k++) { s2 = max(s2, s_i[2 + v][k]); m2 = s_m[v][k] > m2 ? s_m[v][k] : m2; }
      atomicMax(&a.stat_shift[v], s2);
      atomicMax(&a.stat_max[v], m2);
    }
  }
}

enum WinK { W_LENGTH = 0, W_TIME = 1, W_LENGTH_BATCH = 2 };

struct WaWsArgs {
  int32_t kind;
  int64_t param;           // L or T
  int64_t f0, F;           // new filtered positions [f0, F)
  const int32_t* fidx;
  const int64_t* fts;
  const int64_t* now;      // per-event app clock (host ingest); nullptr: now = now_const or the event's ts
  int64_t now_const;       // >= 0: one clock for the whole (device-resident) batch
  int32_t* ws;
  int32_t* maxwin;
};

__global__ void __launch_bounds__(256) k_wa_wstart(WaWsArgs a) {
  int mw = 0;
  for (int64_t p = a.f0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < a.F;
       p += (int64_t)gridDim.x * blockDim.x) {
    int64_t w0;
    if (a.kind == W_LENGTH) {
      w0 = max<int64_t>(0, p - a.param + 1);
    } else {
      const int64_t e = a.fidx[p];
      const int64_t now = a.now ? a.now[e] : (a.now_const >= 0 ? a.now_const : a.fts[p]);
      const int64_t lim = now - a.param;      // expired iff ts <= lim
      int64_t lo = 0, hi = p;                  // first q in [0, p] with fts[q] > lim (p itself stays)
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a.fts[mid] > lim) hi = mid; else lo = mid + 1;
      }
      w0 = lo;
    }
    a.ws[p] = (int32_t)w0;
    mw = max(mw, (int)(p - w0 + 1));
  }
  // one atomic per workgroup (a grid-stride grid of at most a few thousand workgroups)
  __shared__ int s_mw[4];
  mw = wave_max_i(mw);
  if ((threadIdx.x & 63) == 0) s_mw[threadIdx.x >> 6] = mw;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int b = max(max(s_mw[0], s_mw[1]), max(s_mw[2], s_mw[3]));
    if (b > 0) atomicMax(a.maxwin, b);
  }
}

struct WaTileArgs {
  const int32_t* fg;
  const double* fx;
  int64_t cap;
  int32_t nv;
  int32_t shift[WA_MAXV];
  int64_t f0, F;           // outputs for [f0, F); history available from 0
  const int32_t* ws;       // window start of every filtered event
  int32_t T, L, K;         // L: the widest window (LDS halo = L - 1)
  int32_t gmin;
  double* out_sum;         // [nv][cap]
  int64_t* out_cnt;        // [cap]
};

__global__ void __launch_bounds__(WA_B) k_wa_tile(WaTileArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int T = a.T, L = a.L, K = a.K;
  const int64_t p0 = a.f0 + (int64_t)blockIdx.x * T;
  const int64_t p1 = min(p0 + (int64_t)T, a.F);
  const int64_t r0 = a.ws[p0];                   // window starts are non-decreasing
  const int nr = (int)(p1 - r0);
  const int R = T + L;
  int32_t* s_g = (int32_t*)smem;                 // R
  int32_t* s_b = s_g + R;                        // R bucket (region indices)
  int32_t* s_off = s_b + R;                      // K + 1
  int32_t* s_fill = s_off + K + 1;               // K
  int32_t* s_misc = s_fill + K;                  // 16
  int64_t* s_v = (int64_t*)(((uintptr_t)(s_misc + 16) + 15) & ~(uintptr_t)15);   // nv * R fixed point
  const int tid = threadIdx.x;
  for (int k = tid; k < K + 1; k += WA_B) s_off[k] = 0;
  __syncthreads();
  for (int q = tid; q < nr; q += WA_B) {
    int g = a.fg[r0 + q] - a.gmin;
    s_g[q] = g;
    atomicAdd(&s_off[g], 1);
    for (int v = 0; v < a.nv; v++) s_v[v * R + q] = (int64_t)llrint(ldexp(a.fx[(int64_t)v * a.cap + r0 + q], a.shift[v]));
  }
  __syncthreads();
  // exclusive scan of the group histogram (K small: one wave does it)
  if (tid < 64) {
    const int per = (K + 63) / 64;
    const int beg = tid * per, end = min(K, beg + per);
    int s = 0;
    for (int k = beg; k < end; k++) s += s_off[k];
    const int incl = (int)sg_wave_scan((uint32_t)s);
    int run = incl - s;
    for (int k = beg; k < end; k++) { int c = s_off[k]; s_off[k] = run; s_fill[k] = run; run += c; }
    if (tid == 63) s_off[K] = incl;
  }
  __syncthreads();
  for (int q = tid; q < nr; q += WA_B) {
    int pos = atomicAdd(&s_fill[s_g[q]], 1);
    s_b[pos] = q;
  }
  __syncthreads();
  // one lane per group: order its bucket by position, then windowed sums by two pointers
  for (int g = tid; g < K; g += WA_B) {
    const int beg = s_off[g], end = s_off[g + 1];
    for (int p = beg + 1; p < end; p++) {
      int v = s_b[p], q = p - 1;
      while (q >= beg && s_b[q] > v) { s_b[q + 1] = s_b[q]; q--; }
      s_b[q + 1] = v;
    }
    int lo = beg;
    int64_t acc[WA_MAXV] = {0, 0, 0, 0};
    for (int p = beg; p < end; p++) {
      const int q = s_b[p];
      for (int v = 0; v < a.nv; v++) acc[v] += s_v[v * R + q];
      const int64_t wq = a.ws[r0 + q];
      while (r0 + s_b[lo] < wq) {               // expired by the time q is added
        for (int v = 0; v < a.nv; v++) acc[v] -= s_v[v * R + s_b[lo]];
        lo++;
      }
      const int64_t gp = r0 + q;
      if (gp >= p0) {
        for (int v = 0; v < a.nv; v++) a.out_sum[(int64_t)v * a.cap + gp] = ldexp((double)acc[v], -a.shift[v]);
        a.out_cnt[gp] = p - lo + 1;
      }
    }
  }
}

// ---- general path: one lane per group replays the reference's aggregator state machine ----
struct WaAgg {
  int32_t k, v;            // kind, value column (-1 count())
  int32_t t;               // input type
};

// one group's aggregator state, carried across flushes (a persistent slot per group value)
struct WaSt {
  double dsum;
  int64_t lsum, cnt, mv;
  int32_t mvset, dh, dn, pad;
};

struct WaSeqArgs {
  const int32_t* g_off;    // CSR over groups: filtered positions of each group, ascending
  const int32_t* g_pos;
  const int32_t* g_slot;   // state slot of each CSR group
  int32_t ngroups;
  const double* fx;
  const int64_t* fx_raw;   // raw input bits for min/max identity (Float/Double.equals)
  int64_t cap;
  const int32_t* ws;       // window start per filtered event (sliding windows)
  int32_t batchL;          // lengthBatch(L): reset at every batch-first event of the group, no expiry
  int32_t na;
  WaAgg agg[WA_MAXA];
  int64_t* out_raw;        // [na][cap] raw output bits
  uint8_t* out_nul;        // [na][cap]
  WaSt* st;                // [slot][na] carried states
  int64_t* dq;             // deque ring per (slot, aggregator): dq_cap entries (raw bits)
  int32_t dq_cap;
  int32_t* err;
  int32_t destroy;         // group-by: drained states are destroyed and re-created
  int64_t f0;              // positions < f0 were added by earlier flushes (in the carried state)
  int32_t old_add;         // 1: the carried state is stale (an exact-path flush ran): add them again
  int64_t ws_end;          // removals of positions < ws_end are drained before the state is saved
  int64_t save_at;         // lengthBatch: the state saved is the one before this position (the batch
                           // still being filled is replayed by the next flush); sliding: INT64_MAX
};

__device__ __forceinline__ bool lt_raw(int t, int64_t a, int64_t b) {
  switch (t) {
    case T_INT: return (int32_t)a < (int32_t)b;
    case T_LONG: return a < b;
    case T_FLOAT: return bits_f(a) < bits_f(b);
    default: return bits_d(a) < bits_d(b);
  }
}

__device__ __forceinline__ bool eq_boxed(int t, int64_t a, int64_t b) {
  if (t == T_FLOAT) { float x = bits_f(a), y = bits_f(b); if (x != x && y != y) return true; return (uint32_t)a == (uint32_t)b; }
  if (t == T_DOUBLE) { double x = bits_d(a), y = bits_d(b); if (x != x && y != y) return true; return a == b; }
  return a == b;
}

// One lane per group: resumes the group's carried state, replays its removals (events leaving the
// window, in position order, before the group's next add -- the order the global window emits them)
// and adds, then drains the removals the window has made by the flush's last event and saves the state.
// Positions below f0 are already inside the state and only ever expire (old_add: after an exact-path
// flush the state is rebuilt by adding them again; the exact path only runs while every sum is exact,
// so the rebuilt sums equal the reference's).
__global__ void __launch_bounds__(64) k_wa_seq(WaSeqArgs a) {
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= a.ngroups) return;
  const int beg = a.g_off[g], end = a.g_off[g + 1];
  const int64_t slot = a.g_slot[g];
  WaSt* S = a.st + slot * a.na;
  double dsum[WA_MAXA];
  int64_t lsum[WA_MAXA], cnt[WA_MAXA], mv[WA_MAXA];
  int mvnull[WA_MAXA], dh[WA_MAXA], dn[WA_MAXA];
  for (int k = 0; k < a.na; k++) {
    dsum[k] = S[k].dsum; lsum[k] = S[k].lsum; cnt[k] = S[k].cnt; mv[k] = S[k].mv;
    mvnull[k] = !S[k].mvset; dh[k] = S[k].dh; dn[k] = S[k].dn;
  }
  auto remove = [&](int q) {
    for (int k = 0; k < a.na; k++) {
      const WaAgg& A = a.agg[k];
      if (A.k == A_COUNT) { cnt[k]--; continue; }
      const double x = a.fx[(int64_t)A.v * a.cap + q];
      const int64_t xr = a.fx_raw[(int64_t)A.v * a.cap + q];
      if (A.k == A_SUM) {
        if (A.t == T_INT || A.t == T_LONG) {
          double r = (double)lsum[k] - (double)xr;
          lsum[k] = (r != r) ? 0 : (r >= 9.2233720368547758e18 ? INT64_MAX : (r <= -9.2233720368547758e18 ? INT64_MIN : (int64_t)r));
        } else {
          dsum[k] -= x;
        }
        cnt[k]--;
        // PartitionStateHolder destroys a drained group state (canDestroy): -0.0 -> +0.0
        if (a.destroy && cnt[k] == 0 && dsum[k] == 0.0) dsum[k] = 0.0;
      } else if (A.k == A_AVG) {
        cnt[k]--; dsum[k] -= x;
        if (a.destroy && cnt[k] == 0 && dsum[k] == 0.0) dsum[k] = 0.0;
      } else {   // min / max with trackFutureStates deque: removeFirstOccurrence(value)
        int64_t* d = a.dq + (slot * a.na + k) * a.dq_cap;
        for (int i = 0; i < dn[k]; i++) {
          int idx = (dh[k] + i) % a.dq_cap;
          if (eq_boxed(A.t, d[idx], xr)) {
            for (int j = i; j > 0; j--) d[(dh[k] + j) % a.dq_cap] = d[(dh[k] + j - 1) % a.dq_cap];
            dh[k] = (dh[k] + 1) % a.dq_cap;
            dn[k]--;
            break;
          }
        }
        if (dn[k] == 0) mvnull[k] = 1; else { mvnull[k] = 0; mv[k] = d[dh[k]]; }
      }
    }
  };
  auto save = [&]() {
    for (int k = 0; k < a.na; k++) {
      S[k].dsum = dsum[k]; S[k].lsum = lsum[k]; S[k].cnt = cnt[k]; S[k].mv = mv[k];
      S[k].mvset = !mvnull[k]; S[k].dh = dh[k]; S[k].dn = dn[k];
    }
  };
  bool saved = false;
  int lo = beg;   // next event of this group to expire
  for (int p = beg; p < end; p++) {
    const int pos = a.g_pos[p];
    if (!saved && pos >= a.save_at) { save(); saved = true; }
    const bool old = pos < a.f0;
    if (old && !a.old_add) continue;   // inside the carried state: it only expires
    if (a.batchL > 0 && pos % a.batchL == 0) {
      // the batch's RESET event (a copy of its first event) resets this group's aggregators
      for (int k = 0; k < a.na; k++) { dsum[k] = 0; lsum[k] = 0; cnt[k] = 0; mvnull[k] = 1; dh[k] = 0; dn[k] = 0; }
    }
    // removals of this group's events that expire before `pos` is added (window over filtered stream)
    while (a.batchL == 0 && lo < p && a.g_pos[lo] < a.ws[pos]) remove(a.g_pos[lo++]);
    // add
    for (int k = 0; k < a.na; k++) {
      const WaAgg& A = a.agg[k];
      int64_t outv = 0;
      int outn = 0;
      if (A.k == A_COUNT) {
        cnt[k]++;
        outv = cnt[k];
      } else {
        const double x = a.fx[(int64_t)A.v * a.cap + pos];
        const int64_t xr = a.fx_raw[(int64_t)A.v * a.cap + pos];
        if (A.k == A_SUM) {
          if (A.t == T_INT || A.t == T_LONG) { lsum[k] = (int64_t)((uint64_t)lsum[k] + (uint64_t)xr); outv = lsum[k]; }
          else { dsum[k] += x; outv = d_bits(dsum[k]); }
          cnt[k]++;
        } else if (A.k == A_AVG) {
          cnt[k]++; dsum[k] += x;
          outv = d_bits(dsum[k] / (double)cnt[k]);
        } else {
          const bool isMin = A.k == A_MIN;
          int64_t* d = a.dq + (slot * a.na + k) * a.dq_cap;
          while (a.batchL == 0 && dn[k] > 0) {
            int64_t back = d[(dh[k] + dn[k] - 1) % a.dq_cap];
            bool drop = isMin ? lt_raw(A.t, xr, back) : lt_raw(A.t, back, xr);
            if (drop) dn[k]--; else break;
          }
          if (a.batchL == 0) {   // trackFutureStates (sliding windows): the expiry deque
            if (dn[k] >= a.dq_cap) { atomicOr(a.err, 1); return; }
            d[(dh[k] + dn[k]) % a.dq_cap] = xr;
            dn[k]++;
          }
          if (mvnull[k] || (isMin ? lt_raw(A.t, xr, mv[k]) : lt_raw(A.t, mv[k], xr))) { mv[k] = xr; mvnull[k] = 0; }
          outv = mv[k];
        }
      }
      if (!old) {
        a.out_raw[(int64_t)k * a.cap + pos] = outv;
        a.out_nul[(int64_t)k * a.cap + pos] = (uint8_t)outn;
      }
    }
  }
  while (a.batchL == 0 && lo < end && a.g_pos[lo] < a.ws_end) remove(a.g_pos[lo++]);
  if (!saved) save();
}

// re-layout of the deque rings (more slots or a wider window): ring r linearised into the new capacity
__global__ void __launch_bounds__(256) k_wa_dq_grow(const int64_t* __restrict__ od, int32_t ocap, int64_t* __restrict__ nd,
                                                    int32_t ncap, WaSt* st, int64_t nrings) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= nrings) return;
  WaSt& S = st[r];
  for (int i = 0; i < S.dn; i++) nd[r * ncap + i] = od[r * ocap + (S.dh + i) % ocap];
  S.dh = 0;
}

// v -= d for n int32 values (positions / event indices of a compacted buffer)
// projected attribute of each materialised output row: column value at its event, widened to the
// 8-byte raw form (FLOAT bits zero-extended, INT/STRING-id sign-extended)
__global__ void __launch_bounds__(256) k_wa_proj(const uint8_t* __restrict__ col, int w, int is_float,
                                                 const int32_t* __restrict__ idx, int64_t nm, int64_t* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nm) return;
  const int64_t e = idx[p];
  if (w == 8) out[p] = ((const int64_t*)col)[e];
  else {
    const int32_t x = ((const int32_t*)col)[e];
    out[p] = is_float ? (int64_t)(uint32_t)x : (int64_t)x;
  }
}

// device-resident chain (DevChain): the materialised rows of a per-event window query as the inserted stream's
// columns -- timestamp, app clock of the row's send, and every output attribute in the stream's width (a projected
// attribute from the event's column, an aggregate from the device-formed outputs `agg`) -- for NFA consumers
constexpr int WA_MAXO = 8;
struct WaChainArgs {
  const int32_t* fidx; int64_t m0, nm;
  const int64_t* ts; const int64_t* now;
  int32_t no;
  int32_t kind[WA_MAXO], w_in[WA_MAXO], w_out[WA_MAXO], agg[WA_MAXO];
  const uint8_t* col[WA_MAXO];
  const int64_t* aggv;
  int64_t* out_ts; int64_t* out_now;
  uint8_t* out[WA_MAXO];
};
__global__ void __launch_bounds__(256) k_wa_chain_pack(WaChainArgs a) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.nm) return;
  const int64_t e = a.fidx[a.m0 + p];
  a.out_ts[p] = a.ts[e];
  a.out_now[p] = a.now[e];
  for (int o = 0; o < a.no; o++) {
    int64_t v;
    if (a.kind[o] == 0) v = a.w_in[o] == 8 ? ((const int64_t*)a.col[o])[e] : (int64_t)((const int32_t*)a.col[o])[e];
    else v = a.aggv[(int64_t)a.agg[o] * a.nm + p];
    if (a.w_out[o] == 8) ((int64_t*)a.out[o])[p] = v;
    else ((int32_t*)a.out[o])[p] = (int32_t)v;
  }
}

// exact path: aggregator outputs of the materialised rows from the tile sums and counts (sum: the
// integer or double result; avg: sum / count; count), in their raw 8-byte form
struct WaAggOut { WaAgg agg[WA_MAXA]; int32_t na; };
__global__ void __launch_bounds__(256) k_wa_aggout(WaAggOut ao, const double* __restrict__ sum,
                                                   const int64_t* __restrict__ cnt, int64_t cap, int64_t m0,
                                                   int64_t nm, int64_t* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nm) return;
  for (int k = 0; k < ao.na; k++) {
    const WaAgg A = ao.agg[k];
    int64_t v;
    if (A.k == A_COUNT) v = cnt[m0 + p];
    else {
      const double sv = sum[(int64_t)A.v * cap + m0 + p];
      if (A.k == A_SUM) v = (A.t == T_INT || A.t == T_LONG) ? (int64_t)sv : d_bits(sv);
      else v = d_bits(sv / (double)cnt[m0 + p]);
    }
    out[(int64_t)k * nm + p] = v;
  }
}

__global__ void __launch_bounds__(256) k_wa_rebase(int32_t* v, int64_t n, int32_t d) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k < n) v[k] -= d;
}

// ------------------------------------------------------------------------------------------------
struct WindowAggExec : Exec {
  int st = -1;
  int wkind = W_LENGTH;
  int64_t L = 0;            // length / lengthBatch count, or time span (ms)
  DBuf<int64_t> fts, d_now;
  DBuf<int32_t> wsb, maxwin;
  const int64_t* ext_ts = nullptr;
  int64_t ext_now = -1;     // device ingest: one clock for a batch chunk (-1: each event's own ts)
  int64_t emitted_batches = 0;
  Prog filter;
  bool has_filter = false;
  int gcol = -1;            // group-by attribute
  Ty gty = T_INT;
  struct Out { int kind; int col; int agg; };   // kind 0 = attribute, 1 = aggregator
  std::vector<Out> outs;
  std::vector<WaAgg> aggs;
  std::vector<int> vcols;   // distinct aggregated value columns
  std::vector<Ty> vtys;
  bool fast_ok = false;     // all aggregators sum/avg/count
  int tileT = 2048;
  // buffers
  int64_t n = 0, done = 0;
  DBuf<int64_t> ts;
  std::vector<DCol> cols;
  hvec<int64_t> h_seq, h_chunk, h_ts;
  int64_t chunk_ctr = 0;
  DBuf<uint8_t> flags, sel_tmp;
  DBuf<uint32_t> tcnt, toff;   // filter tiles: pass counts -> bases
  DBuf<int32_t> fidx, fg, gsum_off, gsum_pos, gsum_slot, stat_i, dsel_n;
  DBuf<double> fx, out_sum;
  DBuf<int64_t> fx_raw, out_cnt, out_raw, dq, proj;
  std::vector<int32_t> m_hidx, m_hg;
  std::vector<int64_t> m_araw;
  std::vector<uint8_t> m_anul;
  DBuf<uint8_t> out_nul;
  DBuf<unsigned long long> stat_m;
  DBuf<Prog> d_filter;
  DBuf<int32_t> idx_tmp, err;
  int64_t F = 0;            // filtered events held (positions [0, F))
  // general path: one carried aggregator state per group value (slot), deque rings [slot][agg][dq_ring]
  std::unordered_map<int32_t, int32_t> gslot;
  DBuf<WaSt> wst;
  int32_t dq_ring = 0;      // ring capacity of dq
  int64_t dq_slots = 0;     // slots dq is laid out for
  bool state_valid = true;  // wst holds every group's state after position F (false after an exact flush)
  bool inexact_seen = false;   // some flush could round: the exact path is off for good
  DBuf<uint8_t> cmp_tmp;
  DBuf<uint32_t> ts_bad;
  // statistics over the whole filtered history (the window halo reaches back into it)
  int gmin_hist = INT32_MAX, gmax_hist = INT32_MIN;
  int shift_hist[WA_MAXV] = {0, 0, 0, 0};
  double maxabs_hist[WA_MAXV] = {0, 0, 0, 0};
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipEvent_t tev[3] = {};

  ~WindowAggExec() override {
    for (auto& e : tev) if (e) (void)hipEventDestroy(e);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
  }

  WaCols wcols() const {
    WaCols c;
    std::memset(&c, 0, sizeof(c));
    for (size_t k = 0; k < cols.size(); k++) {
      c.c[k] = ext ? (const uint8_t*)ext_cols[k] : cols[k].b.p;
      c.w[k] = cols[k].w;
    }
    return c;
  }

  bool takes_device_batch() const override { return true; }
  void push(const HostBatch& b) override {
    if (b.stream != st) return;
    if (ext) throw Error(-2, "cannot append host events after device-resident ingest");
    if (b.batch && b.n > 1) pending_single = false;
    hipStream_t s = app->stream;
    ts.reserve(n + b.n, true, s, n);
    for (auto& c : cols) c.b.reserve((n + b.n) * c.w, true, s, n * c.w);
    // (a batch staged in HBM: device to device)
    const hipMemcpyKind kts = b.d_ts ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    SG_HIP(hipMemcpyAsync(ts.p + n, b.d_ts ? b.d_ts : b.ts.data(), b.n * 8, kts, s));
    if (wkind == W_TIME) {
      d_now.reserve(n + b.n, true, s, n);
      SG_HIP(hipMemcpyAsync(d_now.p + n, b.d_now ? b.d_now : b.now_ev.data(), b.n * 8,
                            b.d_now ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
    }
    for (size_t k = 0; k < cols.size(); k++) {
      const bool dv = k < b.d_cols.size() && b.d_cols[k];
      SG_HIP(hipMemcpyAsync(cols[k].b.p + n * cols[k].w, dv ? (const void*)b.d_cols[k] : (const void*)b.cols[k].data(),
                            b.n * cols[k].w, dv ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
    }
    const size_t h0 = h_seq.size();
    h_seq.resize(h0 + b.n);
    h_ts.resize(h0 + b.n);
    h_chunk.resize(h0 + b.n);
    const int nth = host_threads(b.n);            // (the host columns over thread ranges while the copies run)
    host_parallel(nth, [&](int t) {
      const int64_t a0 = b.n * t / nth, a1 = b.n * (t + 1) / nth;
      if (b.seqs.empty()) for (int64_t k = a0; k < a1; k++) h_seq[h0 + k] = b.seq0 + k;
      else std::memcpy(h_seq.data() + h0 + a0, b.seqs.data() + a0, (size_t)(a1 - a0) * 8);
      std::memcpy(h_ts.data() + h0 + a0, b.ts.data() + a0, (size_t)(a1 - a0) * 8);
      for (int64_t k = a0; k < a1; k++) h_chunk[h0 + k] = b.batch ? chunk_ctr : chunk_ctr + k;
    });
    SG_HIP(hipStreamSynchronize(s));
    chunk_ctr += b.batch ? 1 : b.n;
    n += b.n;
  }

  // device-resident ingest (bench / zero-copy): columns adopted, outputs stay in HBM (sg_flush_device)
  bool ext = false;
  std::vector<const void*> ext_cols;
  void push_device(int stream, int64_t cnt_, const int64_t* dts, const void* const* dcols, int batch,
                   hipStream_t s) override {
    if (stream != st) return;
    if (n != 0 || ext) throw Error(-2, "device ingest adopts one resident batch per runtime (sg_reset first)");
    ext = true;
    ext_cols.assign(dcols, dcols + cols.size());
    ext_ts = dts;
    n = cnt_;
    // the clock of a device-resident chunk (playback semantics): its last timestamp for one send(Event[]),
    // each event's own timestamp for per-event sends
    ext_now = -1;
    if (batch && cnt_ > 0 && wkind == W_TIME) {
      SG_HIP(hipMemcpyAsync(&ext_now, dts + cnt_ - 1, 8, hipMemcpyDeviceToHost, s));
      SG_HIP(hipStreamSynchronize(s));
    }
    if (wkind == W_LENGTH_BATCH && !batch)
      throw Error(-2, "device-resident lengthBatch ingest takes one chunk (batch=1)");
  }

  void reset() override {
    ext = false; ext_cols.clear(); ext_ts = nullptr; ext_now = -1; emitted_batches = 0; pending_single = true;
    n = done = F = 0; chunk_ctr = 0;
    h_seq.clear(); h_chunk.clear(); h_ts.clear();
    gslot.clear(); dq_slots = 0; dq_ring = 0; state_valid = true; inexact_seen = false;
    gmin_hist = INT32_MAX; gmax_hist = INT32_MIN;
    for (int v = 0; v < WA_MAXV; v++) { shift_hist[v] = 0; maxabs_hist[v] = 0; }
  }

  void flush(std::vector<Callback>& out, bool materialise, hipStream_t s) override {
    flush_run(out, materialise, s);
    compact(s);
    pending_single = true;
  }
  void flush_run(std::vector<Callback>& out, bool materialise, hipStream_t s);
  int64_t buffered() const override { return n; }
  void compact(hipStream_t s);
  void ensure_states(int64_t nslots, int32_t ring, hipStream_t s);
  DevChain* dev_req = nullptr;                     // the next export may stay in HBM (api.hip dispatch)
  bool pending_single = true;                      // every event since the last flush came in a one-event send
  DBuf<int64_t> dx_ts, dx_now;
  DBuf<uint8_t> dx_col[WA_MAXO];
  PinBuf<int32_t> px_hidx;
  PinBuf<uint8_t> px_key;
  hvec<int64_t> dx_seq;
  void set_chain_request(DevChain* dc) override { dev_req = dc; }
  bool flush_export(ChainOut& co, hipStream_t s) override {
    std::vector<Callback> none;
    export_to = &co;
    flush(none, true, s);
    export_to = nullptr;
    return true;
  }
  ChainOut* export_to = nullptr;

  // sg_snapshot / sg_restore after the flush sg_snapshot runs: the window's retained events (the
  // LengthWindowProcessor / LengthBatchWindowProcessor / TimeWindowProcessor queues, e.g.
  // LengthWindowProcessor.java:106-141 state "expiredEventQueue"), the filtered positions the next
  // windows reach back to, and the carried group states (the AttributeAggregatorExecutor states per
  // group-by key of QuerySelector, with the min/max expiry deques).
  bool can_snapshot() const override { return true; }
  void snapshot(SnapWriter& w, hipStream_t s) override {
    if (ext) throw Error(-2, "snapshot after device-resident ingest is not supported (the input is the caller's)");
    if (done != n) throw Error(-5, "window snapshot needs a flushed buffer");
    const int na = std::max<int>((int)aggs.size(), 1);
    const size_t nv = std::max<size_t>(vcols.size(), 1);
    w.pod(n); w.pod(F); w.pod(chunk_ctr); w.pod(emitted_batches);
    w.pod(dq_ring); w.pod(dq_slots); w.pod(state_valid); w.pod(inexact_seen);
    w.pod(gmin_hist); w.pod(gmax_hist);
    for (int v = 0; v < WA_MAXV; v++) { w.pod(shift_hist[v]); w.pod(maxabs_hist[v]); }
    w.dev(ts, (size_t)n, s);
    if (wkind == W_TIME) w.dev(d_now, (size_t)n, s);
    for (auto& c : cols) w.dev(c.b, (size_t)(n * c.w), s);
    w.vec(h_seq); w.vec(h_ts); w.vec(h_chunk);
    w.dev(fidx, (size_t)F, s); w.dev(fg, (size_t)F, s); w.dev(fts, (size_t)F, s); w.dev(wsb, (size_t)F, s);
    const int64_t vcap = F ? (int64_t)(fx.cap / nv) : 0;
    for (size_t v = 0; v < vcols.size(); v++) {
      w.devp(fx.p + v * vcap, (size_t)F, s);
      w.devp(fx_raw.p + v * vcap, (size_t)F, s);
    }
    std::vector<std::pair<int32_t, int32_t>> gs(gslot.begin(), gslot.end());
    w.vec(gs);
    w.dev(wst, (size_t)(dq_slots * na), s);
    w.dev(dq, (size_t)(dq_slots * na * dq_ring), s);
  }
  void restore(SnapReader& r, hipStream_t s) override {
    reset();
    const int na = std::max<int>((int)aggs.size(), 1);
    const size_t nv = std::max<size_t>(vcols.size(), 1);
    const int64_t nn = r.pod<int64_t>(), ff = r.pod<int64_t>();
    chunk_ctr = r.pod<int64_t>(); emitted_batches = r.pod<int64_t>();
    dq_ring = r.pod<int32_t>(); dq_slots = r.pod<int64_t>();
    state_valid = r.pod<bool>(); inexact_seen = r.pod<bool>();
    gmin_hist = r.pod<int>(); gmax_hist = r.pod<int>();
    for (int v = 0; v < WA_MAXV; v++) { shift_hist[v] = r.pod<int>(); maxabs_hist[v] = r.pod<double>(); }
    if (nn < 0 || ff < 0 || ff > nn || nn >= (int64_t)INT32_MAX || dq_ring < 0 || dq_slots < 0)
      throw Error(-1, "snapshot counts out of range");
    auto want = [](size_t got, int64_t need, const char* what) {
      if ((int64_t)got != need) throw Error(-1, std::string("snapshot ") + what + " size does not match its count");
    };
    want(r.dev(ts, s), nn, "event timestamps");
    if (wkind == W_TIME) want(r.dev(d_now, s), nn, "event clocks");
    for (auto& c : cols) want(r.dev(c.b, s), nn * c.w, "column");
    r.vec(h_seq); r.vec(h_ts); r.vec(h_chunk);
    if ((int64_t)h_seq.size() != nn || (int64_t)h_ts.size() != nn || (int64_t)h_chunk.size() != nn)
      throw Error(-1, "snapshot host columns do not match the events");
    want(r.dev(fidx, s), ff, "filtered positions"); want(r.dev(fg, s), ff, "group ids");
    want(r.dev(fts, s), ff, "filtered timestamps"); want(r.dev(wsb, s), ff, "window starts");
    // value columns [v][pitch], pitch = cap / nv as the flush lays them out
    const int64_t ncap = std::max<int64_t>(ff * 2, 1024);
    fx.reserve(nv * (size_t)ncap, false);
    fx_raw.reserve(nv * (size_t)ncap, false);
    const int64_t vcap = (int64_t)(fx.cap / nv);
    if ((int64_t)(fx_raw.cap / nv) != vcap) throw Error(-1, "snapshot value column layout");
    for (size_t v = 0; v < vcols.size(); v++) {
      want(r.devp(fx.p + v * vcap, (size_t)vcap, s), ff, "window values");
      want(r.devp(fx_raw.p + v * vcap, (size_t)vcap, s), ff, "window raw values");
    }
    fg.reserve((size_t)ncap, true, s, (size_t)ff);
    fts.reserve((size_t)ncap, true, s, (size_t)ff);
    wsb.reserve((size_t)ncap, true, s, (size_t)ff);
    std::vector<std::pair<int32_t, int32_t>> gs;
    r.vec(gs);
    gslot = std::unordered_map<int32_t, int32_t>(gs.begin(), gs.end());
    for (auto& g : gs)
      if (g.second < 0 || g.second >= dq_slots) throw Error(-1, "snapshot group slot out of range");
    want(r.dev(wst, s), dq_slots * na, "group states");
    want(r.dev(dq, s), dq_slots * na * dq_ring, "expiry deques");
    n = done = nn; F = ff;
  }
};

// State slots and deque rings for `nslots` groups with rings of `ring` entries (new slots zeroed: empty
// aggregators; a re-layout keeps every ring's contents).
void WindowAggExec::ensure_states(int64_t nslots, int32_t ring, hipStream_t s) {
  const int na = std::max<int>((int)aggs.size(), 1);
  const int64_t have = dq_slots;
  if ((int64_t)wst.cap < nslots * na) {
    wst.reserve((size_t)(nslots * na), true, s, (size_t)(have * na));
  }
  if (nslots > have) SG_HIP(hipMemsetAsync(wst.p + have * na, 0, (size_t)((nslots - have) * na) * sizeof(WaSt), s));
  ring = std::max(ring, dq_ring);
  if (nslots > have || ring > dq_ring) {
    const int64_t cap_slots = std::max<int64_t>(nslots, std::max<int64_t>(2 * have, 64));
    DBuf<int64_t> nd;
    nd.reserve((size_t)(cap_slots * na * ring));
    if (have > 0 && dq_ring > 0) {
      hipLaunchKernelGGL(k_wa_dq_grow, dim3((unsigned)((have * na + 255) / 256)), dim3(256), 0, s, dq.p, dq_ring, nd.p,
                         ring, wst.p, have * na);
      SG_HIP(hipGetLastError());
    }
    SG_HIP(hipStreamSynchronize(s));
    dq = std::move(nd);
    dq_ring = ring;
    wst.reserve((size_t)(cap_slots * na), true, s, (size_t)(nslots * na));
    dq_slots = cap_slots;
    SG_HIP(hipMemsetAsync(wst.p + nslots * na, 0, (size_t)((cap_slots - nslots) * na) * sizeof(WaSt), s));
  }
}

// Compaction (host ingest): after a flush the next one reads only the filtered positions from the last
// window start on -- the sliding windows of later events start there or later, and the carried group
// states hold everything before -- or, for lengthBatch, the batch still being filled.  Events before the
// first kept position are dropped, so memory follows the window, not the events ever pushed.
void WindowAggExec::compact(hipStream_t s) {
  if (ext || n == 0 || done != n) return;
  int64_t P0 = F;
  if (wkind == W_LENGTH_BATCH) {
    P0 = emitted_batches * L;
  } else if (F > 0) {
    int32_t w = 0;
    SG_HIP(hipMemcpyAsync(&w, wsb.p + F - 1, 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    P0 = w;
  }
  int64_t E0 = n;
  if (P0 < F) {
    int32_t e = 0;
    SG_HIP(hipMemcpyAsync(&e, fidx.p + P0, 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    E0 = e;
  }
  if (P0 == 0 && E0 == 0) return;
  const int64_t kf = F - P0, ke = n - E0;
  // shift [off, off + m) of a device array to its front (through a scratch buffer: the ranges overlap)
  auto shift = [&](void* base, size_t elem, int64_t off, int64_t m) {
    if (m <= 0 || off == 0) return;
    cmp_tmp.reserve((size_t)m * elem, false);
    SG_HIP(hipMemcpyAsync(cmp_tmp.p, (uint8_t*)base + (size_t)off * elem, (size_t)m * elem, hipMemcpyDeviceToDevice, s));
    SG_HIP(hipMemcpyAsync(base, cmp_tmp.p, (size_t)m * elem, hipMemcpyDeviceToDevice, s));
  };
  // filtered positions
  shift(fidx.p, 4, P0, kf);
  shift(fg.p, 4, P0, kf);
  shift(fts.p, 8, P0, kf);
  shift(wsb.p, 4, P0, kf);
  const size_t nv = std::max<size_t>(vcols.size(), 1);
  const int64_t vcap = fx.cap / (int64_t)nv;
  for (size_t v = 0; v < vcols.size(); v++) {
    shift(fx.p + v * vcap, 8, P0, kf);
    shift(fx_raw.p + v * vcap, 8, P0, kf);
  }
  if (wkind == W_LENGTH_BATCH) emitted_batches -= P0 / L;   // the batch being filled is replayed
  if (kf > 0) {
    hipLaunchKernelGGL(k_wa_rebase, dim3((unsigned)((kf + 255) / 256)), dim3(256), 0, s, fidx.p, kf, (int32_t)E0);
    if (wkind != W_LENGTH_BATCH)
      hipLaunchKernelGGL(k_wa_rebase, dim3((unsigned)((kf + 255) / 256)), dim3(256), 0, s, wsb.p, kf, (int32_t)P0);
    SG_HIP(hipGetLastError());
  }
  // events
  shift(ts.p, 8, E0, ke);
  if (wkind == W_TIME) shift(d_now.p, 8, E0, ke);
  for (auto& c : cols) shift(c.b.p, (size_t)c.w, E0, ke);
  SG_HIP(hipStreamSynchronize(s));
  h_seq.erase(h_seq.begin(), h_seq.begin() + E0);
  h_ts.erase(h_ts.begin(), h_ts.begin() + E0);
  h_chunk.erase(h_chunk.begin(), h_chunk.begin() + E0);
  F = kf;
  n = done = ke;
}

void WindowAggExec::flush_run(std::vector<Callback>& out, bool materialise, hipStream_t s) {
  last_matches = 0;
  kernel_ms.clear();
  if (n <= done) return;
  PhaseClock pcw(getenv("SG_HOST_TIMING") != nullptr);
  const int64_t nn = n - done;
  if (ext && wkind == W_TIME) check_ts_order(ext_ts, n, ts_bad, s, "time window");   // the window starts bisect ts
  if (!e0) { SG_HIP(hipEventCreate(&e0)); SG_HIP(hipEventCreate(&e1)); }
  for (auto& e : tev) if (!e) SG_HIP(hipEventCreate(&e));
  SG_HIP(hipEventRecord(tev[0], s));
  // 1. filter + compaction (filtered positions continue across flushes)
  const int64_t ntile = (nn + WA_FT - 1) / WA_FT;
  flags.reserve(ntile * WA_FT);
  tcnt.reserve(ntile); toff.reserve(ntile);
  d_filter.reserve(1);
  SG_HIP(hipMemcpyAsync(d_filter.p, &filter, sizeof(Prog), hipMemcpyHostToDevice, s));
  WaAtom atom;
  if (has_filter && wa_atom_of(filter, atom) && !getenv("SG_WA_NO_ATOM")) {   // (env: test hook)
    atom.w = tsize(app->streams[st].types[atom.attr]);
    hipLaunchKernelGGL(k_wa_filter_atom, dim3((unsigned)ntile), dim3(256), 0, s, done, n, wcols().c[atom.attr], atom,
                       flags.p, tcnt.p);
  } else {
    hipLaunchKernelGGL(k_wa_filter, dim3((unsigned)ntile), dim3(256), 0, s, done, n, wcols(), d_filter.p,
                       has_filter ? 1 : 0, flags.p, tcnt.p);
  }
  SG_HIP(hipGetLastError());
  fidx.reserve(F + nn, true, s, F);
  dsel_n.reserve(1);
  {
    size_t tmp = 0;
    SG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, tcnt.p, toff.p, (int)ntile, s));
    sel_tmp.reserve(tmp);
    SG_HIP(hipcub::DeviceScan::ExclusiveSum(sel_tmp.p, tmp, tcnt.p, toff.p, (int)ntile, s));
    hipLaunchKernelGGL(k_wa_place, dim3((unsigned)ntile), dim3(256), 0, s, done, nn, flags.p, toff.p, tcnt.p, ntile,
                       fidx.p + F, dsel_n.p);
    SG_HIP(hipGetLastError());
  }
  SG_HIP(hipEventRecord(tev[1], s));
  int32_t nf = 0;
  SG_HIP(hipMemcpyAsync(&nf, dsel_n.p, 4, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  const int64_t f0 = F, F1 = F + nf;
  // 2. gather group ids + values (cap grows; keep history for the window halo)
  int64_t cap = std::max<int64_t>(F1, 1024);
  if ((int64_t)fg.cap < cap || (int64_t)fts.cap < cap || (int64_t)wsb.cap < cap ||
      (int64_t)fx.cap < cap * (int64_t)std::max<size_t>(vcols.size(), 1)) {
    // re-layout value columns [v][cap]
    DBuf<double> nfx;
    DBuf<int64_t> nraw;
    size_t nv = std::max<size_t>(vcols.size(), 1);
    int64_t ncap = std::max<int64_t>(cap * 2, 1024);
    nfx.reserve(nv * ncap);
    nraw.reserve(nv * ncap);
    if (f0 > 0) {
      // column pitch = cap / nv of each buffer (DBuf rounds capacities up): the same pitch vcap reads with
      const int64_t ocap = fx.cap / nv, npitch = nfx.cap / nv;
      SG_HIP(hipMemcpy2DAsync(nfx.p, npitch * 8, fx.p, ocap * 8, f0 * 8, nv, hipMemcpyDeviceToDevice, s));
      SG_HIP(hipMemcpy2DAsync(nraw.p, npitch * 8, fx_raw.p, ocap * 8, f0 * 8, nv, hipMemcpyDeviceToDevice, s));
    }
    SG_HIP(hipStreamSynchronize(s));
    fx = std::move(nfx);
    fx_raw = std::move(nraw);
    fg.reserve(ncap, true, s, f0);
    fts.reserve(ncap, true, s, f0);
    wsb.reserve(ncap, true, s, f0);
  }
  const int64_t vcap = fx.cap / std::max<size_t>(vcols.size(), 1);
  stat_i.reserve(WA_MAXV + 2);
  stat_m.reserve(WA_MAXV);
  std::vector<int32_t> si(WA_MAXV + 2, 0);
  si[WA_MAXV] = INT32_MIN;       // gmax
  si[WA_MAXV + 1] = INT32_MAX;   // gmin
  SG_HIP(hipMemcpyAsync(stat_i.p, si.data(), si.size() * 4, hipMemcpyHostToDevice, s));
  SG_HIP(hipMemsetAsync(stat_m.p, 0, WA_MAXV * 8, s));
  if (nf > 0) {
    WaGatherArgs ga;
    std::memset(&ga, 0, sizeof(ga));
    ga.fidx = fidx.p; ga.f0 = f0; ga.nf = nf; ga.cols = wcols();
    ga.gcol = gcol; ga.gw = gcol >= 0 ? tsize(gty) : 4;
    ga.nv = (int)vcols.size();
    for (size_t v = 0; v < vcols.size(); v++) { ga.v[v].col = vcols[v]; ga.v[v].t = vtys[v]; }
    ga.fg = fg.p; ga.fx = fx.p; ga.fx_raw = fx_raw.p; ga.cap = vcap;
    ga.stat_shift = stat_i.p; ga.stat_max = stat_m.p; ga.stat_gmax = stat_i.p + WA_MAXV; ga.stat_gmin = stat_i.p + WA_MAXV + 1;
    ga.ts = ext ? ext_ts : ts.p; ga.fts = fts.p;
    hipLaunchKernelGGL(k_wa_gather, dim3((unsigned)std::min<int64_t>((nf + 255) / 256, 4096)), dim3(256), 0, s, ga);
    SG_HIP(hipGetLastError());
  }
  // window start of every new filtered event, and the widest window
  maxwin.reserve(1);
  SG_HIP(hipMemsetAsync(maxwin.p, 0, 4, s));
  if (nf > 0 && wkind != W_LENGTH_BATCH) {
    WaWsArgs wa;
    std::memset(&wa, 0, sizeof(wa));
    wa.kind = wkind; wa.param = L; wa.f0 = f0; wa.F = F1; wa.fidx = fidx.p; wa.fts = fts.p;
    wa.now = (wkind == W_TIME && !ext) ? d_now.p : nullptr;
    wa.now_const = ext ? ext_now : -1;
    wa.ws = wsb.p; wa.maxwin = maxwin.p;
    hipLaunchKernelGGL(k_wa_wstart, dim3((unsigned)std::min<int64_t>((nf + 255) / 256, 8192)), dim3(256), 0, s, wa);
    SG_HIP(hipGetLastError());
  }
  SG_HIP(hipEventRecord(tev[2], s));
  SG_HIP(hipMemcpyAsync(si.data(), stat_i.p, si.size() * 4, hipMemcpyDeviceToHost, s));
  std::vector<unsigned long long> smax(WA_MAXV);
  SG_HIP(hipMemcpyAsync(smax.data(), stat_m.p, WA_MAXV * 8, hipMemcpyDeviceToHost, s));
  int32_t mw = 0;
  SG_HIP(hipMemcpyAsync(&mw, maxwin.p, 4, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  if (wkind == W_LENGTH_BATCH) mw = (int32_t)L;
  F = F1;
  done = n;
  if (nf == 0) return;
  // group ids over the history (needed by both paths)
  int gmin = si[WA_MAXV + 1], gmax = si[WA_MAXV];
  if (f0 > 0) { gmin = std::min(gmin, gmin_hist); gmax = std::max(gmax, gmax_hist); }
  gmin_hist = gmin; gmax_hist = gmax;
  if (gcol < 0) { gmin = gmax = 0; }
  // 3. exact fast path?
  std::vector<int> shift(vcols.size(), 0);
  bool bound_ok = true;
  // (lengthBatch: the per-group resets make it a replay)
  bool exact = fast_ok && wkind != W_LENGTH_BATCH && gmin >= 0 && (int64_t)gmax - gmin + 1 <= WA_MAXK;
  for (size_t v = 0; v < vcols.size(); v++) {          // history statistics always advance
    shift_hist[v] = std::max(shift_hist[v], si[v]);
    double mx;
    std::memcpy(&mx, &smax[v], 8);
    maxabs_hist[v] = std::max(maxabs_hist[v], mx);
    shift[v] = shift_hist[v];
    if (shift[v] > 1000) { bound_ok = false; continue; }
    double bound = std::ldexp(maxabs_hist[v], shift[v]) * (double)(mw + 1);   // widest window + 1
    if (!(bound < 9007199254740992.0)) bound_ok = false;
  }
  // a flush past the bound may have rounded the reference's running sums, and that error stays in
  // them: from then on only the sequential replay reproduces them
  if (!bound_ok) inexact_seen = true;
  if (inexact_seen) exact = false;
  const int nout_agg = (int)aggs.size();
  out_raw.reserve((size_t)std::max(nout_agg, 1) * vcap);
  out_nul.reserve((size_t)std::max(nout_agg, 1) * vcap);
  SG_HIP(hipEventRecord(e0, s));
  if (exact) {
    int K = gmax - gmin + 1;
    out_sum.reserve((size_t)std::max<size_t>(vcols.size(), 1) * vcap);
    out_cnt.reserve(vcap);
    WaTileArgs ta;
    std::memset(&ta, 0, sizeof(ta));
    ta.fg = fg.p; ta.fx = fx.p; ta.cap = vcap; ta.nv = (int)vcols.size();
    for (size_t v = 0; v < vcols.size(); v++) ta.shift[v] = shift[v];
    ta.f0 = f0; ta.F = F1; ta.T = tileT; ta.L = mw; ta.K = K; ta.gmin = gmin; ta.ws = wsb.p;
    ta.out_sum = out_sum.p; ta.out_cnt = out_cnt.p;
    int R = tileT + mw;
    size_t lds = (size_t)R * 8 + (size_t)(2 * K + 1 + 16) * 4 + 16 + (size_t)ta.nv * R * 8;
    if (lds > 160 * 1024) exact = false;
    else {
      int64_t ntiles = (nf + tileT - 1) / tileT;
      SG_HIP(hipFuncSetAttribute((const void*)k_wa_tile, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL(k_wa_tile, dim3((unsigned)ntiles), dim3(WA_B), lds, s, ta);
      SG_HIP(hipGetLastError());
      state_valid = false;   // the carried group states did not see this flush
    }
  }
  if (!exact) {
    // general path: CSR of filtered positions per group (host-built), one lane per group
    std::vector<int32_t> hfg(F1);
    SG_HIP(hipMemcpyAsync(hfg.data(), fg.p, F1 * 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    // (the held positions: the window content carried in the group states, then the new ones; for
    // lengthBatch the batch being filled, replayed from the state saved before it)
    std::unordered_map<int32_t, int> gid;
    std::vector<std::vector<int32_t>> lists;
    std::vector<int32_t> slots;
    for (int64_t p = 0; p < F1; p++) {
      auto it = gid.find(hfg[p]);
      int g;
      if (it == gid.end()) {
        g = (int)lists.size(); gid[hfg[p]] = g; lists.emplace_back();
        auto sl = gslot.emplace(hfg[p], (int32_t)gslot.size()).first;
        slots.push_back(sl->second);
      } else g = it->second;
      lists[g].push_back((int32_t)p);
    }
    std::vector<int32_t> off(1, 0), pos;
    for (auto& l : lists) { pos.insert(pos.end(), l.begin(), l.end()); off.push_back((int32_t)pos.size()); }
    gsum_off.reserve(off.size()); gsum_pos.reserve(pos.size()); gsum_slot.reserve(std::max<size_t>(slots.size(), 1));
    SG_HIP(hipMemcpyAsync(gsum_off.p, off.data(), off.size() * 4, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(gsum_pos.p, pos.data(), pos.size() * 4, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(gsum_slot.p, slots.data(), slots.size() * 4, hipMemcpyHostToDevice, s));
    int ng = (int)lists.size();
    const bool batch = wkind == W_LENGTH_BATCH;
    ensure_states((int64_t)gslot.size(), batch ? 1 : mw + 2, s);   // min/max expiry deques (sliding only)
    const int na = std::max(nout_agg, 1);
    const bool old_add = !batch && !state_valid;
    if (old_add) SG_HIP(hipMemsetAsync(wst.p, 0, (size_t)(dq_slots * na) * sizeof(WaSt), s));
    int32_t ws_end = 0;
    if (!batch) SG_HIP(hipMemcpyAsync(&ws_end, wsb.p + F1 - 1, 4, hipMemcpyDeviceToHost, s));
    err.reserve(1);
    SG_HIP(hipMemsetAsync(err.p, 0, 4, s));
    SG_HIP(hipStreamSynchronize(s));
    WaSeqArgs sa;
    std::memset(&sa, 0, sizeof(sa));
    sa.g_off = gsum_off.p; sa.g_pos = gsum_pos.p; sa.g_slot = gsum_slot.p; sa.ngroups = ng; sa.fx = fx.p;
    sa.fx_raw = fx_raw.p; sa.cap = vcap;
    sa.ws = wsb.p; sa.batchL = batch ? (int32_t)L : 0; sa.na = nout_agg;
    for (int k = 0; k < nout_agg; k++) sa.agg[k] = aggs[k];
    sa.out_raw = out_raw.p; sa.out_nul = out_nul.p; sa.st = wst.p; sa.dq = dq.p; sa.dq_cap = dq_ring; sa.err = err.p;
    sa.destroy = gcol >= 0;
    sa.f0 = batch ? 0 : f0;
    sa.old_add = old_add ? 1 : 0;
    sa.ws_end = ws_end;
    sa.save_at = !batch ? INT64_MAX : (materialise ? (F1 / L) * L : emitted_batches * L);
    hipLaunchKernelGGL(k_wa_seq, dim3((unsigned)((ng + 63) / 64)), dim3(64), 0, s, sa);
    SG_HIP(hipGetLastError());
    int32_t herr = 0;
    SG_HIP(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    if (herr) throw Error(-1, "window aggregator deque overflow");
    state_valid = true;
  }
  SG_HIP(hipEventRecord(e1, s));
  SG_HIP(hipStreamSynchronize(s));
  float ms = 0;
  SG_HIP(hipEventElapsedTime(&ms, e0, e1));
  kernel_ms[exact ? "k_wa_tile" : "k_wa_seq"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, tev[0], tev[1]));
  kernel_ms["k_wa_filter_select"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, tev[1], tev[2]));
  kernel_ms["k_wa_gather"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, tev[0], e1));
  kernel_ms["total"] = ms;
  last_matches = nf;
  if (!materialise) return;
  if (ext) throw Error(-2, "device-resident ingest keeps window outputs in HBM (use sg_flush_device)");
  // 4. materialise: aggregator outputs of the new filtered events, selector batching per chunk.
  //    lengthBatch emits only completed batches, which may have begun in earlier flushes.
  int64_t m0 = f0, m1 = F1;
  if (wkind == W_LENGTH_BATCH) {
    m0 = emitted_batches * L;
    m1 = (F1 / L) * L;
    emitted_batches = F1 / L;
    if (m1 <= m0) return;
  }
  const int64_t nm = m1 - m0;
  pcw.mark("window flush kernels");
  PhaseClock pc(getenv("SG_HOST_TIMING") != nullptr);
  // a chained export that may stay in HBM (DevChain): only per-event sends since the last flush (every filtered
  // event one output row), the aggregates formed on the device, each row's clock on the device (time windows over
  // host ingest); the host takes the rows' source seqs and, pinned, the consumers' key column
  if (export_to && dev_req && pending_single && exact && wkind == W_TIME && !ext && nm > 0 &&
      outs.size() <= (size_t)WA_MAXO && dev_req->widths.size() == outs.size()) {
    DevChain& dc = *dev_req;
    px_hidx.reserve((size_t)nm);
    SG_HIP(hipMemcpyAsync(px_hidx.p, fidx.p + m0, nm * 4, hipMemcpyDeviceToHost, s));
    if (nout_agg > 0) {
      WaAggOut ao;
      std::memset(&ao, 0, sizeof(ao));
      ao.na = nout_agg;
      for (int k = 0; k < nout_agg; k++) ao.agg[k] = aggs[k];
      proj.reserve((size_t)nout_agg * nm);
      hipLaunchKernelGGL(k_wa_aggout, dim3((unsigned)((nm + 255) / 256)), dim3(256), 0, s, ao, out_sum.p, out_cnt.p,
                         (int64_t)vcap, m0, nm, proj.p);
      SG_HIP(hipGetLastError());
    }
    dx_ts.reserve(nm); dx_now.reserve(nm);
    WaChainArgs ca;
    std::memset(&ca, 0, sizeof(ca));
    ca.fidx = fidx.p; ca.m0 = m0; ca.nm = nm; ca.ts = ts.p; ca.now = d_now.p; ca.no = (int32_t)outs.size();
    ca.aggv = proj.p; ca.out_ts = dx_ts.p; ca.out_now = dx_now.p;
    dc.d_cols.assign(outs.size(), nullptr);
    for (size_t o = 0; o < outs.size(); o++) {
      ca.kind[o] = outs[o].kind;
      ca.w_out[o] = dc.widths[o];
      ca.agg[o] = outs[o].agg;
      if (outs[o].kind == 0) {
        ca.col[o] = cols[outs[o].col].b.p;
        ca.w_in[o] = cols[outs[o].col].w;
        if (ca.w_in[o] != ca.w_out[o]) throw Error(SG_E_INVALID, "chained column width differs from the inserted stream");
      }
      dx_col[o].reserve((size_t)nm * dc.widths[o]);
      ca.out[o] = dx_col[o].p;
      dc.d_cols[o] = dx_col[o].p;
    }
    hipLaunchKernelGGL(k_wa_chain_pack, dim3((unsigned)((nm + 255) / 256)), dim3(256), 0, s, ca);
    SG_HIP(hipGetLastError());
    if (dc.key_attr >= 0) {
      px_key.reserve((size_t)nm * dc.widths[dc.key_attr]);
      SG_HIP(hipMemcpyAsync(px_key.p, dx_col[dc.key_attr].p, (size_t)nm * dc.widths[dc.key_attr],
                            hipMemcpyDeviceToHost, s));
    }
    SG_HIP(hipStreamSynchronize(s));
    pc.mark("window export: device chain kernels + copies");
    dx_seq.resize(nm);
    const int nth = host_threads(nm);
    host_parallel(nth, [&](int t) {
      const int64_t a0 = nm * t / nth, a1 = nm * (t + 1) / nth;
      for (int64_t r = a0; r < a1; r++) dx_seq[r] = h_seq[px_hidx.p[r]];
    });
    dc.n = nm; dc.d_ts = dx_ts.p; dc.d_now = dx_now.p;
    dc.seq = dx_seq.data();
    dc.key = dc.key_attr >= 0 ? px_key.p : nullptr;
    dc.done = true;
    pc.mark("window export: device chain seqs");
    return;
  }
  // (host staging kept across flushes: no first-touch page faults)
  std::vector<int32_t>& hidx = m_hidx;
  hidx.resize(nm);
  SG_HIP(hipMemcpyAsync(hidx.data(), fidx.p + m0, nm * 4, hipMemcpyDeviceToHost, s));
  std::vector<int64_t>& araw = m_araw;
  araw.resize((size_t)nout_agg * nm);
  std::vector<uint8_t>& anul = m_anul;
  anul.assign((size_t)nout_agg * nm, 0);
  std::vector<int32_t>& hg = m_hg;
  hg.resize(nm);
  SG_HIP(hipMemcpyAsync(hg.data(), fg.p + m0, nm * 4, hipMemcpyDeviceToHost, s));
  if (exact) {
    if (nout_agg > 0 && nm > 0) {     // outputs formed on the device: one 8-byte value per row crosses PCIe
      WaAggOut ao;
      std::memset(&ao, 0, sizeof(ao));
      ao.na = nout_agg;
      for (int k = 0; k < nout_agg; k++) ao.agg[k] = aggs[k];
      proj.reserve((size_t)nout_agg * nm);
      hipLaunchKernelGGL(k_wa_aggout, dim3((unsigned)((nm + 255) / 256)), dim3(256), 0, s, ao, out_sum.p, out_cnt.p,
                         (int64_t)vcap, m0, nm, proj.p);
      SG_HIP(hipGetLastError());
      SG_HIP(hipMemcpyAsync(araw.data(), proj.p, (size_t)nout_agg * nm * 8, hipMemcpyDeviceToHost, s));
    }
    SG_HIP(hipStreamSynchronize(s));
    pc.mark("window copies + aggregates");
  } else {
    for (int k = 0; k < nout_agg; k++) {
      SG_HIP(hipMemcpyAsync(araw.data() + (size_t)k * nm, out_raw.p + k * vcap + m0, nm * 8, hipMemcpyDeviceToHost, s));
      SG_HIP(hipMemcpyAsync(anul.data() + (size_t)k * nm, out_nul.p + k * vcap + m0, nm, hipMemcpyDeviceToHost, s));
    }
    SG_HIP(hipStreamSynchronize(s));
  }
  // projected attribute values from the host copy of the batch columns
  std::vector<hvec<int64_t>> colv(outs.size());
  for (size_t o = 0; o < outs.size(); o++) {
    if (outs[o].kind != 0) continue;
    const int c = outs[o].col;
    colv[o] = app->take64();
    colv[o].resize(nm);
    if (nm == 0) continue;
    // gathered on the device: only the output rows' values cross PCIe
    proj.reserve(std::max<int64_t>(nm, 1));
    hipLaunchKernelGGL(k_wa_proj, dim3((unsigned)((nm + 255) / 256)), dim3(256), 0, s, cols[c].b.p, cols[c].w,
                       app->streams[st].types[c] == T_FLOAT ? 1 : 0, fidx.p + m0, nm, proj.p);
    SG_HIP(hipGetLastError());
    SG_HIP(hipMemcpyAsync(colv[o].data(), proj.p, nm * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
  }
  pc.mark("window columns");
  if (export_to) {
    // the same selection as the callbacks below, written as columns
    ChainOut& co = *export_to;
    co.raw.assign(outs.size(), {});
    auto put = [&](int64_t p, int64_t sq) {
      co.ts.push_back(h_ts[hidx[p]]);
      co.seq.push_back(sq);
      for (size_t o = 0; o < outs.size(); o++) {
        if (outs[o].kind == 0) co.raw[o].push_back(colv[o][p]);
        else {
          co.raw[o].push_back(araw[(size_t)outs[o].agg * nm + p]);
          co.nulls = co.nulls || anul[(size_t)outs[o].agg * nm + p];
        }
      }
    };
    // per-event sends (every chunk one event): every filtered event is one output row, in order (the check, the
    // row copies and the null scan run over thread ranges)
    const int nth = host_threads(nm);
    bool singles = wkind != W_LENGTH_BATCH;
    if (singles && nm > 1) {
      std::vector<uint8_t> ok((size_t)nth, 1);
      host_parallel(nth, [&](int t) {
        const int64_t a0 = std::max<int64_t>(1, nm * t / nth), a1 = nm * (t + 1) / nth;
        for (int64_t r = a0; r < a1; r++)
          if (h_chunk[hidx[r]] == h_chunk[hidx[r - 1]]) { ok[t] = 0; break; }
      });
      for (int t = 0; t < nth; t++) singles = singles && ok[t];
    }
    pc.mark("window export: per-event check");
    if (singles) {
      co.ts.resize(nm); co.seq.resize(nm); co.singles = true;
      std::vector<size_t> aggo;
      for (size_t o = 0; o < outs.size(); o++)
        if (outs[o].kind != 0) { co.raw[o] = app->take64(); co.raw[o].resize(nm); aggo.push_back(o); }
      std::vector<uint8_t> nul((size_t)nth, 0);
      host_parallel(nth, [&](int t) {
        const int64_t a0 = nm * t / nth, a1 = nm * (t + 1) / nth;
        for (int64_t r = a0; r < a1; r++) {
          const int64_t e = hidx[r];
          co.ts[r] = h_ts[e];
          co.seq[r] = h_seq[e];
        }
        for (size_t o : aggo) {
          const size_t base = (size_t)outs[o].agg * nm;
          std::memcpy(co.raw[o].data() + a0, araw.data() + base + a0, (size_t)(a1 - a0) * 8);
          for (int64_t r = a0; r < a1 && !nul[t]; r++) nul[t] = anul[base + r] != 0;
        }
      });
      pc.mark("window export: row copies");
      for (int t = 0; t < nth; t++) co.nulls = co.nulls || nul[t];
      for (size_t o = 0; o < outs.size(); o++)
        if (outs[o].kind == 0) co.raw[o] = std::move(colv[o]);   // (each is read once)
      pc.mark("window export");
      return;
    }
    co.ts.reserve(nm); co.seq.reserve(nm);
    for (auto& c : co.raw) c.reserve(nm);
    int64_t p = 0;
    std::vector<int32_t> order;
    std::unordered_map<int32_t, int64_t> last;
    while (p < nm) {
      int64_t q = p;
      if (wkind == W_LENGTH_BATCH) q = p + L;
      else {
        const int64_t c = h_chunk[hidx[p]];
        while (q < nm && h_chunk[hidx[q]] == c) q++;
      }
      const int64_t sq = h_seq[hidx[q - 1]];
      if (gcol >= 0) {
        if (q - p == 1) put(p, sq);
        else {
          order.clear(); last.clear();
          for (int64_t r = p; r < q; r++) {
            if (!last.count(hg[r])) order.push_back(hg[r]);
            last[hg[r]] = r;
          }
          for (int32_t g : order) put(last[g], sq);
        }
      } else if (!aggs.empty()) {
        put(q - 1, sq);
      } else {
        for (int64_t r = p; r < q; r++) put(r, sq);
      }
      co.chunk_end.push_back((int64_t)co.ts.size());
      p = q;
    }
    return;
  }
  auto row = [&](int64_t p) {
    OutEvent oe;
    oe.ts = h_ts[hidx[p]];
    for (size_t o = 0; o < outs.size(); o++) {
      if (outs[o].kind == 0) { oe.raw.push_back(colv[o][p]); oe.nul.push_back(0); }
      else { oe.raw.push_back(araw[(size_t)outs[o].agg * nm + p]); oe.nul.push_back(anul[(size_t)outs[o].agg * nm + p]); }
    }
    return oe;
  };
  // output chunks: one per send call (sliding windows), one per completed batch (lengthBatch)
  int64_t p = 0;
  while (p < nm) {
    int64_t q = p;
    if (wkind == W_LENGTH_BATCH) q = p + L;
    else {
      const int64_t c = h_chunk[hidx[p]];
      while (q < nm && h_chunk[hidx[q]] == c) q++;
    }
    Callback cb;
    cb.seq = h_seq[hidx[q - 1]];
    cb.order = qi; cb.kind = 0; cb.target = qi;
    if (gcol >= 0) {   // processInBatchGroupBy (with or without aggregators)
      std::vector<int32_t> order;
      std::unordered_map<int32_t, int64_t> last;
      for (int64_t r = p; r < q; r++) {
        if (!last.count(hg[r])) order.push_back(hg[r]);
        last[hg[r]] = r;
      }
      for (int32_t g : order) cb.ev.push_back(row(last[g]));
    } else if (!aggs.empty()) {
      cb.ev.push_back(row(q - 1));
    } else {
      for (int64_t r = p; r < q; r++) cb.ev.push_back(row(r));
    }
    cb.ts = cb.ev.back().ts;
    out.push_back(std::move(cb));
    p = q;
  }
}

std::unique_ptr<Exec> make_window_agg(App& app, int qi, const J& q, std::string& why) {
  const J& in = q["input"];
  if (in["kind"].s != "single") { why = "not a single-stream query"; return nullptr; }
  if (q.has("partition")) { why = "partitioned window query"; return nullptr; }
  const J& hs = in["handlers"];
  int win = -1;
  std::vector<const J*> filt;
  for (size_t k = 0; k < hs.size(); k++) {
    if (hs[k]["k"].s == "filter") {
      if (win >= 0) { why = "filter after the window"; return nullptr; }
      filt.push_back(&hs[k]["e"]);
    } else {
      if (win >= 0) { why = "two windows"; return nullptr; }
      win = (int)k;
    }
  }
  if (win < 0) { why = "no window"; return nullptr; }
  const J& w = hs[win];
  const std::string wname = w["name"].s;
  if (wname != "length" && wname != "time" && wname != "lengthBatch") { why = "window." + wname + " is not lowered yet"; return nullptr; }
  if (w["params"].size() != 1 || w["params"][0]["op"].s != "const") { why = "window parameter"; return nullptr; }
  const J& s = q["select"];
  if (!s["having"].null() || s["order_by"].size() || !s["limit"].null() || !s["offset"].null()) { why = "selector features"; return nullptr; }
  if (q["output"]["events"].s != "current" && !q["output"]["events"].s.empty()) { why = "expired events output"; return nullptr; }
  auto ex = std::make_unique<WindowAggExec>();
  ex->app = &app; ex->qi = qi; ex->path = 3;
  ex->st = app.stream_idx.at(in["stream"].s);
  ex->wkind = wname == "time" ? W_TIME : wname == "lengthBatch" ? W_LENGTH_BATCH : W_LENGTH;
  ex->L = w["params"][0]["v"].as_int();
  if (ex->L <= 0) { why = "window parameter <= 0"; return nullptr; }
  if (ex->wkind != W_TIME && ex->L > (1 << 30)) { why = "window length"; return nullptr; }
  const auto& types = app.streams[ex->st].types;
  if (types.size() > 12) { why = "too many attributes"; return nullptr; }
  if (s["group_by"].size() > 1) { why = "multi-attribute group by"; return nullptr; }
  if (s["group_by"].size() == 1) {
    const J& g = s["group_by"][0];
    if (g["op"].s != "var") { why = "group by expression"; return nullptr; }
    ex->gcol = (int)g["attr"].as_int();
    ex->gty = types[ex->gcol];
    // (groups are keyed by 32-bit ids here: a LONG key goes to the general window path)
    if (ex->gty != T_STRING && ex->gty != T_INT && ex->gty != T_BOOL) { why = "group by on a float or long"; return nullptr; }
  }
  ex->fast_ok = true;
  for (size_t k = 0; k < s["attrs"].size(); k++) {
    const J& e = s["attrs"][k]["e"];
    if (e["op"].s == "var") { ex->outs.push_back({0, (int)e["attr"].as_int(), -1}); continue; }
    if (e["op"].s != "agg") { why = "select expression is not an attribute or aggregator"; return nullptr; }
    const std::string& nm = e["name"].s;
    WaAgg A;
    A.k = nm == "sum" ? A_SUM : nm == "avg" ? A_AVG : nm == "count" ? A_COUNT : nm == "min" ? A_MIN : nm == "max" ? A_MAX : -1;
    if (A.k < 0) { why = "aggregator " + nm; return nullptr; }
    A.v = -1; A.t = T_INT;
    if (A.k != A_COUNT) {
      if (e["args"].size() != 1 || e["args"][0]["op"].s != "var") { why = "aggregator argument"; return nullptr; }
      int col = (int)e["args"][0]["attr"].as_int();
      Ty t = types[col];
      if (t != T_INT && t != T_LONG && t != T_FLOAT && t != T_DOUBLE) { why = "aggregator over non-numeric"; return nullptr; }
      auto it = std::find(ex->vcols.begin(), ex->vcols.end(), col);
      if (it == ex->vcols.end()) {
        if (ex->vcols.size() >= (size_t)WA_MAXV) { why = "too many aggregated columns"; return nullptr; }
        ex->vcols.push_back(col); ex->vtys.push_back(t); A.v = (int)ex->vcols.size() - 1;
      } else A.v = (int)(it - ex->vcols.begin());
      A.t = t;
      if (A.k == A_MIN || A.k == A_MAX) ex->fast_ok = false;
    }
    if (ex->aggs.size() >= (size_t)WA_MAXA) { why = "too many aggregators"; return nullptr; }
    ex->outs.push_back({1, -1, (int)ex->aggs.size()});
    ex->aggs.push_back(A);
  }
  auto intern = [&](const std::string& str) { return app.intern(str); };
  auto sm = [&](int slot, int chain) -> int { (void)slot; (void)chain; return 0; };
  try {
    if (!filt.empty()) {
      J arr;
      arr.k = J::ARR;
      for (auto* f : filt) arr.a.push_back(*f);
      compile_filters(ex->filter, arr, sm, intern);
      ex->has_filter = true;
    }
  } catch (CompileError& e) {
    why = e.what();
    return nullptr;
  }
  for (Ty t : types) { ex->cols.emplace_back(); ex->cols.back().w = tsize(t); }
  ex->in_streams = {ex->st};
  return ex;
}

}  // namespace sg
