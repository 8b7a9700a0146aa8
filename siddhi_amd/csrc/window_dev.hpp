// window_dev.hpp — device kernels of the general window path (window_gen.hip, GenWindowExec::flush_device).
//
// One flush of a single-stream query runs as:
//   1. k_gw_eval (window_gen.hip): filter + pre-selector values per event.
//   2. k_gwd_mask / DeviceSelect / k_gwd_gather: the filtered events in arrival order, their values appended to
//      the flush's value table behind the rows the windows carried in (host-held window state of earlier
//      flushes), with instance, clock, timestamp and selector-chunk ordinal per event.
//   3. Partitioned: a stable radix sort by instance gives each event its rank inside its instance.
//   4. The window processor as closed forms over those ranks, one thread per event (per clock point for time
//      windows), writing the items of every output chunk -- (type, ts, value row, instance, chunk) -- in the
//      order the reference's processor emits them:
//        LengthWindowProcessor.process      LengthWindowProcessor.java:106-141   k_gwd_len_*
//        LengthBatchWindowProcessor.process LengthBatchWindowProcessor.java:154-351 (both modes) k_gwd_batch_*
//        TimeWindowProcessor.process + its Scheduler TIMER chunks TimeWindowProcessor.java:133-169 k_gwd_time_*
//   5. QuerySelector (QuerySelector.java:76-374): group keys hashed and sorted (stable) into per-(instance,
//      group) segments; sum / count / avg as segmented scans (a RESET item starts a new segment) in exact
//      integer arithmetic -- integral sums as longs, float / double ones in fixed point 2^-S, checked so that
//      the reference's sequential double arithmetic never rounds -- resumed from the carried state;
//      output expressions and having through the expression interpreter (k_gwd_out).
// What stays on the host: the partition-key -> instance map, the per-chunk batching of the selected rows
// (last row per group in first-appearance order, order by / offset / limit) and the carried state between
// flushes (the window queues' held rows and the aggregator states, in the same structures the host path uses).
#pragma once
#include <hip/hip_runtime.h>

#include "compile.hpp"
#include "expr.hpp"

namespace sg {

constexpr int GWD_B = 256;
constexpr int GWD_MAXAGG = 8;
constexpr int GWD_MAXG = 6;      // group-by keys
constexpr int GWD_MAXOUT = 16;   // output attributes

enum { GI_CUR = 0, GI_EXP = 1, GI_RESET = 3 };

// flags[e] &= event e has an instance (partitioned: a null key drops the event)
static __global__ void __launch_bounds__(GWD_B) k_gwd_mask(int64_t n, uint8_t* __restrict__ flags, const int32_t* __restrict__ lid) {
  const int64_t e = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (e < n && lid[e] < 0) flags[e] = 0;
}

struct GwdGatherArgs {
  int64_t F, C, R;            // filtered events, carried rows, value table rows (C + F)
  const int32_t* fidx;        // filtered -> event (flush-relative)
  int32_t nv;
  const int64_t* pv;          // [nv][pitch] k_gw_eval values
  const uint8_t* pn;
  int64_t pitch;
  int64_t* vt;                // [nv][R]
  uint8_t* vn;
  const int32_t* ev_lid;
  const int64_t* ev_ts;
  const int64_t* ev_now;
  const int32_t* ev_ord;
  int32_t* f_lid;
  int64_t* f_ts;
  int64_t* f_now;
  int32_t* f_ord;
  int32_t* cnt;               // per instance (partitioned), nullptr otherwise
};

static __global__ void __launch_bounds__(GWD_B) k_gwd_gather(GwdGatherArgs a) {
  const int64_t f = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (f >= a.F) return;
  const int32_t e = a.fidx[f];
  for (int k = 0; k < a.nv; k++) {
    a.vt[(int64_t)k * a.R + a.C + f] = a.pv[(int64_t)k * a.pitch + e];
    a.vn[(int64_t)k * a.R + a.C + f] = a.pn[(int64_t)k * a.pitch + e];
  }
  const int32_t l = a.ev_lid[e];
  a.f_lid[f] = l;
  a.f_ts[f] = a.ev_ts[e];
  a.f_now[f] = a.ev_now[e];
  a.f_ord[f] = a.ev_ord[e];
  if (a.cnt) atomicAdd(&a.cnt[l], 1);
}

// rank of every filtered event inside its instance, from the instance-sorted order
static __global__ void __launch_bounds__(GWD_B) k_gwd_rank(int64_t F, const int32_t* __restrict__ byinst,
                                                    const int32_t* __restrict__ f_lid, const int32_t* __restrict__ st,
                                                    int32_t* __restrict__ rank) {
  const int64_t p = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (p >= F) return;
  const int32_t f = byinst[p];
  rank[f] = (int32_t)(p - st[f_lid[f]]);
}

// per instance, what the window carried in (host WinState, uploaded per flush)
struct GwdInst {
  int64_t count;     // LengthWindow / LengthBatch count
  int32_t cc, co;    // FIFO head carried: rows [co, co + cc) of the value table
  int32_t cx, cxo;   // lengthBatch (non-stream): the previous batch held for EXPIRED output
  int32_t h0, r0;    // lengthBatch: has_reset and its row
};

struct GwdItems {
  uint8_t* type;
  int64_t* ts;
  int32_t* row;
  int32_t* lid;
  int32_t* ord;
  int64_t cap;        // items allocated (a write past it is dropped, never out of bounds)
};

struct GwdPlanArgs {
  int64_t F, C;
  int64_t L;                       // length / batch count
  int32_t expired_on, stream_current;
  const int32_t* byinst;           // instance-sorted filtered events (identity when unpartitioned)
  const int32_t* st;               // first sorted position per instance
  const int32_t* cnt;              // filtered events per instance
  const int32_t* f_lid;
  const int32_t* rank;
  const int64_t* f_ts;
  const int64_t* f_now;
  const int32_t* f_ord;
  const int64_t* c_ts;             // carried rows' timestamps [C]
  const GwdInst* inst;
  int32_t* nit;                    // items per filtered event
  const int32_t* ioff;             // exclusive scan of nit
  GwdItems it;
};

struct GwdFifo {
  const GwdPlanArgs* a;
  int32_t l;
  __device__ int32_t row(int64_t idx) const {     // FIFO = carried head + the instance's new events
    const GwdInst& I = a->inst[l];
    if (idx < I.cc) return I.co + (int32_t)idx;
    return (int32_t)(a->C + a->byinst[a->st[l] + (idx - I.cc)]);
  }
  __device__ int64_t ts(int64_t idx) const {
    const GwdInst& I = a->inst[l];
    if (idx < I.cc) return a->c_ts[I.co + idx];
    return a->f_ts[a->byinst[a->st[l] + (idx - I.cc)]];
  }
};

// the selector's pre-selector values: value k of row r at v[k * vs + r * rs] (window path: columns of the
// flush's value table; NFA path: the device-projected values of each match, row-major)
struct GwdVals {
  const int64_t* v;
  const uint8_t* n;
  int64_t vs, rs;
  __device__ int64_t val(int k, int64_t r) const { return v[(int64_t)k * vs + r * rs]; }
  __device__ bool nul(int k, int64_t r) const { return n[(int64_t)k * vs + r * rs] != 0; }
};

__device__ __forceinline__ void gwd_put(const GwdItems& it, int64_t k, int type, int64_t ts, int32_t row, int32_t l,
                                        int32_t ord) {
  if (k < 0 || k >= it.cap) return;
  it.type[k] = (uint8_t)type; it.ts[k] = ts; it.row[k] = row; it.lid[k] = l; it.ord[k] = ord;
}

// ---- LengthWindowProcessor (:106-141) ----
// Event of instance rank r, position P = count + r: once L events are held, the oldest (position P - L)
// leaves as EXPIRED stamped with the clock, then the event passes as CURRENT.  length(0): CURRENT, the event
// itself EXPIRED (its own timestamp) and a RESET.
template <bool FILL>
static __global__ void __launch_bounds__(GWD_B) k_gwd_len(GwdPlanArgs a) {
  const int64_t f = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (f >= a.F) return;
  const int32_t l = a.f_lid[f], r = a.rank[f];
  const GwdInst& I = a.inst[l];
  const int64_t P = I.count + r;
  const int32_t me = (int32_t)(a.C + f);
  if (a.L < 0) {                                    // no window: the events pass as they are
    if (!FILL) { a.nit[f] = 1; return; }
    gwd_put(a.it, a.ioff[f], GI_CUR, a.f_ts[f], me, l, a.f_ord[f]);
    return;
  }
  if (a.L == 0) {
    if (!FILL) { a.nit[f] = 3; return; }
    const int64_t k = a.ioff[f];
    gwd_put(a.it, k, GI_CUR, a.f_ts[f], me, l, a.f_ord[f]);
    gwd_put(a.it, k + 1, GI_EXP, a.f_ts[f], me, l, a.f_ord[f]);
    gwd_put(a.it, k + 2, GI_RESET, a.f_ts[f], me, l, a.f_ord[f]);
    return;
  }
  const bool exp = P >= a.L;
  if (!FILL) { a.nit[f] = exp ? 2 : 1; return; }
  int64_t k = a.ioff[f];
  if (exp) {
    // the FIFO holds the carried cc rows (positions count - cc .. count - 1), then the new events
    GwdFifo q{&a, l};
    const int64_t idx = (P - a.L) - (I.count - I.cc);
    gwd_put(a.it, k++, GI_EXP, a.f_now[f], q.row(idx), l, a.f_ord[f]);
  }
  gwd_put(a.it, k, GI_CUR, a.f_ts[f], me, l, a.f_ord[f]);
}

// ---- LengthBatchWindowProcessor (:154-351) ----
// Every event is its own processor call (its own selector chunk).
//   default mode: FIFO = the pending batch carried (count rows) + new events; the event completing batch
//     k (FIFO [kL, kL+L)) emits [previous batch EXPIRED (expired output) | RESET | the batch CURRENT];
//     the previous batch of k = 0 is the carried one, the RESET is a copy of the batch's first event (the
//     carried reset while the carried batch is incomplete).
//   streamCurrentEvents: every event passes as CURRENT at once; the (L+1)-th event since the last flush
//     first emits [that batch EXPIRED (expired output) | RESET]; the RESET is a copy of the first event
//     processed after the previous flush.  FIFO = the carried current batch (when expired output is on) +
//     new events.
// lengthBatch(0): CURRENT, EXPIRED (expired output), RESET -- expired and reset stamped with the clock.
template <bool FILL>
static __global__ void __launch_bounds__(GWD_B) k_gwd_batch(GwdPlanArgs a) {
  const int64_t f = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (f >= a.F) return;
  const int32_t l = a.f_lid[f], r = a.rank[f];
  const GwdInst& I = a.inst[l];
  const int32_t me = (int32_t)(a.C + f);
  const int32_t ord = a.f_ord[f];
  const int64_t now = a.f_now[f];
  GwdFifo q{&a, l};
  const int64_t L = a.L;
  if (L == 0) {
    if (!FILL) { a.nit[f] = a.expired_on ? 3 : 2; return; }
    int64_t k = a.ioff[f];
    gwd_put(a.it, k++, GI_CUR, a.f_ts[f], me, l, ord);
    if (a.expired_on) gwd_put(a.it, k++, GI_EXP, now, me, l, ord);
    gwd_put(a.it, k, GI_RESET, now, me, l, ord);
    return;
  }
  const int64_t b0 = I.count;
  if (!a.stream_current) {
    const bool flush = (b0 + r + 1) % L == 0;
    if (!flush) { if (!FILL) a.nit[f] = 0; return; }
    const int64_t kb = (b0 + r + 1) / L - 1;           // batch index among this flush's batches
    const int64_t nexp = a.expired_on ? (kb == 0 ? I.cx : L) : 0;
    if (!FILL) { a.nit[f] = (int32_t)(nexp + 1 + L); return; }
    int64_t k = a.ioff[f];
    if (a.expired_on) {
      if (kb == 0) for (int32_t x = 0; x < I.cx; x++) gwd_put(a.it, k++, GI_EXP, now, I.cxo + x, l, ord);
      else for (int64_t x = (kb - 1) * L; x < kb * L; x++) gwd_put(a.it, k++, GI_EXP, now, q.row(x), l, ord);
    }
    const int32_t rrow = (kb == 0 && I.h0) ? I.r0 : q.row(kb * L);
    gwd_put(a.it, k++, GI_RESET, now, rrow, l, ord);
    for (int64_t x = kb * L; x < kb * L + L; x++) gwd_put(a.it, k++, GI_CUR, q.ts(x), q.row(x), l, ord);
    return;
  }
  // streamCurrentEvents
  const int64_t t = b0 + r;
  const bool flush = t >= L && t % L == 0;
  const int64_t nexp = (flush && a.expired_on) ? L : 0;
  if (!FILL) { a.nit[f] = (int32_t)(nexp + (flush ? 1 : 0) + 1); return; }
  int64_t k = a.ioff[f];
  if (flush) {
    if (a.expired_on) {
      const int64_t base = I.cc + r - L;                  // FIFO index of the batch's first event
      for (int64_t x = base; x < base + L; x++) gwd_put(a.it, k++, GI_EXP, now, q.row(x), l, ord);
    }
    int32_t rrow;
    if (t >= 2 * L) rrow = (int32_t)(a.C + a.byinst[a.st[l] + (r - L + 1)]);   // after the previous flush
    else rrow = I.h0 ? I.r0 : (int32_t)(a.C + a.byinst[a.st[l]]);
    gwd_put(a.it, k++, GI_RESET, now, rrow, l, ord);
  }
  gwd_put(a.it, k, GI_CUR, a.f_ts[f], me, l, ord);
}

// ---- TimeWindowProcessor (:133-169), one instance ----
// Clock points: the filtered events (expiry runs before each one, with its chunk's clock) and the
// Scheduler ticks (a due notifyAt fires one TIMER chunk that expires everything due).  With non-decreasing
// timestamps and clocks, held row j (FIFO = carried queue + new events) leaves at the first clock point
// after its insertion whose clock reaches ts_j + T.
struct GwdTimeArgs {
  int64_t F, C, NT, NC;            // filtered events, carried rows, ticks, clock points (F + NT)
  int64_t T;
  const int32_t* fidx;             // filtered -> event position
  const int64_t* tk_pos;           // tick positions (fire before the event at pos)
  const int64_t* tk_now;
  const int32_t* tk_ord;
  const int64_t* f_ts;
  const int64_t* f_now;
  const int32_t* f_ord;
  const int64_t* c_ts;
  int64_t* cp_now;                 // [NC]
  int32_t* cp_ev;                  // [NC] filtered event or -1 (tick)
  int32_t* cp_ord;                 // [NC]
  int32_t* f_cp;                   // [F] clock point of each filtered event
  int32_t* x;                      // [C + F] expiry clock point (NC: still held)
  int32_t* cnt_exp;                // [NC]
  const int32_t* e_off;            // exclusive scan of cnt_exp
  int32_t* nit;                    // [NC]
  const int32_t* ioff;             // exclusive scan of nit
  GwdItems it;
};

static __global__ void __launch_bounds__(GWD_B) k_gwd_time_cp(GwdTimeArgs a) {
  const int64_t i = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (i < a.F) {
    const int64_t pos = a.fidx[i];
    int64_t lo = 0, hi = a.NT;                    // ticks with pos <= this event's position
    while (lo < hi) { const int64_t m = (lo + hi) >> 1; if (a.tk_pos[m] <= pos) lo = m + 1; else hi = m; }
    const int64_t c = i + lo;
    a.cp_now[c] = a.f_now[i]; a.cp_ev[c] = (int32_t)i; a.cp_ord[c] = a.f_ord[i];
    a.f_cp[i] = (int32_t)c;
  } else if (i < a.F + a.NT) {
    const int64_t t = i - a.F;
    const int64_t pos = a.tk_pos[t];
    int64_t lo = 0, hi = a.F;                     // filtered events before the tick
    while (lo < hi) { const int64_t m = (lo + hi) >> 1; if (a.fidx[m] < pos) lo = m + 1; else hi = m; }
    const int64_t c = t + lo;
    a.cp_now[c] = a.tk_now[t]; a.cp_ev[c] = -1; a.cp_ord[c] = a.tk_ord[t];
  }
}

static __global__ void __launch_bounds__(GWD_B) k_gwd_time_exp(GwdTimeArgs a) {
  const int64_t j = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (j >= a.C + a.F) return;
  const int64_t ins = j < a.C ? -1 : a.f_cp[j - a.C];
  const int64_t lim = (j < a.C ? a.c_ts[j] : a.f_ts[j - a.C]) + a.T;   // expires once the clock reaches it
  int64_t lo = ins + 1, hi = a.NC;
  while (lo < hi) { const int64_t m = (lo + hi) >> 1; if (a.cp_now[m] >= lim) hi = m; else lo = m + 1; }
  a.x[j] = (int32_t)lo;
  if (lo < a.NC) atomicAdd(&a.cnt_exp[lo], 1);
}

static __global__ void __launch_bounds__(GWD_B) k_gwd_time_nit(GwdTimeArgs a) {
  const int64_t c = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (c < a.NC) a.nit[c] = a.cnt_exp[c] + (a.cp_ev[c] >= 0 ? 1 : 0);
}

static __global__ void __launch_bounds__(GWD_B) k_gwd_time_fill(GwdTimeArgs a) {
  const int64_t j = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (j < a.C + a.F) {
    const int32_t c = a.x[j];
    if (c < a.NC) {
      const int64_t k = a.ioff[c] + (j - a.e_off[c]);
      gwd_put(a.it, k, GI_EXP, a.cp_now[c], (int32_t)j, 0, a.cp_ord[c]);
    }
  }
  if (j < a.NC && a.cp_ev[j] >= 0) {
    const int32_t f = a.cp_ev[j];
    gwd_put(a.it, a.ioff[j] + a.cnt_exp[j], GI_CUR, a.f_ts[f], (int32_t)(a.C + f), 0, a.cp_ord[j]);
  }
}

// ---- TimeWindowProcessor per partition instance (current-events output) ----
// Expired rows are invisible without expired output: a tick's removal reaches the aggregates before the
// instance's next CURRENT event either way, so each instance expires at its own events only (the Scheduler's
// map order, which decides which instance a tick drains, plays no part).  Held row j of instance l -- the
// carried queue, then the new events in rank order -- leaves at the instance's first later event whose clock
// reaches ts_j + T.
struct GwdPTimeArgs {
  int64_t F, C, T;
  const int32_t* byinst;
  const int32_t* st;
  const int32_t* cnt;
  const int32_t* f_lid;
  const int32_t* rank;
  const int64_t* f_ts;
  const int64_t* f_now;
  const int32_t* f_ord;
  const int64_t* c_ts;
  const int32_t* c_lid;            // [C] instance of each carried row
  const GwdInst* inst;
  int32_t* x;                      // [C + F] expiry rank inside the instance (cnt[l]: still held)
  int32_t* cnt_exp;                // [F] rows expiring at each filtered event
  const int32_t* es;               // [F + 1] exclusive scan of cnt_exp in instance-sorted order
  int32_t* nit;                    // [F + 1]
  const int32_t* ioff;
  GwdItems it;
};

static __global__ void __launch_bounds__(GWD_B) k_gwd_ptime_exp(GwdPTimeArgs a) {
  const int64_t j = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (j >= a.C + a.F) return;
  const int32_t l = j < a.C ? a.c_lid[j] : a.f_lid[j - a.C];
  const int64_t lim = (j < a.C ? a.c_ts[j] : a.f_ts[j - a.C]) + a.T;
  const int32_t base = a.st[l], n = a.cnt[l];
  int32_t lo = j < a.C ? 0 : a.rank[j - a.C] + 1, hi = n;
  while (lo < hi) {
    const int32_t m = (lo + hi) >> 1;
    if (a.f_now[a.byinst[base + m]] >= lim) hi = m; else lo = m + 1;
  }
  a.x[j] = lo;
  if (lo < n) atomicAdd(&a.cnt_exp[a.byinst[base + lo]], 1);
}

// counts in instance-sorted order (for the exclusive scan) and items per event
static __global__ void __launch_bounds__(GWD_B) k_gwd_ptime_nit(GwdPTimeArgs a, int32_t* __restrict__ sorted_cnt) {
  const int64_t p = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (p >= a.F) return;
  const int32_t f = a.byinst[p];
  sorted_cnt[p] = a.cnt_exp[f];
  a.nit[f] = a.cnt_exp[f] + 1;
}

static __global__ void __launch_bounds__(GWD_B) k_gwd_ptime_fill(GwdPTimeArgs a) {
  const int64_t j = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (j < a.C + a.F) {
    const bool carried = j < a.C;
    const int32_t l = carried ? a.c_lid[j] : a.f_lid[j - a.C];
    const int32_t xr = a.x[j];
    if (xr < a.cnt[l]) {
      const GwdInst& I = a.inst[l];
      const int32_t p = a.st[l] + xr;                 // sorted position of the expiring event
      const int32_t f = a.byinst[p];
      const int64_t fifo = carried ? (j - I.co) : (I.cc + a.rank[j - a.C]);
      const int64_t before = a.es[p] - a.es[a.st[l]];  // rows of the instance expiring at its earlier events
      gwd_put(a.it, a.ioff[f] + (fifo - before), GI_EXP, a.f_now[f], (int32_t)j, l, a.f_ord[f]);
    }
  }
  if (j < a.F) gwd_put(a.it, a.ioff[j] + a.cnt_exp[j], GI_CUR, a.f_ts[j], (int32_t)(a.C + j), a.f_lid[j], a.f_ord[j]);
}

// ---- QuerySelector ----
struct GwdSelArgs {
  int64_t M;
  GwdItems it;
  GwdVals vals;
  int32_t ng;                      // group-by keys (pre-selector value indices)
  int32_t gcol[GWD_MAXG];
  int32_t keyed_lid;               // the instance is part of the aggregator key (partitioned)
  uint64_t* hkey;                  // [M] key hash
  int32_t* iota;
  // sorted by key (stable): item index per sorted position, group segment per position
  const uint64_t* shkey;
  const int32_t* sidx;
  int32_t* head;                   // [M] group head flag
  int32_t* head2;                  // [M] group head or RESET item
  const int32_t* gnum;             // inclusive scan of head: group number + 1 per sorted position
  int32_t* rep;                    // [G] first item of each group
  int32_t* gstart;                 // [G + 1] first sorted position of each group (min / max lanes)
  int32_t* bad;                    // key hash collision
  int32_t* gid;                    // [M] group of each item (item order)
};

__device__ __forceinline__ uint64_t gwd_mix(uint64_t h, uint64_t v) {
  h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
  h ^= h >> 31; h *= 0xbf58476d1ce4e5b9ull; h ^= h >> 29;
  return h;
}

__device__ __forceinline__ void gwd_keyval(const GwdSelArgs& a, int32_t row, int g, int64_t& v, int64_t& n) {
  n = a.vals.nul(a.gcol[g], row);
  v = n ? INT64_MIN : a.vals.val(a.gcol[g], row);
}

static __global__ void __launch_bounds__(GWD_B) k_gwd_hash(GwdSelArgs a) {
  const int64_t i = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (i >= a.M) return;
  uint64_t h = 0x1234567ull;
  if (a.keyed_lid) h = gwd_mix(h, (uint64_t)(uint32_t)a.it.lid[i]);
  const int32_t row = a.it.row[i];
  for (int g = 0; g < a.ng; g++) {
    int64_t v, n;
    gwd_keyval(a, row, g, v, n);
    h = gwd_mix(gwd_mix(h, (uint64_t)v), (uint64_t)n);
  }
  a.hkey[i] = h;
  a.iota[i] = (int32_t)i;
}

static __global__ void __launch_bounds__(GWD_B) k_gwd_heads(GwdSelArgs a, int32_t* __restrict__ rflag) {
  const int64_t p = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (p >= a.M) return;
  const bool h = p == 0 || a.shkey[p] != a.shkey[p - 1];
  const bool rs = a.it.type[a.sidx[p]] == GI_RESET;
  a.head[p] = h;
  a.head2[p] = h || rs;
  rflag[p] = rs;
}

// after the scan of `head` into `gnum` (group number + 1): representative item and group of every item
static __global__ void __launch_bounds__(GWD_B) k_gwd_groups(GwdSelArgs a) {
  const int64_t p = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (p >= a.M) return;
  const int32_t g = a.gnum[p] - 1;
  const int32_t i = a.sidx[p];
  a.gid[i] = g;
  if (p == 0 || a.gnum[p] != a.gnum[p - 1]) { a.rep[g] = i; if (a.gstart) a.gstart[g] = (int32_t)p; }
}

// items sharing a hash must share the key (a collision sends the flush to the host path)
static __global__ void __launch_bounds__(GWD_B) k_gwd_verify(GwdSelArgs a) {
  const int64_t p = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (p >= a.M) return;
  const int32_t i = a.sidx[p], i0 = a.rep[a.gnum[p] - 1];
  if (i == i0) return;
  bool same = !a.keyed_lid || a.it.lid[i] == a.it.lid[i0];
  for (int k = 0; k < a.ng && same; k++) {
    int64_t v0, n0, v1, n1;
    gwd_keyval(a, a.it.row[i0], k, v0, n0);
    gwd_keyval(a, a.it.row[i], k, v1, n1);
    same = v0 == v1 && n0 == n1;
  }
  if (!same) atomicOr(a.bad, 1);
}

// the key fields of each group (host lookup of the carried aggregator states)
static __global__ void __launch_bounds__(GWD_B) k_gwd_repkeys(GwdSelArgs a, int64_t G, int64_t* __restrict__ keys) {
  const int64_t g = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (g >= G) return;
  const int32_t i = a.rep[g];
  const int w = 2 * a.ng + 1;
  for (int k = 0; k < a.ng; k++) {
    int64_t v, n;
    gwd_keyval(a, a.it.row[i], k, v, n);
    keys[g * w + 2 * k] = v;
    keys[g * w + 2 * k + 1] = n;
  }
  keys[g * w + 2 * a.ng] = a.it.lid[i];
}

struct GwdAgg {
  int32_t k;        // SA_SUM / SA_AVG / SA_COUNT
  int32_t arg;      // pre-selector value index (-1 count())
  int32_t in_t;
  int32_t shift;    // fixed point 2^-shift (float / double input); 0 integral
};

// contributions of every sorted position to aggregator a: value (fixed point) and non-null count
static __global__ void __launch_bounds__(GWD_B) k_gwd_contrib(GwdSelArgs s, GwdAgg A, int64_t* __restrict__ xc,
                                                       int64_t* __restrict__ nc) {
  const int64_t p = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (p >= s.M) return;
  const int32_t i = s.sidx[p];
  const int ty = s.it.type[i];
  const int sg = ty == GI_CUR ? 1 : (ty == GI_EXP ? -1 : 0);
  if (A.k == SA_COUNT) { xc[p] = 0; nc[p] = sg; return; }
  const int32_t row = s.it.row[i];
  const bool nul = s.vals.nul(A.arg, row);
  if (nul || sg == 0) { xc[p] = 0; nc[p] = 0; return; }
  const int64_t r = s.vals.val(A.arg, row);
  int64_t v;
  switch (A.in_t) {
    case T_INT: v = (int64_t)(int32_t)r; break;
    case T_LONG: v = r; break;
    case T_FLOAT: v = (int64_t)llrint(ldexp((double)bits_f(r), A.shift)); break;
    default: v = (int64_t)llrint(ldexp(bits_d(r), A.shift)); break;
  }
  xc[p] = sg * v;
  nc[p] = sg;
}

// statistics for the exactness check of a float / double argument: max required shift, max |x|
static __global__ void __launch_bounds__(GWD_B) k_gwd_xstat(int64_t R, GwdVals vals, int32_t arg, int32_t in_t,
                                                     int32_t* __restrict__ need, unsigned long long* __restrict__ mx) {
  const int64_t r = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  int nd = 0;
  unsigned long long m = 0;
  if (r < R && !vals.nul(arg, r)) {
    const int64_t raw = vals.val(arg, r);
    double x;
    switch (in_t) {
      case T_INT: x = (double)(int32_t)raw; break;
      case T_LONG: x = (double)raw; break;
      case T_FLOAT: x = (double)bits_f(raw); break;
      default: x = bits_d(raw); break;
    }
    if (!isfinite(x)) nd = 4096;
    else if (x != 0.0) {
      int e;
      const double fm = frexp(x, &e);
      const uint64_t bits = (uint64_t)__double_as_longlong(ldexp(fabs(fm), 53));
      const int lsb = e - 53 + (__ffsll((long long)bits) - 1);
      nd = lsb < 0 ? -lsb : 0;
      if (in_t == T_LONG && fabs(x) >= 9007199254740992.0) nd = 4096;   // a long not exact as a double
    }
    m = (unsigned long long)__double_as_longlong(fabs(x));
  }
  for (int d = 32; d >= 1; d >>= 1) {
    nd = max(nd, __shfl_xor(nd, d, 64));
    const unsigned long long o = __shfl_xor(m, d, 64);
    m = o > m ? o : m;
  }
  if ((threadIdx.x & 63) == 0) { atomicMax(need, nd); atomicMax(mx, m); }
}

struct GwdAggOutArgs {
  int64_t M;
  const int32_t* sidx;
  const int32_t* head;             // group number + 1 per sorted position
  const int32_t* rcnt;             // RESET items so far in the group (inclusive)
  const int64_t* X;                // scanned value contributions (by group segment and RESET)
  const int64_t* N;                // scanned counts
  const int64_t* init_x;           // [G] carried state
  const int64_t* init_n;
  GwdAgg A;
  int64_t* av;                     // [M] result raw (item order)
  uint8_t* an;
  int64_t* fin_x;                  // [G] state after the group's last item
  int64_t* fin_n;
};

static __global__ void __launch_bounds__(GWD_B) k_gwd_aggout(GwdAggOutArgs a) {
  const int64_t p = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (p >= a.M) return;
  const int32_t g = a.head[p] - 1;
  const bool epoch0 = a.rcnt[p] == 0;
  const int64_t x = a.X[p] + (epoch0 ? a.init_x[g] : 0);
  const int64_t n = a.N[p] + (epoch0 ? a.init_n[g] : 0);
  const int32_t i = a.sidx[p];
  int64_t v = 0;
  bool nul = false;
  switch (a.A.k) {
    case SA_COUNT: v = n; break;
    case SA_SUM:
      nul = n == 0;
      if (!nul) v = (a.A.in_t == T_INT || a.A.in_t == T_LONG) ? x : d_bits(ldexp((double)x, -a.A.shift));
      break;
    default:   // SA_AVG
      nul = n == 0;
      if (!nul) v = d_bits(ldexp((double)x, -a.A.shift) / (double)n);
      break;
  }
  a.av[i] = v;
  a.an[i] = (uint8_t)nul;
  if (p == a.M - 1 || a.head[p + 1] != a.head[p]) { a.fin_x[g] = x; a.fin_n[g] = n; }
}

// ---- min / max: one lane per group replays the aggregator's deque (Min/MaxAttributeAggregatorExecutor:
// with trackFutureStates a monotone deque, EXPIRED removes the first element equal to the value --
// Float/Double.equals -- whether or not it is the same event; without it the running extreme, cleared when
// an EXPIRED value equals it).  The group's items are contiguous in the sorted order.
struct GwdMinMaxArgs {
  int64_t G;
  const int32_t* gstart;           // [G + 1] first sorted position of each group
  const int32_t* sidx;
  GwdItems it;
  GwdVals vals;
  int32_t arg, in_t, is_min, track;
  const int32_t* dq_off;           // [G + 1] carried deque of each group: rows [dq_off[g], dq_off[g + 1]) of dq_in
  const int64_t* dq_in;
  const int64_t* mv0;              // [G] carried extreme
  const uint8_t* mvn0;
  const int64_t* wo;               // [G + 1] workspace offsets (carried deque + the group's items)
  int64_t* ws;
  int64_t* av;                     // [M] result per item (item order)
  uint8_t* an;
  int64_t* fin_mv;                 // [G]
  uint8_t* fin_mvn;
  int32_t* fin_h;                  // [G] final deque: ws[wo[g] + fin_h[g] .. wo[g] + fin_t[g])
  int32_t* fin_t;
};

__device__ __forceinline__ bool gwd_lt(int t, int64_t a, int64_t b) {
  switch (t) {
    case T_INT: return (int32_t)a < (int32_t)b;
    case T_LONG: return a < b;
    case T_FLOAT: return bits_f(a) < bits_f(b);
    default: return bits_d(a) < bits_d(b);
  }
}
__device__ __forceinline__ bool gwd_eq(int t, int64_t a, int64_t b) {
  if (t == T_FLOAT) { const float x = bits_f(a), y = bits_f(b); if (x != x && y != y) return true; return (uint32_t)a == (uint32_t)b; }
  if (t == T_DOUBLE) { const double x = bits_d(a), y = bits_d(b); if (x != x && y != y) return true; return a == b; }
  if (t == T_INT) return (int32_t)a == (int32_t)b;
  return a == b;
}

static __global__ void __launch_bounds__(64) k_gwd_minmax(GwdMinMaxArgs a) {
  const int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (g >= a.G) return;
  int64_t* q = a.ws + a.wo[g];
  int32_t h = 0, t = 0;
  for (int32_t k = a.dq_off[g]; k < a.dq_off[g + 1]; k++) q[t++] = a.dq_in[k];
  int64_t mv = a.mv0[g];
  bool mvn = a.mvn0[g] != 0;
  const int ty = a.in_t;
  for (int32_t p = a.gstart[g]; p < a.gstart[g + 1]; p++) {
    const int32_t i = a.sidx[p];
    const int type = a.it.type[i];
    if (type == GI_RESET) { h = t = 0; mvn = true; a.av[i] = 0; a.an[i] = 1; continue; }
    const int32_t row = a.it.row[i];
    if (a.vals.nul(a.arg, row)) { a.av[i] = mv; a.an[i] = mvn; continue; }
    const int64_t in = a.vals.val(a.arg, row);
    if (type == GI_CUR) {
      if (a.track) {
        while (t > h && (a.is_min ? gwd_lt(ty, in, q[t - 1]) : gwd_lt(ty, q[t - 1], in))) t--;
        q[t++] = in;
      }
      if (mvn || (a.is_min ? gwd_lt(ty, in, mv) : gwd_lt(ty, mv, in))) { mv = in; mvn = false; }
    } else if (a.track) {
      for (int32_t k = h; k < t; k++)
        if (gwd_eq(ty, q[k], in)) {                 // erase: shift the front part up by one
          for (int32_t x = k; x > h; x--) q[x] = q[x - 1];
          h++;
          break;
        }
      mvn = h == t;
      if (!mvn) mv = q[h];
    } else if (!mvn && gwd_eq(ty, mv, in)) {
      mvn = true;
    }
    a.av[i] = mv;
    a.an[i] = mvn;
  }
  a.fin_mv[g] = mv; a.fin_mvn[g] = mvn; a.fin_h[g] = h; a.fin_t[g] = t;
}

struct GwdOutArgs {
  int64_t M;
  GwdItems it;
  GwdVals vals;
  int32_t naggs;
  const int64_t* av;               // [naggs][M]
  const uint8_t* an;
  int32_t nout;
  int32_t akind[GWD_MAXOUT];       // 0 plain (value index aidx), 2 program aidx
  int32_t aidx[GWD_MAXOUT];
  const Prog* progs;               // sp.host
  int32_t has_having;
  const Prog* having;
  int32_t current_on, expired_on;
  int64_t* out;                    // [M][nout]
  uint8_t* onul;
  uint8_t* pass;                   // [M]
};

struct GwdLoader {
  const GwdOutArgs* a;
  int64_t i;
  int32_t row;
  __device__ bool load(int slot, int attr, int64_t& v) const {
    if (slot == 255) {
      if (attr < 0 || attr >= a->nout || a->onul[i * a->nout + attr]) return false;
      v = a->out[i * a->nout + attr];
      return true;
    }
    if (slot == 254) {
      if (a->an[(int64_t)attr * a->M + i]) return false;
      v = a->av[(int64_t)attr * a->M + i];
      return true;
    }
    if (a->vals.nul(attr, row)) return false;
    v = a->vals.val(attr, row);
    return true;
  }
};

static __global__ void __launch_bounds__(GWD_B) k_gwd_out(GwdOutArgs a) {
  __shared__ int64_t rf[MAX_REG * GWD_B];
  const int64_t i = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (i >= a.M) return;
  const int ty = a.it.type[i];
  if (ty == GI_RESET) { a.pass[i] = 0; return; }
  const int32_t row = a.it.row[i];
  GwdLoader ld{&a, i, row};
  for (int k = 0; k < a.nout; k++) {
    int64_t v = 0;
    bool nul;
    if (a.akind[k] == 0) {
      nul = a.vals.nul(a.aidx[k], row);
      v = a.vals.val(a.aidx[k], row);
    } else {
      nul = true;
      run(a.progs[a.aidx[k]], ld, v, nul, rf + threadIdx.x, GWD_B);
    }
    a.out[i * a.nout + k] = v;
    a.onul[i * a.nout + k] = (uint8_t)nul;
  }
  bool ok = (ty == GI_CUR && a.current_on) || (ty == GI_EXP && a.expired_on);
  if (ok && a.has_having) ok = run_pred(*a.having, ld, rf + threadIdx.x, GWD_B);
  a.pass[i] = (uint8_t)ok;
}

// held new rows (the window state the host keeps for the next flush): rank >= hold_from[instance]
static __global__ void __launch_bounds__(GWD_B) k_gwd_held(int64_t F, const int32_t* __restrict__ byinst,
                                                    const int32_t* __restrict__ f_lid, const int32_t* __restrict__ rank,
                                                    const int32_t* __restrict__ hold_from, const int32_t* __restrict__ x,
                                                    int64_t C, int64_t NC, uint8_t* __restrict__ held) {
  const int64_t p = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (p >= F) return;
  const int32_t f = byinst[p];
  if (NC < 0) held[p] = (uint8_t)(x[C + f] >= hold_from[f_lid[f]]);   // partitioned time: hold_from = the count
  else held[p] = x ? (uint8_t)(x[C + f] >= NC) : (uint8_t)(rank[f] >= hold_from[f_lid[f]]);
}

// rows of selected positions packed for the host: [ts, value row values..] of the held rows
static __global__ void __launch_bounds__(GWD_B) k_gwd_pack_held(int64_t H, const int32_t* __restrict__ hpos,
                                                         const int32_t* __restrict__ byinst, int64_t C, int64_t R,
                                                         int32_t nv, const int64_t* __restrict__ vt,
                                                         const uint8_t* __restrict__ vn, const int64_t* __restrict__ f_ts,
                                                         const int32_t* __restrict__ f_lid, int64_t* __restrict__ o,
                                                         uint8_t* __restrict__ on, int32_t* __restrict__ ol) {
  const int64_t h = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (h >= H) return;
  const int32_t f = byinst[hpos[h]];
  o[h * (nv + 1)] = f_ts[f];
  for (int k = 0; k < nv; k++) {
    o[h * (nv + 1) + 1 + k] = vt[(int64_t)k * R + C + f];
    on[h * nv + k] = vn[(int64_t)k * R + C + f];
  }
  ol[h] = f_lid[f];
}

// selected items packed for the host: ts, type, chunk, group and the output row
static __global__ void __launch_bounds__(GWD_B) k_gwd_pack_out(int64_t P, const int32_t* __restrict__ pidx, GwdItems it,
                                                        const int32_t* __restrict__ gid, int32_t nout,
                                                        const int64_t* __restrict__ out, const uint8_t* __restrict__ onul,
                                                        int64_t* __restrict__ o_ts, int32_t* __restrict__ o_meta,
                                                        int64_t* __restrict__ o_raw, uint8_t* __restrict__ o_nul) {
  const int64_t q = (int64_t)blockIdx.x * GWD_B + threadIdx.x;
  if (q >= P) return;
  const int32_t i = pidx[q];
  o_ts[q] = it.ts[i];
  o_meta[3 * q] = it.type[i];
  o_meta[3 * q + 1] = it.ord[i];
  o_meta[3 * q + 2] = gid ? gid[i] : 0;
  for (int k = 0; k < nout; k++) {
    o_raw[q * nout + k] = out[(int64_t)i * nout + k];
    o_nul[q * nout + k] = onul[(int64_t)i * nout + k];
  }
}

}  // namespace sg
