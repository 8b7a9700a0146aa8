// nfa.hip — execution path SG_PATH_NFA: the general pattern / sequence engine.
//
// Covers every StateElement shape the followed-by path does not: count / Kleene states
// (<n:m>, +, *, ?), logical and/or, sequences (strict contiguity), non-`every` starts, nested
// every, multi-stream patterns and `partition with (attr of S)`, and absent states (`not S[f] for
// T`, AbsentStreamPreStateProcessor.java:35-343) in unpartitioned queries: a lane's timeline
// interleaves its events with the app's Scheduler ticks (every playback send whose timestamp
// advances the clock, every sleep / advance_time: TimestampGeneratorImpl.java:78-122), and each tick
// fires the lane's due deadlines per absent processor, earliest first (Scheduler.java:64-212).  In a
// partitioned query the Scheduler keeps one partition instance per distinct deadline
// (SchedulerState.compareTo == 0), which couples the keys' lanes: such queries are not lowered.
//
// Design.  The NFA is the processor graph StateInputStreamParser builds
// (CORE/util/parser/StateInputStreamParser.java:148-408), lowered on the host to a flat table:
// per pre/post processor pair its kind, slot, links (next / every / within-every / callback /
// logical partner), count bounds and filter bytecode, plus the init / reset / update orders of the
// InnerStateRuntime tree and the receivers' processor lists.  One device lane runs one partition
// instance (PartitionStateHolder keys, CORE/util/snapshot/state/PartitionStateHolder.java:43-49):
// it walks that key's events in arrival order and executes the exact per-event algorithm of
// MultiProcessStreamReceiver / SingleProcessStreamReceiver (stabilize = expire + update or
// reset+update, then the receiver's processors in reverse setup order).  The Java object graph is
// restated with fixed-capacity, reference-counted pools in HBM (struct-of-arrays over lanes, so the
// lanes of a wave touch consecutive addresses):
//   StateEvent   slots[S] (chain heads), ts, type            StateEvent.java:42-258
//   StreamEvent  event index + next (chains of count states) StreamEvent.java, StateEvent.addEvent :212-222
//   lists        pending / newAndEvery per processor         StreamPreStateProcessor.java:435-498
// Shared objects stay shared (logical partners, the count self/next lists, shallow clones of
// addEveryState share chain heads), so the reference's aliasing quirks reproduce bit for bit.
// A pool overflow raises SG_E_CAPACITY — never a silently different result.
// Matches are projected on the device (select bytecode) and tagged with (trigger event,
// receiver holder, order) so the host can rebuild the reference's callback grouping.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <thread>
#include <tuple>
#include <unordered_map>

#include "runtime.hpp"
#include "selector.hpp"
#include "selector_dev.hpp"

#include "nfa_rtc.hpp"

namespace sg {

// Tick indexes of one launch (NArgs::tick_ub / tick_lb), one binary search per rank and per millisecond of
// the ticks' clock range, all in parallel (the lanes then look each up with one load).
__global__ void __launch_bounds__(256) k_nfa_tick_index(const int64_t* __restrict__ tick_now,
                                                         const int32_t* __restrict__ tick_ev, int32_t nt, int64_t x0,
                                                         int64_t nx, int32_t* __restrict__ ub, int64_t t0, int64_t ntm,
                                                         int32_t* __restrict__ lb) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < max(nx, ntm); i += stride) {
    if (i < nx) {
      const int64_t x = x0 + i;
      int lo = 0, hi = nt;
      while (lo < hi) { const int mid = (lo + hi) >> 1; if (tick_ev[mid] > x) hi = mid; else lo = mid + 1; }
      ub[i] = lo;
    }
    if (i < ntm) {
      const int64_t t = t0 + i;
      int lo = 0, hi = nt;
      while (lo < hi) { const int mid = (lo + hi) >> 1; if (tick_now[mid] >= t) hi = mid; else lo = mid + 1; }
      lb[i] = lo;
    }
  }
}


// several device copies in one launch (the exact sweep's pool checkpoints: NfaExec::pools_copy); addresses are
// 4-byte aligned, a length that is not a multiple of 4 ends with single bytes
struct CopySegs {
  static constexpr int MAX = 32;
  const uint8_t* src[MAX];
  uint8_t* dst[MAX];
  size_t bytes[MAX];
  int n;
};
__global__ void __launch_bounds__(256) k_copy_segs(CopySegs c) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (int k = 0; k < c.n; k++) {
    const size_t nw = c.bytes[k] / 4;
    const uint32_t* s = (const uint32_t*)c.src[k];
    uint32_t* d = (uint32_t*)c.dst[k];
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += stride) d[i] = s[i];
    if (blockIdx.x == 0 && threadIdx.x < (c.bytes[k] & 3)) c.dst[k][nw * 4 + threadIdx.x] = c.src[k][nw * 4 + threadIdx.x];
  }
}

// the exact sweep's round: the deferred instances' pools back to the window's checkpoint (element x of lane l at
// [x * L + l] in each pool and in its checkpoint copy)
struct LaneSegs {
  static constexpr int MAX = 32;
  const uint8_t* ck[MAX];
  uint8_t* pool[MAX];
  int64_t per[MAX];
  int32_t esz[MAX];
  int n;
};
__global__ void __launch_bounds__(256) k_restore_lanes(LaneSegs g, const int32_t* __restrict__ lanes, int nd, int64_t L) {
  const int k = blockIdx.x;
  if (k >= g.n) return;
  const int64_t tot = g.per[k] * nd;
  const int e = g.esz[k];
  for (int64_t i = threadIdx.x; i < tot; i += blockDim.x) {
    const int64_t o = ((i / nd) * L + lanes[i % nd]) * e;
    for (int b = 0; b < e; b++) g.pool[k][o + b] = g.ck[k][o + b];
  }
}
// the sweep's base pools (saved with Ls lanes) back into the pools of Ld >= Ls lanes
__global__ void __launch_bounds__(256) k_pools_relayout(LaneSegs g, int64_t Ls, int64_t Ld) {
  const int k = blockIdx.y;
  if (k >= g.n) return;
  const int64_t tot = g.per[k] * Ls;
  const int e = g.esz[k];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = i / Ls, l = i % Ls;
    for (int b = 0; b < e; b++) g.pool[k][(x * Ld + l) * e + b] = g.ck[k][(x * Ls + l) * e + b];
  }
}
// and the records those instances wrote in the window [r0, r1) superseded (task 0, which emit drops)
__global__ void k_rec_supersede(const int32_t* __restrict__ rec_lane, int32_t* __restrict__ rec_task, int64_t r0,
                                int64_t r1, const int32_t* __restrict__ lanes, int nd) {
  const int64_t k = r0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= r1) return;
  const int32_t l = rec_lane[k];
  for (int i = 0; i < nd; i++)
    if (lanes[i] == l) { rec_task[k] = 0; return; }
}

__global__ void k_nfa_iota(int32_t* out, int32_t v0, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[k] = v0 + (int32_t)k;
}

__global__ void k_nfa_gather_ts(const int64_t* __restrict__ ts, const int32_t* __restrict__ idx, int64_t m,
                                int64_t* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < m) out[k] = ts[idx[k]];
}

__global__ void k_nfa_ev_fill(int8_t* st, int32_t* row, int64_t* now, int8_t ls, int32_t row0, int64_t now_v,
                              int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  st[k] = ls;
  row[k] = row0 + (int32_t)k;
  if (now) now[k] = now_v;
}

__global__ void k_nfa_pool_init(NState s, int64_t lane0, int64_t nlanes) {
  int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nlanes) return;
  nfa_pool_init_one(s, lane0 + q);
}

// copy lane sl of src into lane dl of dst (every pool; a verified speculative end state becomes the
// instance's state)
__global__ void k_nfa_lane_xfer(NState dst, NState src_all, const int32_t* __restrict__ pairs, int32_t npairs,
                                int32_t blocked) {
  // the scratch lanes may run with smaller pools: ids below the source capacities keep their meaning, and
  // the ids the source never had join the destination's free stacks
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= npairs) return;
  const int64_t dl = pairs[2 * k];
  int64_t sl = pairs[2 * k + 1];
  const NState src = blocked ? nfa_block_view(src_all, sl >> 6) : src_all;   // (blocked scratch pools: the lane's block)
  if (blocked) sl &= 63;
  auto cp = [&](auto* dp, auto* sp, int64_t n) { for (int64_t x = 0; x < n; x++) dp[x * dst.L + dl] = sp[x * src.L + sl]; };
  cp(dst.se_slot, src.se_slot, (int64_t)src.se_cap * NS); cp(dst.se_ts, src.se_ts, src.se_cap);
  cp(dst.se_type, src.se_type, src.se_cap); cp(dst.se_ref, src.se_ref, src.se_cap);
  cp(dst.nd_ev, src.nd_ev, src.nd_cap); cp(dst.nd_next, src.nd_next, src.nd_cap); cp(dst.nd_ref, src.nd_ref, src.nd_cap);
  int32_t top = src.se_top[sl];
  for (int32_t x = 0; x < top; x++) dst.se_free[(int64_t)x * dst.L + dl] = src.se_free[(int64_t)x * src.L + sl];
  for (int32_t id = src.se_cap; id < dst.se_cap; id++) dst.se_free[(int64_t)(top++) * dst.L + dl] = id;
  dst.se_top[dl] = top;
  top = src.nd_top[sl];
  for (int32_t x = 0; x < top; x++) dst.nd_free[(int64_t)x * dst.L + dl] = src.nd_free[(int64_t)x * src.L + sl];
  for (int32_t id = src.nd_cap; id < dst.nd_cap; id++) dst.nd_free[(int64_t)(top++) * dst.L + dl] = id;
  dst.nd_top[dl] = top;
  for (int p = 0; p < NP; p++)
    for (int x = 0; x < src.list_cap; x++) {
      dst.pend[((int64_t)p * dst.list_cap + x) * dst.L + dl] = src.pend[((int64_t)p * src.list_cap + x) * src.L + sl];
      dst.nev[((int64_t)p * dst.list_cap + x) * dst.L + dl] = src.nev[((int64_t)p * src.list_cap + x) * src.L + sl];
    }
  cp(dst.npend, src.npend, NP); cp(dst.nnev, src.nnev, NP); cp(dst.flags, src.flags, NP);
  cp(dst.created, src.created, 1); cp(dst.err, src.err, 1); cp(dst.lst, src.lst, NP);
  cp(dst.tq, src.tq, (int64_t)src.nq * NTQ); cp(dst.ntq, src.ntq, src.nq);
  cp(dst.tqc, src.tqc, (int64_t)src.nq * NTQ); cp(dst.tqh, src.tqh, src.nq);
}

// verification: task q > first of its key is valid when its post-warm-up state equals the end state of q - 1
__global__ void k_nfa_spec_verify(const int32_t* __restrict__ prev, const int32_t* __restrict__ canon, int32_t ntask,
                                  uint8_t* __restrict__ ok) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= ntask) return;
  if (prev[q] < 0) { ok[q] = 1; return; }            // the key's first segment: runs from the true state
  const int32_t* wq = canon + (size_t)q * 2 * (SG_CANON + 1);
  const int32_t* fp = canon + (size_t)prev[q] * 2 * (SG_CANON + 1) + SG_CANON + 1;
  const int32_t n = wq[0];
  bool eq = n >= 0 && fp[0] == n;
  for (int k = 1; eq && k <= n; k++) eq = wq[k] == fp[k];
  ok[q] = eq ? 1 : 0;
}

// Scheduler-collision pre-check on the device (NfaExec::flush): one 64-bit key per logged firing -- tick (relative to
// the launch) << 32 | scheduler << 24 | the head deadline's low 24 bits -- so that two firings under one (tick,
// scheduler, head) have equal keys; firings of speculative segments that did not verify get unique keys (bit 63
// and their index).  After a radix sort, equal neighbours mean a possible collision (an alias of two heads only
// sends the flush to the exact host check).
__global__ void k_fire_keys(const FireRec* __restrict__ f, int64_t n, const uint8_t* __restrict__ task_ok,
                            uint64_t* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const FireRec r = f[i];
  const bool gone = task_ok && r.task >= 0 && !task_ok[r.task];
  keys[i] = gone ? ((1ull << 63) | (uint64_t)i)
                 : ((uint64_t)(uint32_t)r.tau << 32) | ((uint64_t)(uint8_t)r.sched << 24) | ((uint64_t)r.head & 0xffffffull);
}
__global__ void k_adj_dup(const uint64_t* __restrict__ k, int64_t n, uint32_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i + 1 >= n) return;
  if (k[i] == k[i + 1] && !(k[i] >> 63)) atomicOr(flag, 1u);
}

// repair round (NfaExec::run_spec): fix task i re-ran a segment from the key's true state; the next segment (task
// nxt[i], -1: none) stands if its post-warm-up state equals that true end state
__global__ void k_nfa_fix_verify(const int32_t* __restrict__ fcanon, const int32_t* __restrict__ canon,
                                 const int32_t* __restrict__ nxt, int32_t nfix, uint8_t* __restrict__ ok) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nfix) return;
  if (nxt[i] < 0) { ok[i] = 0; return; }
  const int32_t* fe = fcanon + (size_t)i * 2 * (SG_CANON + 1) + SG_CANON + 1;
  const int32_t* wq = canon + (size_t)nxt[i] * 2 * (SG_CANON + 1);
  const int32_t n = wq[0];
  bool eq = n >= 0 && fe[0] == n;
  for (int k = 1; eq && k <= n; k++) eq = wq[k] == fe[k];
  ok[i] = eq ? 1 : 0;
}

// The launch's events packed lane-major (NEvRec, one per CSR entry): the per-event fields nfa_run_lane reads, gathered
// by one thread per entry with full occupancy, so that each lane then streams its events from consecutive records.
// The attributes are read exactly as Lane::prefetch_attrs reads them (8-B columns whole, 4-B ones sign-extended).
__device__ __forceinline__ NEvRec nfa_pack_rec(const NArgs& a, const NCols* __restrict__ cols, int x) {
  NEvRec r;
  r.x = x;
  r.ts = a.ev_ts[x];
  r.rank = a.ev_rank[x];
  r.row = a.ev_row[x];
  const int st = a.ev_stream[x];
  r.stream = (int8_t)st;
  r.skip = a.ev_skip ? a.ev_skip[x] : (uint16_t)0;
  const int64_t ro = (int64_t)r.rank - a.tub0;
  r.tub = a.tick_ub && ro >= 0 && ro < a.ntub ? a.tick_ub[ro] : -1;
  r.cok = cols->nul[st] ? 0 : 1;
  const int na = cols->na[st];
#pragma unroll
  for (int k = 0; k < NFA_CA; k++) {
    int64_t v = 0;
    if (k < na) {
      const uint8_t* col = cols->col[st][k];
      v = cols->w[st][k] == 8 ? ((const int64_t*)col)[r.row] : (int64_t)((const int32_t*)col)[r.row];
    }
    r.v[k] = v;
  }
  r.pad = 0;
  return r;
}

// one thread per CSR entry: the entry's event fields gathered at random event indices (any CSR, broadcast events
// placed in several lanes included)
__global__ void __launch_bounds__(256) k_nfa_pack(NArgs a, const NCols* __restrict__ cols, int64_t ne,
                                                  NEvRec* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ne) return;
  out[e] = nfa_pack_rec(a, cols, a.lane_ev[e]);
}

// A CSR where every event has at most one entry (no broadcast stream): the entry of each event, then one thread per
// event in store order, so the per-event arrays and columns are read in order (the gather form reads a 64-B sector
// per field per entry: 19 GB per config-5 step for 1.3 GB of records) and each record is one 64-B store
__global__ void __launch_bounds__(256) k_nfa_inv(const int32_t* __restrict__ lane_ev, int64_t ne,
                                                 int32_t* __restrict__ inv) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < ne) inv[lane_ev[i]] = (int32_t)i;
}
__global__ void __launch_bounds__(256) k_nfa_pack_ev(NArgs a, const NCols* __restrict__ cols, int64_t x0, int64_t x1,
                                                     const int32_t* __restrict__ inv, NEvRec* __restrict__ out) {
  const int64_t x = x0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= x1) return;
  const int32_t i = inv[x];
  if (i >= 0) out[i] = nfa_pack_rec(a, cols, (int)x);
}

// ------------------------------------------------------------------------------------------------
// Host side: table builder (StateInputStreamParser.parse restated) and executor
// ------------------------------------------------------------------------------------------------
struct NBuilder {
  NTable& t;
  std::vector<const J*> filters;   // per processor
  bool seq;
  int np = 0;
  std::string err;

  struct In { int k; int first, last; std::vector<std::string> streams; std::vector<int> firsts; int a = -1, b = -1; };
  std::vector<In> ins;

  int new_proc(int kind) {
    if (np >= NP) throw CompileError("too many states for the device NFA table");
    NProc& P = t.p[np];
    std::memset(&P, 0, sizeof(P));
    P.kind = (int8_t)kind;
    P.withinEvery = P.thisLast = P.partner = P.nextPre = P.nextEveryPre = P.callbackPre = P.partnerPost = -1;
    P.filter = -1;
    P.absIdx = -1;
    P.thisLast = (int8_t)np;
    filters.push_back(nullptr);
    return np++;
  }

  void set_next(int post, int pre) {            // Post.setNextStatePre (+ Logical / Count overrides)
    NProc& P = t.p[post];
    P.nextPre = (int8_t)pre;
    if (P.kind == K_LOGICAL) t.p[P.partnerPost].nextPre = (int8_t)pre;
    if (P.kind == K_COUNT && P.isStart && seq && P.minCount == 0) t.p[pre].callbackPre = (int8_t)post;
  }
  void set_next_every(int post, int pre) {
    NProc& P = t.p[post];
    P.nextEveryPre = (int8_t)pre;
    if (P.kind == K_LOGICAL) t.p[P.partnerPost].nextEveryPre = (int8_t)pre;
  }

  // returns inner-runtime index
  int parse(const J& el, int pre, std::vector<int>& preList, bool isStart, std::map<std::string, int>& sidx) {
    const std::string& k = el["k"].s;
    if (k == "stream" || k == "absent") {
      const bool own = pre < 0;
      if (own) pre = new_proc(k == "absent" ? K_ABSENT : K_STREAM);
      NProc& P = t.p[pre];
      if (k == "absent" && own) {      // AbsentStreamPreStateProcessor + its Scheduler (parse order)
        t.waiting[pre] = el["wait"].as_int();
        P.absIdx = (int8_t)t.nabs;
        t.absOrder[t.nabs++] = (int8_t)pre;
      }
      P.stateId = (int8_t)el["slot"].as_int();
      P.isStart = isStart;
      filters[pre] = &el["filters"];
      P.thisLast = (int8_t)pre;
      In in;
      in.k = 0; in.first = pre; in.last = pre;
      in.streams.push_back(el["stream"].s);
      in.firsts.push_back(pre);
      preList.push_back(pre);
      ins.push_back(in);
      return (int)ins.size() - 1;
    }
    if (k == "next") {
      int a = parse(el["a"], pre, preList, isStart, sidx);
      int b = parse(el["b"], pre, preList, false, sidx);
      set_next(ins[a].last, ins[b].first);
      In in;
      in.k = 1; in.first = ins[a].first; in.last = ins[b].last; in.a = a; in.b = b;
      ins.push_back(in);
      return (int)ins.size() - 1;
    }
    if (k == "every") {
      std::vector<int> withinEvery;
      int a = parse(el["e"], pre, withinEvery, isStart, sidx);
      In in;
      in.k = 2; in.first = ins[a].first; in.last = ins[a].last; in.a = a;
      set_next_every(in.last, in.first);
      for (int p : withinEvery) t.p[p].withinEvery = (int8_t)in.first;
      for (int p : withinEvery) preList.push_back(p);
      ins.push_back(in);
      return (int)ins.size() - 1;
    }
    if (k == "logical") {
      bool isAnd = el["op"].s == "AND";
      int p1 = new_proc(K_LOGICAL), p2 = new_proc(K_LOGICAL);
      // AbsentLogicalPreStateProcessor for a `not S[f] [for T]` side; its Scheduler is created with the
      // processor, element 1 before element 2 (StateInputStreamParser.java:289-335)
      const J* sides[2] = {&el["a"], &el["b"]};
      const int procs[2] = {p1, p2};
      for (int z = 0; z < 2; z++) {
        if ((*sides[z])["k"].s != "absent") continue;
        const int pz = procs[z];
        t.p[pz].absLog = 1;
        t.waiting[pz] = (*sides[z])["wait"].null() ? -1 : (*sides[z])["wait"].as_int();
        t.p[pz].absIdx = (int8_t)t.nabs;
        t.absOrder[t.nabs++] = (int8_t)pz;
      }
      t.p[p1].isAnd = t.p[p2].isAnd = isAnd;
      t.p[p1].partner = (int8_t)p2; t.p[p2].partner = (int8_t)p1;
      t.p[p1].partnerPost = (int8_t)p2; t.p[p2].partnerPost = (int8_t)p1;
      int r2 = parse(el["b"], p2, preList, isStart, sidx);
      int r1 = parse(el["a"], p1, preList, isStart, sidx);
      In in;
      in.k = 3; in.first = ins[r1].first; in.last = ins[r2].last; in.a = r1; in.b = r2;
      ins.push_back(in);
      return (int)ins.size() - 1;
    }
    if (k == "count") {
      int mn = (int)el["min"].as_int(), mx = (int)el["max"].as_int();
      if (mn == -1) mn = 0;
      if (mx == -1) mx = INT32_MAX;
      int p = new_proc(K_COUNT);
      t.p[p].minCount = mn;
      t.p[p].maxCount = mx;
      int r = parse(el["e"], p, preList, isStart, sidx);
      ins[r].k = 4;
      return r;
    }
    throw CompileError("unknown state element " + k);
  }

  void orders(int r, std::vector<int>& init, std::vector<int>& reset, std::vector<int>& update) {
    const In& in = ins[r];
    switch (in.k) {
      case 0: case 4: init.push_back(in.first); break;
      case 1: orders(in.a, init, reset, update); orders(in.b, init, reset, update); break;
      case 2: orders(in.a, init, reset, update); break;
      case 3: orders(in.b, init, reset, update); orders(in.a, init, reset, update); break;
    }
  }
  void resets(int r, std::vector<int>& out) {
    const In& in = ins[r];
    switch (in.k) {
      case 0: case 4: case 2: out.push_back(in.first); break;
      case 1: resets(in.b, out); resets(in.a, out); break;
      case 3: resets(in.b, out); break;
    }
  }
  void updates(int r, std::vector<int>& out) {
    const In& in = ins[r];
    switch (in.k) {
      case 0: case 4: case 2: out.push_back(in.first); break;
      case 1: updates(in.a, out); updates(in.b, out); break;
      case 3: updates(in.b, out); break;
    }
  }
  void sel_last(int r) {                         // setQuerySelector
    const In& in = ins[r];
    switch (in.k) {
      case 0: case 4: t.p[in.last].hasNext = 1; break;
      case 1: sel_last(in.b); break;
      case 2: sel_last(in.a); break;
      case 3: sel_last(in.b); sel_last(in.a); break;
    }
  }
  void setup(int r, std::vector<std::vector<int>>& nexts, std::map<std::string, int>& sidx) {
    const In& in = ins[r];
    switch (in.k) {
      case 0: case 4: nexts[sidx.at(in.streams[0])].push_back(in.first); break;
      case 1: setup(in.a, nexts, sidx); setup(in.b, nexts, sidx); break;
      case 2: setup(in.a, nexts, sidx); break;
      case 3: setup(in.b, nexts, sidx); setup(in.a, nexts, sidx); break;
    }
  }
};

// ---- event prefilter (NArgs::ev_skip) ----
// In a pattern (not a sequence) an event a processor's filter rejects leaves the processor's partials as they
// were: each gets the event in its slot, fails, and loses it again (StreamPreStateProcessor.processAndReturn
// :363-403 with stateChanged false; AbsentStreamPreStateProcessor and the AND of LogicalPreStateProcessor
// alike).  When the filter reads only the arriving event, its verdict is the same for every partial and can be
// taken once per event, before the lanes run: the lane then skips that processor for the event.  Count
// states (removeIfNextStateProcessed on every arrival), OR and absent logical states are never skipped.
struct NfaPfLoader {
  const NCols* c;
  int st;
  int64_t row;
  __device__ bool load(int code, int attr, int64_t& v) const {
    const int chain = (code & 15) - 8;     // the slot holds the arriving event alone: [0] and [last] are it
    if (chain != 0 && chain != -1) return false;
    if (c->nul[st] && c->nul[st][row * c->na[st] + attr]) return false;
    const uint8_t* col = c->col[st][attr];
    v = c->w[st][attr] == 8 ? ((const int64_t*)col)[row] : (int64_t)((const int32_t*)col)[row];
    return true;
  }
};
__global__ void __launch_bounds__(256) k_nfa_prefilter(int64_t e0, int64_t e1, const int8_t* __restrict__ ev_stream,
                                                       const int32_t* __restrict__ ev_row, const NTable* __restrict__ tab,
                                                       const NCols* __restrict__ cols, const Prog* __restrict__ progs,
                                                       const uint8_t* __restrict__ elig, uint16_t* __restrict__ skip) {
  __shared__ int64_t rf[MAX_REG * 256];
  const int64_t e = e0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= e1) return;
  const int st = ev_stream[e];
  uint32_t m = 0;
  for (int k = 0; k < tab->nnext[st]; k++) {
    if (!elig[st * NP + k]) continue;
    const NProc& P = tab->p[tab->nexts[st][k]];
    NfaPfLoader ld{cols, st, ev_row[e]};
    if (!run_pred(progs[P.filter], ld, rf + threadIdx.x, 256)) m |= 1u << k;
  }
  skip[e] = (uint16_t)m;
}

// ---- event-store compaction (NfaExec::compact) ----
// After a flush the only references into the event store are the chain nodes of the instances' pools.  A node
// is allocated unless its lane's free stack holds it (a free node's fields are stale, and a never-used one's
// are whatever the allocation held); an allocated node names its event (nd_ev).  Those events are kept.
__global__ void __launch_bounds__(256) k_nfa_free_nodes(NState g, uint8_t* __restrict__ fr) {
  const int64_t l = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (l >= g.L) return;
  const int32_t top = g.nd_top[l];
  for (int32_t x = 0; x < top && x < g.nd_cap; x++) {
    const int32_t nd = g.nd_free[(int64_t)x * g.L + l];
    if (nd >= 0 && nd < g.nd_cap) fr[(int64_t)nd * g.L + l] = 1;
  }
}
__global__ void __launch_bounds__(256) k_nfa_mark_live(NState g, const uint8_t* __restrict__ fr, int64_t n,
                                                       uint8_t* __restrict__ mark) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;   // node x of lane l at [x * L + l]
  if (k >= (int64_t)g.nd_cap * g.L || fr[k]) return;
  const int32_t ev = g.nd_ev[k];
  if (ev >= 0 && ev < n) mark[ev] = 1;
}
__global__ void __launch_bounds__(256) k_nfa_cmp_map(int64_t m, const int32_t* __restrict__ list, int32_t* __restrict__ map) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k < m) map[list[k]] = (int32_t)k;
}
__global__ void __launch_bounds__(256) k_nfa_remap_nodes(NState g, const uint8_t* __restrict__ fr, int64_t n,
                                                         const int32_t* __restrict__ map) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= (int64_t)g.nd_cap * g.L || fr[k]) return;
  const int32_t ev = g.nd_ev[k];
  if (ev >= 0 && ev < n) g.nd_ev[k] = map[ev];
}
__global__ void __launch_bounds__(256) k_nfa_cmp_gather(int64_t m, const int32_t* __restrict__ list,
                                                        const int32_t* __restrict__ rank, const int32_t* __restrict__ row,
                                                        const int8_t* __restrict__ st, int32_t* __restrict__ grank,
                                                        int32_t* __restrict__ grow, int8_t* __restrict__ gst) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= m) return;
  const int32_t e = list[k];
  grank[k] = rank[e]; grow[k] = row[e]; gst[k] = st[e];
}
// rows of w bytes: dst[k] = src[idx[k]]
__global__ void __launch_bounds__(256) k_nfa_gather_rows(const uint8_t* __restrict__ src, const int64_t* __restrict__ idx,
                                                         int64_t m, int w, uint8_t* __restrict__ dst) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= m) return;
  for (int b = 0; b < w; b++) dst[k * w + b] = src[idx[k] * w + b];
}

struct NfaExec : Exec {
  NTable tab;
  std::vector<Prog> progs;          // [filters per processor (index = proc)] + [select programs]
  std::vector<int> streams;         // local stream index -> app stream
  std::map<int, int> local;         // app stream -> local
  std::map<int, int> part_attr;     // local stream -> partition attribute (partitioned)
  bool partitioned = false;
  int nsel = 0;                     // device-projected values per match (select, or pre-selector values)
  SelSpec selspec;                  // host QuerySelector stage (aggregators / group-by / having / order / limit)
  std::unique_ptr<SelectorStage> selector;
  DevSelector dsel;                 // the selector stage on the device (selector_dev.hpp)
  DBuf<uint8_t> sel_ty;
  DBuf<int64_t> sel_ts;
  DBuf<int32_t> sel_row, sel_lid, sel_ord;
  // capacities
  int se_cap = 64, nd_cap = 256, list_cap = 48;
  int64_t L = 0;                    // lanes allocated
  std::unordered_map<int64_t, int> key_lane;
  PurgeClock* purge = nullptr;                       // @purge of the partition (runtime.hpp)
  std::unordered_map<int64_t, int64_t> last_seen;    // @purge: key -> its last initPartition time
  std::vector<int64_t> lane_key;        // partition key value per lane (string id / int)
  std::vector<int32_t> dense_lane;      // key -> lane for keys in [0, 2^24)
  hvec<int32_t> rank_ev;                // arrival rank -> event index (stable by seq)
  DBuf<int32_t> ev_rank;                // event index -> arrival rank
  Ty key_ty = T_STRING;                 // type of the partition attribute
  // (lane, absolute tick << 8 | scheduler): firings deferred because another instance won the deadline
  std::vector<std::pair<int32_t, int64_t>> deferrals;   // (lane, tick << 8 | scheduler), in key order
  void defer(int32_t lane, int64_t key) {
    auto at = deferrals.end();
    if (!deferrals.empty() && deferrals.back().second > key)
      at = std::upper_bound(deferrals.begin(), deferrals.end(), key,
                            [](int64_t k, const std::pair<int32_t, int64_t>& d) { return k < d.second; });
    deferrals.insert(at, {lane, key});
  }
  DBuf<int32_t> d_def_off;
  DBuf<int64_t> d_def_key, ev_now;
  DBuf<FireRec> d_fire;
  DBuf<OpRec> d_ops;
  DBuf<int8_t> rec_sched;
  // device state
  DBuf<int32_t> se_slot, se_ref, se_free, se_top, nd_ev, nd_next, nd_ref, nd_free, nd_top, pend, npend, nev, nnev,
      created, err, ret;
  DBuf<int64_t> se_ts;
  DBuf<int8_t> se_type;
  DBuf<uint32_t> flags;
  // events (device, growing)
  int64_t n = 0;
  DBuf<int64_t> ev_ts;
  DBuf<int8_t> ev_stream;
  DBuf<int32_t> ev_row;
  std::vector<std::vector<DCol>> cols;   // per local stream
  std::vector<int64_t> rows;             // rows per local stream
  DBuf<uint8_t> nulcol[NSTR];            // per local stream: null flags [row][attr] (once a null arrived)
  bool has_nul[NSTR] = {};
  bool supports_nulls() const override { return true; }
  hvec<int64_t> h_seq;                   // arrival seq per event
  hvec<int8_t> h_stream;
  hvec<int> h_lane;                      // lane per event (-1: a broadcast event)
  bool bcast[NSTR] = {};                 // local stream not keyed by the partition (broadcast)
  std::vector<int32_t> create_rank;      // per lane: arrival rank of its first keyed event
  std::vector<int32_t> lane_hash_c;      // per lane: spread Java hash of the key string (HashSet order)
  int64_t flushed = 0;                   // events [0, flushed) processed
  DBuf<NTable> d_tab;
  DBuf<NCols> d_cols;
  DBuf<Prog> d_progs;
  DBuf<int32_t> lane_off, lane_ev, lane_id;
  DBuf<NEvRec> lane_rec;                 // the launch's events packed per CSR entry (k_nfa_pack)
  DBuf<int32_t> pack_inv;                // each event's CSR entry (-1: none), for k_nfa_pack_ev
  DBuf<uint64_t> rec_key;
  DBuf<int64_t> rec_val, rec_ts, rec_dl;
  DBuf<int32_t> rec_tick, rec_lane;
  DBuf<uint8_t> rec_nul;
  DBuf<uint32_t> counter;
  DBuf<int64_t> lst, tq, d_tick_now;
  DBuf<int32_t> ntq, tqc, tqh, d_tick_ev, d_tick_ub, d_tick_lb;
  // Scheduler ticks (absent states): app clock, next event index, arrival seq
  pvec<int64_t> tick_now;                // (pinned: uploaded whole each flush)
  hvec<int64_t> tick_seq;
  pvec<int32_t> tick_ev;
  size_t ticks_flushed = 0;
  int64_t start_now = 0;
  hipEvent_t e0 = nullptr, e1 = nullptr;

  void on_tick(int64_t now, int64_t seq, int stream, int64_t k) override {
    (void)stream; (void)k;
    if (tab.nabs == 0) return;
    tick_now.push_back(now);
    tick_seq.push_back(seq);
    tick_ev.push_back(-1);          // arrival rank of the next event, placed at flush (place_new)
  }
  void on_ticks(const TickBuf& t, int stream) override {
    (void)stream;
    if (tab.nabs == 0) return;
    const size_t m = t.now.size(), o = tick_now.size();
    tick_now.resize(o + m); tick_seq.resize(o + m); tick_ev.resize(o + m);
    const int nth = host_threads((int64_t)m);
    host_parallel(nth, [&](int th) {
      const size_t a0 = m * th / nth, a1 = m * (th + 1) / nth;
      std::memcpy(tick_now.data() + o + a0, t.now.data() + a0, (a1 - a0) * 8);
      std::memcpy(tick_seq.data() + o + a0, t.seq.data() + a0, (a1 - a0) * 8);
      std::fill(tick_ev.data() + o + a0, tick_ev.data() + o + a1, -1);
    });
  }

  // Arrival ranks of the events pushed since the last flush (stable by seq: events derived from one
  // send by an upstream query arrive with that send's seq, in subscription order), and the rank of the
  // next event at each new tick.
  std::vector<int32_t> place_tmp, place_idx, place_cnt;
  pvec<int32_t> csr_evs;
  PinBuf<int32_t> place_rk;
  void place_new(hipStream_t s) {
    PhaseClock pc(getenv("SG_HOST_TIMING") != nullptr);
    const int64_t r0 = (int64_t)rank_ev.size();
    const int64_t m_ = n - r0;
    const int nth = m_ >= (1 << 20) ? (int)std::min<int64_t>(16, std::max(1u, std::thread::hardware_concurrency())) : 1;
    auto par = [&](auto&& f) {            // f(t, e0, e1) over events [r0, n) split across nth threads
      if (nth == 1) { f(0, r0, n); return; }
      host_parallel(nth, [&](int t) { f(t, r0 + m_ * t / nth, r0 + m_ * (t + 1) / nth); });
    };
    std::vector<uint8_t> run_ok(nth, 1);
    par([&](int t, int64_t e0, int64_t e1) {      // (thread-local flag: no shared cache line in the loop)
      bool ok = true;
      for (int64_t e = std::max(e0, r0 + 1); e < e1 && ok; e++) ok = h_seq[e] >= h_seq[e - 1];
      run_ok[t] = ok;
    });
    const bool one_run = std::all_of(run_ok.begin(), run_ok.end(), [](uint8_t x) { return x != 0; });
    pc.mark("place: run check");
    if (n > r0 && one_run) {       // arrival order is array order: ranks are the identity
      rank_ev.resize((size_t)n);
      par([&](int, int64_t e0, int64_t e1) { for (int64_t e = e0; e < e1; e++) rank_ev[e] = (int32_t)e; });
      pc.mark("place: identity ranks");
      if (partitioned) {
        create_rank.resize(lane_key.size(), INT32_MAX);
        // first keyed event of each lane: per-thread minima, then the smallest
        std::vector<std::vector<int32_t>> tfirst(nth);
        par([&](int t, int64_t e0, int64_t e1) {
          auto& f = tfirst[t];
          f.assign(lane_key.size(), INT32_MAX);
          for (int64_t e = e0; e < e1; e++) {
            const int l = h_lane[e];
            if (l >= 0 && f[l] == INT32_MAX) f[l] = (int32_t)e;
          }
        });
        for (int t = 0; t < nth; t++)
          for (size_t l = 0; l < lane_key.size(); l++)
            if (create_rank[l] == INT32_MAX) create_rank[l] = tfirst[t][l];
      }
      ev_rank.reserve(n, true, s, r0);
      hipLaunchKernelGGL(k_nfa_iota, dim3((unsigned)((n - r0 + 255) / 256)), dim3(256), 0, s, ev_rank.p + r0,
                         (int32_t)r0, n - r0);
      SG_HIP(hipGetLastError());
      pc.mark("place ranks (one run)");
    } else if (n > r0) {
      // (member buffers: their pages stay mapped from one flush to the next)
      std::vector<int32_t>& idx = place_idx;
      idx.resize(n - r0);
      // the pushes since the last flush are runs already ordered by seq (each push is).  Dense seqs (the
      // usual case: every send one seq, an upstream query's rows carrying their send's): a stable counting
      // sort by seq, O(n + range); otherwise a stable merge of the runs, O(n log runs)
      int64_t smin = INT64_MAX, smax = INT64_MIN;
      const int64_t m = n - r0;
      std::vector<size_t> runs(1, 0);
      // two runs (one push of each of two streams, config 5's StockStream and chained VolStream): a parallel
      // stable merge, split by merge path (the first run wins ties: it was pushed first)
      std::vector<std::vector<size_t>> tb(nth);
      if (nth > 1 && !one_run)
        par([&](int t, int64_t e0, int64_t e1) {
          for (int64_t e = std::max(e0, r0 + 1); e < e1; e++)
            if (h_seq[e] < h_seq[e - 1]) tb[t].push_back((size_t)(e - r0));
        });
      size_t nbreak = 0;
      for (auto& v : tb) nbreak += v.size();
      const bool two_runs = nth > 1 && !one_run && nbreak == 1;
      if (two_runs) {
        size_t a = 0;
        for (auto& v : tb) if (!v.empty()) a = v[0];
        const int64_t na = (int64_t)a, nb = m - (int64_t)a;
        std::vector<int32_t>& tmp2 = place_tmp;
        tmp2.resize((size_t)m);
        auto sq = [&](int64_t rel) { return h_seq[r0 + rel]; };
        host_parallel(nth, [&](int t) {
          auto split = [&](int64_t d) {          // elements of run A among the first d of the merge
            int64_t lo = std::max<int64_t>(0, d - nb), hi = std::min<int64_t>(d, na);
            while (lo < hi) {
              const int64_t mid = (lo + hi) >> 1;
              if (sq(mid) <= sq(na + d - mid - 1)) lo = mid + 1; else hi = mid;
            }
            return lo;
          };
          const int64_t d0 = m * t / nth, d1 = m * (t + 1) / nth;
          int64_t i = split(d0), j = d0 - i;
          const int64_t i1 = split(d1), j1 = d1 - i1;
          for (int64_t o = d0; o < d1; o++) {
            const bool takeA = i < i1 && (j >= j1 || sq(i) <= sq(na + j));
            tmp2[(size_t)o] = (int32_t)(r0 + (takeA ? i++ : na + j++));
          }
        });
        idx.swap(tmp2);
      } else if (!one_run &&
                 [&] { for (int64_t e = r0; e < n; e++) { smin = std::min(smin, h_seq[e]); smax = std::max(smax, h_seq[e]); }
                       return smax - smin < 4 * m && smax - smin < (1ll << 30); }()) {
        std::vector<int32_t>& cnt = place_cnt;
        cnt.assign((size_t)(smax - smin + 2), 0);
        for (int64_t e = r0; e < n; e++) cnt[(size_t)(h_seq[e] - smin) + 1]++;
        for (size_t k = 1; k < cnt.size(); k++) cnt[k] += cnt[k - 1];
        for (int64_t e = r0; e < n; e++) idx[(size_t)cnt[(size_t)(h_seq[e] - smin)]++] = (int32_t)e;
      } else {                           // the runs the pushes left
        par([&](int, int64_t e0, int64_t e1) { for (int64_t e = e0; e < e1; e++) idx[e - r0] = (int32_t)e; });
        for (int64_t e = r0 + 1; e < n; e++)
          if (h_seq[e] < h_seq[e - 1]) runs.push_back((size_t)(e - r0));
      }
      runs.push_back(idx.size());
      auto by_seq = [&](int32_t x, int32_t y) { return h_seq[x] < h_seq[y]; };
      std::vector<int32_t> tmp(runs.size() > 2 ? idx.size() : 0);
      while (runs.size() > 2) {               // pairwise merges into a buffer (linear, no rotations)
        std::vector<size_t> nr(1, 0);
        size_t k = 0;
        for (; k + 2 < runs.size(); k += 2) {
          std::merge(idx.begin() + runs[k], idx.begin() + runs[k + 1], idx.begin() + runs[k + 1],
                     idx.begin() + runs[k + 2], tmp.begin() + runs[k], by_seq);
          nr.push_back(runs[k + 2]);
        }
        if (k + 1 < runs.size())              // an odd run out: carried over as it is
          std::copy(idx.begin() + runs[k], idx.begin() + runs[k + 1], tmp.begin() + runs[k]);
        if (runs.size() % 2 == 0) nr.push_back(runs.back());
        idx.swap(tmp);
        runs.swap(nr);
      }
      pc.mark("place merge");
      PinBuf<int32_t>& rk = place_rk;      // (pinned: the ranks go to the device)
      rk.reserve((size_t)(n - r0));
      rank_ev.resize((size_t)n);
      par([&](int, int64_t e0, int64_t e1) {      // (rank ranges: [e0 - r0, e1 - r0) of idx)
        for (int64_t r = e0 - r0; r < e1 - r0; r++) { rank_ev[r0 + r] = idx[r]; rk.p[idx[r] - r0] = (int32_t)(r0 + r); }
      });
      if (partitioned) {                 // instance creation: the first keyed event of each key, in rank order
        create_rank.resize(lane_key.size(), INT32_MAX);
        std::vector<std::vector<int32_t>> tfirst(nth);
        par([&](int t, int64_t e0, int64_t e1) {
          auto& f = tfirst[t];
          f.assign(lane_key.size(), INT32_MAX);
          for (int64_t r = e0 - r0; r < e1 - r0; r++) {
            const int l = h_lane[idx[r]];
            if (l >= 0 && f[l] == INT32_MAX) f[l] = (int32_t)(r0 + r);
          }
        });
        for (int t = 0; t < nth; t++)
          for (size_t l = 0; l < lane_key.size(); l++)
            if (create_rank[l] == INT32_MAX) create_rank[l] = tfirst[t][l];
      }
      ev_rank.reserve(n, true, s, r0);
      SG_HIP(hipMemcpyAsync(ev_rank.p + r0, rk.p, (size_t)(n - r0) * 4, hipMemcpyHostToDevice, s));
      SG_HIP(hipStreamSynchronize(s));
      pc.mark("place ranks");
    }
    // first rank whose seq >= the tick's seq (tick seqs and the seqs in rank order are non-decreasing), and at
    // least the rank of every tick placed before it.  Placed ticks (earlier flushes) are a prefix; the new ones
    // search the rank order in parallel.
    int32_t r = 0;
    size_t t = 0;
    for (; t < tick_ev.size() && tick_ev[t] >= 0; t++) r = std::max(r, tick_ev[t]);
    const int32_t nr = (int32_t)rank_ev.size();
    const size_t nt_new = tick_ev.size() - t;
    const int tth = nt_new >= (1u << 18) ? nth : 1;
    const size_t tb0 = t;
    auto place_ticks = [&](size_t a, size_t b) {   // one search for the range's first tick, then a sweep
      if (a >= b) return;
      int32_t lo = r, hi = nr;
      while (lo < hi) { const int32_t mid = (lo + hi) >> 1; if (h_seq[rank_ev[mid]] < tick_seq[a]) lo = mid + 1; else hi = mid; }
      int32_t q = lo;
      for (size_t k = a; k < b; k++) {
        while (q < nr && h_seq[rank_ev[q]] < tick_seq[k]) q++;
        tick_ev[k] = q;
      }
    };
    if (tth > 1) host_parallel(tth, [&](int q) { place_ticks(tb0 + nt_new * q / tth, tb0 + nt_new * (q + 1) / tth); });
    else place_ticks(tb0, tick_ev.size());
  }
  void start(int64_t now) override { start_now = now; }
  int nq() const { return std::max<int>(1, tab.nabs); }
  bool chunk_sensitive() const override { return false; }   // selector output is 1:1 per StateEvent

  ~NfaExec() override {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    for (auto& e : sp_ev) if (e) (void)hipEventDestroy(e);
    if (sw_cnt) (void)hipHostFree(sw_cnt);
  }

  NState state() {
    NState s;
    s.L = L; s.se_cap = se_cap; s.nd_cap = nd_cap; s.list_cap = list_cap;
    s.se_slot = se_slot.p; s.se_ts = se_ts.p; s.se_type = se_type.p; s.se_ref = se_ref.p; s.se_free = se_free.p;
    s.se_top = se_top.p; s.nd_ev = nd_ev.p; s.nd_next = nd_next.p; s.nd_ref = nd_ref.p; s.nd_free = nd_free.p;
    s.nd_top = nd_top.p; s.pend = pend.p; s.npend = npend.p; s.nev = nev.p; s.nnev = nnev.p; s.flags = flags.p;
    s.created = created.p; s.err = err.p; s.ret = ret.p;
    s.lst = lst.p; s.tq = tq.p; s.ntq = ntq.p; s.tqc = tqc.p; s.tqh = tqh.p; s.nq = nq();
    return s;
  }

  // every per-lane pool with its elements per lane (SoA, element x of lane l at [x * L + l])
  template <class F>
  void for_each_pool(F&& f) {
    f(se_slot, (int64_t)se_cap * NS); f(se_ts, se_cap); f(se_type, se_cap); f(se_ref, se_cap);
    f(se_free, se_cap); f(se_top, 1); f(nd_ev, nd_cap); f(nd_next, nd_cap); f(nd_ref, nd_cap);
    f(nd_free, nd_cap); f(nd_top, 1); f(pend, (int64_t)NP * list_cap); f(npend, NP);
    f(nev, (int64_t)NP * list_cap); f(nnev, NP); f(flags, NP); f(created, 1); f(err, 1);
    f(ret, list_cap); f(lst, NP); f(tq, (int64_t)nq() * NTQ); f(ntq, nq());
    f(tqc, (int64_t)nq() * NTQ); f(tqh, nq());
  }

  // Snapshot of a flushed runtime: the per-lane pools (per partition instance and processor: the pending
  // and new-and-every StateEvent lists, the StateEvent / chain-node pools they reference, the
  // initialized / started / changed flags, lastScheduledTime and the Scheduler queues -- the fields of
  // StreamPreStateProcessor.StreamPreState.snapshot, StreamPreStateProcessor.java:450-469, and
  // AbsentStreamPreStateProcessor's), the event store those StateEvents index, the key -> instance map,
  // the clock ticks and the selector's aggregator states.
  bool can_snapshot() const override { return true; }

  // sg_query_state_json: StreamPreStateProcessor.StreamPreState.snapshot (:450-469) read back from the lane pools --
  // per instance (lane, creation order) and pre-state processor (allPre, the parser's preStateProcessors order)
  // the initialized flag and the pending / new-and-every StateEvent lists, each StateEvent with its slots' event
  // chains (StateEvent.getStreamEvents) as (ts, raw attribute slots); absent processors add lastScheduledTime.
  template <class T>
  std::vector<T> fetch(const DBuf<T>& b, size_t cnt, hipStream_t s) {
    std::vector<T> h(std::max<size_t>(cnt, 1));
    if (cnt) SG_HIP(hipMemcpyAsync(h.data(), b.p, cnt * sizeof(T), hipMemcpyDeviceToHost, s));
    return h;
  }
  bool state_json(std::string& out, hipStream_t s) override {
    const int64_t nl = partitioned ? (int64_t)lane_key.size() : std::min<int64_t>(L, 1);
    const auto hslot = fetch(se_slot, (size_t)(se_cap * NS * L), s);
    const auto hsts = fetch(se_ts, (size_t)(se_cap * L), s);
    const auto hsty = fetch(se_type, (size_t)(se_cap * L), s);
    const auto hnev = fetch(nd_ev, (size_t)(nd_cap * L), s);
    const auto hnnx = fetch(nd_next, (size_t)(nd_cap * L), s);
    const auto hpend = fetch(pend, (size_t)(NP * list_cap * L), s);
    const auto hnpend = fetch(npend, (size_t)(NP * L), s);
    const auto hnew = fetch(nev, (size_t)(NP * list_cap * L), s);
    const auto hnnew = fetch(nnev, (size_t)(NP * L), s);
    const auto hfl = fetch(flags, (size_t)(NP * L), s);
    const auto hlst = fetch(lst, (size_t)(NP * L), s);
    const auto hets = fetch(ev_ts, (size_t)n, s);
    const auto hest = fetch(ev_stream, (size_t)n, s);
    const auto herow = fetch(ev_row, (size_t)n, s);
    std::vector<std::vector<std::vector<uint8_t>>> hcol(streams.size());
    std::vector<std::vector<uint8_t>> hnul(streams.size());
    for (size_t ls = 0; ls < streams.size(); ls++) {
      for (auto& c : cols[ls]) hcol[ls].push_back(fetch(c.b, (size_t)(rows[ls] * c.w), s));
      if (has_nul[ls]) hnul[ls] = fetch(nulcol[ls], (size_t)(rows[ls] * (int64_t)cols[ls].size()), s);
    }
    SG_HIP(hipStreamSynchronize(s));
    std::string& o = out;
    auto num = [&](int64_t v) { o += std::to_string(v); };
    auto event = [&](int ev) {
      o += '[';
      if (ev < 0) { num(-1); o += ']'; return; }    // StreamEventFactory.newInstance(): ts -1, no attributes
      num(hets[(size_t)ev]);
      const int ls = hest[(size_t)ev];
      const int64_t row = herow[(size_t)ev];
      const auto& types = app->streams[streams[(size_t)ls]].types;
      for (size_t k = 0; k < cols[(size_t)ls].size(); k++) {
        o += ',';
        if (has_nul[ls] && hnul[(size_t)ls][(size_t)(row * (int64_t)cols[(size_t)ls].size() + (int64_t)k)]) { o += "null"; continue; }
        const auto& c = hcol[(size_t)ls][k];
        int64_t v;
        if (cols[(size_t)ls][k].w == 8) std::memcpy(&v, c.data() + row * 8, 8);
        else {
          int32_t x;
          std::memcpy(&x, c.data() + row * 4, 4);
          v = types[k] == T_FLOAT ? (int64_t)(uint32_t)x : (int64_t)x;   // the ABI's raw slot
        }
        num(v);
      }
      o += ']';
    };
    auto stev = [&](int64_t l, int se) {
      o += "{\"ts\":"; num(hsts[(size_t)(se * L + l)]);
      o += ",\"type\":"; num(hsty[(size_t)(se * L + l)]);
      o += ",\"slots\":[";
      for (int k = 0; k < tab.nslots; k++) {
        if (k) o += ',';
        o += '[';
        int nd = hslot[(size_t)(((int64_t)se * NS + k) * L + l)];
        for (bool first = true; nd >= 0; first = false) {
          if (!first) o += ',';
          event(hnev[(size_t)((int64_t)nd * L + l)]);
          nd = hnnx[(size_t)((int64_t)nd * L + l)];
        }
        o += ']';
      }
      o += "]}";
    };
    auto list = [&](int64_t l, int p, const std::vector<int32_t>& arr, const std::vector<int32_t>& cnt) {
      o += '[';
      const int m = cnt[(size_t)((int64_t)p * L + l)];
      for (int k = 0; k < m; k++) {
        if (k) o += ',';
        stev(l, arr[(size_t)(((int64_t)p * list_cap + k) * L + l)]);
      }
      o += ']';
    };
    o = "{\"instances\":[";
    for (int64_t l = 0; l < nl; l++) {
      if (l) o += ',';
      o += "{\"key\":";
      if (partitioned) num(lane_key[(size_t)l]); else o += "null";
      o += ",\"processors\":[";
      for (int a = 0; a < tab.nall; a++) {
        const int p = tab.allPre[a];
        if (a) o += ',';
        o += "{\"initialized\":";
        o += (hfl[(size_t)((int64_t)p * L + l)] & 2u) ? "true" : "false";
        o += ",\"pending\":"; list(l, p, hpend, hnpend);
        o += ",\"new_and_every\":"; list(l, p, hnew, hnnew);
        if (tab.p[p].kind == K_ABSENT) { o += ",\"last_scheduled\":"; num(hlst[(size_t)((int64_t)p * L + l)]); }
        o += '}';
      }
      o += "]}";
    }
    o += "]}";
    return true;
  }

  void snapshot(SnapWriter& w, hipStream_t s) override {
    // the exact sweep's base (partitioned absent states) is moved to the present first (a replay of the flushes
    // since, which ends in the same pools), so that only its maps are saved
    if (tab.nabs > 0 && partitioned && !shard && !f_fresh && !base_current() && flushed == n && ticks_flushed == tick_now.size()) {
      int r = 0;
      double a = 0, b = 0;
      (void)sweep(s, (int64_t)tick_now.size() << 8, r, a, b);
    }
    w.pod(L); w.pod(se_cap); w.pod(nd_cap); w.pod(list_cap);
    w.pod(n); w.pod(flushed); w.pod<uint64_t>(ticks_flushed); w.pod(start_now);
    for_each_pool([&](auto& buf, int64_t per_lane) { w.dev(buf, (size_t)(per_lane * L), s); });
    w.dev(ev_ts, (size_t)n, s); w.dev(ev_stream, (size_t)n, s); w.dev(ev_row, (size_t)n, s);
    w.dev(ev_now, (size_t)n, s); w.dev(ev_rank, (size_t)n, s);
    w.pod<uint64_t>(streams.size());
    for (size_t ls = 0; ls < streams.size(); ls++) {
      w.pod(rows[ls]);
      for (auto& c : cols[ls]) w.dev(c.b, (size_t)(rows[ls] * c.w), s);
      w.pod(has_nul[ls]);
      if (has_nul[ls]) w.dev(nulcol[ls], (size_t)rows[ls] * cols[ls].size(), s);
    }
    w.vec(h_seq); w.vec(h_stream); w.vec(h_lane); w.vec(lane_key); w.vec(rank_ev); w.vec(deferrals);
    w.vec(tick_now); w.vec(tick_seq); w.vec(tick_ev); w.vec(create_rank);
    {
      std::vector<std::pair<int64_t, int64_t>> ls(last_seen.begin(), last_seen.end());
      w.vec(ls);
    }
    w.pod<uint8_t>(selector ? 1 : 0);
    if (selector) selector->snapshot(w);
    const bool fb = !f_fresh && base_current();
    w.pod<uint8_t>(fb ? 1 : 0);
    if (fb) {
      w.pod<uint64_t>(fmaps.size());
      for (const SchedMap& m : fmaps) {
        w.pod<uint64_t>(m.tab.size()); w.pod<uint64_t>(m.size); w.pod<uint64_t>(m.thr);
        for (const auto& bin : m.tab) w.vec(bin);
      }
    }
  }
  void restore(SnapReader& r, hipStream_t s) override {
    reset();
    L = r.pod<int64_t>(); se_cap = r.pod<int>(); nd_cap = r.pod<int>(); list_cap = r.pod<int>();
    n = r.pod<int64_t>(); flushed = r.pod<int64_t>(); ticks_flushed = (size_t)r.pod<uint64_t>(); start_now = r.pod<int64_t>();
    for_each_pool([&](auto& buf, int64_t per_lane) {
      if ((int64_t)r.dev(buf, s) != per_lane * L) throw Error(-1, "snapshot pool size does not match the query");
    });
    // every device array must hold exactly what the counts say: the kernels index them by those counts
    auto want = [](size_t got, int64_t need, const char* what) {
      if ((int64_t)got != need) throw Error(-1, std::string("snapshot ") + what + " size does not match its count");
    };
    want(r.dev(ev_ts, s), n, "event timestamps"); want(r.dev(ev_stream, s), n, "event streams");
    want(r.dev(ev_row, s), n, "event rows"); want(r.dev(ev_now, s), n, "event clocks");
    want(r.dev(ev_rank, s), n, "event ranks");
    if (r.pod<uint64_t>() != streams.size()) throw Error(-1, "snapshot streams do not match the query");
    int64_t rows_total = 0;
    for (size_t ls = 0; ls < streams.size(); ls++) {
      rows[ls] = r.pod<int64_t>();
      if (rows[ls] < 0) throw Error(-1, "snapshot row count is negative");
      rows_total += rows[ls];
      for (auto& c : cols[ls]) want(r.dev(c.b, s), rows[ls] * c.w, "column");
      has_nul[ls] = r.pod<bool>();
      if (has_nul[ls]) want(r.dev(nulcol[ls], s), rows[ls] * (int64_t)cols[ls].size(), "null flags");
    }
    if (rows_total != n) throw Error(-1, "snapshot rows do not add up to its events");
    r.vec(h_seq); r.vec(h_stream); r.vec(h_lane); r.vec(lane_key); r.vec(rank_ev); r.vec(deferrals);
    std::stable_sort(deferrals.begin(), deferrals.end(), [](const auto& x, const auto& y) { return x.second < y.second; });
    r.vec(tick_now); r.vec(tick_seq); r.vec(tick_ev); r.vec(create_rank);
    {
      std::vector<std::pair<int64_t, int64_t>> ls;
      r.vec(ls);
      last_seen = std::unordered_map<int64_t, int64_t>(ls.begin(), ls.end());
    }
    key_lane.clear();
    dense_lane.clear();
    for (size_t l = 0; l < lane_key.size(); l++) {
      const int64_t key = lane_key[l];
      key_lane[key] = (int)l;
      if (key >= 0 && key < (1 << 24)) {
        if ((size_t)key >= dense_lane.size()) dense_lane.resize(std::max<size_t>((size_t)key + 1, dense_lane.size() * 2), -1);
        dense_lane[(size_t)key] = (int32_t)l;
      }
    }
    const bool has_sel = r.pod<uint8_t>() != 0;
    if (has_sel != (selector != nullptr)) throw Error(-1, "snapshot selector does not match the query");
    if (selector) selector->restore(r);
    if (r.pod<uint8_t>()) {
      fmaps.assign((size_t)r.pod<uint64_t>(), SchedMap());
      if ((int)fmaps.size() != tab.nabs) throw Error(-1, "snapshot Scheduler maps do not match the query");
      for (SchedMap& m : fmaps) {
        m.tab.resize((size_t)r.pod<uint64_t>()); m.size = (size_t)r.pod<uint64_t>(); m.thr = (size_t)r.pod<uint64_t>();
        for (auto& bin : m.tab) r.vec(bin);
      }
      base_save(s);
    }
  }

  // grow the lane pools to `want` lanes (SoA: re-layout by copying per element)
  void grow_lanes(int64_t want, hipStream_t s) {
    if (want <= L) return;
    int64_t nl = std::max<int64_t>(want, std::max<int64_t>(64, L * 2));
    NState old = state();
    int64_t oldL = L;
    auto regrow = [&](auto& buf, int64_t per_lane) {
      using T = typename std::remove_reference<decltype(*buf.p)>::type;
      DBuf<T> nb;
      nb.reserve((size_t)per_lane * nl);
      if (oldL) SG_HIP(hipMemcpy2DAsync(nb.p, nl * sizeof(T), buf.p, oldL * sizeof(T), oldL * sizeof(T), per_lane,
                                        hipMemcpyDeviceToDevice, s));
      SG_HIP(hipStreamSynchronize(s));
      buf = std::move(nb);
    };
    (void)old;
    for_each_pool(regrow);
    L = nl;
    NState ns = state();
    hipLaunchKernelGGL(k_nfa_pool_init, dim3((unsigned)((nl - oldL + 255) / 256)), dim3(256), 0, s, ns, oldL, nl - oldL);
    SG_HIP(hipGetLastError());
    SG_HIP(hipStreamSynchronize(s));
  }

  bool takes_device_batch() const override { return true; }
  void push(const HostBatch& b) override {
    auto it = local.find(b.stream);
    if (it == local.end()) return;
    int ls = it->second;
    hipStream_t s = app->stream;
    int64_t need = n + b.n;
    ev_ts.reserve(need, true, s, n);
    ev_stream.reserve(need, true, s, n);
    ev_row.reserve(need, true, s, n);
    ev_now.reserve(need, true, s, n);
    auto& cs = cols[ls];
    for (auto& c : cs) c.b.reserve((rows[ls] + b.n) * c.w, true, s, rows[ls] * c.w);
    // (a batch staged in HBM: device to device)
    SG_HIP(hipMemcpyAsync(ev_ts.p + n, b.d_ts ? b.d_ts : b.ts.data(), b.n * 8,
                          b.d_ts ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
    // stream index, row and (one-clock batches) app clock of each event are generated on the device
    const bool now_dev = b.now_uniform || b.now_ev.empty();
    hipLaunchKernelGGL(k_nfa_ev_fill, dim3((unsigned)((b.n + 255) / 256)), dim3(256), 0, s, ev_stream.p + n,
                       ev_row.p + n, now_dev ? ev_now.p + n : nullptr, (int8_t)ls, (int32_t)rows[ls], b.now, b.n);
    SG_HIP(hipGetLastError());
    if (!now_dev)
      SG_HIP(hipMemcpyAsync(ev_now.p + n, b.d_now ? b.d_now : b.now_ev.data(), b.n * 8,
                            b.d_now ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
    for (size_t k = 0; k < cs.size(); k++) {
      const bool dv = k < b.d_cols.size() && b.d_cols[k];
      SG_HIP(hipMemcpyAsync(cs[k].b.p + rows[ls] * cs[k].w, dv ? (const void*)b.d_cols[k] : (const void*)b.cols[k].data(),
                            b.n * cs[k].w, dv ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
    }
    // null flags: a stream's flag column exists from its first null on (earlier rows zeroed)
    const size_t na = cs.size();
    if (!b.nulls.empty() && !has_nul[ls]) {
      has_nul[ls] = true;
      nulcol[ls].reserve(std::max<size_t>((rows[ls] + b.n) * na, 1));
      SG_HIP(hipMemsetAsync(nulcol[ls].p, 0, std::max<size_t>(rows[ls] * na, 1), s));
    }
    if (has_nul[ls]) {
      nulcol[ls].reserve((rows[ls] + b.n) * na, true, s, rows[ls] * na);
      if (b.nulls.empty()) SG_HIP(hipMemsetAsync(nulcol[ls].p + rows[ls] * na, 0, b.n * na, s));
      else SG_HIP(hipMemcpyAsync(nulcol[ls].p + rows[ls] * na, b.nulls.data(), b.n * na, hipMemcpyHostToDevice, s));
    }
    // lanes: partition key -> lane (first appearance creates the instance), while the copies run
    auto pa = part_attr.find(ls);
    const bool keyed = partitioned && pa != part_attr.end();
    book(ls, b.n, keyed ? b.cols[pa->second].data() : nullptr,
         keyed && b.n ? (int)(b.cols[pa->second].size() / (size_t)b.n) : 4,
         b.nulls.empty() ? nullptr : b.nulls.data(), b.seq0, b.seqs.empty() ? nullptr : b.seqs.data(),
         b.now_ev.empty() ? nullptr : b.now_ev.data(), b.now);
    SG_HIP(hipStreamSynchronize(s));
    rows[ls] += b.n;
    n += b.n;
  }

  // Host bookkeeping of pushed events [n, n + cnt) of local stream ls: arrival seq, stream and partition
  // instance (lane) per event.  keycol: the partition attribute's host column (keyw bytes per value), null
  // for an unpartitioned query or a broadcast stream; nulls: [cnt][attrs] flags or null.
  void book(int ls, int64_t cnt, const uint8_t* keycol, int keyw, const uint8_t* nulls, int64_t seq0,
            const int64_t* seqs, const int64_t* now_ev, int64_t now) {
    const size_t h0 = h_lane.size();
    h_lane.resize(h0 + cnt);
    h_seq.resize(h0 + cnt);
    h_stream.resize(h0 + cnt);
    const int nth = cnt >= (1 << 20) ? (int)std::min<int64_t>(16, std::max(1u, std::thread::hardware_concurrency())) : 1;
    auto par = [&](auto&& f) {            // f(k0, k1) over [0, cnt) split across nth threads
      if (nth == 1) { f((int64_t)0, cnt); return; }
      host_parallel(nth, [&](int t) { f(cnt * t / nth, cnt * (t + 1) / nth); });
    };
    par([&](int64_t a0, int64_t a1) { std::memset(h_stream.data() + h0 + a0, ls, (size_t)(a1 - a0)); });
    if (!seqs) par([&](int64_t a0, int64_t a1) { for (int64_t k = a0; k < a1; k++) h_seq[h0 + k] = seq0 + k; });
    else par([&](int64_t a0, int64_t a1) { std::memcpy(h_seq.data() + h0 + a0, seqs + a0, (size_t)(a1 - a0) * 8); });
    int* hl = h_lane.data() + h0;
    auto pa = part_attr.find(ls);
    if (!partitioned) {
      std::fill(hl, hl + cnt, 0);
      return;
    }
    if (pa == part_attr.end() || !keycol) {   // broadcast: placed into every lane created before it (run_lanes)
      std::fill(hl, hl + cnt, -1);
      return;
    }
    const bool w8 = keyw == 8;
    const int64_t* k8 = (const int64_t*)keycol;
    const int32_t* k4 = (const int32_t*)keycol;
    const size_t na_ = cols[ls].size();
    auto keyat = [&](int64_t k) { return w8 ? k8[k] : (int64_t)k4[k]; };
    auto new_lane = [&](int64_t key) {
      const int lane = (int)lane_key.size();
      key_lane[key] = lane;
      lane_key.push_back(key);
      if (key >= 0 && key < (1 << 24)) {
        if ((size_t)key >= dense_lane.size()) dense_lane.resize(std::max<size_t>((size_t)key + 1, dense_lane.size() * 2), -1);
        dense_lane[(size_t)key] = lane;
      }
      return lane;
    };
    if (!purge && !nulls && nth > 1) {
      // large batch of dense keys: new keys take lanes in first-appearance order (each thread notes the
      // first occurrence in its range of every key without a lane; merged by position), then every event's
      // lane is a parallel table lookup
      std::vector<int64_t> tmin(nth, INT64_MAX), tmax(nth, -1);
      host_parallel(nth, [&](int t) {
        int64_t lo = INT64_MAX, hi = -1;               // (thread-local: no shared cache line in the loop)
        for (int64_t k = cnt * t / nth, e = cnt * (t + 1) / nth; k < e; k++) {
          const int64_t key = keyat(k);
          lo = std::min(lo, key); hi = std::max(hi, key);
        }
        tmin[t] = lo; tmax[t] = hi;
      });
      const int64_t kmin = *std::min_element(tmin.begin(), tmin.end()), kmax = *std::max_element(tmax.begin(), tmax.end());
      if (kmin >= 0 && kmax < (1 << 24)) {
        if ((size_t)kmax >= dense_lane.size()) dense_lane.resize(std::max<size_t>((size_t)kmax + 1, dense_lane.size() * 2), -1);
        std::vector<std::vector<std::pair<int64_t, int64_t>>> firsts(nth);   // (position, key)
        host_parallel(nth, [&](int t) {
          std::vector<uint8_t> seen((size_t)kmax + 1, 0);
          for (int64_t k = cnt * t / nth, e = cnt * (t + 1) / nth; k < e; k++) {
            const int64_t key = keyat(k);
            if (dense_lane[(size_t)key] < 0 && !seen[(size_t)key]) { seen[(size_t)key] = 1; firsts[t].push_back({k, key}); }
          }
        });
        for (int t = 0; t < nth; t++)            // thread ranges are in position order
          for (auto& f : firsts[t])
            if (dense_lane[(size_t)f.second] < 0) new_lane(f.second);
        par([&](int64_t a0, int64_t a1) { for (int64_t k = a0; k < a1; k++) hl[k] = dense_lane[(size_t)keyat(k)]; });
        return;
      }
    }
    for (int64_t k = 0; k < cnt; k++) {
      if (nulls && nulls[(size_t)k * na_ + pa->second]) { hl[k] = -2; continue; }   // null key: dropped
      const int64_t key = keyat(k);
      int lane;
      if (key >= 0 && key < (1 << 24)) {          // dictionary ids / small ints: direct index
        if ((size_t)key >= dense_lane.size()) dense_lane.resize(std::max<size_t>((size_t)key + 1, dense_lane.size() * 2), -1);
        const int32_t dl = dense_lane[(size_t)key];
        lane = dl < 0 ? new_lane(key) : dl;
      } else {
        auto f = key_lane.find(key);
        lane = f == key_lane.end() ? new_lane(key) : f->second;
      }
      if (purge) {
        // initPartition of this chunk: a purge task since the key's last chunk cleaned its states, so the
        // key continues as a new partition instance (a new lane; the old one never runs again)
        const int64_t now_k = now_ev ? now_ev[k] : now;
        auto it = last_seen.find(key);
        if (it != last_seen.end() && purge->task_in(it->second + purge->idle, now_k)) lane = new_lane(key);
        purge->note(now_k);
        last_seen[key] = now_k;
      }
      hl[k] = lane;
    }
  }

  // Device-resident ingest (sg_push_device): the columns are copied device to device into the event
  // store; only the partition attribute comes to the host, for the instance bookkeeping.
  PinBuf<uint8_t> dkeys;
  void push_device(int stream, int64_t cnt, const int64_t* dts, const void* const* dcols, int batch,
                   hipStream_t s) override {
    (void)batch;
    auto it = local.find(stream);
    if (it == local.end() || cnt <= 0) return;
    const int ls = it->second;
    PhaseClock pc(getenv("SG_HOST_TIMING") != nullptr);
    if (tab.nabs > 0) throw Error(-2, "device-resident ingest of a query with absent states (its Scheduler ticks "
                                      "follow the host clock): use sg_push");
    const int64_t need = n + cnt;
    ev_ts.reserve(need, true, s, n);
    ev_stream.reserve(need, true, s, n);
    ev_row.reserve(need, true, s, n);
    ev_now.reserve(need, true, s, n);
    auto& cs = cols[ls];
    for (auto& c : cs) c.b.reserve((rows[ls] + cnt) * c.w, true, s, rows[ls] * c.w);
    SG_HIP(hipMemcpyAsync(ev_ts.p + n, dts, cnt * 8, hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_nfa_ev_fill, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, ev_stream.p + n,
                       ev_row.p + n, ev_now.p + n, (int8_t)ls, (int32_t)rows[ls], app->now, cnt);
    SG_HIP(hipGetLastError());
    for (size_t k = 0; k < cs.size(); k++) {
      if (!dcols[k]) {                 // an attribute the caller did not provide: zeros (never read by the query)
        SG_HIP(hipMemsetAsync(cs[k].b.p + rows[ls] * cs[k].w, 0, cnt * cs[k].w, s));
        continue;
      }
      SG_HIP(hipMemcpyAsync(cs[k].b.p + rows[ls] * cs[k].w, dcols[k], cnt * cs[k].w, hipMemcpyDeviceToDevice, s));
    }
    if (has_nul[ls]) {               // (device batches carry no nulls)
      nulcol[ls].reserve((rows[ls] + cnt) * cs.size(), true, s, rows[ls] * cs.size());
      SG_HIP(hipMemsetAsync(nulcol[ls].p + rows[ls] * cs.size(), 0, cnt * cs.size(), s));
    }
    auto pa = part_attr.find(ls);
    const bool keyed = partitioned && pa != part_attr.end();
    int keyw = 4;
    if (keyed) {
      if (!dcols[pa->second]) throw Error(-1, "device push without the partition attribute's column");
      keyw = cs[pa->second].w;
      dkeys.reserve((size_t)cnt * keyw);
      SG_HIP(hipMemcpyAsync(dkeys.p, dcols[pa->second], (size_t)cnt * keyw, hipMemcpyDeviceToHost, s));
    }
    SG_HIP(hipStreamSynchronize(s));
    pc.mark("push_device: copies + keys to host");
    book(ls, cnt, keyed ? dkeys.p : nullptr, keyw, nullptr, app->seq, nullptr, nullptr, app->now);
    pc.mark("push_device: instance bookkeeping");
    rows[ls] += cnt;
    dev_push_h0 = n;
    dev_push_n = cnt;
    n += cnt;
  }
  // Chained input kept in HBM (DevChain, api.hip dispatch): an upstream window query's output rows, packed on the
  // device in this stream's widths, are copied device to device with their app clocks; the host keeps only the
  // partition attribute and the source seqs, for the instance bookkeeping (the same as push with those columns).
  int chain_key_attr(int stream) const override {
    auto it = local.find(stream);
    if (it == local.end() || purge) return -2;           // (a purge task reads each event's clock on the host)
    auto pa = part_attr.find(it->second);
    return partitioned && pa != part_attr.end() ? pa->second : -1;
  }
  void push_device_chain(int stream, const DevChain& dc, int64_t now, hipStream_t s) override {
    auto it = local.find(stream);
    if (it == local.end() || dc.n <= 0) return;
    const int ls = it->second;
    const int64_t cnt = dc.n, need = n + cnt;
    ev_ts.reserve(need, true, s, n);
    ev_stream.reserve(need, true, s, n);
    ev_row.reserve(need, true, s, n);
    ev_now.reserve(need, true, s, n);
    auto& cs = cols[ls];
    if (dc.d_cols.size() != cs.size()) throw Error(SG_E_INVALID, "chained output arity differs from the inserted stream");
    for (auto& c : cs) c.b.reserve((rows[ls] + cnt) * c.w, true, s, rows[ls] * c.w);
    SG_HIP(hipMemcpyAsync(ev_ts.p + n, dc.d_ts, cnt * 8, hipMemcpyDeviceToDevice, s));
    SG_HIP(hipMemcpyAsync(ev_now.p + n, dc.d_now, cnt * 8, hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_nfa_ev_fill, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, ev_stream.p + n,
                       ev_row.p + n, (int64_t*)nullptr, (int8_t)ls, (int32_t)rows[ls], now, cnt);
    SG_HIP(hipGetLastError());
    for (size_t k = 0; k < cs.size(); k++) {
      if (dc.widths[k] != cs[k].w) throw Error(SG_E_INVALID, "chained column width differs from the inserted stream");
      SG_HIP(hipMemcpyAsync(cs[k].b.p + rows[ls] * cs[k].w, dc.d_cols[k], cnt * cs[k].w, hipMemcpyDeviceToDevice, s));
    }
    if (has_nul[ls]) {               // (chained rows carry no nulls)
      nulcol[ls].reserve((rows[ls] + cnt) * cs.size(), true, s, rows[ls] * cs.size());
      SG_HIP(hipMemsetAsync(nulcol[ls].p + rows[ls] * cs.size(), 0, cnt * cs.size(), s));
    }
    const bool keyed = dc.key_attr >= 0;
    book(ls, cnt, keyed ? dc.key : nullptr, keyed ? dc.widths[dc.key_attr] : 4, nullptr, 0, dc.seq,
         nullptr, now);
    SG_HIP(hipStreamSynchronize(s));
    rows[ls] += cnt;
    n += cnt;
    chain_dev_rows += cnt;
  }
  int64_t chain_dev_rows = 0;
  // sg_push_device_seq: the events of the last device push carry global arrival seqs (a rank's key-routed
  // share of the stream, siddhi_amd/shard.py): callbacks take them, and the merge by seq across ranks restores
  // the single runtime's order.  They must increase (source-rank order of the all-to-all keeps them so).
  int64_t dev_push_h0 = 0, dev_push_n = 0;
  void set_device_seq(const int64_t* d_seq) override {
    if (dev_push_n <= 0 || !d_seq) return;
    if (tab.nabs > 0) throw Error(-2, "device arrival seqs for a query with absent states: use sg_push_shard");
    SG_HIP(hipMemcpy(h_seq.data() + dev_push_h0, d_seq, (size_t)dev_push_n * 8, hipMemcpyDeviceToHost));
    for (int64_t e = std::max<int64_t>(dev_push_h0, 1); e < dev_push_h0 + dev_push_n; e++)
      if (h_seq[e] <= h_seq[e - 1]) throw Error(SG_E_INVALID, "device arrival seqs must increase");
    dev_push_n = 0;
  }

  void reset() override {
    PhaseClock pc(getenv("SG_HOST_TIMING") != nullptr);
    if (selector) selector->clear();
    n = 0; flushed = 0; h_seq.clear(); h_stream.clear(); h_lane.clear(); key_lane.clear(); lane_key.clear();
    last_seen.clear();
    skip_done = 0;
    rank_ev.clear(); dense_lane.clear(); create_rank.clear(); lane_hash_c.clear();
    deferrals.clear();
    fx = 0; fk = 0; f_fresh = true; fL = 0; fmaps.clear();
    shard_run = RunOut(); shard_dirty = false;
    tick_now.clear(); tick_seq.clear(); tick_ev.clear(); ticks_flushed = 0;
    for (auto& r : rows) r = 0;
    for (auto& h : has_nul) h = false;
    pc.mark("reset: host state");
    if (L) {
      NState ns = state();
      hipLaunchKernelGGL(k_nfa_pool_init, dim3((unsigned)((L + 255) / 256)), dim3(256), 0, app->stream, ns, 0, L);
      SG_HIP(hipStreamSynchronize(app->stream));
    }
    pc.mark("reset");
  }

  // Java HashMap iteration order of one Scheduler's key -> SchedulerState map (JDK 8 computeIfAbsent
  // inserts at the head of its bin and resizes when size > threshold; resize keeps relative order;
  // a bin of 8 at capacity < 64 resizes).  Only the exact replay below uses it.
  struct SchedMap {
    std::vector<std::vector<std::pair<int32_t, int32_t>>> tab;   // bin -> chain of (hash, lane)
    size_t size = 0, thr = 0;
    void resize() {
      const size_t oc = tab.size();
      if (!oc) { tab.assign(16, {}); thr = 12; return; }
      std::vector<std::vector<std::pair<int32_t, int32_t>>> nt(oc * 2);
      for (size_t b = 0; b < oc; b++)
        for (auto& e : tab[b]) nt[((uint32_t)e.first & (uint32_t)oc) ? b + oc : b].push_back(e);
      tab.swap(nt);
      thr *= 2;
    }
    void touch(int32_t h, int32_t lane) {
      if (size > thr || tab.empty()) resize();
      auto& bin = tab[(uint32_t)h & (uint32_t)(tab.size() - 1)];
      for (auto& e : bin) if (e.second == lane) return;
      const size_t cnt = bin.size();
      bin.insert(bin.begin(), {h, lane});
      if (cnt >= 7) {
        if (tab.size() < 64) resize();
        else throw Error(-2, "partition Scheduler map bin would be treeified (not lowered)");
      }
      size++;
    }
    void remove(int32_t h, int32_t lane) {
      if (tab.empty()) return;
      auto& bin = tab[(uint32_t)h & (uint32_t)(tab.size() - 1)];
      for (size_t i = 0; i < bin.size(); i++)
        if (bin[i].second == lane) { bin.erase(bin.begin() + i); size--; return; }
    }
    int64_t rank(int32_t h, int32_t lane) const {   // position in iteration order
      const size_t b = (uint32_t)h & (uint32_t)(tab.size() - 1);
      for (size_t i = 0; i < tab[b].size(); i++)
        if (tab[b][i].second == lane) return ((int64_t)b << 32) | (int64_t)i;
      return INT64_MAX;
    }
  };

  // HashMap.hash(String.hashCode()) of the partition key's toString()
  int32_t lane_hash(int lane) const { return java_key_hash(*app, key_ty, lane_key[lane]); }

  struct RunOut {
    uint32_t nrec = 0;
    std::vector<uint8_t> task_ok;   // speculative run: records of task t are kept iff task_ok[t] (-1: kept)
    std::vector<FireRec> fires;
    std::vector<OpRec> ops;
    int64_t fires_dev = 0;          // firings left in d_fire (fire_lazy: not copied to the host yet)
    size_t fire_tk0 = 0;            // their ticks are relative to this one
  };
  bool fire_lazy = false;           // run_lanes leaves the firing log on the device (flush's pre-check)
  DBuf<uint64_t> fk_keys, fk_sorted;
  DBuf<uint8_t> fk_tmp, fk_ok;
  DBuf<uint32_t> fk_flag;
  // Could two firings of the run share (tick, scheduler, head)?  On the device: keys, a radix sort, a neighbour
  // test and one flag copied back -- instead of copying the whole log and checking it on the host.  False means
  // no collision; true only a possible one (the caller then copies the log and checks it exactly).
  bool fires_may_collide(const RunOut& ro, hipStream_t s) {
    const int64_t n = ro.fires_dev;
    if (n < 2) return false;
    fk_keys.reserve(n); fk_sorted.reserve(n); fk_flag.reserve(1);
    const uint8_t* okp = nullptr;
    if (!ro.task_ok.empty()) {
      fk_ok.reserve(ro.task_ok.size());
      SG_HIP(hipMemcpyAsync(fk_ok.p, ro.task_ok.data(), ro.task_ok.size(), hipMemcpyHostToDevice, s));
      okp = fk_ok.p;
    }
    hipLaunchKernelGGL(k_fire_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_fire.p, n, okp, fk_keys.p);
    SG_HIP(hipGetLastError());
    size_t tb = 0;
    SG_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, fk_keys.p, fk_sorted.p, (int)n, 0, 64, s));
    fk_tmp.reserve(std::max<size_t>(tb, 1));
    SG_HIP(hipcub::DeviceRadixSort::SortKeys(fk_tmp.p, tb, fk_keys.p, fk_sorted.p, (int)n, 0, 64, s));
    SG_HIP(hipMemsetAsync(fk_flag.p, 0, 4, s));
    hipLaunchKernelGGL(k_adj_dup, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, fk_sorted.p, n, fk_flag.p);
    SG_HIP(hipGetLastError());
    uint32_t flag = 0;
    SG_HIP(hipMemcpyAsync(&flag, fk_flag.p, 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    return flag != 0;
  }
  // the firing log the pre-check left on the device, as run_lanes would have returned it
  void fetch_fires(RunOut& ro, hipStream_t s) {
    if (ro.fires_dev <= 0) return;
    ro.fires.resize((size_t)ro.fires_dev);
    SG_HIP(hipMemcpyAsync(ro.fires.data(), d_fire.p, (size_t)ro.fires_dev * sizeof(FireRec), hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    if (!ro.task_ok.empty())
      ro.fires.erase(std::remove_if(ro.fires.begin(), ro.fires.end(),
                                    [&](const FireRec& f) { return f.task >= 0 && !ro.task_ok[(size_t)f.task]; }),
                     ro.fires.end());
    for (auto& f : ro.fires) f.tau += (int32_t)ro.fire_tk0;
    ro.fires_dev = 0;
  }

  // kinds and modes the lowered table uses (FM_*)
  int feature_mask() const {
    int fm = tab.seq ? FM_SEQ : FM_PAT;
    if (tab.within >= 0) fm |= FM_WITHIN;
    if (tab.nabs > 0) fm |= FM_ABS;
    for (int p = 0; p < tab.nproc; p++) {
      if (tab.p[p].kind == K_ABSENT || tab.p[p].absLog) fm |= FM_ABS;
      if (tab.p[p].kind == K_LOGICAL) fm |= FM_LOG;
      if (tab.p[p].kind == K_COUNT) fm |= FM_CNT;
    }
    if (getenv("SG_NFA_GENERIC")) fm = FM_ALL;      // measurement hook: the unspecialised interpreter
    return fm;
  }
  // the smallest instantiated interpreter whose mask covers `fm`
  static const void* lanes_kernel(int fm) {
    static const int masks[] = {FM_SEQ, FM_SEQ | FM_CNT, FM_SEQ | FM_WITHIN, FM_SEQ | FM_CNT | FM_WITHIN,
                                FM_PAT, FM_PAT | FM_CNT, FM_PAT | FM_WITHIN, FM_PAT | FM_CNT | FM_WITHIN,
                                FM_PAT | FM_LOG, FM_PAT | FM_ABS, FM_PAT | FM_LOG | FM_ABS, FM_ALL};
    static const void* fns[] = {
        (const void*)k_nfa_lanes<FM_SEQ>, (const void*)k_nfa_lanes<FM_SEQ | FM_CNT>,
        (const void*)k_nfa_lanes<FM_SEQ | FM_WITHIN>, (const void*)k_nfa_lanes<FM_SEQ | FM_CNT | FM_WITHIN>,
        (const void*)k_nfa_lanes<FM_PAT>, (const void*)k_nfa_lanes<FM_PAT | FM_CNT>,
        (const void*)k_nfa_lanes<FM_PAT | FM_WITHIN>, (const void*)k_nfa_lanes<FM_PAT | FM_CNT | FM_WITHIN>,
        (const void*)k_nfa_lanes<FM_PAT | FM_LOG>, (const void*)k_nfa_lanes<FM_PAT | FM_ABS>,
        (const void*)k_nfa_lanes<FM_PAT | FM_LOG | FM_ABS>, (const void*)k_nfa_lanes<FM_ALL>};
    for (size_t k = 0; k < sizeof(masks) / sizeof(masks[0]); k++)
      if ((fm & ~masks[k]) == 0) return fns[k];
    return (const void*)k_nfa_lanes<FM_ALL>;
  }

  // One launch of the lane interpreter over nl lanes (speculative tasks when spec is given).  Lanes per
  // workgroup (<= NFA_B; the register file keeps its NFA_B stride): a lane is a long chain of dependent pool
  // accesses, so with few lanes (e.g. K = 1000 partition keys) they are spread over as many waves (CUs) as
  // possible: halve the workgroup until there are >= 1024 of them, down to one lane per workgroup (config 3,
  // K = 1000, LDS pools: 4 lanes/wave 465 ms, 1 lane 374 ms).
  int64_t lds_max_lanes() const {
    return getenv("SG_NFA_LDS_MAX_LANES") ? atoll(getenv("SG_NFA_LDS_MAX_LANES")) : 8192;
  }
  bool blocked_launch = false;      // the launch runs scratch tasks on blocked pools (run_spec)
  void launch_lanes(NArgs& a, int nl, const NSpec* d_spec, hipStream_t s, const int* caps = nullptr) {
    if (nl <= 0) return;
    a.nl = nl;
    // pool capacities of the lanes (speculative scratch lanes may run smaller ones)
    const int c_se = caps ? caps[0] : se_cap, c_nd = caps ? caps[1] : nd_cap, c_list = caps ? caps[2] : list_cap;
    // the lanes' pools go to LDS when at least one lane fits beside the table, programs and register file
    NLds lay;
    lay.build(c_se, c_nd, c_list, nq(), 1, std::max(1, (int)tab.nslots), std::max(1, (int)tab.nproc));
    const size_t lane_b = lay.bytes + MAX_REG * sizeof(int64_t) + 64;
    const size_t fixed = NLds::al(progs.size() * sizeof(Prog)) + sizeof(NCols) + sizeof(NTable) + 1024;
    const size_t cu_lds = 160 * 1024;
    const int lds_lanes = (int)std::min<size_t>(NFA_B, cu_lds > fixed ? (cu_lds - fixed) / lane_b : 0);
    // (a window of the exact sweep runs a few events per lane: staging whole pools through LDS costs more than it saves;
    // and a launch of many lanes -- speculative segments -- keeps its pools in global memory too: LDS caps a CU at ~50
    // lanes of 3 KB, while from L2 the lanes of every resident wave run, config 5's 79,000 segments 17.1 -> 8.4 ms,
    // config 3's 78,620 14.9 -> 11.4 ms; SG_NFA_LDS_MAX_LANES, default 8192)
    const bool use_lds = lds_lanes >= 1 && !in_sweep && !getenv("SG_NFA_NO_LDS") && nl < lds_max_lanes();
    // lanes per workgroup (one wave): measured wider is better (config 3, 20K speculative tasks: 1 lane per
    // workgroup 148 ms, 2: 125, 4-8: 113, 16-32: 110): the lanes of a wave share its issue slots almost for
    // free while the workgroups per CU are LDS-bound.  Halve from 64 only to keep >= 1024 workgroups (few
    // lanes: config 3 without segments, K = 1000, runs one lane per workgroup on as many CUs as possible).
    int tpb = NFA_B;
    while (tpb > 1 && (nl + tpb - 1) / tpb < 1024) tpb /= 2;
    if (in_sweep) tpb = NFA_B;
    if (use_lds) tpb = std::min(tpb, lds_lanes);
    if (const char* x = getenv("SG_NFA_TPB")) tpb = std::max(1, std::min(use_lds ? lds_lanes : NFA_B, atoi(x)));   // tuning hook
    if (blocked_launch) while (tpb & (tpb - 1)) tpb &= tpb - 1;   // (blocked scratch pools: a workgroup within one block)
    // one lane per workgroup on LDS pools: the lane takes the whole wavefront (wide mode, NArgs::wide) -- the same
    // waves and LDS as one-thread workgroups, with the wave's other 63 threads splitting the list-parallel steps
    // (within expiry as a ballot + popc-rank compaction) and the pool staging
    const bool wide = tpb == 1 && use_lds && !(getenv("SG_NFA_WIDE") && atoi(getenv("SG_NFA_WIDE")) == 0);
    a.wide = wide ? 1 : 0;
    if (use_lds) lay.build(c_se, c_nd, c_list, nq(), tpb, lay.ns, lay.np);
    else lay.bytes = 0;
    lay.finish((int)progs.size(), tpb);
    kernel_ms["nfa_lanes_per_wg"] = tpb;
    kernel_ms["nfa_wide"] = wide ? 1 : 0;
    kernel_ms["nfa_lane_pool_lds_bytes"] = use_lds ? (double)lay.bytes / tpb : 0.0;   // 0: pools in HBM
    kernel_ms["nfa_lane_pool_bytes_needed"] = (double)lane_b;
    NState st = state();
    const NTable* dt = d_tab.p;
    const NCols* dc = d_cols.p;
    const Prog* dp = d_progs.p;
    void* kargs[] = {&a, &st, &lay, &dt, &dc, &dp, &d_spec};
    const unsigned nwg = (unsigned)((nl + tpb - 1) / tpb);
    const unsigned nthr = wide ? 64u : (unsigned)tpb;
    if (const hipFunction_t cf = compiled_kernel()) {  // the query's compiled kernel (nfa_rtc.hpp)
      kernel_ms["nfa_compiled"] = 1;
      SG_HIP(hipModuleLaunchKernel(cf, nwg, 1, 1, nthr, 1, 1, (unsigned)lay.total, s, kargs, nullptr));
      SG_HIP(hipGetLastError());
      return;
    }
    kernel_ms["nfa_compiled"] = 0;
    const void* kfn = lanes_kernel(feature_mask());
    if (kfn != attr_fn || (int)lay.total > attr_lds) {   // (a host call per launch otherwise)
      SG_HIP(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lay.total));
      attr_fn = kfn;
      attr_lds = (int)lay.total;
    }
    SG_HIP(hipLaunchKernel(kfn, dim3(nwg), dim3(nthr), kargs, lay.total, s));
    SG_HIP(hipGetLastError());
  }

  bool kernel_source(std::string& out) override {
    out = nfa_rtc_source(tab, progs, feature_mask());
    return true;
  }
  bool compile_kernel(double& ms, bool& from_disk, std::string& err) override {
    std::vector<char> code;
    RtcKernel k;
    const bool ok = rtc_code(nfa_rtc_source(tab, progs, feature_mask()), code, k);
    ms = k.compile_ms; from_disk = k.from_disk; err = k.err;
    return ok;
  }

  // ---- the query's compiled kernel (nfa_rtc.hpp) ----
  // SG_NFA_RTC=0: never (the interpreter runs every launch); =1: every launch, compiled synchronously at the first
  // (tests).  Default: from the first launch if the code object is in the process or disk cache (a file read and a
  // module load); otherwise, once the query has run SG_NFA_RTC_MIN events (65,536, summed over its flushes, so a
  // streaming caller that flushes small chunks gets there too), hipRTC compiles it on a background thread
  // (nfa_rtc.hpp rtc_compile_async, 10-70 s) while the interpreter keeps serving, and every launch after it is ready
  // runs the compiled kernel, whatever its size.  No flush waits for hipRTC.  A query whose source fails to compile
  // keeps the interpreter, with the reason on stderr.
  RtcKernel rtc;
  bool rtc_tried = false;             // the caches were looked up (default mode)
  bool rtc_started = false;           // a background compile was started (or, with SG_NFA_RTC=1, a synchronous one)
  std::string rtc_src;
  std::shared_ptr<RtcJob> rtc_job;
  int64_t launch_events = 0;          // events of the current run (run_lanes)
  int64_t seen_events = 0;            // events run so far (run_lanes, summed)
  hipFunction_t compiled_kernel() {
    const char* e = getenv("SG_NFA_RTC");
    if (e && e[0] == '0') return nullptr;
    if (rtc.fn) return rtc.fn;
    if (e && e[0] == '1') {
      if (!rtc_started) {
        rtc_started = true;
        rtc = nfa_rtc_get(nfa_rtc_source(tab, progs, feature_mask()));
        kernel_ms["nfa_rtc_compile_ms"] = rtc.compile_ms;
        if (!rtc.err.empty()) fprintf(stderr, "[sg nfa] compiled kernel unavailable, the interpreter runs: %s\n", rtc.err.c_str());
      }
      return rtc.fn;
    }
    if (!rtc_tried) {
      rtc_tried = true;
      rtc_src = nfa_rtc_source(tab, progs, feature_mask());
      if (nfa_rtc_cached(rtc_src, rtc)) {
        kernel_ms["nfa_rtc_compile_ms"] = 0;
        return rtc.fn;
      }
    }
    if (rtc_job) {
      if (!rtc_job->done.load(std::memory_order_acquire)) return nullptr;
      rtc = nfa_rtc_from_job(rtc_src, *rtc_job);
      rtc_job.reset();
      kernel_ms["nfa_rtc_compile_ms"] = rtc.compile_ms;
      if (!rtc.err.empty()) fprintf(stderr, "[sg nfa] compiled kernel unavailable, the interpreter runs: %s\n", rtc.err.c_str());
      return rtc.fn;
    }
    const int64_t lim = getenv("SG_NFA_RTC_MIN") ? atoll(getenv("SG_NFA_RTC_MIN")) : (1 << 16);
    if (!rtc_started && seen_events >= lim) {
      rtc_started = true;
      rtc_job = rtc_compile_async(rtc_src);
      kernel_ms["nfa_rtc_background"] = 1;
    }
    return nullptr;
  }

  // ---- speculative time segments (NSpec) ----
  struct SpecPlan {
    std::vector<int32_t> w0, e0, e1, pool, lane, prev;   // per task: the keys' first segments, then the rest
    std::vector<uint8_t> tail;                           // per task: the key's last segment
    std::vector<int32_t> ks0, kn;                  // per CSR lane: its first scratch task, its segments
    int32_t nkeys = 0, nscratch = 0;
    std::vector<uint8_t> ok;                       // per task: records kept
  };
  // scratch pools (grown when too many segments overflow): StateEvents, chain nodes, list entries.  (16 / 64 / 16 until
  // round 6; with the pools in global memory a smaller footprint is faster -- config 3 k_nfa_lanes 9.8 -> 9.35 ms,
  // config 5 11.2 -> 10.4 ms, profiles/r06o_b*caps_*)
  int sp_caps[3] = {8, 32, 8};
  bool sp_caps_env = false;
  DBuf<int32_t> sp_w0, sp_e0, sp_e1, sp_pool, sp_lane, sp_prev, sp_canon, sp_cmap, sp_fix_off, sp_fix_ev, sp_fix_lid, sp_pairs;
  DBuf<int32_t> rp_arr, rp_canon, rp_cmap;         // repair rounds: per fix task e0 / e1 / lane / next task, forms
  DBuf<int32_t> rec_task;
  DBuf<uint8_t> sp_ok, sp_scratch, sp_tail, rp_tail, rp_ok;
  DBuf<NSpec> d_spec;
  hipEvent_t sp_ev[4] = {nullptr, nullptr, nullptr, nullptr};

  // Segment the long lanes of a flush (events per CSR lane in off) when the lanes are too few to fill the
  // chip: segments of S events, each after the first with a warm-up of H events.  Not for broadcast streams (their
  // events enter several instances), shard mode, nor logged runs (the exact Scheduler sweep); absent states are
  // segmented too (a segment runs the ticks before each of its events, its firings count only once it verifies).
  bool plan_spec(const std::vector<int32_t>& off, const std::vector<int32_t>& lid, SpecPlan& p) {
    const char* force = getenv("SG_NFA_SPEC");
    if (force && force[0] == '0') return false;
    if (shard || std::any_of(std::begin(bcast), std::end(bcast), [](bool x) { return x; })) return false;
    // segment / warm-up lengths (config 3, 10M events over 1000 keys, round 3 interpreter: 512 events 60 ms, 256: 61,
    // 128: 50; warm-ups of 16-48 events rebuilt every segment's state, none re-ran.  Round 6, compiled kernel with its
    // pools in global memory, `k_nfa_lanes`: 64 / 32 events 13.1 ms, 96 / 32 10.4, 128 / 32 11.5, 128 / 16 10.5,
    // 192 / 32 14.5, 256 / 48 17.4 -- profiles/r06l_t3_*).  Absent states need a longer warm-up:
    // a drained absent processor re-arms itself every `for` period (notifyAt(ct + waiting) when nothing fired), and
    // that chain of deadlines ends only when it fires over a pending partial, so a segment's Scheduler queue is
    // rebuilt once its warm-up spans a few waits with partials in them (config 5, 256-event segments: 128-event
    // warm-ups leave 0.3 % of the segments unverified, and the repair rounds of run_spec re-run just those)
    const bool abs_q = tab.nabs > 0;
    const int64_t S = getenv("SG_NFA_SEG") ? std::max(16, atoi(getenv("SG_NFA_SEG"))) : abs_q ? 256 : 96;
    const int64_t H = getenv("SG_NFA_WARM") ? std::max(1, atoi(getenv("SG_NFA_WARM"))) : abs_q ? 128 : 32;
    const int nl = (int)lid.size();
    int32_t longest = 0;
    for (int q = 0; q < nl; q++) longest = std::max(longest, off[q + 1] - off[q]);
    // worth it when a few long lanes would leave the chip idle: fewer lanes than ~16 per CU
    if (!force && (longest < 4 * S || nl > 4096)) return false;
    // tasks [0, nl): each key's first segment on its own pools; then the later segments, key by key
    std::vector<int64_t> G(nl);
    for (int q = 0; q < nl; q++) {
      const int32_t c = off[q + 1] - off[q];
      G[q] = c >= 2 * S ? (c + S - 1) / S : 1;
      p.e0.push_back(off[q]);
      p.e1.push_back(G[q] == 1 ? off[q + 1] : off[q] + (int32_t)S);
      p.w0.push_back(off[q]);
      p.pool.push_back(lid[q]);
      p.lane.push_back(lid[q]);
      p.prev.push_back(-1);
      p.tail.push_back(G[q] == 1);
    }
    p.nkeys = nl;
    for (int q = 0; q < nl; q++) {
      p.ks0.push_back((int32_t)p.w0.size());
      p.kn.push_back((int32_t)G[q]);
      for (int64_t g = 1; g < G[q]; g++) {
        const int32_t e0 = off[q] + (int32_t)(g * S);
        p.prev.push_back(g == 1 ? q : (int32_t)p.w0.size() - 1);
        p.e0.push_back(e0);
        p.e1.push_back(g + 1 == G[q] ? off[q + 1] : e0 + (int32_t)S);
        p.w0.push_back(std::max<int32_t>(off[q], e0 - (int32_t)H));
        p.pool.push_back(-(++p.nscratch));
        p.lane.push_back(lid[q]);
        p.tail.push_back(g + 1 == G[q]);
      }
    }
    return p.nscratch > 0;
  }

  // pools of L lanes carved from one device buffer (the scratch lanes of speculative tasks)
  NState carve(DBuf<uint8_t>& buf, int64_t nl, int se_cap, int nd_cap, int list_cap, bool blocked = false) {
    if (blocked) nl = (nl + 63) / 64 * 64;          // whole blocks of 64 lanes (nfa_block_view)
    NState g;
    g.L = nl; g.se_cap = se_cap; g.nd_cap = nd_cap; g.list_cap = list_cap; g.nq = nq();
    const int64_t per[24] = {(int64_t)se_cap * NS * 4, (int64_t)se_cap * 8, se_cap, (int64_t)se_cap * 4, (int64_t)se_cap * 4, 4,
                             (int64_t)nd_cap * 4, (int64_t)nd_cap * 4, (int64_t)nd_cap * 4, (int64_t)nd_cap * 4, 4,
                             (int64_t)NP * list_cap * 4, NP * 4, (int64_t)NP * list_cap * 4, NP * 4, NP * 4, 4, 4,
                             (int64_t)list_cap * 4, NP * 8, (int64_t)nq() * NTQ * 8, (int64_t)nq() * 4,
                             (int64_t)nq() * NTQ * 4, (int64_t)nq() * 4};
    size_t tot = 0;
    for (int k = 0; k < 24; k++) tot += (size_t)((per[k] * nl + 255) / 256 * 256);
    buf.reserve(tot);
    uint8_t* b = buf.p;
    void* q[24];
    for (int k = 0; k < 24; k++) { q[k] = b; b += (per[k] * nl + 255) / 256 * 256; }
    g.se_slot = (int32_t*)q[0]; g.se_ts = (int64_t*)q[1]; g.se_type = (int8_t*)q[2]; g.se_ref = (int32_t*)q[3];
    g.se_free = (int32_t*)q[4]; g.se_top = (int32_t*)q[5]; g.nd_ev = (int32_t*)q[6]; g.nd_next = (int32_t*)q[7];
    g.nd_ref = (int32_t*)q[8]; g.nd_free = (int32_t*)q[9]; g.nd_top = (int32_t*)q[10]; g.pend = (int32_t*)q[11];
    g.npend = (int32_t*)q[12]; g.nev = (int32_t*)q[13]; g.nnev = (int32_t*)q[14]; g.flags = (uint32_t*)q[15];
    g.created = (int32_t*)q[16]; g.err = (int32_t*)q[17]; g.ret = (int32_t*)q[18]; g.lst = (int64_t*)q[19];
    g.tq = (int64_t*)q[20]; g.ntq = (int32_t*)q[21]; g.tqc = (int32_t*)q[22]; g.tqh = (int32_t*)q[23];
    return g;
  }

  // Run the tasks, verify them, move each key's verified end state into its lane and re-run a key from
  // the end of its last verified segment where a segment did not verify.  p.ok: records of task t kept.
  void run_spec(NArgs& a, SpecPlan& p, const pvec<int32_t>& evs, hipStream_t s) {
    const int nt = (int)p.w0.size();
    auto up = [&](DBuf<int32_t>& d, const std::vector<int32_t>& h) {
      d.reserve(std::max<size_t>(h.size(), 1));
      if (!h.empty()) SG_HIP(hipMemcpyAsync(d.p, h.data(), h.size() * 4, hipMemcpyHostToDevice, s));
    };
    up(sp_w0, p.w0); up(sp_e0, p.e0); up(sp_e1, p.e1); up(sp_pool, p.pool); up(sp_lane, p.lane); up(sp_prev, p.prev);
    sp_tail.reserve(nt);
    SG_HIP(hipMemcpyAsync(sp_tail.p, p.tail.data(), nt, hipMemcpyHostToDevice, s));
    if (const char* c = getenv("SG_NFA_SPEC_CAPS")) {   // measurement hook: "se,nd,list" of the scratch pools
      int v[3] = {0, 0, 0};
      if (sscanf(c, "%d,%d,%d", &v[0], &v[1], &v[2]) == 3 && !sp_caps_env) {
        for (int k = 0; k < 3; k++) sp_caps[k] = std::max(4, v[k]);
        sp_caps_env = true;
      }
    }
    for (int k = 0; k < 3; k++) sp_caps[k] = std::min(sp_caps[k], k == 0 ? se_cap : k == 1 ? nd_cap : list_cap);
    if (getenv("SG_NFA_SPEC_FULLCAPS")) { sp_caps[0] = se_cap; sp_caps[1] = nd_cap; sp_caps[2] = list_cap; }
    const size_t cstride = 2 * (SG_CANON + 1), mstride = 2 * (size_t)se_cap + nd_cap;
    sp_canon.reserve((size_t)nt * cstride);
    sp_cmap.reserve((size_t)nt * mstride);
    sp_ok.reserve(nt);
    // scratch pools in blocks of 64 lanes when their launch keeps them in global memory (launch_lanes)
    const bool blocked = p.nscratch >= lds_max_lanes() && !getenv("SG_NFA_NO_BLOCK");
    NSpec h[2];
    std::memset(h, 0, sizeof(h));
    for (int k = 0; k < 2; k++) {
      h[k].w0 = sp_w0.p; h[k].e0 = sp_e0.p; h[k].e1 = sp_e1.p; h[k].pool = sp_pool.p; h[k].tail = sp_tail.p;
      h[k].gs = carve(sp_scratch, p.nscratch, sp_caps[0], sp_caps[1], sp_caps[2], blocked);
      h[k].canon = sp_canon.p; h[k].cmap = sp_cmap.p; h[k].ntask = nt; h[k].cmap_stride = (int32_t)mstride;
    }
    h[0].q0 = 0;            // the keys' first segments, on the instances' pools
    h[1].q0 = p.nkeys;      // the later segments, on scratch pools
    h[1].blocked = blocked ? 1 : 0;
    kernel_ms["nfa_spec_blocked"] = blocked ? 1 : 0;
    d_spec.reserve(3);
    SG_HIP(hipMemcpyAsync(d_spec.p, h, sizeof(h), hipMemcpyHostToDevice, s));
    const int32_t* key_lane_ids = a.lane_id;
    a.lane_id = sp_lane.p;
    rec_task.reserve((size_t)a.rec_cap);
    a.rec_task = rec_task.p;
    if (!sp_ev[0]) for (auto& e : sp_ev) SG_HIP(hipEventCreate(&e));
    SG_HIP(hipEventRecord(sp_ev[0], s));
    blocked_launch = blocked;
    launch_lanes(a, p.nscratch, d_spec.p + 1, s, sp_caps);
    blocked_launch = false;
    launch_lanes(a, p.nkeys, d_spec.p, s);
    SG_HIP(hipEventRecord(sp_ev[1], s));
    hipLaunchKernelGGL(k_nfa_spec_verify, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, sp_prev.p, sp_canon.p, nt,
                       sp_ok.p);
    SG_HIP(hipGetLastError());
    std::vector<uint8_t> ok(nt);
    std::vector<int32_t> serr(p.nscratch);
    SG_HIP(hipMemcpyAsync(ok.data(), sp_ok.p, nt, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(serr.data(), h[1].gs.err, (size_t)p.nscratch * 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    // per key: its segments that did not verify (or failed in their scratch pools).  Repair rounds re-run such a
    // segment from the key's true state; once its true end state equals the next segment's post-warm-up state, the
    // segments up to the next unverified one stand as they ran.  A key still unrepaired after SG_NFA_REPAIR_ROUNDS
    // rounds (default 8; 0: none, the whole rest of every unverified key re-runs at once) re-runs its rest in one go.
    std::vector<int32_t> pairs, fix_off(1, 0), fix_ev, fix_lid;
    int64_t nbad = 0, nover = 0;
    for (int32_t e : serr) nover += e != 0;
    p.ok.assign(nt, 1);
    auto task_of = [&](int q, int32_t g) { return g == 0 ? q : p.ks0[q] + g - 1; };
    auto bad_seg = [&](int q, int32_t g) {
      const int32_t t = task_of(q, g);
      return !ok[t] || serr[-p.pool[t] - 1] != 0;
    };
    auto next_bad = [&](int q, int32_t g) {        // first unverified segment >= g (kn[q] if none)
      while (g < p.kn[q] && !bad_seg(q, g)) g++;
      return g;
    };
    std::vector<int32_t> cur(p.nkeys, -1);          // per key: the segment the next round re-runs (-1: done)
    int64_t ncur = 0;
    for (int q = 0; q < p.nkeys; q++) {
      const int32_t n_seg = p.kn[q];
      const int32_t g = next_bad(q, 1), key = p.lane[q];
      if (g == n_seg) {                      // every segment verified: the last one's end state is the key's
        if (n_seg > 1) { pairs.push_back(key); pairs.push_back(-p.pool[task_of(q, n_seg - 1)] - 1); }
        continue;
      }
      cur[q] = g;
      ncur++;
      if (g > 1) { pairs.push_back(key); pairs.push_back(-p.pool[task_of(q, g - 1)] - 1); }
    }
    kernel_ms["nfa_spec_tasks"] = nt;
    kernel_ms["nfa_spec_overflows"] = (double)nover;
    if (getenv("SG_NFA_SPEC_STATS")) {     // diagnostics: canonical forms that did not fit, their longest
      std::vector<int32_t> cl((size_t)nt * cstride);
      SG_HIP(hipMemcpy(cl.data(), sp_canon.p, cl.size() * 4, hipMemcpyDeviceToHost));
      int64_t nfit = 0, mx = 0, nmis = 0;
      for (int t = 0; t < nt; t++)
        for (int k = 0; k < 2; k++) {
          const int32_t len = cl[(size_t)t * cstride + k * (SG_CANON + 1)];
          if (k == 0 && p.prev[t] < 0) continue;
          nfit += len < 0;
          mx = std::max<int64_t>(mx, len);
        }
      for (int t = 0; t < nt; t++) nmis += p.prev[t] >= 0 && !ok[t];
      if (atoi(getenv("SG_NFA_SPEC_STATS")) > 1) {   // the first mismatched pairs: prev's end form, then t's warm-up form
        int shown = 0;
        for (int t = 0; t < nt && shown < 6; t++) {
          if (p.prev[t] < 0 || ok[t]) continue;
          shown++;
          for (int k = 0; k < 2; k++) {
            const int32_t* f = cl.data() + (size_t)(k ? t : p.prev[t]) * cstride + (k ? 0 : SG_CANON + 1);
            fprintf(stderr, "[sg spec] task %d %s len %d:", t, k ? "warm" : "prev-end", f[0]);
            for (int z = 0; z < std::min(f[0], 96); z++) fprintf(stderr, " %d", f[1 + z]);
            fprintf(stderr, "\n");
          }
        }
      }
      kernel_ms["nfa_spec_canon_unfit"] = (double)nfit;
      kernel_ms["nfa_spec_canon_max"] = (double)mx;
      kernel_ms["nfa_spec_mismatch"] = (double)nmis;
    }
    // scratch pools too small for this stream (more than 1 % of the segments overflowed): larger next flush
    if (nover * 100 > p.nscratch) {
      sp_caps[0] = std::min(se_cap, sp_caps[0] * 2);
      sp_caps[1] = std::min(nd_cap, sp_caps[1] * 2);
      sp_caps[2] = std::min(list_cap, sp_caps[2] * 2);
    }
    auto xfer = [&]() {
      if (pairs.empty()) return;
      up(sp_pairs, pairs);
      hipLaunchKernelGGL(k_nfa_lane_xfer, dim3((unsigned)((pairs.size() / 2 + 63) / 64)), dim3(64), 0, s, state(),
                         h[1].gs, sp_pairs.p, (int32_t)(pairs.size() / 2), h[1].blocked);
      SG_HIP(hipGetLastError());
      pairs.clear();
    };
    xfer();
    SG_HIP(hipEventRecord(sp_ev[2], s));
    const int max_rounds = getenv("SG_NFA_REPAIR_ROUNDS") ? std::max(0, atoi(getenv("SG_NFA_REPAIR_ROUNDS"))) : 8;
    int rounds = 0;
    int64_t nrep = 0;
    // repair rounds: fix task i re-runs segment cur[q] of key q on the instance's pools (NSpec without a warm-up, its
    // task index i < nkeys: a key's first segment's index, whose records are always kept) and writes its end form
    std::vector<int32_t> rq, rhost;
    std::vector<uint8_t> rtail, rok;
    while (ncur > 0 && rounds < max_rounds) {
      rounds++;
      rq.clear();
      for (int q = 0; q < p.nkeys; q++) if (cur[q] >= 0) rq.push_back(q);
      const int nf = (int)rq.size();
      rhost.assign((size_t)nf * 4, 0);               // e0 | e1 | lane | next task (-1: none)
      rtail.assign(nf, 0);
      for (int i = 0; i < nf; i++) {
        const int q = rq[i];
        const int32_t g = cur[q], t = task_of(q, g);
        rhost[i] = p.e0[t];
        rhost[nf + i] = p.e1[t];
        rhost[2 * nf + i] = p.lane[q];
        rhost[3 * nf + i] = g + 1 < p.kn[q] ? task_of(q, g + 1) : -1;
        rtail[i] = g + 1 == p.kn[q];
        p.ok[t] = 0;                                  // its speculative records go, the re-run's stay
        nrep++;
      }
      up(rp_arr, rhost);
      rp_tail.reserve(nf);
      SG_HIP(hipMemcpyAsync(rp_tail.p, rtail.data(), nf, hipMemcpyHostToDevice, s));
      rp_canon.reserve((size_t)nf * cstride);
      rp_cmap.reserve((size_t)nf * mstride);
      NSpec hf = h[0];
      hf.w0 = rp_arr.p; hf.e0 = rp_arr.p; hf.e1 = rp_arr.p + nf; hf.pool = rp_arr.p + 2 * nf; hf.tail = rp_tail.p;
      hf.canon = rp_canon.p; hf.cmap = rp_cmap.p; hf.ntask = nf; hf.q0 = 0;
      SG_HIP(hipMemcpyAsync(d_spec.p + 2, &hf, sizeof(hf), hipMemcpyHostToDevice, s));
      a.lane_id = rp_arr.p + 2 * nf;
      launch_lanes(a, nf, d_spec.p + 2, s);
      a.lane_id = sp_lane.p;
      rp_ok.reserve(nf);
      hipLaunchKernelGGL(k_nfa_fix_verify, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, s, rp_canon.p, sp_canon.p,
                         rp_arr.p + 3 * nf, nf, rp_ok.p);
      SG_HIP(hipGetLastError());
      rok.resize(nf);
      SG_HIP(hipMemcpyAsync(rok.data(), rp_ok.p, nf, hipMemcpyDeviceToHost, s));
      SG_HIP(hipStreamSynchronize(s));
      for (int i = 0; i < nf; i++) {
        const int q = rq[i];
        const int32_t g = cur[q];
        if (g + 1 == p.kn[q]) { cur[q] = -1; ncur--; continue; }      // the instance holds the key's final state
        if (!rok[i] || serr[-p.pool[task_of(q, g + 1)] - 1]) { cur[q] = g + 1; continue; }
        const int32_t g2 = next_bad(q, g + 2);     // g + 1 stands on g's true end state: so do the segments up to g2
        if (g2 == p.kn[q]) {
          pairs.push_back(p.lane[q]); pairs.push_back(-p.pool[task_of(q, g2 - 1)] - 1);
          cur[q] = -1; ncur--;
        } else {
          pairs.push_back(p.lane[q]); pairs.push_back(-p.pool[task_of(q, g2 - 1)] - 1);
          cur[q] = g2;
        }
      }
      xfer();
    }
    // the keys the rounds did not finish: their rest in one re-run from the state the instance holds
    for (int q = 0; q < p.nkeys; q++) {
      if (cur[q] < 0) continue;
      const int32_t n_seg = p.kn[q];
      nbad += n_seg - cur[q];
      for (int32_t g = cur[q]; g < n_seg; g++) p.ok[task_of(q, g)] = 0;
      fix_lid.push_back(p.lane[q]);
      for (int32_t e = p.e0[task_of(q, cur[q])]; e < p.e1[task_of(q, n_seg - 1)]; e++) fix_ev.push_back(evs[e]);
      fix_off.push_back((int32_t)fix_ev.size());
    }
    kernel_ms["nfa_spec_repair_rounds"] = rounds;
    kernel_ms["nfa_spec_repaired_tasks"] = (double)nrep;
    kernel_ms["nfa_spec_rerun_tasks"] = (double)nbad;
    kernel_ms["nfa_spec_rerun_keys"] = (double)fix_lid.size();
    if (!fix_lid.empty()) {
      up(sp_fix_off, fix_off); up(sp_fix_ev, fix_ev); up(sp_fix_lid, fix_lid);
      a.lane_off = sp_fix_off.p; a.lane_ev = sp_fix_ev.p; a.lane_id = sp_fix_lid.p;
      a.lane_rec = nullptr;                       // (the records follow the flush's CSR, not the re-run's)
      launch_lanes(a, (int)fix_lid.size(), nullptr, s);
    }
    SG_HIP(hipEventRecord(sp_ev[3], s));
    SG_HIP(hipEventSynchronize(sp_ev[3]));
    float ms = 0;
    SG_HIP(hipEventElapsedTime(&ms, sp_ev[0], sp_ev[1])); kernel_ms["k_nfa_spec"] = ms;
    SG_HIP(hipEventElapsedTime(&ms, sp_ev[2], sp_ev[3])); kernel_ms["k_nfa_fixup"] = ms;
    a.lane_id = key_lane_ids;
    a.rec_task = nullptr;
  }

  // One launch of k_nfa_lanes over events [ev0, n) and ticks [tk0, #ticks) with the given
  // deferrals; logs firings (partitioned absent) and, in exact mode, every notifyAt.
  //
  // A window of the exact sweep (flush) passes ev1 / tk1: events of arrival ranks [ev0, ev1) and ticks [tk0, tk1)
  // (tk1's tick precedes rank ev1), its records appended after record slot rbase of a buffer of rcap slots, and
  // their ticks absolute.
  // sweep diagnostics (SG_HOST_TIMING): host time per phase of run_lanes summed over the sweep's windows
  double sw_t[4] = {0, 0, 0, 0};
  std::chrono::steady_clock::time_point sw_t0;
  void sw_mark(int k) {
    if (!in_sweep) return;
    const auto t = std::chrono::steady_clock::now();
    sw_t[k] += std::chrono::duration<double, std::milli>(t - sw_t0).count();
    sw_t0 = t;
  }
  RunOut run_lanes(int64_t ev0, size_t tk0, bool log_fire, bool log_ops, hipStream_t s, int64_t ev1 = -1,
                   int64_t tk1 = -1, uint32_t rbase = 0, int64_t rcap = 0, const std::vector<uint8_t>* only = nullptr) {
    sw_t0 = std::chrono::steady_clock::now();
    PhaseClock pc(getenv("SG_HOST_TIMING") != nullptr);
    const bool absent = tab.nabs > 0;
    const bool window = ev1 >= 0;
    const int64_t xe = window ? ev1 : n;
    const int64_t lanes_needed = partitioned ? (int64_t)lane_key.size() : 1;
    grow_lanes(std::max<int64_t>(lanes_needed, 1), s);
    const size_t nt = (window ? (size_t)tk1 : tick_now.size()) - tk0;
    // CSR of the events per lane (arrival order inside each lane); with pending ticks every created
    // lane runs (its deadlines fire at ticks even without events of its own)
    std::vector<int32_t> cnt(lanes_needed, 0);
    bool any_bcast = false;
    // counting sort of the events by lane, in arrival-rank order; parallel over rank ranges (per-thread
    // histograms, then each thread scatters its range behind the lower threads' counts)
    const int64_t ne = xe - ev0;
    launch_events = ne;
    seen_events += ne;
    const int nth = (!std::any_of(std::begin(bcast), std::end(bcast), [](bool x) { return x; }) && ne >= (1 << 20))
                        ? (int)std::min<int64_t>(16, std::max(1u, std::thread::hardware_concurrency()))
                        : 1;
    std::vector<std::vector<int32_t>> tcnt(nth, std::vector<int32_t>(nth > 1 ? lanes_needed : 0, 0));
    if (nth > 1) {
      host_parallel(nth, [&](int t) {
        const int64_t r0 = ev0 + ne * t / nth, r1 = ev0 + ne * (t + 1) / nth;
        int32_t* c = tcnt[t].data();
        for (int64_t r = r0; r < r1; r++) { const int l = h_lane[rank_ev[r]]; if (l >= 0) c[l]++; }
      });
      for (int t = 0; t < nth; t++)
        for (int64_t l = 0; l < lanes_needed; l++) cnt[l] += tcnt[t][l];
    } else if (!window) {
      for (int64_t e = ev0; e < n; e++) {          // ranks [ev0, n) are exactly the events [ev0, n)
        if (h_lane[e] >= 0) cnt[h_lane[e]]++;
        else if (h_lane[e] == -1) any_bcast = true;
      }
    } else {
      for (int64_t r = ev0; r < xe; r++) {
        const int32_t e = rank_ev[r];
        if (h_lane[e] >= 0) cnt[h_lane[e]]++;
        else if (h_lane[e] == -1) any_bcast = true;
      }
    }
    if (any_bcast)                               // a broadcast event reaches the lanes created before it
      for (int64_t r = ev0; r < xe; r++) {
        if (h_lane[rank_ev[r]] != -1) continue;
        for (int64_t l = 0; l < lanes_needed; l++) if (create_rank[l] < r) cnt[l]++;
      }
    std::vector<int32_t> lid, off(1, 0), start(lanes_needed, -1);
    for (int64_t l = 0; l < lanes_needed; l++) {
      if (only && !(*only)[(size_t)l]) continue;   // a round of the sweep re-runs only the deferred instances
      // (a window runs only the instances created before its end: a later one has no state yet)
      if (cnt[l] || (absent && nt > 0 && (!window || !partitioned || create_rank[l] < xe))) { start[l] = (int32_t)lid.size(); lid.push_back((int32_t)l); off.push_back(off.back() + cnt[l]); }
    }
    pvec<int32_t>& evs = csr_evs;           // (kept across flushes: no first-touch faults)
    std::vector<int32_t> fill(lid.size(), 0);
    evs.resize(off.back());
    if (nth > 1) {
      // thread t's first slot in lane l: the lane's offset + the lower threads' counts
      for (int64_t l = 0; l < lanes_needed; l++) {
        if (start[l] < 0) continue;
        int32_t run = off[start[l]];
        for (int t = 0; t < nth; t++) { const int32_t c = tcnt[t][l]; tcnt[t][l] = run; run += c; }
      }
      host_parallel(nth, [&](int t) {
        const int64_t r0 = ev0 + ne * t / nth, r1 = ev0 + ne * (t + 1) / nth;
        int32_t* pos = tcnt[t].data();
        for (int64_t r = r0; r < r1; r++) {
          const int32_t e = rank_ev[r];
          if (h_lane[e] >= 0 && start[h_lane[e]] >= 0) evs[pos[h_lane[e]]++] = e;
        }
      });
    } else
    for (int64_t r = ev0; r < xe; r++) {
      const int32_t e = rank_ev[r];
      if (h_lane[e] == -2) continue;                 // null partition key: no instance
      if (h_lane[e] < 0) {
        for (int64_t l = 0; l < lanes_needed; l++)
          if (create_rank[l] < r && start[l] >= 0) { const int q = start[l]; evs[off[q] + fill[q]++] = e; }
        continue;
      }
      int q = start[h_lane[e]];
      if (q >= 0) evs[off[q] + fill[q]++] = e;
    }
    const int nl = (int)lid.size();
    pc.mark("lanes csr");
    sw_mark(0);
    RunOut ro;
    ro.nrec = rbase;
    if (nl == 0) return ro;
    // a sweep window stages its small per-launch arrays in one pinned block and uploads them with one copy (each
    // separate copy is a queue operation of its own, which dominates a window's launch)
    sw_stage.clear();
    size_t so_off = 0, so_ev = 0, so_id = 0, so_doff = SIZE_MAX, so_dkey = SIZE_MAX, so_cnt = 0;
    if (in_sweep) {
      so_off = sw_stage.put(off.data(), (nl + 1) * 4);
      so_ev = sw_stage.put(evs.data(), evs.size() * 4);
      so_id = sw_stage.put(lid.data(), (size_t)nl * 4);
    } else {
      lane_off.reserve(nl + 1); lane_ev.reserve(std::max<size_t>(evs.size(), 1)); lane_id.reserve(nl);
      SG_HIP(hipMemcpyAsync(lane_off.p, off.data(), (nl + 1) * 4, hipMemcpyHostToDevice, s));
      if (!evs.empty()) SG_HIP(hipMemcpyAsync(lane_ev.p, evs.data(), evs.size() * 4, hipMemcpyHostToDevice, s));
      SG_HIP(hipMemcpyAsync(lane_id.p, lid.data(), nl * 4, hipMemcpyHostToDevice, s));
    }
    // (the sweep uploads every tick once: a window reads its range in place)
    const int64_t* tnow = d_tick_now.p + (in_sweep ? tk0 : 0);
    const int32_t* tev = d_tick_ev.p + (in_sweep ? tk0 : 0);
    if (absent && nt > 0 && !in_sweep) {
      d_tick_now.reserve(nt); d_tick_ev.reserve(nt);
      tnow = d_tick_now.p; tev = d_tick_ev.p;
      SG_HIP(hipMemcpyAsync(d_tick_now.p, tick_now.data() + tk0, nt * 8, hipMemcpyHostToDevice, s));
      SG_HIP(hipMemcpyAsync(d_tick_ev.p, tick_ev.data() + tk0, nt * 4, hipMemcpyHostToDevice, s));
    }
    // tick indexes over this launch's event ranks [ev0, n) and its ticks' clock range (dense while that range
    // is within 8 ms per tick or 4M ms; a sparser clock keeps the binary search for due deadlines)
    int64_t tub0 = 0, ntub = 0, tlb0 = 0, ntlb = 0;
    bool use_ub = false, use_lb = false;
    if (absent && nt > 0 && !getenv("SG_NFA_TICK_SEARCH")) {
      ntub = std::max<int64_t>(xe - ev0, 0);
      tub0 = ev0;
      tlb0 = tick_now[tk0];
      ntlb = tick_now[tk0 + nt - 1] - tlb0 + 1;
      use_ub = ntub > 0;
      use_lb = ntlb > 0 && ntlb <= std::max<int64_t>(8 * (int64_t)nt, (int64_t)1 << 22);
      if (!use_lb) ntlb = 0;
      if (use_ub) d_tick_ub.reserve(ntub);
      if (use_lb) d_tick_lb.reserve(ntlb);
      const int64_t work = std::max(use_ub ? ntub : 0, ntlb);
      // (a sweep's round re-runs its window: the same ranks and ticks, the same index)
      const int64_t tkey[4] = {ev0, (int64_t)tk0, xe, (int64_t)nt};
      const bool cached = in_sweep && std::equal(tkey, tkey + 4, ti_key);
      if (in_sweep) std::copy(tkey, tkey + 4, ti_key);
      if (work > 0 && !cached) {
        hipLaunchKernelGGL(k_nfa_tick_index, dim3((unsigned)std::min<int64_t>(8192, (work + 255) / 256)), dim3(256), 0, s,
                           tnow, tev, (int32_t)nt, tub0, use_ub ? ntub : 0, d_tick_ub.p, tlb0, ntlb,
                           d_tick_lb.p);
        SG_HIP(hipGetLastError());
      }
    }
    // deferred firings (relative tick index << 8 | scheduler), per CSR lane, ascending
    std::vector<int32_t> doff;
    std::vector<int64_t> dkey;
    if (!deferrals.empty()) {
      std::vector<std::vector<int64_t>> per(nl);
      // deferrals are kept in tick order (defer()): the launch's ticks are one range of them
      const auto lo = std::lower_bound(deferrals.begin(), deferrals.end(), (int64_t)tk0 << 8,
                                       [](const std::pair<int32_t, int64_t>& d, int64_t k) { return d.second < k; });
      for (auto it = lo; it != deferrals.end(); ++it) {
        const auto& d = *it;
        const int64_t tau = d.second >> 8;
        if (tau >= (int64_t)(tk0 + nt)) break;
        if (start[d.first] < 0) continue;
        per[start[d.first]].push_back(((tau - (int64_t)tk0) << 8) | (d.second & 255));
      }
      doff.push_back(0);
      for (auto& v : per) { std::sort(v.begin(), v.end()); dkey.insert(dkey.end(), v.begin(), v.end()); doff.push_back((int32_t)dkey.size()); }
      if (in_sweep) {
        so_doff = sw_stage.put(doff.data(), doff.size() * 4);
        so_dkey = sw_stage.put(dkey.data(), dkey.size() * 8);
      } else {
        d_def_off.reserve(doff.size()); d_def_key.reserve(std::max<size_t>(dkey.size(), 1));
        SG_HIP(hipMemcpyAsync(d_def_off.p, doff.data(), doff.size() * 4, hipMemcpyHostToDevice, s));
        if (!dkey.empty()) SG_HIP(hipMemcpyAsync(d_def_key.p, dkey.data(), dkey.size() * 8, hipMemcpyHostToDevice, s));
      }
    }
    NCols hc;
    std::memset(&hc, 0, sizeof(hc));
    for (size_t ls = 0; ls < streams.size(); ls++) {
      for (size_t k = 0; k < cols[ls].size(); k++) { hc.col[ls][k] = cols[ls][k].b.p; hc.w[ls][k] = cols[ls][k].w; }
      hc.nul[ls] = has_nul[ls] ? nulcol[ls].p : nullptr;
      hc.na[ls] = (int32_t)cols[ls].size();
    }
    if (!in_sweep || !sweep_uploaded) {          // (constant over a sweep's windows)
      d_cols.reserve(1);
      d_tab.reserve(1);
      d_progs.reserve(progs.size());
      SG_HIP(hipMemcpyAsync(d_cols.p, &hc, sizeof(hc), hipMemcpyHostToDevice, s));
      SG_HIP(hipMemcpyAsync(d_tab.p, &tab, sizeof(tab), hipMemcpyHostToDevice, s));
      SG_HIP(hipMemcpyAsync(d_progs.p, progs.data(), progs.size() * sizeof(Prog), hipMemcpyHostToDevice, s));
      prefilter(s);
      sweep_uploaded = in_sweep;
    }
    // (a speculative run may write a re-run key's records twice: the discarded copy and the re-run's)
    const int64_t cap = rcap > 0 ? std::max<int64_t>(rcap, (int64_t)rbase + std::max<int64_t>(1024, (xe - ev0 + (int64_t)nt) * 8))
                                 : std::max<int64_t>(1024, (n - ev0 + (int64_t)nt) * 8);
    {
      // (a sweep window appends after rbase records: growing keeps them, superseded ones included)
      const size_t u = rbase, w = (size_t)std::max(nsel, 1);
      rec_key.reserve(cap, true, s, u); rec_val.reserve((size_t)cap * w, true, s, u * w); rec_nul.reserve((size_t)cap * w, true, s, u * w);
      rec_ts.reserve(cap, true, s, u); rec_tick.reserve(cap, true, s, u); rec_lane.reserve(cap, true, s, u);
      rec_dl.reserve(cap, true, s, u); rec_sched.reserve(cap, true, s, u);
      if (in_sweep) rec_task.reserve(cap, true, s, u);
    }
    counter.reserve(4);
    const uint32_t c0[4] = {rbase, 0, 0, 0};
    if (in_sweep) so_cnt = sw_stage.put(c0, 16);
    else if (rbase) SG_HIP(hipMemcpyAsync(counter.p, c0, 16, hipMemcpyHostToDevice, s));
    else SG_HIP(hipMemsetAsync(counter.p, 0, 16, s));
    const int64_t fcap = log_fire ? std::max<int64_t>(4096, (xe - ev0 + (int64_t)nt) * 2) : 0;
    const int64_t ocap = log_ops ? std::max<int64_t>(4096, (xe - ev0 + (int64_t)nt) * 8) : 0;
    if (log_fire && !in_sweep) d_fire.reserve(fcap);
    if (log_ops && !in_sweep) d_ops.reserve(ocap);
    FireRec* fire_dev = d_fire.p;
    OpRec* ops_dev = d_ops.p;
    if (in_sweep) {                 // a window's logs are small: the lanes write them into host memory directly
      if (log_fire) fire_dev = sw_fire.get(fcap);
      if (log_ops) ops_dev = sw_ops.get(ocap);
    }
    NArgs a;
    std::memset(&a, 0, sizeof(a));
    a.ev_ts = ev_ts.p; a.ev_stream = ev_stream.p; a.ev_row = ev_row.p; a.ev_rank = ev_rank.p;
    a.lane_off = lane_off.p; a.lane_ev = lane_ev.p; a.lane_id = lane_id.p; a.nl = nl;
    a.rec_key = rec_key.p; a.rec_val = rec_val.p; a.rec_nul = rec_nul.p; a.nrec = counter.p; a.rec_cap = cap;
    a.rec_ts = rec_ts.p; a.rec_tick = rec_tick.p; a.rec_lane = rec_lane.p; a.rec_dl = rec_dl.p; a.rec_sched = rec_sched.p;
    a.tick_now = tnow; a.tick_ev = tev; a.ntick = absent ? (int32_t)nt : 0;
    a.tick_base = window ? (int32_t)tk0 : 0;
    a.tick_ub = use_ub ? d_tick_ub.p : nullptr; a.tub0 = tub0; a.ntub = ntub;
    a.tick_lb = use_lb ? d_tick_lb.p : nullptr; a.tlb0 = tlb0; a.ntlb = ntlb;
    a.start_now = start_now;
    a.ev_now = partitioned ? ev_now.p : nullptr;
    a.def_off = doff.empty() ? nullptr : d_def_off.p;
    a.def_key = doff.empty() ? nullptr : d_def_key.p;
    a.fire = log_fire ? fire_dev : nullptr; a.nfire = counter.p + 1; a.fire_cap = fcap;
    a.ops = log_ops ? ops_dev : nullptr; a.nops = counter.p + 2; a.ops_cap = ocap;
    a.ev_skip = pf_any ? ev_skip.p : nullptr;
    uint32_t* cnt_dev = counter.p;
    if (in_sweep) {                 // (records a later round supersedes are marked through their task: emit drops 0)
      a.rec_task = rec_task.p;
      sw_arena.reserve(sw_stage.n, false);
      SG_HIP(hipMemcpyAsync(sw_arena.p, sw_stage.p, sw_stage.n, hipMemcpyHostToDevice, s));
      a.lane_off = (const int32_t*)(sw_arena.p + so_off);
      a.lane_ev = (const int32_t*)(sw_arena.p + so_ev);
      a.lane_id = (const int32_t*)(sw_arena.p + so_id);
      if (!doff.empty()) {
        a.def_off = (const int32_t*)(sw_arena.p + so_doff);
        a.def_key = (const int64_t*)(sw_arena.p + so_dkey);
      }
      cnt_dev = (uint32_t*)(sw_arena.p + so_cnt);
      a.nrec = cnt_dev; a.nfire = cnt_dev + 1; a.nops = cnt_dev + 2;
    }
    if (!e0) { SG_HIP(hipEventCreate(&e0)); SG_HIP(hipEventCreate(&e1)); }
#ifdef SG_NFA_PROBE
    probe_buf.reserve(8, false);
    SG_HIP(hipMemsetAsync(probe_buf.p, 0, 64, s));
    a.probe = probe_buf.p;
#endif
    // the launch's events packed lane-major (not in a sweep window: a few events per lane, one more launch each)
    if (!in_sweep && !evs.empty() && !getenv("SG_NFA_NO_PACK")) {
      lane_rec.reserve(evs.size());
      const bool unique = !std::any_of(std::begin(bcast), std::end(bcast), [](bool x) { return x; });
      const int64_t x0 = ev0, x1 = n;              // the launch's events are among the events [ev0, n)
      if (unique && (int64_t)evs.size() * 2 >= x1 - x0 && !getenv("SG_NFA_PACK_GATHER")) {
        pack_inv.reserve((size_t)n);
        SG_HIP(hipMemsetAsync(pack_inv.p + x0, 0xff, (size_t)(x1 - x0) * 4, s));
        hipLaunchKernelGGL(k_nfa_inv, dim3((unsigned)((evs.size() + 255) / 256)), dim3(256), 0, s, a.lane_ev,
                           (int64_t)evs.size(), pack_inv.p);
        hipLaunchKernelGGL(k_nfa_pack_ev, dim3((unsigned)((x1 - x0 + 255) / 256)), dim3(256), 0, s, a, d_cols.p, x0,
                           x1, (const int32_t*)pack_inv.p, lane_rec.p);
      } else {
        hipLaunchKernelGGL(k_nfa_pack, dim3((unsigned)((evs.size() + 255) / 256)), dim3(256), 0, s, a, d_cols.p,
                           (int64_t)evs.size(), lane_rec.p);
      }
      SG_HIP(hipGetLastError());
      a.lane_rec = lane_rec.p;
    }
    pc.mark("lanes upload");
    sw_mark(1);
    SpecPlan sp;
    const bool spec_on = !log_ops && plan_spec(off, lid, sp);
    if (!in_sweep) SG_HIP(hipEventRecord(e0, s));   // (a sweep window is not timed: kernel_ms keeps the flush's run)
    if (spec_on) {
      run_spec(a, sp, evs, s);
      ro.task_ok = std::move(sp.ok);
    } else {
      launch_lanes(a, nl, nullptr, s);
    }
    if (!in_sweep) SG_HIP(hipEventRecord(e1, s));
    uint32_t cnts[4] = {0, 0, 0, 0};
    std::vector<int32_t> errs;
    if (in_sweep) {                  // a failed lane also sets counter word 3 (Lane::fail): the pools' flags only then
      uint32_t* hc = sw_cnt_host();
      SG_HIP(hipMemcpyAsync(hc, cnt_dev, 16, hipMemcpyDeviceToHost, s));
      SG_HIP(hipStreamSynchronize(s));
      std::memcpy(cnts, hc, 16);
      if (cnts[3]) {
        errs.resize(L);
        SG_HIP(hipMemcpy(errs.data(), err.p, L * 4, hipMemcpyDeviceToHost));
      }
    } else {
      errs.resize(L);
      SG_HIP(hipMemcpyAsync(cnts, counter.p, 16, hipMemcpyDeviceToHost, s));
      SG_HIP(hipMemcpyAsync(errs.data(), err.p, L * 4, hipMemcpyDeviceToHost, s));
      SG_HIP(hipStreamSynchronize(s));
    }
    pc.mark("lanes kernel + sync");
    sw_mark(2);
    if (!in_sweep) {
      float ms = 0;
      SG_HIP(hipEventElapsedTime(&ms, e0, e1));
      kernel_ms["k_nfa_lanes"] = ms;
    }
#ifdef SG_NFA_PROBE
    {
      unsigned long long pr[8];
      SG_HIP(hipMemcpy(pr, probe_buf.p, 64, hipMemcpyDeviceToHost));
      // wall_clock64 runs at 100 MHz: ticks * 10 ns, summed over lanes; per event
      const double ev = std::max<double>(1.0, (double)pr[5]);
      fprintf(stderr, "[sg probe] events %.0f, ns per event: ticks %.0f expire %.0f update %.0f process %.0f\n", ev,
              pr[0] * 10.0 / ev, pr[1] * 10.0 / ev, pr[2] * 10.0 / ev, pr[3] * 10.0 / ev);
    }
#endif
    for (int64_t l = 0; l < (int64_t)errs.size(); l++)
      if (errs[l]) throw Error(-4, "device NFA pool overflow (code " + std::to_string(errs[l]) +
                                   "): raise SG_NFA_SE_CAP / SG_NFA_ND_CAP / SG_NFA_LIST_CAP");
    ro.nrec = cnts[0];
    if (in_sweep) {                 // (written in place: the stream is synchronised)
      if (log_fire && cnts[1]) ro.fires.assign(sw_fire.h, sw_fire.h + cnts[1]);
      if (log_ops && cnts[2]) ro.ops.assign(sw_ops.h, sw_ops.h + cnts[2]);
    } else {
      if (log_fire && cnts[1] && fire_lazy) {
        ro.fires_dev = cnts[1];
        ro.fire_tk0 = tk0;
      } else if (log_fire && cnts[1]) {
        ro.fires.resize(cnts[1]);
        SG_HIP(hipMemcpyAsync(ro.fires.data(), d_fire.p, cnts[1] * sizeof(FireRec), hipMemcpyDeviceToHost, s));
      }
      if (log_ops && cnts[2]) {
        ro.ops.resize(cnts[2]);
        SG_HIP(hipMemcpyAsync(ro.ops.data(), d_ops.p, cnts[2] * sizeof(OpRec), hipMemcpyDeviceToHost, s));
      }
      if ((log_fire && cnts[1] && !fire_lazy) || (log_ops && cnts[2])) SG_HIP(hipStreamSynchronize(s));
    }
    if (!ro.task_ok.empty())          // firings of segments that did not verify never happened
      ro.fires.erase(std::remove_if(ro.fires.begin(), ro.fires.end(),
                                    [&](const FireRec& f) { return f.task >= 0 && !ro.task_ok[(size_t)f.task]; }),
                     ro.fires.end());
    pc.mark("lanes logs copy");
    sw_mark(3);
    for (auto& f : ro.fires) f.tau += (int32_t)tk0;
    for (auto& o : ro.ops) if (o.tau >= 0) o.tau += (int32_t)tk0;
    return ro;
  }

  // Earliest (tick, scheduler) at which two instances fired under the same head deadline.
  // The earliest (tick, scheduler) at which two instances fired under one head deadline: firings are
  // bucketed by tick (counting sort, O(firings)); only ticks with several firings are compared.
  static bool first_collision(const std::vector<FireRec>& fires, int64_t& key) {
    if (fires.size() < 2) return false;
    int32_t tmax = INT32_MIN, tmin = INT32_MAX;       // (a window of the sweep logs a short range of ticks)
    for (const FireRec& f : fires) { tmax = std::max(tmax, f.tau); tmin = std::min(tmin, f.tau); }
    // tick ranges in parallel (each thread buckets the firings of its range); the earliest range with a
    // collision holds the earliest one
    const int nth = fires.size() >= (1u << 16) ? (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency())) : 1;
    std::vector<int64_t> found(nth, -1);
    auto scan = [&](int t) {
      const int64_t span = (int64_t)tmax - tmin + 1;
      const int32_t lo = tmin + (int32_t)(span * t / nth), hi = tmin + (int32_t)(span * (t + 1) / nth);
      if (lo >= hi) return;
      std::vector<uint32_t> off((size_t)(hi - lo) + 1, 0), idx, fill;
      for (const FireRec& f : fires) if (f.tau >= lo && f.tau < hi) off[(size_t)(f.tau - lo) + 1]++;
      for (size_t k = 1; k < off.size(); k++) off[k] += off[k - 1];
      idx.resize(off.back());
      fill.assign(off.begin(), off.end() - 1);
      for (uint32_t i = 0; i < fires.size(); i++)
        if (fires[i].tau >= lo && fires[i].tau < hi) idx[fill[(size_t)(fires[i].tau - lo)]++] = i;
      std::vector<std::pair<int, int64_t>> grp;
      for (size_t k = 0; k + 1 < off.size(); k++) {
        if (off[k + 1] - off[k] < 2) continue;
        grp.clear();
        for (uint32_t q = off[k]; q < off[k + 1]; q++) grp.push_back({fires[idx[q]].sched, fires[idx[q]].head});
        std::sort(grp.begin(), grp.end());
        for (size_t q = 1; q < grp.size(); q++)
          if (grp[q] == grp[q - 1]) {          // sorted: the first hit has the smallest scheduler
            found[t] = ((int64_t)(lo + (int32_t)k) << 8) | grp[q].first;
            return;
          }
      }
    };
    if (nth > 1) host_parallel(nth, scan); else scan(0);
    for (int t = 0; t < nth; t++)
      if (found[t] >= 0) { key = found[t]; return true; }
    return false;
  }

  // Replay the Scheduler maps (from an empty app) over a run's logs; at the first colliding (tick, scheduler)
  // the instances that lose (not first in the map's iteration order) are deferred.  The replay then goes on
  // and resolves later collisions in the same round while the run's logs still describe them exactly:
  //   * a deferred instance fires its deferred head at a later tick (nobody else holds that head any more),
  //     and every deadline it arms from then on lies at least the shortest `for` wait after the first
  //     collision's clock, so up to that clock its firings are the logged ones except the deferred head;
  //   * so a later collision whose tick is earlier than that clock, among instances none of which was
  //     deferred, under a head none of them was deferred with, and with no firing of a deferred instance
  //     logged since the first collision, has the logged participants, and its winner depends only on their
  //     relative map order -- unless the map resized in between or came within the deferred count of its
  //     threshold (a deferred instance stays in the map where the log removed it).
  // The first collision that fails a condition ends the round (the caller re-runs the lanes with the
  // deferrals and replays again).  False when the run had no collision.
  bool resolve_first_collision(const RunOut& ro) {
    int64_t ck = 0;
    if (!first_collision(ro.fires, ck)) return false;
    std::vector<SchedMap> maps(tab.nabs);
    return replay_maps(ro, maps, true, ck);
  }
  // One window of the exact sweep (flush): with a collision among its logged firings, the collisions the logs
  // still describe are resolved (deferrals added: the window re-runs from its checkpoint) and true is returned;
  // without one, `base` (the maps at the window's start) is advanced over the window's logs.
  std::set<int32_t> last_dlanes;
  bool resolve_window(const RunOut& ro, std::vector<SchedMap>& base) {
    int64_t ck = 0;
    if (!first_collision(ro.fires, ck)) { replay_maps(ro, base, false, 0); return false; }
    std::vector<SchedMap> maps(base);
    return replay_maps(ro, maps, true, ck);
  }
  // The replay itself over a run's logs, from `maps`; resolve = false only applies the logged map operations.
  bool replay_maps(const RunOut& ro, std::vector<SchedMap>& maps, bool resolve, int64_t ck) {
    const int32_t ctau = (int32_t)(ck >> 8);
    const int csched = (int)(ck & 255);
    int64_t min_wait = INT64_MAX;
    for (int k = 0; k < tab.nabs; k++) {
      const int64_t w = tab.waiting[(int)tab.absOrder[k]];
      min_wait = std::min(min_wait, w < 0 ? 0 : w);
    }
    if (getenv("SG_NFA_COLLIDE_ONE")) min_wait = 0;   // test hook: one collision per round
    // global order: (x, phase, tau, kfire, stage 0 collect / 1 ops / 2 remove, head, sub)
    struct Item { int32_t x; int8_t phase; int32_t tau; int8_t kf; int8_t stage; int64_t head; int32_t sub; int32_t idx; };
    std::vector<Item> items;
    std::set<std::pair<int32_t, int>> ticks;   // (tau, sched) with firings
    for (auto& f : ro.fires) ticks.insert({f.tau, f.sched});
    for (size_t i = 0; i < ro.ops.size(); i++) {
      const OpRec& o = ro.ops[i];
      items.push_back({o.x, o.phase, o.phase ? -1 : o.tau, o.phase ? (int8_t)-1 : o.kfire, 1, o.phase ? 0 : o.head, o.sub, (int32_t)i});
    }
    for (auto& tk : ticks) {
      items.push_back({tick_ev[tk.first], 0, tk.first, (int8_t)tk.second, 0, INT64_MIN, 0, -1});
      items.push_back({tick_ev[tk.first], 0, tk.first, (int8_t)tk.second, 2, INT64_MAX, 0, -2});
    }
    std::stable_sort(items.begin(), items.end(), [](const Item& a, const Item& b) {
      return std::tie(a.x, a.phase, a.tau, a.kf, a.stage, a.head, a.sub) < std::tie(b.x, b.phase, b.tau, b.kf, b.stage, b.head, b.sub);
    });
    // firings per (tau, sched)
    std::map<std::pair<int32_t, int>, std::vector<const FireRec*>> fired;
    for (auto& f : ro.fires) fired[{f.tau, f.sched}].push_back(&f);
    std::vector<size_t> cap0(tab.nabs, 0), smax(tab.nabs, 0);   // capacity and peak size since the first collision
    bool first = false;                        // the first collision is resolved
    int64_t clock_end = 0;                     // resolvable collisions lie before this clock
    std::set<int32_t>& dlanes = last_dlanes;   // instances deferred this round
    dlanes.clear();
    std::set<std::pair<int, int64_t>> dheads;  // (scheduler, head) they were deferred under
    for (const Item& it : items) {
      if (it.idx >= 0) {
        const OpRec& o = ro.ops[it.idx];
        maps[o.ktarget].touch(lane_hash(o.lane), o.lane);
        smax[o.ktarget] = std::max(smax[o.ktarget], maps[o.ktarget].size);
        continue;
      }
      const auto& fl = fired[{it.tau, (int)it.kf}];
      if (it.idx == -1) {
        if (!resolve) continue;
        if (first) {
          if (tick_now[it.tau] >= clock_end) return true;
          for (auto* f : fl) if (dlanes.count(f->lane)) return true;   // a deferred instance's logged firing
        } else if (it.tau != ctau || it.kf != csched) {
          continue;
        }
        // the collection at a colliding (tick, scheduler): per shared head, the instance first in iteration
        // order wins; the others are deferred to a later tick
        std::map<int64_t, std::vector<const FireRec*>> byhead;
        for (auto* f : fl) byhead[f->head].push_back(f);
        if (first) {
          bool any = false;
          for (auto& kv : byhead) any |= kv.second.size() >= 2;
          if (any) {
            const SchedMap& m = maps[it.kf];
            const size_t slack = dlanes.size() + 1;
            if (m.tab.size() != cap0[it.kf] || smax[it.kf] + slack > m.thr) return true;
            for (auto& kv : byhead)
              if (kv.second.size() >= 2 && dheads.count({(int)it.kf, kv.first})) return true;
          }
        }
        for (auto& kv : byhead) {
          if (kv.second.size() < 2) continue;
          const FireRec* win = nullptr;
          int64_t best = INT64_MAX;
          for (auto* f : kv.second) {
            const int64_t r = maps[it.kf].rank(lane_hash(f->lane), f->lane);
            if (r < best) { best = r; win = f; }
          }
          for (auto* f : kv.second)
            if (f != win) {
              defer(f->lane, ((int64_t)it.tau << 8) | it.kf);
              dlanes.insert(f->lane);
              dheads.insert({(int)it.kf, kv.first});
            }
        }
        if (!first) {
          first = true;
          if (min_wait <= 0) return true;
          clock_end = tick_now[it.tau] + min_wait;
          for (int k = 0; k < tab.nabs; k++) { cap0[k] = maps[k].tab.size(); smax[k] = maps[k].size; }
        }
        continue;
      }
      for (auto* f : fl)   // returnAllStates: a state whose queue is empty is dropped
        if (f->empty_after && !dlanes.count(f->lane)) maps[it.kf].remove(lane_hash(f->lane), f->lane);
    }
    if (first || !resolve) return first;
    throw Error(-3, "scheduler replay did not reach the collision");
  }

  // The exact sweep: instances shared a deadline at one tick (the flush's run logged a collision at `ck`), so
  // the app is replayed from its start in windows of ticks, each from a checkpoint of the lane pools and the
  // Scheduler maps at its start.  A window whose logs show a collision has it (and the later ones the logs
  // still describe) resolved by deferrals, and re-runs from its checkpoint; one without a collision advances
  // the maps over its logs and keeps its records.  Cost: O(events + ticks) for the runs without collisions,
  // plus one window per round -- O(collisions * window) instead of a whole-app run per round.
  DBuf<uint8_t> ckpt;
  bool in_sweep = false, sweep_uploaded = false;
  const void* attr_fn = nullptr;          // the lanes kernel whose dynamic-LDS limit was last raised, and to what
  int attr_lds = 0;
  int64_t ti_key[4] = {-1, -1, -1, -1};   // the window whose tick index d_tick_ub / d_tick_lb hold (sweep only)
  // The sweep's base: events of arrival rank < fx and ticks < fk are settled (their collisions resolved), with the
  // lane pools (fbase, fL lanes) and the Scheduler maps (fmaps) at that point; f_fresh: the base is the app's start.
  // A sweep starts there and moves the base to its end, so the events before it are needed only through the
  // chains that reference them (compaction) and the deferrals before it never again.
  int64_t fx = 0;
  size_t fk = 0;
  bool f_fresh = true;
  int64_t fL = 0;
  std::vector<SchedMap> fmaps;
  DBuf<uint8_t> fbase;
  bool base_current() const { return f_fresh ? (n == 0 && tick_now.empty()) : (fx == n && fk == tick_now.size()); }
  void base_save(hipStream_t s) {
    pools_copy(true, s, &fbase);
    fL = L;
    fx = n;
    fk = tick_now.size();
    f_fresh = false;
  }
  void base_load(hipStream_t s) {
    if (f_fresh || fL <= 0) {
      hipLaunchKernelGGL(k_nfa_pool_init, dim3((unsigned)((L + 255) / 256)), dim3(256), 0, s, state(), 0, L);
      SG_HIP(hipGetLastError());
      return;
    }
    LaneSegs g;
    std::memset(&g, 0, sizeof(g));
    size_t off = 0;
    for_each_pool([&](auto& b, int64_t per) {
      g.ck[g.n] = fbase.p + off;
      g.pool[g.n] = (uint8_t*)b.p;
      g.per[g.n] = per;
      g.esz[g.n++] = (int32_t)sizeof(*b.p);
      off += ((size_t)per * fL * sizeof(*b.p) + 15) / 16 * 16;
    });
    hipLaunchKernelGGL(k_pools_relayout, dim3(256, (unsigned)g.n), dim3(256), 0, s, g, fL, L);
    SG_HIP(hipGetLastError());
    if (L > fL) {                                 // instances created since the base start fresh
      hipLaunchKernelGGL(k_nfa_pool_init, dim3((unsigned)((L - fL + 255) / 256)), dim3(256), 0, s, state(), fL, L - fL);
      SG_HIP(hipGetLastError());
    }
  }
  // every pool to (save) or from its copy in `buf` (the window checkpoint by default), element layout kept
  void pools_copy(bool save, hipStream_t s, DBuf<uint8_t>* into = nullptr) {
    DBuf<uint8_t>& buf = into ? *into : ckpt;
    CopySegs cs;
    std::memset(&cs, 0, sizeof(cs));
    size_t tot = 0;
    for_each_pool([&](auto& b, int64_t per) { tot += ((size_t)per * L * sizeof(*b.p) + 15) / 16 * 16; });
    buf.reserve(tot, false);
    size_t off = 0;
    for_each_pool([&](auto& b, int64_t per) {
      const size_t by = (size_t)per * L * sizeof(*b.p);
      if (cs.n >= CopySegs::MAX) throw Error(-3, "pool checkpoint: too many pools");
      cs.src[cs.n] = save ? (const uint8_t*)b.p : buf.p + off;
      cs.dst[cs.n] = save ? buf.p + off : (uint8_t*)b.p;
      cs.bytes[cs.n++] = by;
      off += (by + 15) / 16 * 16;
    });
    hipLaunchKernelGGL(k_copy_segs, dim3(1024), dim3(256), 0, s, cs);
    SG_HIP(hipGetLastError());
  }
  DBuf<int32_t> d_dl;
  // the sweep's staging: one pinned block per launch (NfaExec::run_lanes) and its device copy
  struct PinStage {
    uint8_t* p = nullptr;
    size_t n = 0, cap = 0;
    ~PinStage() { if (p) (void)hipHostFree(p); }
    void clear() { n = 0; }
    size_t put(const void* src, size_t by) {
      const size_t at = (n + 15) / 16 * 16;
      if (at + by > cap) {
        size_t nc = std::max<size_t>(cap * 2, 1 << 16);
        while (nc < at + by) nc *= 2;
        uint8_t* q = nullptr;
        SG_HIP(hipHostMalloc((void**)&q, nc, hipHostMallocDefault));
        if (p) { std::memcpy(q, p, n); (void)hipHostFree(p); }
        p = q;
        cap = nc;
      }
      if (by) std::memcpy(p + at, src, by);
      n = at + by;
      return at;
    }
  } sw_stage;
  DBuf<uint8_t> sw_arena;
  // host-resident log buffers the lanes of a sweep window write into (coherent, mapped pinned memory)
  template <class T>
  struct HostLog {
    T* h = nullptr;
    T* d = nullptr;
    int64_t cap = 0;
    ~HostLog() { if (h) (void)hipHostFree(h); }
    T* get(int64_t need) {
      if (need > cap) {
        if (h) SG_HIP(hipHostFree(h));
        cap = std::max<int64_t>(need, cap * 2);
        SG_HIP(hipHostMalloc((void**)&h, (size_t)cap * sizeof(T), hipHostMallocMapped | hipHostMallocCoherent));
        SG_HIP(hipHostGetDevicePointer((void**)&d, h, 0));
      }
      return d;
    }
  };
  HostLog<FireRec> sw_fire;
  HostLog<OpRec> sw_ops;
  uint32_t* sw_cnt = nullptr;
  uint32_t* sw_cnt_host() {
    if (!sw_cnt) SG_HIP(hipHostMalloc((void**)&sw_cnt, 16, hipHostMallocDefault));
    return sw_cnt;
  }
  void restore_lanes(const std::vector<int32_t>& dl, hipStream_t s) {
    LaneSegs g;
    std::memset(&g, 0, sizeof(g));
    size_t off = 0;
    for_each_pool([&](auto& b, int64_t per) {
      const size_t by = (size_t)per * L * sizeof(*b.p);
      g.ck[g.n] = ckpt.p + off;
      g.pool[g.n] = (uint8_t*)b.p;
      g.per[g.n] = per;
      g.esz[g.n++] = (int32_t)sizeof(*b.p);
      off += (by + 15) / 16 * 16;
    });
    d_dl.reserve(std::max<size_t>(dl.size(), 1));
    SG_HIP(hipMemcpyAsync(d_dl.p, dl.data(), dl.size() * 4, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_restore_lanes, dim3((unsigned)g.n), dim3(256), 0, s, g, d_dl.p, (int)dl.size(), (int64_t)L);
    SG_HIP(hipGetLastError());
  }
  RunOut sweep(hipStream_t s, int64_t ck0, int& rounds, double& t_run, double& t_res) {
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    const size_t NT = tick_now.size();
    const int64_t rcap = std::max<int64_t>(1024, (n - fx + (int64_t)(NT - fk)) * 8);
    grow_lanes(std::max<int64_t>(partitioned ? (int64_t)lane_key.size() : 1, 1), s);
    base_load(s);
    std::vector<SchedMap> maps = f_fresh ? std::vector<SchedMap>(tab.nabs) : fmaps;
    const size_t hmin = getenv("SG_NFA_SWEEP_TICKS") ? (size_t)std::max(1, atoi(getenv("SG_NFA_SWEEP_TICKS"))) : 128;
    if (tab.nabs > 0 && NT > 0) {
      d_tick_now.reserve(NT); d_tick_ev.reserve(NT);
      SG_HIP(hipMemcpyAsync(d_tick_now.p, tick_now.data(), NT * 8, hipMemcpyHostToDevice, s));
      SG_HIP(hipMemcpyAsync(d_tick_ev.p, tick_ev.data(), NT * 4, hipMemcpyHostToDevice, s));
    }
    in_sweep = true;
    sweep_uploaded = false;
    std::fill(ti_key, ti_key + 4, -1);
    for (double& x : sw_t) x = 0;
    struct Off { bool& f; ~Off() { f = false; } } off_{in_sweep};
    // the first window ends at the flush's first collision: every earlier tick ran without one
    size_t k0 = f_fresh ? 0 : fk;
    size_t H = std::max<size_t>(1, (size_t)(ck0 >> 8) > k0 ? (size_t)(ck0 >> 8) - k0 : 1);
    int64_t x0 = f_fresh ? 0 : fx, runs = 0;
    uint32_t rbase = 0;
    bool superseded = false;
    RunOut ro;
    for (;;) {
      const size_t k1 = std::min(NT, k0 + H);
      const int64_t x1 = k1 < NT ? (int64_t)tick_ev[k1] : n;
      pools_copy(true, s);
      bool collided = false;
      auto r0 = clk::now();
      ro = run_lanes(x0, k0, true, true, s, x1, (int64_t)k1, rbase, rcap);
      runs++;
      t_run += ms(r0);
      for (;;) {
        const auto r1 = clk::now();
        const bool more = shard == 3 ? resolve_window_shard(ro) : resolve_window(ro, maps);
        t_res += ms(r1);
        if (!more) break;
        rounds++;
        collided = true;
        // a deferral changes only its own instance: the deferred ones go back to the checkpoint and re-run the
        // window; their earlier records and logs are superseded, every other instance's stand
        r0 = clk::now();
        const std::vector<int32_t> dl(last_dlanes.begin(), last_dlanes.end());
        if (dl.empty() && shard == 3) continue;   // (the losers were other ranks' instances: this rank's logs stand)
        if (dl.empty()) throw Error(-3, "scheduler replay resolved a collision without deferring an instance");
        std::vector<uint8_t> only((size_t)L, 0);
        for (int32_t l : dl) only[(size_t)l] = 1;
        restore_lanes(dl, s);
        if (ro.nrec > rbase) {
          hipLaunchKernelGGL(k_rec_supersede, dim3((unsigned)((ro.nrec - rbase + 255) / 256)), dim3(256), 0, s,
                             rec_lane.p, rec_task.p, (int64_t)rbase, (int64_t)ro.nrec, d_dl.p, (int)dl.size());
          SG_HIP(hipGetLastError());
          superseded = true;
        }
        RunOut r2 = run_lanes(x0, k0, true, true, s, x1, (int64_t)k1, ro.nrec, rcap, &only);
        runs++;
        auto gone = [&](int32_t l) { return only[(size_t)l] != 0; };
        ro.fires.erase(std::remove_if(ro.fires.begin(), ro.fires.end(), [&](const FireRec& f) { return gone(f.lane); }), ro.fires.end());
        ro.ops.erase(std::remove_if(ro.ops.begin(), ro.ops.end(), [&](const OpRec& o) { return gone(o.lane); }), ro.ops.end());
        ro.fires.insert(ro.fires.end(), r2.fires.begin(), r2.fires.end());
        ro.ops.insert(ro.ops.end(), r2.ops.begin(), r2.ops.end());
        ro.nrec = r2.nrec;
        t_run += ms(r0);
      }
      rbase = ro.nrec;
      x0 = x1;
      k0 = k1;
      if (k0 >= NT && x0 >= n) break;
      H = collided ? hmin : std::min<size_t>(H * 2, (size_t)1 << 20);
    }
    kernel_ms["nfa_sweep_runs"] = (double)runs;      // diagnostic: launches (windows, and rounds' re-runs)
    if (getenv("SG_HOST_TIMING"))
      fprintf(stderr, "[sg sweep] runs %lld rounds %d: csr %.1f upload %.1f kernel+sync %.1f logs %.1f ms, resolve %.1f ms\n",
              (long long)runs, rounds, sw_t[0], sw_t[1], sw_t[2], sw_t[3], t_res);
    ro.nrec = rbase;
    ro.fires.clear();
    ro.ops.clear();
    if (superseded) ro.task_ok.assign(1, 0);          // task 0: superseded records (the live ones are -1)
    // the end is the new base; the deferrals lie before it
    fmaps = std::move(maps);
    base_save(s);
    deferrals.clear();
    return ro;
  }

  // shard mode (sg_query_shard_mode): collisions are resolved across ranks by the driver; every flush
  // re-runs the instances from the start with the deferrals given so far and keeps its logs
  int shard = 0;
  bool shard_dirty = false;
  RunOut shard_run;
  sg_shard_resolver_fn shard_cb = nullptr;   // mode 3 (streaming): the driver's answers to the Scheduler-map questions
  void* shard_user = nullptr;

  bool shard_mode(int mode) override {
    if (!(partitioned && tab.nabs > 0)) return false;
    if (mode && selector) throw Error(-2, "shard mode re-emits every match: the query's selector must be stateless");
    if (mode != shard) shard_dirty = true;
    shard = mode;
    shard_cb = nullptr;
    return true;
  }
  // Streaming shard mode: every flush runs from the settled base as a single runtime does, and where that runtime
  // reads its own Scheduler maps -- is there a collision in this run, and which instances lose in this window of the
  // sweep -- the driver answers from every rank's logs (sg_query_shard_resolver).  The rank re-runs only its own
  // deferred instances, from the window's checkpoint, so a settled window is never run again.
  bool shard_resolver(sg_shard_resolver_fn fn, void* user) override {
    if (!(partitioned && tab.nabs > 0)) return false;
    if (selector) throw Error(-2, "shard mode merges the ranks' matches by seq: the query's selector must be stateless");
    if (shard != 3) shard_dirty = true;
    shard = 3;
    shard_cb = fn;
    shard_user = user;
    return true;
  }
  void to_global(const RunOut& ro, std::vector<sg_sched_fire>& fv, std::vector<sg_sched_op>* ov) const {
    fv.resize(ro.fires.size());
    for (size_t i = 0; i < ro.fires.size(); i++) {
      const FireRec& f = ro.fires[i];
      fv[i] = sg_sched_fire{lane_key[f.lane], f.head, tick_seq[f.tau], f.tau, f.sched, f.empty_after, 0};
    }
    if (!ov) return;
    ov->resize(ro.ops.size());
    for (size_t i = 0; i < ro.ops.size(); i++) {
      const OpRec& o = ro.ops[i];
      sg_sched_op r;
      std::memset(&r, 0, sizeof(r));
      r.seq = o.phase == 0 ? tick_seq[o.tau] : h_seq[rank_ev[o.x]];
      r.head = o.phase == 0 ? o.head : 0;
      r.key = lane_key[o.lane];
      r.tick = o.phase == 0 ? o.tau : -1;
      r.sub = o.sub;
      r.pos = o.phase == 0 ? 0 : o.x;
      r.phase = o.phase;
      r.kfire = o.phase == 0 ? o.kfire : -1;
      r.ktarget = o.ktarget;
      (*ov)[i] = r;
    }
  }
  // kind 0: the first collision across the ranks' runs (-1: none)
  bool shard_first_collision(const RunOut& ro, int64_t& ck) {
    std::vector<sg_sched_fire> fv;
    to_global(ro, fv, nullptr);
    int64_t nd = 0;
    const int64_t r = shard_cb(shard_user, 0, fv.data(), (int64_t)fv.size(), nullptr, 0, nullptr, 0, &nd);
    if (r < -1) throw Error(SG_E_INVALID, "shard resolver failed (first collision)");
    ck = r;
    return r >= 0;
  }
  // kind 1: one window of the sweep; this rank's losers are deferred (last_dlanes: its instances to re-run)
  std::vector<int64_t> shard_defer_buf;
  bool resolve_window_shard(const RunOut& ro) {
    std::vector<sg_sched_fire> fv;
    std::vector<sg_sched_op> ov;
    to_global(ro, fv, &ov);
    shard_defer_buf.resize((size_t)3 * std::max<int64_t>(L, 1));
    int64_t nd = 0;
    const int64_t r = shard_cb(shard_user, 1, fv.data(), (int64_t)fv.size(), ov.data(), (int64_t)ov.size(),
                               shard_defer_buf.data(), (int64_t)shard_defer_buf.size() / 3, &nd);
    if (r < 0) throw Error(SG_E_INVALID, "shard resolver failed (window)");
    last_dlanes.clear();
    if (r == 0) return false;
    for (int64_t i = 0; i < nd; i++) {
      const int64_t key = shard_defer_buf[3 * i], tick = shard_defer_buf[3 * i + 1], sc = shard_defer_buf[3 * i + 2];
      const auto f = key_lane.find(key);
      if (f == key_lane.end()) throw Error(SG_E_INVALID, "shard resolver deferred a key this rank does not own");
      defer(f->second, (tick << 8) | sc);
      last_dlanes.insert(f->second);
    }
    return true;
  }
  int64_t sched_fires(sg_sched_fire* out, int64_t cap) const override {
    if (!shard) return -1;
    const int64_t c = (int64_t)shard_run.fires.size();
    for (int64_t i = 0; i < std::min(c, cap); i++) {
      const FireRec& f = shard_run.fires[i];
      out[i] = sg_sched_fire{lane_key[f.lane], f.head, tick_seq[f.tau], f.tau, f.sched, f.empty_after, 0};
    }
    return c;
  }
  int64_t sched_clock(int64_t* now, int64_t cap, int64_t* min_wait) const override {
    if (!(partitioned && tab.nabs > 0)) return -1;
    const int64_t c = (int64_t)tick_now.size();
    for (int64_t i = 0; i < std::min(c, cap); i++) now[i] = tick_now[(size_t)i];
    if (min_wait) {
      int64_t w = INT64_MAX;
      for (int k = 0; k < tab.nabs; k++) w = std::min<int64_t>(w, std::max<int64_t>(0, tab.waiting[(int)tab.absOrder[k]]));
      *min_wait = w;
    }
    return c;
  }
  int64_t sched_ops(sg_sched_op* out, int64_t cap) const override {
    if (shard != 2) return -1;
    const int64_t c = (int64_t)shard_run.ops.size();
    for (int64_t i = 0; i < std::min(c, cap); i++) {
      const OpRec& o = shard_run.ops[i];
      sg_sched_op r;
      std::memset(&r, 0, sizeof(r));
      // a tick-phase op belongs to its tick (the send the tick precedes); an event-phase op to its event
      r.seq = o.phase == 0 ? tick_seq[o.tau] : h_seq[rank_ev[o.x]];
      r.head = o.phase == 0 ? o.head : 0;
      r.key = lane_key[o.lane];
      r.tick = o.phase == 0 ? o.tau : -1;
      r.sub = o.sub;
      r.pos = o.phase == 0 ? 0 : o.x;
      r.phase = o.phase;
      r.kfire = o.phase == 0 ? o.kfire : -1;
      r.ktarget = o.ktarget;
      out[i] = r;
    }
    return c;
  }
  bool sched_defer(int64_t key, int32_t tick, int sched) override {
    if (!shard) return false;
    const auto f = key_lane.find(key);
    if (f == key_lane.end()) return false;
    defer(f->second, ((int64_t)tick << 8) | sched);
    shard_dirty = true;
    return true;
  }

  // ---- event-store compaction ----
  // A long-running runtime would otherwise keep every event it was ever sent (the chains index the store)
  // and fail at 2^31.  Once the store has doubled since the last compaction (at least 2^20 events;
  // SG_NFA_COMPACT_MIN for tests), the events the instances' chains still reference are renumbered in order,
  // with their stream rows, arrival ranks and host bookkeeping, and the rest are dropped.  Not with Scheduler
  // ticks (the exact collision replay re-runs from the first event), broadcast streams (instance creation
  // ranks order their HashSet) or shard mode.
  int64_t compact_at = 0;
  int64_t buffered() const override { return n; }
  DBuf<uint8_t> cmp_mark, cmp_tmp, cmp_fr;
  DBuf<unsigned long long> probe_buf;     // SG_NFA_PROBE builds
  // event prefilter: which (stream, next-processor) pairs may be skipped, and the per-event masks so far
  std::vector<uint8_t> pf_elig;           // [NSTR * NP]
  bool pf_any = false;
  DBuf<uint8_t> d_pf_elig;
  DBuf<uint16_t> ev_skip;
  int64_t skip_done = 0;                  // events [0, skip_done) have their mask
  void build_prefilter() {
    pf_elig.assign((size_t)NSTR * NP, 0);
    pf_any = false;
    if (tab.seq || getenv("SG_NFA_NO_PREFILTER")) return;
    for (int st = 0; st < (int)streams.size() && st < NSTR; st++)
      for (int k = 0; k < tab.nnext[st]; k++) {
        const NProc& P = tab.p[tab.nexts[st][k]];
        const bool kind_ok = P.kind == K_STREAM || P.kind == K_ABSENT || (P.kind == K_LOGICAL && P.isAnd && !P.absLog);
        if (!kind_ok || P.filter < 0 || tab.slotStream[P.stateId] != st) continue;
        const Prog& pr = progs[(size_t)P.filter];
        bool own = true;
        for (int pc = 0; pc < pr.n && own; pc++)
          if (pr.ins[pc].op == BC_LD) {
            const int code = pr.ins[pc].a, chain = (code & 15) - 8;
            own = (code >> 4) == P.stateId && (chain == 0 || chain == -1);
          }
        if (own) { pf_elig[(size_t)st * NP + k] = 1; pf_any = true; }
      }
  }
  void prefilter(hipStream_t s) {
    if (!pf_any || skip_done >= n) return;
    ev_skip.reserve((size_t)n, true, s, (size_t)skip_done);
    if (d_pf_elig.cap == 0) {
      d_pf_elig.reserve(pf_elig.size(), false);
      SG_HIP(hipMemcpyAsync(d_pf_elig.p, pf_elig.data(), pf_elig.size(), hipMemcpyHostToDevice, s));
    }
    const int64_t m = n - skip_done;
    hipLaunchKernelGGL(k_nfa_prefilter, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, skip_done, n, ev_stream.p,
                       ev_row.p, d_tab.p, d_cols.p, d_progs.p, d_pf_elig.p, ev_skip.p);
    SG_HIP(hipGetLastError());
    skip_done = n;
  }
  DBuf<int32_t> cmp_list, cmp_map, cmp_n, cmp_i32;
  DBuf<int64_t> cmp_idx;
  // Absent states: partitioned, only when the sweep's base is the present (an exact replay starts there, so no
  // event before it is read again except through live chains); unpartitioned ones never replay.
  bool compactable() const {
    if (shard || getenv("SG_NFA_NO_COMPACT")) return false;
    for (int k = 0; k < NSTR; k++) if (bcast[k]) return false;
    if (tab.nabs > 0 && partitioned && !base_current()) return false;
    return true;
  }
  void compact(hipStream_t s) {
    if (compact_at == 0) {
      const char* e = getenv("SG_NFA_COMPACT_MIN");
      compact_at = e ? std::max<int64_t>(1, atoll(e)) : (int64_t)1 << 20;
    }
    if (!compactable() || n < compact_at || L <= 0) return;
    PhaseClock pc(getenv("SG_HOST_TIMING") != nullptr);
    const NState g = state();
    const int64_t nodes = (int64_t)nd_cap * L;
    cmp_fr.reserve((size_t)nodes, false);
    SG_HIP(hipMemsetAsync(cmp_fr.p, 0, (size_t)nodes, s));
    hipLaunchKernelGGL(k_nfa_free_nodes, dim3((unsigned)((L + 255) / 256)), dim3(256), 0, s, g, cmp_fr.p);
    cmp_mark.reserve((size_t)n, false);
    SG_HIP(hipMemsetAsync(cmp_mark.p, 0, (size_t)n, s));
    hipLaunchKernelGGL(k_nfa_mark_live, dim3((unsigned)((nodes + 255) / 256)), dim3(256), 0, s, g, cmp_fr.p, n, cmp_mark.p);
    SG_HIP(hipGetLastError());
    cmp_list.reserve((size_t)n, false);
    cmp_n.reserve(1, false);
    hipcub::CountingInputIterator<int32_t> cidx(0);
    size_t tb = 0;
    SG_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb, cidx, cmp_mark.p, cmp_list.p, cmp_n.p, (int)n, s));
    cmp_tmp.reserve(std::max<size_t>(tb, 1), false);
    SG_HIP(hipcub::DeviceSelect::Flagged(cmp_tmp.p, tb, cidx, cmp_mark.p, cmp_list.p, cmp_n.p, (int)n, s));
    int32_t m32 = 0;
    SG_HIP(hipMemcpyAsync(&m32, cmp_n.p, 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    const int64_t m = m32;
    // the nodes take the new event indices
    cmp_map.reserve((size_t)n, false);
    SG_HIP(hipMemsetAsync(cmp_map.p, 0xff, (size_t)n * 4, s));
    if (m > 0) hipLaunchKernelGGL(k_nfa_cmp_map, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, m, cmp_list.p, cmp_map.p);
    hipLaunchKernelGGL(k_nfa_remap_nodes, dim3((unsigned)((nodes + 255) / 256)), dim3(256), 0, s, g, cmp_fr.p, n, cmp_map.p);
    SG_HIP(hipGetLastError());
    // the kept events' old index, arrival rank, stream and row, gathered on the device (O(kept) to the host)
    std::vector<int32_t> list((size_t)m), grank((size_t)m), grow((size_t)m);
    std::vector<int8_t> gst((size_t)m);
    if (m > 0) {
      cmp_i32.reserve((size_t)m * 2, false);
      cmp_tmp.reserve((size_t)m, false);
      hipLaunchKernelGGL(k_nfa_cmp_gather, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, m, cmp_list.p, ev_rank.p,
                         ev_row.p, ev_stream.p, cmp_i32.p, cmp_i32.p + m, (int8_t*)cmp_tmp.p);
      SG_HIP(hipMemcpyAsync(list.data(), cmp_list.p, (size_t)m * 4, hipMemcpyDeviceToHost, s));
      SG_HIP(hipMemcpyAsync(grank.data(), cmp_i32.p, (size_t)m * 4, hipMemcpyDeviceToHost, s));
      SG_HIP(hipMemcpyAsync(grow.data(), cmp_i32.p + m, (size_t)m * 4, hipMemcpyDeviceToHost, s));
      SG_HIP(hipMemcpyAsync(gst.data(), cmp_tmp.p, (size_t)m, hipMemcpyDeviceToHost, s));
    }
    SG_HIP(hipStreamSynchronize(s));
    pc.mark("compact: mark + remap");
    // arrival ranks: the kept events in their old rank order
    std::vector<int32_t> by_rank((size_t)m);
    for (int64_t k = 0; k < m; k++) by_rank[(size_t)k] = (int32_t)k;
    std::sort(by_rank.begin(), by_rank.end(), [&](int32_t x, int32_t y) { return grank[(size_t)x] < grank[(size_t)y]; });
    std::vector<int32_t> ev_rank2((size_t)std::max<int64_t>(m, 1));
    for (int64_t r = 0; r < m; r++) ev_rank2[(size_t)by_rank[(size_t)r]] = (int32_t)r;
    // per-event host bookkeeping gathered in place (list ascends: k <= list[k]), keeping the vectors' capacity
    // (freeing them would make the next push fault their pages in again)
    std::vector<int64_t> idx64((size_t)std::max<int64_t>(m, 1));
    std::vector<int32_t> row2((size_t)std::max<int64_t>(m, 1));
    std::vector<std::vector<int64_t>> srows(streams.size());
    for (int64_t k = 0; k < m; k++) {
      const int32_t e = list[(size_t)k];
      h_seq[(size_t)k] = h_seq[(size_t)e]; h_stream[(size_t)k] = h_stream[(size_t)e]; h_lane[(size_t)k] = h_lane[(size_t)e];
      idx64[(size_t)k] = e;
      auto& sr = srows[(size_t)gst[(size_t)k]];
      row2[(size_t)k] = (int32_t)sr.size();
      sr.push_back(grow[(size_t)k]);
    }
    h_seq.resize((size_t)m); h_stream.resize((size_t)m); h_lane.resize((size_t)m);
    rank_ev.resize((size_t)m);
    for (int64_t r = 0; r < m; r++) rank_ev[(size_t)r] = by_rank[(size_t)r];
    pc.mark("compact: host bookkeeping");
    cmp_idx.reserve(idx64.size(), false);
    SG_HIP(hipMemcpyAsync(cmp_idx.p, idx64.data(), idx64.size() * 8, hipMemcpyHostToDevice, s));
    compact_rows(ev_ts.p, cmp_idx.p, m, cmp_tmp, s);
    compact_rows(ev_now.p, cmp_idx.p, m, cmp_tmp, s);
    compact_rows(ev_stream.p, cmp_idx.p, m, cmp_tmp, s);
    if (pf_any && skip_done >= n) compact_rows(ev_skip.p, cmp_idx.p, m, cmp_tmp, s);
    SG_HIP(hipMemcpyAsync(ev_row.p, row2.data(), (size_t)m * 4, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(ev_rank.p, ev_rank2.data(), (size_t)m * 4, hipMemcpyHostToDevice, s));
    for (size_t ls = 0; ls < streams.size(); ls++) {
      const auto& sr = srows[ls];
      const int64_t ml = (int64_t)sr.size();
      if (ml > 0) {
        SG_HIP(hipStreamSynchronize(s));               // (cmp_idx is reused per stream)
        SG_HIP(hipMemcpyAsync(cmp_idx.p, sr.data(), (size_t)ml * 8, hipMemcpyHostToDevice, s));
        for (auto& c : cols[ls]) compact_col(c.b.p, c.w, cmp_idx.p, ml, cmp_tmp, s);
        if (has_nul[ls]) {
          const int w = (int)cols[ls].size();
          cmp_tmp.reserve((size_t)ml * w, false);
          hipLaunchKernelGGL(k_nfa_gather_rows, dim3((unsigned)((ml + 255) / 256)), dim3(256), 0, s, nulcol[ls].p, cmp_idx.p,
                             ml, w, cmp_tmp.p);
          SG_HIP(hipMemcpyAsync(nulcol[ls].p, cmp_tmp.p, (size_t)ml * w, hipMemcpyDeviceToDevice, s));
        }
      }
      rows[ls] = ml;
    }
    SG_HIP(hipGetLastError());
    SG_HIP(hipStreamSynchronize(s));
    kernel_ms["nfa_compacted_from"] = (double)n;
    kernel_ms["nfa_compacted_to"] = (double)m;
    skip_done = (pf_any && skip_done >= n) ? m : 0;
    n = m;
    flushed = m;
    dev_push_n = 0;
    compact_at = std::max<int64_t>(compact_at, 2 * m);
    if (tab.nabs > 0) {
      // every tick so far is settled: each precedes the next event to come (place_new starts from their ranks),
      // and every instance was created before it
      for (auto& te : tick_ev) te = (int32_t)m;
      for (auto& cr : create_rank) cr = std::min<int32_t>(cr, 0);
      if (partitioned) base_save(s);               // the base's pools hold the renumbered chains
    }
    pc.mark("compact: gathers");
  }

  void flush(std::vector<Callback>& out, bool materialise, hipStream_t s) override {
    last_matches = 0;
    kernel_ms["nfa_chain_device_rows"] = (double)chain_dev_rows;   // diagnostic: rows chained in HBM since the last flush
    chain_dev_rows = 0;
    if (shard && shard != 3) {
      // shard mode: every flush reports the whole run (the protocol compares complete runs across ranks),
      // so a rank with nothing new since its last run reports that run again
      if (n <= flushed && ticks_flushed == tick_now.size() && !shard_dirty) {
        emit(shard_run.nrec, 0, 0, 0, true, materialise, out, s);
        return;
      }
      place_new(s);
      if (L > 0) {
        hipLaunchKernelGGL(k_nfa_pool_init, dim3((unsigned)((L + 255) / 256)), dim3(256), 0, s, state(), 0, L);
        SG_HIP(hipGetLastError());
      }
      shard_run = run_lanes(0, 0, true, shard == 2, s);
      flushed = n;
      ticks_flushed = tick_now.size();
      shard_dirty = false;
      kernel_ms["nfa_exact_rounds"] = 0;
      emit(shard_run.nrec, 0, 0, 0, true, materialise, out, s);
      return;
    }
    // (streaming shard mode: every rank asks the driver at every flush, new events or not, to stay in step)
    if (n <= flushed && ticks_flushed == tick_now.size() && shard != 3) return;
    const auto th0 = std::chrono::steady_clock::now();
    auto hms = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count(); };
    const bool ht = getenv("SG_HOST_TIMING") != nullptr;
    place_new(s);
    if (ht) fprintf(stderr, "[sg nfa] place %.1f ms\n", hms());
    const size_t t0 = ticks_flushed;
    const int64_t f0 = flushed;
    const bool sched_log = partitioned && tab.nabs > 0;
    size_t tk_base = t0;
    fire_lazy = sched_log && shard != 3 && !getenv("SG_NFA_HOST_COLLISION_CHECK");
    RunOut ro = run_lanes(flushed, t0, sched_log, false, s);
    fire_lazy = false;
    int rounds = 0;
    bool replayed = false;
    PhaseClock pc(getenv("SG_HOST_TIMING") != nullptr);
    if (sched_log) {
      int64_t ck;
      bool col;
      if (shard == 3) {
        col = shard_first_collision(ro, ck);
      } else if (ro.fires_dev > 0 && !fires_may_collide(ro, s)) {
        col = false;                                       // (the device pre-check: the log never leaves HBM)
        ro.fires_dev = 0;
      } else {
        fetch_fires(ro, s);
        col = first_collision(ro.fires, ck);
      }
      kernel_ms["nfa_host_collision_check"] = (double)!ro.fires.empty();
      pc.mark("collision check");
      replayed = col;
      if (col && (shard == 3 || !getenv("SG_NFA_REPLAY_ROUNDS"))) {
        double t_run = 0, t_res = 0;
        ro = sweep(s, ck, rounds, t_run, t_res);
        kernel_ms["nfa_replay_run_ms"] = t_run;
        kernel_ms["nfa_replay_resolve_ms"] = t_res;
        tk_base = 0;
      } else if (col) {
        // (SG_NFA_REPLAY_ROUNDS, the round-3 form kept for comparison) replay the app from its start with
        // the exact map order, deferring the losers, until no tick has a collision
        double t_run = 0, t_res = 0;
        for (int round = 0;; round++) {
          if (round > 100000) throw Error(-3, "scheduler collision replay did not converge");
          const double r0 = hms();
          NState ns = state();
          hipLaunchKernelGGL(k_nfa_pool_init, dim3((unsigned)((L + 255) / 256)), dim3(256), 0, s, ns, 0, L);
          SG_HIP(hipGetLastError());
          ro = run_lanes(0, 0, true, true, s);
          rounds++;
          const double r1 = hms();
          const bool more = resolve_first_collision(ro);
          t_run += r1 - r0;
          t_res += hms() - r1;
          if (!more) break;
        }
        kernel_ms["nfa_replay_run_ms"] = t_run;     // diagnostics: lane re-runs and host map replays
        kernel_ms["nfa_replay_resolve_ms"] = t_res;
        tk_base = 0;
      }
    }
    kernel_ms["nfa_exact_rounds"] = rounds;   // diagnostic: exact Scheduler replays of this flush
    if (ht) fprintf(stderr, "[sg nfa] run %.1f ms (kernel %.1f)\n", hms(), kernel_ms["k_nfa_lanes"]);
    flushed = n;
    ticks_flushed = tick_now.size();
    emit(ro.nrec, tk_base, t0, f0, replayed, materialise, out, s, ro.task_ok);
    compact(s);
  }

  // The records of a run as callbacks: those of ticks >= t0 and events >= f0 (a replay from the start,
  // `replayed`, re-emits earlier flushes' records); tk_base = the run's first tick
  void emit(uint32_t nrec_all, size_t tk_base, size_t t0, int64_t f0, bool replayed, bool materialise,
            std::vector<Callback>& out, hipStream_t s, const std::vector<uint8_t>& task_ok = {}) {
    if (nrec_all == 0) return;
    // a speculative run: records of segments that did not verify are dropped
    // (host staging in pinned members: full-rate copies, no allocation per flush)
    pvec<int32_t>& rtask = em_task;
    rtask.clear();
    if (!task_ok.empty()) {
      rtask.resize(nrec_all);
      SG_HIP(hipMemcpyAsync(rtask.data(), rec_task.p, nrec_all * 4, hipMemcpyDeviceToHost, s));
      SG_HIP(hipStreamSynchronize(s));
    }
    auto kept = [&](uint32_t k) { return rtask.empty() || rtask[k] < 0 || task_ok[(size_t)rtask[k]]; };
    // without an exact replay the launch ran only this flush's events and ticks: every record is new,
    // and a device-resident flush needs only their count
    if (!materialise && !replayed) {
      if (rtask.empty()) { last_matches = nrec_all; return; }
      int64_t c = 0;
      for (uint32_t k = 0; k < nrec_all; k++) c += kept(k);
      last_matches = c;
      return;
    }
    PhaseClock pc(getenv("SG_HOST_TIMING") != nullptr);
    pvec<uint64_t>& key = em_key;
    pvec<int32_t>& rtick = em_tick;
    key.resize(nrec_all);
    rtick.resize(nrec_all);
    SG_HIP(hipMemcpyAsync(key.data(), rec_key.p, nrec_all * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(rtick.data(), rec_tick.p, nrec_all * 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    // records of this flush only (an exact replay re-emits earlier flushes' records)
    std::vector<uint32_t> idx;
    idx.reserve(nrec_all);
    for (uint32_t k = 0; k < nrec_all; k++) {
      const bool mine = rtick[k] >= 0 ? (size_t)(rtick[k] + (int32_t)tk_base) >= t0 : (int64_t)(key[k] >> 24) >= f0;
      if (mine && kept(k)) idx.push_back(k);
    }
    last_matches = idx.size();
    if (!materialise || idx.empty()) return;
    pvec<int64_t>& rts = em_ts;
    pvec<int64_t>& rdl = em_dl;
    pvec<int8_t>& rsched = em_sched;
    pvec<int64_t>& val = em_val;
    pvec<uint8_t>& nul = em_nul;
    rts.resize(nrec_all); rdl.resize(nrec_all); rsched.resize(nrec_all);
    val.resize((size_t)nrec_all * nsel); nul.resize((size_t)nrec_all * nsel);
    if (!tab.nabs) {
      std::fill(rdl.begin(), rdl.end(), 0);
      std::fill(rsched.begin(), rsched.end(), 0);
    }
    if (nsel) {
      SG_HIP(hipMemcpyAsync(val.data(), rec_val.p, val.size() * 8, hipMemcpyDeviceToHost, s));
      SG_HIP(hipMemcpyAsync(nul.data(), rec_nul.p, nul.size(), hipMemcpyDeviceToHost, s));
    }
    // the timestamps of the records' trigger events only, gathered on the device (not all n events' across PCIe)
    pvec<int64_t>& hts = em_hts;
    hts.resize(nrec_all);
    {
      pvec<int32_t>& evi = em_evi;
      evi.resize(nrec_all);
      const int eth = host_threads((int64_t)nrec_all * 8);
      host_parallel(eth, [&](int t) {
        for (uint32_t k = (uint32_t)((int64_t)nrec_all * t / eth), e = (uint32_t)((int64_t)nrec_all * (t + 1) / eth); k < e; k++)
          evi[k] = rtick[k] >= 0 ? 0 : rank_ev[(size_t)(key[k] >> 24)];
      });
      emit_evi.reserve(nrec_all); emit_ts.reserve(nrec_all);
      SG_HIP(hipMemcpyAsync(emit_evi.p, evi.data(), (size_t)nrec_all * 4, hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(k_nfa_gather_ts, dim3((unsigned)((nrec_all + 255) / 256)), dim3(256), 0, s, ev_ts.p, emit_evi.p,
                         (int64_t)nrec_all, emit_ts.p);
      SG_HIP(hipGetLastError());
      SG_HIP(hipMemcpyAsync(hts.data(), emit_ts.p, (size_t)nrec_all * 8, hipMemcpyDeviceToHost, s));
      SG_HIP(hipStreamSynchronize(s));
    }
    SG_HIP(hipMemcpyAsync(rts.data(), rec_ts.p, nrec_all * 8, hipMemcpyDeviceToHost, s));
    std::vector<int32_t> rlane;
    const bool bc_any = partitioned && std::any_of(std::begin(bcast), std::end(bcast), [](bool x) { return x; });
    if (selector || bc_any) {
      rlane.resize(nrec_all);
      SG_HIP(hipMemcpyAsync(rlane.data(), rec_lane.p, nrec_all * 4, hipMemcpyDeviceToHost, s));
    }
    if (tab.nabs) {
      SG_HIP(hipMemcpyAsync(rdl.data(), rec_dl.p, nrec_all * 8, hipMemcpyDeviceToHost, s));
      SG_HIP(hipMemcpyAsync(rsched.data(), rec_sched.p, nrec_all, hipMemcpyDeviceToHost, s));
    }
    SG_HIP(hipStreamSynchronize(s));
    // reference order: by trigger position; a tick's records before the event's holders, ordered by
    // tick, Scheduler (listener order), head deadline (TreeMultimap key), then emission
    // a broadcast event runs in every instance in turn, in the iteration order of the partition-key
    // HashSet at that moment (PartitionRuntimeImpl.getPartitionKeys copied into a HashSet: capacity
    // tableSizeFor(max(n / .75 + 1, 16)), bins by the spread String hash, creation order inside a bin)
    std::vector<int32_t> sorted_cr;
    if (bc_any) {
      sorted_cr = create_rank;
      std::sort(sorted_cr.begin(), sorted_cr.end());
      while (lane_hash_c.size() < lane_key.size())      // lane_hash is already spread (h ^ h >>> 16)
        lane_hash_c.push_back(lane_hash((int)lane_hash_c.size()));
    }
    auto hs_pos = [&](int64_t r, int32_t lane) -> uint64_t {
      const size_t nr = (size_t)(std::lower_bound(sorted_cr.begin(), sorted_cr.end(), (int32_t)r) - sorted_cr.begin());
      const size_t want = std::max<size_t>((size_t)((float)nr / .75f) + 1, 16);
      size_t cap = 1;
      while (cap < want) cap <<= 1;
      return ((uint64_t)((uint32_t)lane_hash_c[lane] & (uint32_t)(cap - 1)) << 32) | (uint32_t)create_rank[lane];
    };
    auto is_bcast_rec = [&](uint32_t x) { return bc_any && rtick[x] < 0 && h_lane[rank_ev[(size_t)(key[x] >> 24)]] == -1; };
    pc.mark("emit: records to host");
    if (!bc_any) {
      // the same order as the comparator below without broadcast events, as one flat key per record (a non-tick
      // record's tick fields equal: -1, 0, 0) sorted over thread ranges; the record index keeps it stable
      struct SortRec { uint64_t px; int32_t tick; int32_t sched; int64_t dl; uint32_t low, k; };
      std::vector<SortRec> sr(idx.size());
      const int sth = host_threads((int64_t)idx.size() * 8);
      host_parallel(sth, [&](int t) {
        for (size_t q = idx.size() * t / sth, e = idx.size() * (t + 1) / sth; q < e; q++) {
          const uint32_t k = idx[q];
          const bool tk_ = rtick[k] >= 0;
          sr[q] = SortRec{key[k] >> 20, tk_ ? rtick[k] : -1, tk_ ? (int32_t)rsched[k] : 0, tk_ ? rdl[k] : 0,
                          (uint32_t)(key[k] & 0xfffff), k};
        }
      });
      par_sort(sr, [](const SortRec& a, const SortRec& b) {
        if (a.px != b.px) return a.px < b.px;
        if (a.tick != b.tick) return a.tick < b.tick;
        if (a.sched != b.sched) return a.sched < b.sched;
        if (a.dl != b.dl) return a.dl < b.dl;
        if (a.low != b.low) return a.low < b.low;
        return a.k < b.k;
      }, host_threads((int64_t)sr.size() * 4));
      for (size_t q = 0; q < idx.size(); q++) idx[q] = sr[q].k;
    } else
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) {
      const uint64_t ex = key[x] >> 24, ey = key[y] >> 24;
      if (ex != ey) return ex < ey;
      if (is_bcast_rec(x) && is_bcast_rec(y) && rlane[x] != rlane[y])
        return hs_pos((int64_t)ex, rlane[x]) < hs_pos((int64_t)ex, rlane[y]);
      const uint64_t px = key[x] >> 20, py = key[y] >> 20;   // (event, holder field)
      if (px != py) return px < py;
      if (rtick[x] >= 0) {
        if (rtick[x] != rtick[y]) return rtick[x] < rtick[y];
        if (rsched[x] != rsched[y]) return rsched[x] < rsched[y];
        if (rdl[x] != rdl[y]) return rdl[x] < rdl[y];
      }
      return (key[x] & 0xfffff) < (key[y] & 0xfffff);
    });
    // callbacks: one per (event, holder) for a multi receiver; one per match for a single receiver
    // with a selector stage each match is one chunk through QuerySelector.process
    // (StreamPostStateProcessor -> QuerySelector per returned StateEvent); a match it drops emits nothing
    // QuerySelector on the device (selector_dev.hpp): each match is one chunk, in callback order; the host
    // SelectorStage runs instead when the device declines (a group-key hash collision, a sum that could round)
    DevSelRows dsr;
    std::vector<int64_t> sel_at;                     // per position in idx: its selected row, or -1
    bool dev_sel = false;
    if (selector && !getenv("SG_NFA_HOST_SELECTOR")) {
      const int64_t M = (int64_t)idx.size();
      std::vector<uint8_t> ity((size_t)M, (uint8_t)GI_CUR);
      std::vector<int64_t> its((size_t)M);
      std::vector<int32_t> irow((size_t)M), ilid((size_t)M), iord((size_t)M);
      for (int64_t q = 0; q < M; q++) {
        const uint32_t k = idx[(size_t)q];
        its[(size_t)q] = rtick[k] >= 0 ? rts[k] : hts[k];
        irow[(size_t)q] = (int32_t)k; ilid[(size_t)q] = rlane[k]; iord[(size_t)q] = (int32_t)q;
      }
      DevSelector::h2d(sel_ty, ity.data(), ity.size(), s);
      DevSelector::h2d(sel_ts, its.data(), its.size(), s);
      DevSelector::h2d(sel_row, irow.data(), irow.size(), s);
      DevSelector::h2d(sel_lid, ilid.data(), ilid.size(), s);
      DevSelector::h2d(sel_ord, iord.data(), iord.size(), s);
      const GwdItems it{sel_ty.p, sel_ts.p, sel_row.p, sel_lid.p, sel_ord.p, M};
      const GwdVals vals{rec_val.p, rec_nul.p, 1, std::max(nsel, 1)};
      if (dsel.run(selspec, *selector, partitioned, M, it, vals, (int64_t)nrec_all, [](int32_t l) { return (int64_t)l; },
                   s, dsr)) {
        dev_sel = true;
        sel_at.assign((size_t)M, -1);
        for (int64_t r = 0; r < dsr.P; r++) sel_at[(size_t)dsr.ord(r)] = r;
      }
      kernel_ms["nfa_device_selector"] = dev_sel ? 1 : 0;
    }
    pc.mark("emit: order");
    if (!selector && host_threads((int64_t)idx.size() * 256) > 1) {   // (4,096 records and up)
      // the callback boundaries first (sequential: a multi receiver's holder groups, the loop below restated), then
      // the callbacks and their rows over thread ranges
      std::vector<uint32_t> cstart;
      cstart.reserve(idx.size() + 1);
      uint64_t cg = ~0ull;
      int32_t cl = -1;
      for (size_t pos = 0; pos < idx.size(); pos++) {
        const uint32_t k = idx[pos];
        const uint64_t kk = key[k];
        const int ev = rank_ev[(size_t)(kk >> 24)];
        const uint64_t grp = kk >> 20;
        const int32_t glane = is_bcast_rec(k) ? rlane[k] : -1;
        const bool timer = rtick[k] >= 0;
        const bool multi = !timer && tab.multi[h_stream[ev]] != 0;
        if (!multi || cstart.empty() || grp != cg || glane != cl) {
          cl = glane;
          cstart.push_back((uint32_t)pos);
          cg = timer ? ~0ull : grp;
        }
      }
      const size_t nc = cstart.size(), o0 = out.size();
      cstart.push_back((uint32_t)idx.size());
      out.resize(o0 + nc);
      const int nth = host_threads((int64_t)idx.size() * 8);
      host_parallel(nth, [&](int t) {
        for (size_t c = nc * t / nth, ce = nc * (t + 1) / nth; c < ce; c++) {
          Callback& cb = out[o0 + c];
          const uint32_t k0 = idx[cstart[c]];
          const bool timer = rtick[k0] >= 0;
          cb.seq = timer ? tick_seq[tk_base + rtick[k0]] : h_seq[rank_ev[(size_t)(key[k0] >> 24)]];
          cb.tsched = timer ? (int32_t)rsched[k0] : -1;
          cb.tdl = timer ? rdl[k0] : 0;
          cb.order = qi;
          cb.kind = 0;
          cb.target = qi;
          cb.ev.reserve(cstart[c + 1] - cstart[c]);
          for (uint32_t pos = cstart[c]; pos < cstart[c + 1]; pos++) {
            const uint32_t k = idx[pos];
            OutEvent oe;
            oe.ts = rtick[k] >= 0 ? rts[k] : hts[k];
            oe.raw.assign(val.begin() + (size_t)k * nsel, val.begin() + (size_t)(k + 1) * nsel);
            oe.nul.assign(nul.begin() + (size_t)k * nsel, nul.begin() + (size_t)(k + 1) * nsel);
            cb.ts = oe.ts;
            cb.ev.push_back(std::move(oe));
          }
        }
      });
      pc.mark("emit: callbacks");
      return;
    }
    Callback* cur = nullptr;
    uint64_t curgrp = ~0ull;
    int32_t curlane = -1;
    std::vector<SelIn> chunk(1);
    out.reserve(out.size() + idx.size());
    for (size_t pos = 0; pos < idx.size(); pos++) {
      const uint32_t k = idx[pos];
      uint64_t kk = key[k];
      int ev = rank_ev[(size_t)(kk >> 24)];
      uint64_t grp = kk >> 20;
      const int32_t glane = is_bcast_rec(k) ? rlane[k] : -1;   // a broadcast event: one holder per instance
      const bool timer = rtick[k] >= 0;              // fired by a Scheduler tick: one callback per match
      bool multi = !timer && tab.multi[h_stream[ev]] != 0;
      const int64_t ts = timer ? rts[k] : hts[k];
      std::vector<SelOut> so;
      if (selector) {
        if (dev_sel) {
          const int64_t r = sel_at[pos];
          if (r < 0) continue;
          DevSelector::batch(selspec, *selector, dsr, r, r + 1, so);
        } else {
          chunk[0] = SelIn{SE_CURRENT, ts, val.data() + (size_t)k * nsel, nul.data() + (size_t)k * nsel, rlane[k]};
          so = selector->process(chunk);
        }
        if (so.empty()) continue;
      }
      if (!multi || cur == nullptr || grp != curgrp || glane != curlane) {
        curlane = glane;
        out.emplace_back();
        cur = &out.back();
        cur->seq = timer ? tick_seq[tk_base + rtick[k]] : h_seq[ev];
        cur->tsched = timer ? (int32_t)rsched[k] : -1;
        cur->tdl = timer ? rdl[k] : 0;
        cur->order = qi;
        cur->kind = 0;
        cur->target = qi;
        curgrp = timer ? ~0ull : grp;
      }
      if (selector) {
        for (auto& o : so) {
          OutEvent oe;
          oe.ts = o.ts;
          oe.raw = std::move(o.raw);
          oe.nul = std::move(o.nul);
          cur->ts = oe.ts;
          cur->ev.push_back(std::move(oe));
        }
        continue;
      }
      OutEvent oe;
      oe.ts = ts;
      oe.raw.assign(val.begin() + (size_t)k * nsel, val.begin() + (size_t)(k + 1) * nsel);
      oe.nul.assign(nul.begin() + (size_t)k * nsel, nul.begin() + (size_t)(k + 1) * nsel);
      cur->ts = oe.ts;
      cur->ev.push_back(std::move(oe));
    }
    pc.mark("emit: callbacks");
  }
  DBuf<int32_t> emit_evi;
  DBuf<int64_t> emit_ts;
  pvec<uint64_t> em_key;
  pvec<int32_t> em_task, em_tick, em_evi;
  pvec<int64_t> em_ts, em_dl, em_val, em_hts;
  pvec<int8_t> em_sched;
  pvec<uint8_t> em_nul;
};

std::unique_ptr<Exec> make_nfa(App& app, int qi, const J& q, std::string& why) {
  const J& in = q["input"];
  if (in["kind"].s != "state") { why = "not a state query"; return nullptr; }
  const J& s = q["select"];
  if (q["output"]["events"].s == "expired") { why = "expired-events output"; return nullptr; }
  auto ex = std::make_unique<NfaExec>();
  ex->app = &app;
  ex->qi = qi;
  ex->path = 2;
  NTable& t = ex->tab;
  std::memset(&t, 0, sizeof(t));
  t.seq = in["type"].s == "SEQUENCE";
  t.nslots = (int)in["slots"].size();
  if (t.nslots > NS) { why = "too many states"; return nullptr; }
  // local streams in order of first appearance in the slots
  std::map<std::string, int> sidx;
  for (auto& sl : in["slots"].a) {
    const std::string& nm = sl["stream"].s;
    if (!sidx.count(nm)) {
      int ls = (int)ex->streams.size();
      if (ls >= NSTR) { why = "too many input streams"; return nullptr; }
      sidx[nm] = ls;
      ex->streams.push_back(app.stream_idx.at(nm));
      ex->local[app.stream_idx.at(nm)] = ls;
    }
  }
  for (int k = 0; k < t.nslots; k++) t.slotStream[k] = (int8_t)sidx.at(in["slots"][k]["stream"].s);
  for (size_t ls = 0; ls < ex->streams.size(); ls++) {
    ex->cols.emplace_back();
    const auto& ty = app.streams[ex->streams[ls]].types;
    if (ty.size() > 12) { why = "too many attributes"; return nullptr; }
    for (Ty tt : ty) { ex->cols.back().emplace_back(); ex->cols.back().back().w = tsize(tt); }
    ex->rows.push_back(0);
  }
  if (q.has("partition")) {
    ex->partitioned = true;
    for (auto& kv : q["partition"].o) {
      int as = app.stream_idx.at(kv.first);
      if (ex->local.count(as)) ex->part_attr[ex->local[as]] = (int)kv.second.as_int();
    }
    // a stream the partition does not key is broadcast to every existing instance
    // (PartitionStreamReceiver.send -> every partition key, PartitionStreamReceiver.java:275)
    for (size_t ls = 0; ls < ex->streams.size(); ls++)
      if (!ex->part_attr.count((int)ls)) ex->bcast[ls] = true;
    if (ex->part_attr.empty()) { why = "partitioned query without a keyed stream"; return nullptr; }
  }
  for (int k = 0; k < NP; k++) t.waiting[k] = -1;
  NBuilder b{t, {}, (bool)t.seq};
  std::vector<int> allPre;
  int root;
  try {
    root = b.parse(in["element"], -1, allPre, true, sidx);
  } catch (CompileError& e) {
    why = e.what();
    return nullptr;
  }
  t.nproc = b.np;
  t.partitioned = ex->partitioned;
  if (ex->partitioned) {
    const auto& pa = *ex->part_attr.begin();
    ex->key_ty = app.streams[ex->streams[pa.first]].types.at(pa.second);
  }
  if (!in["within"].null()) {
    t.within = in["within"].as_int();
    std::vector<int> ids;
    for (int p : allPre) if (t.p[p].isStart) ids.push_back(t.p[p].stateId);
    t.nstart = (int)ids.size();
    for (size_t k = 0; k < ids.size(); k++) t.startIds[k] = (int8_t)ids[k];
  } else {
    t.within = -1;
  }
  t.p[b.ins[root].first].thisLast = (int8_t)b.ins[root].last;
  b.sel_last(root);
  std::vector<int> init, reset, update;
  b.orders(root, init, reset, update);
  b.resets(root, reset);
  b.updates(root, update);
  t.nall = (int8_t)allPre.size();
  for (size_t k = 0; k < allPre.size(); k++) t.allPre[k] = (int8_t)allPre[k];
  t.ninit = (int8_t)init.size();
  for (size_t k = 0; k < init.size(); k++) t.initOrder[k] = (int8_t)init[k];
  t.nreset = (int8_t)reset.size();
  for (size_t k = 0; k < reset.size(); k++) t.resetOrder[k] = (int8_t)reset[k];
  t.nupdate = (int8_t)update.size();
  for (size_t k = 0; k < update.size(); k++) t.updateOrder[k] = (int8_t)update[k];
  std::vector<std::vector<int>> nexts(ex->streams.size());
  b.setup(root, nexts, sidx);
  t.nstreams = (int)ex->streams.size();
  for (size_t ls = 0; ls < nexts.size(); ls++) {
    t.nnext[ls] = t.nfor[ls] = (int8_t)nexts[ls].size();
    t.multi[ls] = nexts[ls].size() > 1;
    for (size_t k = 0; k < nexts[ls].size(); k++) t.nexts[ls][k] = t.forStream[ls][k] = (int8_t)nexts[ls][k];
  }
  // bytecode: filters (index = processor) then select programs
  auto intern = [&](const std::string& str) { return app.intern(str); };
  auto sm = [&](int slot, int chain) -> int {
    if (slot < 0 || slot >= t.nslots || chain < -8 || chain > 7) return -1;
    return slot * 16 + (chain + 8);
  };
  try {
    ex->progs.resize(t.nproc);
    for (int p = 0; p < t.nproc; p++) {
      const J* f = b.filters[p];
      if (f && f->size() > 0) { compile_filters(ex->progs[p], *f, sm, intern); t.p[p].filter = (int16_t)p; }
    }
    std::vector<const J*> dev;   // expressions the device projects per match
    if (!build_selector(s, q, false, ex->selspec, dev, intern, why)) return nullptr;
    if (dev.size() > 64) { why = "selector reads more than 64 values"; return nullptr; }
    for (const J* e : dev) {
      Prog p;
      compile_expr(p, *e, sm, intern);
      ex->progs.push_back(p);
    }
    t.nsel = (int)dev.size();
  } catch (CompileError& e) {
    why = e.what();
    return nullptr;
  }
  ex->nsel = t.nsel;
  ex->selspec.partitioned = ex->partitioned;
  if (ex->partitioned) {
    std::string pw;
    ex->purge = purge_of(app, q, pw);
    if (!pw.empty()) { why = pw; return nullptr; }
    if (ex->purge) {
      // a purged key continues as a new lane: exact when nothing reaches the old lane afterwards
      if (t.nabs > 0) { why = "@purge with absent states (Scheduler timers of cleaned keys)"; return nullptr; }
      for (size_t ls = 0; ls < ex->streams.size(); ls++)
        if (ex->bcast[ls]) { why = "@purge with a broadcast stream (partitionKeys membership)"; return nullptr; }
      for (auto& kv : q["partition"].o)
        if (!ex->local.count(app.stream_idx.at(kv.first))) { why = "@purge with a partition stream the query does not read"; return nullptr; }
    }
  }
  if (ex->selspec.active) ex->selector = std::make_unique<SelectorStage>(ex->selspec, &app.strings);
  if (const char* e = getenv("SG_NFA_SE_CAP")) ex->se_cap = std::max(8, atoi(e));
  if (const char* e = getenv("SG_NFA_ND_CAP")) ex->nd_cap = std::max(8, atoi(e));
  if (const char* e = getenv("SG_NFA_LIST_CAP")) ex->list_cap = std::max(8, atoi(e));
  ex->in_streams = ex->streams;
  ex->build_prefilter();
  return ex;
}

}  // namespace sg
