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
#include <cstring>
#include <functional>
#include <unordered_map>

#include "runtime.hpp"

namespace sg {

constexpr int NP = 12;        // max processors
constexpr int NS = 10;        // max slots
constexpr int NSTR = 4;       // max input streams per query
constexpr int NFA_B = 64;     // lanes per workgroup

enum { K_STREAM = 0, K_COUNT = 1, K_LOGICAL = 2, K_ABSENT = 3 };
constexpr int NTQ = 32;       // pending deadlines per absent processor and lane

struct NProc {
  int8_t kind, stateId, isStart, withinEvery;
  int8_t thisLast, partner, isAnd, hasNext;
  int8_t nextPre, nextEveryPre, callbackPre, partnerPost;
  int16_t filter;
  int16_t pad;
  int32_t minCount, maxCount;
};

struct NTable {
  int32_t nproc, nslots, seq, nstart;
  int64_t within;
  int8_t startIds[NS];
  int8_t nall, ninit, nreset, nupdate;
  int8_t allPre[NP], initOrder[NP], resetOrder[NP], updateOrder[NP];
  int32_t nstreams;
  int8_t nnext[NSTR], nfor[NSTR], multi[NSTR];
  int8_t nexts[NSTR][NP], forStream[NSTR][NP];
  int8_t slotStream[NS];
  NProc p[NP];
  int32_t nsel;
  int64_t waiting[NP];     // absent: waitingTime (`for T`), else -1
  int8_t nabs;             // absent processors, in Scheduler creation order
  int8_t absOrder[NP];
};

struct NCols {
  const uint8_t* col[NSTR][12];
  int32_t w[NSTR][12];
};

struct NState {          // SoA pools, element x of lane l at [x * L + l]
  int64_t L;
  int32_t se_cap, nd_cap, list_cap;
  int32_t* se_slot;      // [se_cap * NS]
  int64_t* se_ts;        // [se_cap]
  int8_t* se_type;       // [se_cap]
  int32_t* se_ref;       // [se_cap]
  int32_t* se_free;      // [se_cap] free stack
  int32_t* se_top;       // [1]
  int32_t* nd_ev;        // [nd_cap]
  int32_t* nd_next;
  int32_t* nd_ref;
  int32_t* nd_free;
  int32_t* nd_top;
  int32_t* pend;         // [NP * list_cap]
  int32_t* npend;        // [NP]
  int32_t* nev;          // [NP * list_cap]
  int32_t* nnev;         // [NP]
  uint32_t* flags;       // [NP] bit0 stateChanged, bit1 initialized, bit2 success, bit3 startStateReset, bit4 returned(post)
  int32_t* created;      // [1]
  int32_t* err;          // [1]
  int32_t* ret;          // [list_cap] StateEvents returned by one processAndReturn (selected after the walk)
  int64_t* lst;          // [NP] absent: lastScheduledTime
  int64_t* tq;           // [NP * NTQ] absent: pending Scheduler deadlines (sorted ascending)
  int32_t* ntq;          // [NP]
};

struct NArgs {
  const int64_t* ev_ts;
  const int8_t* ev_stream;   // local stream index per event
  const int32_t* ev_row;     // row in that stream's columns
  const int32_t* lane_off;   // CSR over lanes of this flush
  const int32_t* lane_ev;
  const int32_t* lane_id;    // pool lane of CSR entry
  int32_t nl;
  // Scheduler ticks: lane_ev entries < 0 are ticks -(k+1)
  const int64_t* tick_now;   // [k] app clock the tick moved to
  const int32_t* tick_ev;    // [k] index of the next event (records fired by the tick sort before it)
  int64_t start_now;         // app clock at start (partitionCreated of absent start states)
  // output
  int64_t* rec_ts;           // output event timestamp (StateEvent ts)
  int32_t* rec_tick;         // tick that fired the record, -1 for event-driven ones
  uint64_t* rec_key;
  int64_t* rec_val;
  uint8_t* rec_nul;
  uint32_t* nrec;
  int64_t rec_cap;
};

enum { F_CHANGED = 1, F_INIT = 2, F_SUCCESS = 4, F_RESET = 8, F_RET = 16, F_INACTIVE = 32 };
enum { E_SE = 1, E_ND = 2, E_LIST = 4, E_REC = 8 };

struct Lane {
  const NTable& t;
  const NState& s;
  const NCols& c;
  const NArgs& a;
  const Prog* progs;
  int64_t l;
  int32_t cur_ev;
  int32_t holder;
  int32_t sub;
  int32_t tick;        // tick being processed (-1: an event)
  int64_t now;         // app clock (TimestampGenerator.currentTime)

  __device__ int32_t& SS(int se, int k) const { return s.se_slot[((int64_t)se * NS + k) * s.L + l]; }
  __device__ int64_t& STS(int se) const { return s.se_ts[(int64_t)se * s.L + l]; }
  __device__ int8_t& STY(int se) const { return s.se_type[(int64_t)se * s.L + l]; }
  __device__ int32_t& SREF(int se) const { return s.se_ref[(int64_t)se * s.L + l]; }
  __device__ int32_t& NEV(int nd) const { return s.nd_ev[(int64_t)nd * s.L + l]; }
  __device__ int32_t& NNX(int nd) const { return s.nd_next[(int64_t)nd * s.L + l]; }
  __device__ int32_t& NREF(int nd) const { return s.nd_ref[(int64_t)nd * s.L + l]; }
  __device__ int32_t& PEND(int p, int k) const { return s.pend[((int64_t)p * s.list_cap + k) * s.L + l]; }
  __device__ int32_t& NPEND(int p) const { return s.npend[(int64_t)p * s.L + l]; }
  __device__ int32_t& NEW(int p, int k) const { return s.nev[((int64_t)p * s.list_cap + k) * s.L + l]; }
  __device__ int32_t& NNEW(int p) const { return s.nnev[(int64_t)p * s.L + l]; }
  __device__ uint32_t& FL(int p) const { return s.flags[(int64_t)p * s.L + l]; }
  __device__ int64_t& LST(int p) const { return s.lst[(int64_t)p * s.L + l]; }
  __device__ int64_t& TQ(int p, int k) const { return s.tq[((int64_t)p * NTQ + k) * s.L + l]; }
  __device__ int32_t& NTQA(int p) const { return s.ntq[(int64_t)p * s.L + l]; }
  // Scheduler.notifyAt: a TreeMultimap of deadlines (ascending, duplicates kept)
  __device__ void notify_at(int p, int64_t t2) const {
    int n = NTQA(p);
    if (n >= NTQ) { fail(E_LIST); return; }
    int q = n;
    while (q > 0 && TQ(p, q - 1) > t2) { TQ(p, q) = TQ(p, q - 1); q--; }
    TQ(p, q) = t2;
    NTQA(p) = n + 1;
  }
  __device__ bool flag(int p, uint32_t f) const { return (FL(p) & f) != 0; }
  __device__ void setf(int p, uint32_t f, bool v) const { if (v) FL(p) |= f; else FL(p) &= ~f; }
  __device__ void fail(int e) const { s.err[l] |= e; }
  __device__ bool bad() const { return s.err[l] != 0; }

  // ---- node (StreamEvent) pool ----
  __device__ int nd_alloc(int ev) const {
    int& top = s.nd_top[l];
    if (top <= 0) { fail(E_ND); return -1; }
    int nd = s.nd_free[(int64_t)(--top) * s.L + l];
    NEV(nd) = ev; NNX(nd) = -1; NREF(nd) = 0;
    return nd;
  }
  __device__ void nd_inc(int nd) const { if (nd >= 0) NREF(nd)++; }
  __device__ void nd_dec(int nd) const {
    while (nd >= 0) {
      if (--NREF(nd) > 0) return;
      int nx = NNX(nd);
      int& top = s.nd_top[l];
      s.nd_free[(int64_t)(top++) * s.L + l] = nd;
      nd = nx;          // the freed node's `next` reference goes away too
    }
  }
  __device__ int64_t nd_ts(int nd) const { return a.ev_ts[NEV(nd)]; }

  // ---- StateEvent pool ----
  __device__ int se_alloc() const {
    int& top = s.se_top[l];
    if (top <= 0) { fail(E_SE); return -1; }
    int se = s.se_free[(int64_t)(--top) * s.L + l];
    for (int k = 0; k < t.nslots; k++) SS(se, k) = -1;
    STS(se) = -1; STY(se) = 0; SREF(se) = 0;
    return se;
  }
  __device__ void se_inc(int se) const { SREF(se)++; }
  __device__ void se_dec(int se) const {
    if (--SREF(se) > 0) return;
    for (int k = 0; k < t.nslots; k++) { nd_dec(SS(se, k)); SS(se, k) = -1; }
    int& top = s.se_top[l];
    s.se_free[(int64_t)(top++) * s.L + l] = se;
  }
  __device__ void set_slot(int se, int k, int nd) const {   // StateEvent.setEvent
    int old = SS(se, k);
    nd_inc(nd);
    SS(se, k) = nd;
    nd_dec(old);
  }
  __device__ int clone(int se) const {                       // StateEventCloner.copyStateEvent (shallow)
    int c2 = se_alloc();
    if (c2 < 0) return -1;
    for (int k = 0; k < t.nslots; k++) { int nd = SS(se, k); nd_inc(nd); SS(c2, k) = nd; }
    STS(c2) = STS(se); STY(c2) = STY(se);
    return c2;
  }

  // ---- lists ----
  __device__ void push_new(int p, int se) const {
    int& n = NNEW(p);
    if (n >= s.list_cap) { fail(E_LIST); return; }
    NEW(p, n++) = se;
    se_inc(se);
  }
  __device__ void clear_new(int p) const {
    for (int k = 0; k < NNEW(p); k++) se_dec(NEW(p, k));
    NNEW(p) = 0;
  }
  __device__ void clear_pend(int p) const {
    for (int k = 0; k < NPEND(p); k++) se_dec(PEND(p, k));
    NPEND(p) = 0;
  }
  // updateState: stable sort newAndEvery by ts (-1 last), append to pending
  __device__ void move_new_to_pending(int p) const {
    int n = NNEW(p);
    for (int k = 1; k < n; k++) {
      int v = NEW(p, k);
      int64_t tv = STS(v);
      int q = k - 1;
      while (q >= 0) {
        int64_t tq = STS(NEW(p, q));
        bool gt = (tq == -1) ? (tv != -1) : (tv != -1 && tq > tv);
        if (!gt) break;
        NEW(p, q + 1) = NEW(p, q);
        q--;
      }
      NEW(p, q + 1) = v;
    }
    int& np = NPEND(p);
    if (np + n > s.list_cap) { fail(E_LIST); return; }
    for (int k = 0; k < n; k++) PEND(p, np++) = NEW(p, k);   // references move
    NNEW(p) = 0;
  }

  // ---- chains (StateEvent.getStreamEvent(int[]) :138-182) ----
  __device__ int chain_at(int head, int idx) const {
    if (head < 0) return -1;
    int e = head;
    if (idx >= 0) {
      for (int k = 1; k <= idx; k++) { e = NNX(e); if (e < 0) return -1; }
      return e;
    }
    if (idx == -1) { while (NNX(e) >= 0) e = NNX(e); return e; }
    if (idx == -2) {
      if (NNX(e) < 0) return -1;
      while (NNX(NNX(e)) >= 0) e = NNX(e);
      return e;
    }
    int len = 0;
    for (int x = e; x >= 0; x = NNX(x)) len++;
    int k = len + idx;
    if (k < 0) return -1;
    for (int q = 0; q < k; q++) e = NNX(e);
    return e;
  }

  // loader for the bytecode: slot id = slot * 16 + (chain + 8)
  struct Ld {
    const Lane* ln;
    int se;
    __device__ bool load(int code, int attr, int64_t& v) const {
      int slot = code >> 4, chain = (code & 15) - 8;
      int nd = ln->chain_at(ln->SS(se, slot), chain);
      if (nd < 0) return false;
      int ev = ln->NEV(nd);
      int st = ln->t.slotStream[slot];
      int row = ln->a.ev_row[ev];
      const uint8_t* col = ln->c.col[st][attr];
      v = ln->c.w[st][attr] == 8 ? ((const int64_t*)col)[row] : (int64_t)((const int32_t*)col)[row];
      return true;
    }
  };

  __device__ bool filter_ok(int p, int se, int64_t* rf) const {
    int f = t.p[p].filter;
    if (f < 0) return true;
    Ld ld{this, se};
    return run_pred(progs[f], ld, rf, NFA_B);
  }

  // ---- processors (mirrors oracle/siddhi_oracle.cpp Pre / Post) ----
  __device__ void init(int p) const {
    const NProc& P = t.p[p];
    if (P.isStart && (!flag(p, F_INIT) || P.nextEveryPre >= 0 ||
                      (t.seq && P.nextPre >= 0 && t.p[P.nextPre].kind == K_ABSENT))) {
      int se = se_alloc();
      if (se < 0) return;
      se_inc(se);
      add_state(p, se);
      se_dec(se);
      setf(p, F_INIT, true);
    }
  }

  __device__ void add_state(int p, int se) const {
    const NProc& P = t.p[p];
    if (P.kind == K_ABSENT) {            // AbsentStreamPreStateProcessor.addState (:78-100)
      if (flag(p, F_INACTIVE)) return;
      if (t.seq) clear_new(p);
      push_new(p, se);
      if (!P.isStart) { LST(p) = STS(se) + t.waiting[p]; notify_at(p, LST(p)); }
      return;
    }
    if (P.kind == K_LOGICAL) {          // LogicalPreStateProcessor.addState (:43-62)
      if (P.isStart || t.seq) {
        if (NNEW(p) == 0) push_new(p, se);
        if (NNEW(P.partner) == 0) push_new(P.partner, se);
      } else {
        push_new(p, se);
        push_new(P.partner, se);
      }
      return;
    }
    if (t.seq) { if (NNEW(p) == 0) push_new(p, se); }
    else push_new(p, se);
    if (P.kind == K_COUNT && P.minCount == 0 && SS(se, P.stateId) < 0) min_count_reached(p, se);  // :126-134
  }

  __device__ void add_every_state(int p, int se) const {
    const NProc& P = t.p[p];
    int c2 = clone(se);
    if (c2 < 0) return;
    STY(c2) = 0;
    for (int k = P.stateId; k < t.nslots; k++) set_slot(c2, k, -1);
    se_inc(c2);
    push_new(p, c2);
    if (P.kind == K_LOGICAL) {
      set_slot(c2, t.p[P.partner].stateId, -1);
      push_new(P.partner, c2);
    }
    if (P.kind == K_ABSENT) { LST(p) = STS(se) + t.waiting[p]; notify_at(p, LST(p)); }
    se_dec(c2);
  }

  __device__ void reset_state(int p) const {
    const NProc& P = t.p[p];
    if (P.kind == K_LOGICAL) {
      if (!P.isAnd || NPEND(p) == NPEND(P.partner)) {
        clear_pend(p);
        clear_pend(P.partner);
        if (P.isStart && NNEW(p) == 0) {
          if (t.seq && P.nextEveryPre < 0 && P.nextPre >= 0 && NPEND(P.nextPre) != 0) return;
          init(p);
        }
      }
      return;
    }
    clear_pend(p);
    if (P.isStart && NNEW(p) == 0) {
      if (t.seq && P.nextEveryPre < 0 && P.nextPre >= 0 && NPEND(P.nextPre) != 0) return;
      init(p);
    }
  }

  __device__ void update_state(int p) const {
    const NProc& P = t.p[p];
    if (P.kind == K_COUNT && flag(p, F_RESET)) { setf(p, F_RESET, false); init(p); }
    move_new_to_pending(p);
    if (P.kind == K_LOGICAL) move_new_to_pending(P.partner);
  }

  __device__ bool is_expired(int se, int64_t ts) const {
    if (t.within < 0) return false;
    for (int k = 0; k < t.nstart; k++) {
      int nd = SS(se, t.startIds[k]);
      if (nd >= 0) {
        int64_t d = nd_ts(nd) - ts;
        if (d < 0) d = -d;
        if (d > t.within) return true;
      }
    }
    return false;
  }

  __device__ void expire_events(int p, int64_t ts) const {   // StreamPreStateProcessor.expireEvents (:325-361)
    int expired = -1;
    int n = NPEND(p), r = 0;
    while (r < n) {
      int se = PEND(p, r);
      if (!is_expired(se, ts)) break;
      if (STY(se) != 1) { STY(se) = 1; if (expired >= 0) se_dec(expired); expired = se; se_inc(se); }
      se_dec(se);
      r++;
    }
    if (r) { for (int k = r; k < n; k++) PEND(p, k - r) = PEND(p, k); NPEND(p) = n - r; }
    int m = NNEW(p), w = 0;
    for (int k = 0; k < m; k++) {
      int se = NEW(p, k);
      if (is_expired(se, ts)) {
        if (STY(se) != 1) { STY(se) = 1; if (expired >= 0) se_dec(expired); expired = se; se_inc(se); }
        se_dec(se);
      } else {
        NEW(p, w++) = se;
      }
    }
    NNEW(p) = w;
    if (expired >= 0) {
      int we = t.p[p].withinEvery;
      if (we >= 0) { add_every_state(we, expired); update_state(we); }
      se_dec(expired);
    }
  }

  __device__ void count_start_state_reset(int p) const {     // CountPreStateProcessor.startStateReset
    // the reference re-invokes startStateReset on countPost.thisStatePreProcessor (itself) when its own
    // post carries a callback; setting the flag once is the observable effect
    setf(p, F_RESET, true);
  }

  __device__ void stream_post(int p, int se) const {         // StreamPostStateProcessor.process (:64-83)
    const NProc& P = t.p[p];
    setf(p, F_CHANGED, true);
    STS(se) = nd_ts(SS(se, P.stateId));
    if (P.hasNext) setf(p, F_RET, true);
    if (P.nextPre >= 0) add_state(P.nextPre, se);
    if (P.nextEveryPre >= 0) add_every_state(P.nextEveryPre, se);
    if (P.callbackPre >= 0) count_start_state_reset(P.callbackPre);
  }

  __device__ void min_count_reached(int p, int se) const {   // CountPostStateProcessor (:67-79)
    const NProc& P = t.p[p];
    if (P.hasNext) { setf(p, F_CHANGED, true); setf(p, F_RET, true); }
    if (P.nextPre >= 0) add_state(P.nextPre, se);
    if (P.nextEveryPre >= 0) add_every_state(P.nextEveryPre, se);
  }

  __device__ void post_process(int p, int se) const {
    const NProc& P = t.p[p];
    if (P.kind == K_ABSENT) {                                 // AbsentStreamPostStateProcessor.process (:36-56)
      setf(p, F_CHANGED, true);
      const int64_t ts = nd_ts(SS(se, P.stateId));
      STS(se) = ts;
      setf(p, F_RET, true);
      if (P.isStart && P.nextEveryPre == p) add_every_state(p, se);
      LST(p) = ts + t.waiting[p];                            // updateLastArrivalTime
      notify_at(p, LST(p));
      return;
    }
    if (P.kind == K_COUNT) {                                  // CountPostStateProcessor.process (:39-65)
      int e = SS(se, P.stateId);
      int n = 1;
      while (NNX(e) >= 0) { n++; e = NNX(e); }
      setf(p, F_SUCCESS, true);
      STS(se) = nd_ts(e);
      if (n >= P.minCount) {
        if (t.seq) {
          if (P.nextPre >= 0) add_state(P.nextPre, se);
          if (n != P.maxCount) add_state(p, se);
        } else if (n == P.minCount) {
          min_count_reached(p, se);
        }
        if (n == P.maxCount) setf(p, F_CHANGED, true);
      }
      return;
    }
    if (P.kind == K_LOGICAL) {                                // LogicalPostStateProcessor.process (:59-87)
      if (P.isAnd) {
        if (SS(se, t.p[P.partner].stateId) >= 0) stream_post(p, se);
        else setf(p, F_CHANGED, true);
      } else {
        stream_post(p, se);
        int pp = P.partnerPost;
        if (t.p[pp].hasNext && P.thisLast == pp) setf(pp, F_RET, true);
      }
      return;
    }
    stream_post(p, se);
  }

  __device__ void process_chain(int p, int se, int64_t* rf) const {
    setf(p, F_CHANGED, false);
    if (filter_ok(p, se, rf)) post_process(p, se);
  }

  __device__ void emit(int se, int64_t* rf) const {
    uint32_t k = atomicAdd(a.nrec, 1u);
    if ((int64_t)k >= a.rec_cap) { fail(E_REC); return; }
    // order: trigger event, then tick records (holder field 0) before the event's holders (1 + k)
    const uint32_t hf = tick >= 0 ? 0u : (uint32_t)((holder + 1) & 15);
    a.rec_key[k] = ((uint64_t)(uint32_t)cur_ev << 24) | ((uint64_t)hf << 20) | (uint64_t)(sub & 0xfffff);
    a.rec_ts[k] = STS(se);
    a.rec_tick[k] = tick;
    Ld ld{this, se};
    for (int q = 0; q < t.nsel; q++) {
      int64_t v = 0;
      bool isnull = false;
      run(progs[t.nproc + q], ld, v, isnull, rf, NFA_B);
      a.rec_val[(int64_t)k * t.nsel + q] = v;
      a.rec_nul[(int64_t)k * t.nsel + q] = isnull;
    }
  }

  // processAndReturn (StreamPreStateProcessor :363-403 / Count :53-95 / Logical :128-165);
  // matches are projected immediately (QuerySelector.process on the returned StateEvent)
  __device__ void process_and_return(int p, int ev, int64_t* rf) {
    const NProc& P = t.p[p];
    const int last = P.thisLast;
    int nret = 0;
    if (P.kind == K_ABSENT && flag(p, F_INACTIVE)) return;   // AbsentStreamPreStateProcessor.processAndReturn
    int n = NPEND(p), w = 0;
    for (int r = 0; r < n; r++) {
      if (bad()) { NPEND(p) = w; return; }
      int se = PEND(p, r);
      if (P.kind == K_COUNT) {
        if ((P.stateId + 1 < t.nslots && SS(se, P.stateId + 1) >= 0) ||
            (P.stateId + 2 < t.nslots && SS(se, P.stateId + 2) >= 0)) {
          se_dec(se);
          continue;
        }
        int nd = nd_alloc(ev);
        if (nd < 0) return;
        int h = SS(se, P.stateId);
        if (h < 0) set_slot(se, P.stateId, nd);
        else { while (NNX(h) >= 0) h = NNX(h); NNX(h) = nd; nd_inc(nd); }
        setf(p, F_SUCCESS, false);
        se_inc(se);
        process_chain(p, se, rf);
        if (flag(last, F_RET)) { setf(last, F_RET, false); ret_push(se, nret); }
        bool removed = false;
        if (flag(p, F_CHANGED)) removed = true;
        if (!flag(p, F_SUCCESS)) {
          // StateEvent.removeLastEvent (:224-236)
          int hh = SS(se, P.stateId);
          if (hh >= 0) {
            if (NNX(hh) < 0) set_slot(se, P.stateId, -1);
            else {
              int x = hh;
              while (NNX(NNX(x)) >= 0) x = NNX(x);
              int victim = NNX(x);
              NNX(x) = -1;
              nd_dec(victim);
            }
          }
          if (t.seq) removed = true;
        }
        if (removed) se_dec(se);
        else PEND(p, w++) = se;
        se_dec(se);
        continue;
      }
      if (P.kind == K_LOGICAL && !P.isAnd && SS(se, t.p[P.partner].stateId) >= 0) {
        se_dec(se);
        continue;
      }
      int nd = nd_alloc(ev);
      if (nd < 0) return;
      set_slot(se, P.stateId, nd);
      se_inc(se);
      process_chain(p, se, rf);
      if (flag(last, F_RET)) {
        setf(last, F_RET, false);
        if (P.kind != K_ABSENT) ret_push(se, nret);     // an absent state returns nothing on arrivals
      }
      if (flag(p, F_CHANGED)) {
        se_dec(se);                                    // removed from pending
      } else {
        set_slot(se, P.stateId, -1);
        if (t.seq) {
          if (P.kind == K_ABSENT) PEND(p, w++) = se;   // removeOnNoStateChange is false for absent
          else se_dec(se);
          if ((P.kind == K_STREAM || P.kind == K_ABSENT) && P.callbackPre >= 0) count_start_state_reset(P.callbackPre);
        } else {
          PEND(p, w++) = se;
        }
      }
      se_dec(se);
    }
    // entries appended to pending during the walk cannot happen (only newAndEvery grows)
    NPEND(p) = w;
    // QuerySelector.process on each returned StateEvent, after the walk (StateMultiProcessStreamReceiver :47-68)
    for (int k = 0; k < nret; k++) {
      int se = s.ret[(int64_t)k * s.L + l];
      emit(se, rf);
      sub++;
      se_dec(se);
    }
  }

  __device__ void ret_push(int se, int& nret) const {
    if (nret >= s.list_cap) { fail(E_LIST); return; }
    s.ret[(int64_t)(nret++) * s.L + l] = se;
    se_inc(se);
  }

  // AbsentStreamPreStateProcessor.process(TIMER chunk) (:150-227) for deadline `ct`
  __device__ void absent_timer(int p, int64_t ct, int64_t* rf) {
    const NProc& P = t.p[p];
    if (flag(p, F_INACTIVE)) return;
    bool initialize = P.isStart && NNEW(p) == 0 && NPEND(p) == 0;
    if (initialize && t.seq && P.nextEveryPre < 0 && LST(p) > 0) initialize = false;
    if (initialize) {
      int se = se_alloc();
      if (se < 0) return;
      se_inc(se);
      add_state(p, se);
      se_dec(se);
    } else if (t.seq && NNEW(p) != 0) {
      reset_state(p);
    }
    update_state(p);
    int nret = 0;
    int n = NPEND(p), w = 0;
    for (int r = 0; r < n; r++) {
      int se = PEND(p, r);
      if (is_expired(se, ct)) {
        if (P.withinEvery >= 0 && P.nextEveryPre != p && P.nextEveryPre >= 0) add_every_state(P.nextEveryPre, se);
        se_dec(se);
        continue;
      }
      const int64_t sts = STS(se);
      if ((sts == -1 && ct >= LST(p)) || (sts != -1 && ct >= sts + t.waiting[p])) {
        STS(se) = ct;
        ret_push(se, nret);
        se_dec(se);
        continue;
      }
      PEND(p, w++) = se;
    }
    NPEND(p) = w;
    if (P.withinEvery >= 0) update_state(P.withinEvery);
    const bool notProcessed = nret == 0;
    for (int k = 0; k < nret; k++) {            // sendEvent
      int se = s.ret[(int64_t)k * s.L + l];
      if (P.hasNext) { emit(se, rf); sub++; }
      if (P.nextPre >= 0) add_state(P.nextPre, se);
      if (P.nextEveryPre >= 0) add_every_state(P.nextEveryPre, se);
      else if (P.isStart) setf(p, F_INACTIVE, true);
      if (P.callbackPre >= 0) count_start_state_reset(P.callbackPre);
      se_dec(se);
    }
    if (now > t.waiting[p] + ct) LST(p) = now + t.waiting[p];
    if (notProcessed && LST(p) < ct) { LST(p) = ct + t.waiting[p]; notify_at(p, LST(p)); }
  }

  // Scheduler.onTimeChange for this instance: every absent processor's due deadlines, earliest first
  __device__ void fire_timers(int64_t* rf) {
    for (int k = 0; k < t.nabs; k++) {
      const int p = t.absOrder[k];
      while (NTQA(p) > 0 && TQ(p, 0) <= now) {
        const int64_t tt = TQ(p, 0);
        const int n = NTQA(p);
        for (int q = 1; q < n; q++) TQ(p, q - 1) = TQ(p, q);
        NTQA(p) = n - 1;
        absent_timer(p, tt, rf);
        if (bad()) return;
      }
    }
  }

  __device__ void on_tick(int k, int64_t* rf) {
    now = a.tick_now[k];
    tick = k;
    cur_ev = a.tick_ev[k];
    sub = 0;
    fire_timers(rf);
    tick = -1;
  }

  // PartitionRuntime.initPartition / App.start: inner.init(), then partitionCreated of absent start states
  __device__ void create(int64_t* rf) {
    (void)rf;
    for (int k = 0; k < t.ninit; k++) init(t.initOrder[k]);
    for (int k = 0; k < t.nabs; k++) {
      const int p = t.absOrder[k];
      if (t.p[p].isStart && !flag(p, F_INACTIVE)) { LST(p) = a.start_now + t.waiting[p]; notify_at(p, LST(p)); }
    }
  }

  __device__ void on_event(int ev, int64_t* rf) {
    const int st = a.ev_stream[ev];
    const int64_t ts = a.ev_ts[ev];
    cur_ev = ev;
    sub = 0;
    for (int k = 0; k < t.nall; k++) expire_events(t.allPre[k], ts);
    if (t.seq) {
      for (int k = 0; k < t.nreset; k++) reset_state(t.resetOrder[k]);
      for (int k = 0; k < t.nupdate; k++) update_state(t.updateOrder[k]);
    } else if (t.multi[st]) {
      for (int k = 0; k < t.nfor[st]; k++) update_state(t.forStream[st][k]);
    } else if (t.nfor[st] > 0) {
      update_state(t.forStream[st][0]);
    }
    if (t.multi[st]) {
      for (int k = t.nnext[st] - 1; k >= 0; k--) {
        holder = k;
        sub = 0;
        process_and_return(t.nexts[st][k], ev, rf);
      }
    } else {
      holder = 0;
      process_and_return(t.nexts[st][0], ev, rf);
    }
  }
};

__global__ void __launch_bounds__(NFA_B) k_nfa_lanes(NArgs a, NState s, const NTable* __restrict__ tab,
                                                     const NCols* __restrict__ cols, const Prog* __restrict__ progs) {
  __shared__ int64_t rf[MAX_REG * NFA_B];
  int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.nl) return;
  Lane ln{*tab, s, *cols, a, progs, (int64_t)a.lane_id[q], 0, 0, 0, -1, a.start_now};
  int64_t* myrf = rf + threadIdx.x;
  if (!s.created[ln.l]) {
    // first event of the partition key: PartitionRuntimeImpl.initPartition -> innerStateRuntime.init()
    s.created[ln.l] = 1;
    ln.create(myrf);
  }
  for (int e = a.lane_off[q]; e < a.lane_off[q + 1]; e++) {
    if (ln.bad()) return;
    const int x = a.lane_ev[e];
    if (x < 0) ln.on_tick(-x - 1, myrf);
    else ln.on_event(x, myrf);
  }
}

__global__ void k_nfa_pool_init(NState s, int64_t lane0, int64_t nlanes) {
  int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nlanes) return;
  int64_t l = lane0 + q;
  for (int k = 0; k < s.se_cap; k++) s.se_free[(int64_t)k * s.L + l] = s.se_cap - 1 - k;
  for (int k = 0; k < s.nd_cap; k++) s.nd_free[(int64_t)k * s.L + l] = s.nd_cap - 1 - k;
  s.se_top[l] = s.se_cap;
  s.nd_top[l] = s.nd_cap;
  for (int p = 0; p < NP; p++) {
    s.npend[(int64_t)p * s.L + l] = 0; s.nnev[(int64_t)p * s.L + l] = 0; s.flags[(int64_t)p * s.L + l] = 0;
    s.lst[(int64_t)p * s.L + l] = 0; s.ntq[(int64_t)p * s.L + l] = 0;
  }
  s.created[l] = 0;
  s.err[l] = 0;
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
      if (pre < 0) pre = new_proc(k == "absent" ? K_ABSENT : K_STREAM);
      else if (k == "absent") throw CompileError("logical absent states are not lowered to the device NFA yet");
      NProc& P = t.p[pre];
      if (k == "absent") {
        t.waiting[pre] = el["wait"].as_int();
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
        if (el["a"]["k"].s != "stream" || el["b"]["k"].s != "stream")
        throw CompileError("logical absent states are not lowered to the device NFA yet");
      int p1 = new_proc(K_LOGICAL), p2 = new_proc(K_LOGICAL);
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

struct NfaExec : Exec {
  NTable tab;
  std::vector<Prog> progs;          // [filters per processor (index = proc)] + [select programs]
  std::vector<int> streams;         // local stream index -> app stream
  std::map<int, int> local;         // app stream -> local
  std::map<int, int> part_attr;     // local stream -> partition attribute (partitioned)
  bool partitioned = false;
  int nsel = 0;
  // capacities
  int se_cap = 64, nd_cap = 256, list_cap = 48;
  int64_t L = 0;                    // lanes allocated
  std::unordered_map<int64_t, int> key_lane;
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
  std::vector<int64_t> h_seq;            // arrival seq per event
  std::vector<int8_t> h_stream;
  std::vector<int> h_lane;               // lane per event
  int64_t flushed = 0;                   // events [0, flushed) processed
  DBuf<NTable> d_tab;
  DBuf<NCols> d_cols;
  DBuf<Prog> d_progs;
  DBuf<int32_t> lane_off, lane_ev, lane_id;
  DBuf<uint64_t> rec_key;
  DBuf<int64_t> rec_val, rec_ts;
  DBuf<int32_t> rec_tick;
  DBuf<uint8_t> rec_nul;
  DBuf<uint32_t> counter;
  DBuf<int64_t> lst, tq, d_tick_now;
  DBuf<int32_t> ntq, d_tick_ev;
  // Scheduler ticks (absent states): app clock, next event index, arrival seq
  std::vector<int64_t> tick_now, tick_seq;
  std::vector<int32_t> tick_ev;
  size_t ticks_flushed = 0;
  int64_t start_now = 0;
  hipEvent_t e0 = nullptr, e1 = nullptr;

  void on_tick(int64_t now, int64_t seq, int stream, int64_t k) override {
    if (tab.nabs == 0) return;
    tick_now.push_back(now);
    tick_seq.push_back(seq);
    tick_ev.push_back((int32_t)(n + (local.count(stream) ? k : 0)));
  }
  void start(int64_t now) override { start_now = now; }

  ~NfaExec() override {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
  }

  NState state() {
    NState s;
    s.L = L; s.se_cap = se_cap; s.nd_cap = nd_cap; s.list_cap = list_cap;
    s.se_slot = se_slot.p; s.se_ts = se_ts.p; s.se_type = se_type.p; s.se_ref = se_ref.p; s.se_free = se_free.p;
    s.se_top = se_top.p; s.nd_ev = nd_ev.p; s.nd_next = nd_next.p; s.nd_ref = nd_ref.p; s.nd_free = nd_free.p;
    s.nd_top = nd_top.p; s.pend = pend.p; s.npend = npend.p; s.nev = nev.p; s.nnev = nnev.p; s.flags = flags.p;
    s.created = created.p; s.err = err.p; s.ret = ret.p;
    s.lst = lst.p; s.tq = tq.p; s.ntq = ntq.p;
    return s;
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
    regrow(se_slot, (int64_t)se_cap * NS); regrow(se_ts, se_cap); regrow(se_type, se_cap); regrow(se_ref, se_cap);
    regrow(se_free, se_cap); regrow(se_top, 1); regrow(nd_ev, nd_cap); regrow(nd_next, nd_cap); regrow(nd_ref, nd_cap);
    regrow(nd_free, nd_cap); regrow(nd_top, 1); regrow(pend, (int64_t)NP * list_cap); regrow(npend, NP);
    regrow(nev, (int64_t)NP * list_cap); regrow(nnev, NP); regrow(flags, NP); regrow(created, 1); regrow(err, 1);
    regrow(ret, list_cap); regrow(lst, NP); regrow(tq, (int64_t)NP * NTQ); regrow(ntq, NP);
    L = nl;
    NState ns = state();
    hipLaunchKernelGGL(k_nfa_pool_init, dim3((unsigned)((nl - oldL + 255) / 256)), dim3(256), 0, s, ns, oldL, nl - oldL);
    SG_HIP(hipGetLastError());
    SG_HIP(hipStreamSynchronize(s));
  }

  void push(const HostBatch& b) override {
    auto it = local.find(b.stream);
    if (it == local.end()) return;
    int ls = it->second;
    hipStream_t s = app->stream;
    int64_t need = n + b.n;
    ev_ts.reserve(need, true, s, n);
    ev_stream.reserve(need, true, s, n);
    ev_row.reserve(need, true, s, n);
    auto& cs = cols[ls];
    for (auto& c : cs) c.b.reserve((rows[ls] + b.n) * c.w, true, s, rows[ls] * c.w);
    std::vector<int8_t> st(b.n, (int8_t)ls);
    std::vector<int32_t> rw(b.n);
    for (int64_t k = 0; k < b.n; k++) rw[k] = (int32_t)(rows[ls] + k);
    SG_HIP(hipMemcpyAsync(ev_ts.p + n, b.ts.data(), b.n * 8, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(ev_stream.p + n, st.data(), b.n, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(ev_row.p + n, rw.data(), b.n * 4, hipMemcpyHostToDevice, s));
    for (size_t k = 0; k < cs.size(); k++)
      SG_HIP(hipMemcpyAsync(cs[k].b.p + rows[ls] * cs[k].w, b.cols[k].data(), b.n * cs[k].w, hipMemcpyHostToDevice, s));
    SG_HIP(hipStreamSynchronize(s));
    // lanes: partition key -> lane (first appearance creates the instance)
    for (int64_t k = 0; k < b.n; k++) {
      int lane = 0;
      if (partitioned) {
        auto pa = part_attr.find(ls);
        if (pa == part_attr.end()) throw Error(-2, "stream not named in `partition with` (broadcast) is not lowered to the device NFA");
        const auto& col = b.cols[pa->second];
        int w = (int)col.size() / (int)b.n;
        int64_t key = w == 8 ? ((const int64_t*)col.data())[k] : (int64_t)((const int32_t*)col.data())[k];
        auto f = key_lane.find(key);
        if (f == key_lane.end()) { lane = (int)key_lane.size(); key_lane[key] = lane; }
        else lane = f->second;
      }
      h_lane.push_back(lane);
      h_seq.push_back(b.seq0 + k);
      h_stream.push_back((int8_t)ls);
    }
    rows[ls] += b.n;
    n += b.n;
  }

  void reset() override {
    n = 0; flushed = 0; h_seq.clear(); h_stream.clear(); h_lane.clear(); key_lane.clear();
    tick_now.clear(); tick_seq.clear(); tick_ev.clear(); ticks_flushed = 0;
    for (auto& r : rows) r = 0;
    if (L) {
      NState ns = state();
      hipLaunchKernelGGL(k_nfa_pool_init, dim3((unsigned)((L + 255) / 256)), dim3(256), 0, app->stream, ns, 0, L);
      SG_HIP(hipStreamSynchronize(app->stream));
    }
  }

  void flush(std::vector<Callback>& out, bool materialise, hipStream_t s) override {
    last_matches = 0;
    if (n <= flushed && ticks_flushed == tick_now.size()) return;
    int64_t lanes_needed = partitioned ? (int64_t)key_lane.size() : 1;
    grow_lanes(lanes_needed, s);
    // CSR of this flush's events per lane (arrival order inside each lane)
    std::vector<int> order;
    std::vector<int32_t> cnt(lanes_needed, 0);
    for (int64_t e = flushed; e < n; e++) cnt[h_lane[e]]++;
    std::vector<int32_t> lid, off(1, 0);
    std::vector<int32_t> start(lanes_needed, -1);
    for (int64_t l = 0; l < lanes_needed; l++)
      if (cnt[l]) { start[l] = (int32_t)lid.size(); lid.push_back((int32_t)l); off.push_back(off.back() + cnt[l]); }
    std::vector<int32_t> evs(n - flushed), fill(lid.size(), 0);
    for (int64_t e = flushed; e < n; e++) {
      int q = start[h_lane[e]];
      evs[off[q] + fill[q]++] = (int32_t)e;
    }
    // unpartitioned query with absent states: the lane's timeline interleaves the Scheduler ticks
    // (tick k before event tick_ev[k]); entries < 0 are ticks -(k+1), k relative to this flush
    const size_t t0 = ticks_flushed, nt = tick_now.size() - t0;
    if (nt > 0) {
      std::vector<int32_t> tl;
      tl.reserve(evs.size() + nt);
      size_t k = 0;
      for (int32_t e : evs) {
        while (k < nt && tick_ev[t0 + k] <= e) { tl.push_back(-(int32_t)k - 1); k++; }
        tl.push_back(e);
      }
      while (k < nt) { tl.push_back(-(int32_t)k - 1); k++; }
      evs.swap(tl);
      if (lid.empty()) { lid.push_back(0); off.push_back(0); }
      off[1] = (int32_t)evs.size();
      d_tick_now.reserve(nt); d_tick_ev.reserve(nt);
      SG_HIP(hipMemcpyAsync(d_tick_now.p, tick_now.data() + t0, nt * 8, hipMemcpyHostToDevice, s));
      SG_HIP(hipMemcpyAsync(d_tick_ev.p, tick_ev.data() + t0, nt * 4, hipMemcpyHostToDevice, s));
    }
    int nl = (int)lid.size();
    lane_off.reserve(nl + 1); lane_ev.reserve(evs.size()); lane_id.reserve(nl);
    SG_HIP(hipMemcpyAsync(lane_off.p, off.data(), (nl + 1) * 4, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(lane_ev.p, evs.data(), evs.size() * 4, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(lane_id.p, lid.data(), nl * 4, hipMemcpyHostToDevice, s));
    NCols hc;
    std::memset(&hc, 0, sizeof(hc));
    for (size_t ls = 0; ls < streams.size(); ls++)
      for (size_t k = 0; k < cols[ls].size(); k++) { hc.col[ls][k] = cols[ls][k].b.p; hc.w[ls][k] = cols[ls][k].w; }
    d_cols.reserve(1);
    d_tab.reserve(1);
    d_progs.reserve(progs.size());
    SG_HIP(hipMemcpyAsync(d_cols.p, &hc, sizeof(hc), hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(d_tab.p, &tab, sizeof(tab), hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(d_progs.p, progs.data(), progs.size() * sizeof(Prog), hipMemcpyHostToDevice, s));
    int64_t cap = std::max<int64_t>(1024, (n - flushed + (int64_t)nt) * 4);
    rec_key.reserve(cap); rec_val.reserve((size_t)cap * std::max(nsel, 1)); rec_nul.reserve((size_t)cap * std::max(nsel, 1));
    rec_ts.reserve(cap); rec_tick.reserve(cap);
    counter.reserve(1);
    SG_HIP(hipMemsetAsync(counter.p, 0, 4, s));
    NArgs a;
    a.ev_ts = ev_ts.p; a.ev_stream = ev_stream.p; a.ev_row = ev_row.p;
    a.lane_off = lane_off.p; a.lane_ev = lane_ev.p; a.lane_id = lane_id.p; a.nl = nl;
    a.rec_key = rec_key.p; a.rec_val = rec_val.p; a.rec_nul = rec_nul.p; a.nrec = counter.p; a.rec_cap = cap;
    a.rec_ts = rec_ts.p; a.rec_tick = rec_tick.p;
    a.tick_now = d_tick_now.p; a.tick_ev = d_tick_ev.p; a.start_now = start_now;
    if (!e0) { SG_HIP(hipEventCreate(&e0)); SG_HIP(hipEventCreate(&e1)); }
    SG_HIP(hipEventRecord(e0, s));
    // lanes per workgroup (<= NFA_B; the register file keeps its NFA_B stride).  A lane is a long chain
    // of dependent pool accesses, so with few lanes (e.g. K = 1000 partition keys) they are spread over
    // as many waves (CUs) as possible: halve the workgroup until there are >= 1024 of them or 4 lanes
    // per wave (measured on config 3, K = 1000: 64 lanes/wave 722 ms, 16: 643 ms, 4: 572 ms)
    int tpb = NFA_B;
    while (tpb > 4 && (nl + tpb - 1) / tpb < 1024) tpb /= 2;
    if (const char* x = getenv("SG_NFA_TPB")) tpb = std::max(1, std::min(NFA_B, atoi(x)));   // tuning hook
    hipLaunchKernelGGL(k_nfa_lanes, dim3((unsigned)((nl + tpb - 1) / tpb)), dim3(tpb), 0, s, a, state(), d_tab.p,
                       d_cols.p, d_progs.p);
    SG_HIP(hipGetLastError());
    SG_HIP(hipEventRecord(e1, s));
    uint32_t nrec = 0;
    SG_HIP(hipMemcpyAsync(&nrec, counter.p, 4, hipMemcpyDeviceToHost, s));
    std::vector<int32_t> errs(lanes_needed);
    SG_HIP(hipMemcpyAsync(errs.data(), err.p, lanes_needed * 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    float ms = 0;
    SG_HIP(hipEventElapsedTime(&ms, e0, e1));
    kernel_ms["k_nfa_lanes"] = ms;
    for (int64_t l = 0; l < lanes_needed; l++)
      if (errs[l]) throw Error(-4, "device NFA pool overflow (code " + std::to_string(errs[l]) +
                                   "): raise SG_NFA_SE_CAP / SG_NFA_ND_CAP / SG_NFA_LIST_CAP");
    flushed = n;
    ticks_flushed = tick_now.size();
    last_matches = nrec;
    if (!materialise || nrec == 0) return;
    std::vector<uint64_t> key(nrec);
    std::vector<int64_t> val((size_t)nrec * nsel);
    std::vector<uint8_t> nul((size_t)nrec * nsel);
    SG_HIP(hipMemcpyAsync(key.data(), rec_key.p, nrec * 8, hipMemcpyDeviceToHost, s));
    if (nsel) {
      SG_HIP(hipMemcpyAsync(val.data(), rec_val.p, val.size() * 8, hipMemcpyDeviceToHost, s));
      SG_HIP(hipMemcpyAsync(nul.data(), rec_nul.p, nul.size(), hipMemcpyDeviceToHost, s));
    }
    std::vector<int64_t> hts(n), rts(nrec);
    std::vector<int32_t> rtick(nrec);
    SG_HIP(hipMemcpyAsync(hts.data(), ev_ts.p, n * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(rts.data(), rec_ts.p, nrec * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(rtick.data(), rec_tick.p, nrec * 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    std::vector<uint32_t> idx(nrec);
    for (uint32_t k = 0; k < nrec; k++) idx[k] = k;
    // stable: records of one lane with equal keys (several ticks before one event) keep emission order
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) { return key[x] < key[y]; });
    // callbacks: one per (event, holder) for a multi receiver; one per match for a single receiver
    Callback* cur = nullptr;
    uint64_t curgrp = ~0ull;
    for (uint32_t k : idx) {
      uint64_t kk = key[k];
      int ev = (int)(kk >> 24);
      uint64_t grp = kk >> 20;
      const bool timer = rtick[k] >= 0;              // fired by a Scheduler tick: one callback per match
      bool multi = !timer && tab.multi[h_stream[ev]] != 0;
      if (!multi || cur == nullptr || grp != curgrp) {
        out.emplace_back();
        cur = &out.back();
        cur->seq = timer ? tick_seq[t0 + rtick[k]] : h_seq[ev];
        cur->order = qi;
        cur->kind = 0;
        cur->target = qi;
        curgrp = timer ? ~0ull : grp;
      }
      OutEvent oe;
      oe.ts = timer ? rts[k] : hts[ev];
      oe.raw.assign(val.begin() + (size_t)k * nsel, val.begin() + (size_t)(k + 1) * nsel);
      oe.nul.assign(nul.begin() + (size_t)k * nsel, nul.begin() + (size_t)(k + 1) * nsel);
      cur->ts = oe.ts;
      cur->ev.push_back(std::move(oe));
    }
  }
};

static bool has_agg(const J& e) {
  if (e["op"].s == "agg" || e["op"].s == "multivar") return true;
  for (const char* c : {"a", "b"})
    if (e.has(c) && has_agg(e[c])) return true;
  return false;
}

std::unique_ptr<Exec> make_nfa(App& app, int qi, const J& q, std::string& why) {
  const J& in = q["input"];
  if (in["kind"].s != "state") { why = "not a state query"; return nullptr; }
  const J& s = q["select"];
  if (s["group_by"].size() || !s["having"].null() || s["order_by"].size() || !s["limit"].null() ||
      !s["offset"].null()) {
    why = "selector with group-by / having / order / limit is not lowered to the device NFA yet";
    return nullptr;
  }
  for (size_t k = 0; k < s["attrs"].size(); k++)
    if (has_agg(s["attrs"][k]["e"])) { why = "aggregators in a pattern selector are not lowered yet"; return nullptr; }
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
    // a stream the partition does not key is broadcast to every instance (Java HashSet order):
    // not lowered to the lanes yet
    for (size_t ls = 0; ls < ex->streams.size(); ls++)
      if (!ex->part_attr.count((int)ls)) { why = "stream not named in `partition with` (broadcast)"; return nullptr; }
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
  if (t.nabs > 0 && ex->partitioned) {
    // Scheduler.onTimeChange keeps ONE partition instance per distinct deadline (SchedulerState.compareTo
    // == 0, Scheduler.java:364-366): instances sharing a deadline fire at different ticks, which couples
    // the partition lanes
    why = "absent states in a partitioned query (the Scheduler couples partition instances)";
    return nullptr;
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
    for (size_t k = 0; k < s["attrs"].size(); k++) {
      Prog p;
      compile_expr(p, s["attrs"][k]["e"], sm, intern);
      ex->progs.push_back(p);
    }
  } catch (CompileError& e) {
    why = e.what();
    return nullptr;
  }
  t.nsel = (int)s["attrs"].size();
  ex->nsel = t.nsel;
  if (const char* e = getenv("SG_NFA_SE_CAP")) ex->se_cap = std::max(8, atoi(e));
  if (const char* e = getenv("SG_NFA_ND_CAP")) ex->nd_cap = std::max(8, atoi(e));
  if (const char* e = getenv("SG_NFA_LIST_CAP")) ex->list_cap = std::max(8, atoi(e));
  ex->in_streams = ex->streams;
  return ex;
}

}  // namespace sg
