// nfa_lane.hpp -- the NFA lane interpreter (device side of SG_PATH_NFA; see nfa.hip for the design).
//
// Compiled twice: ahead of time into libsiddhi_gfx.so (nfa.hip: k_nfa_lanes<FM>, the table, bytecode and column
// table read from LDS at run time), and per query at run time by hipRTC (nfa_rtc.hpp: the table is a constexpr
// struct and every filter / projection a generated straight-line function, so the processor dispatch and the
// bytecode interpreter fold away).  One source, so both evaluate the reference semantics identically.
#pragma once
#ifndef SG_RTC
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>

#include "expr.hpp"

namespace sg {


constexpr int NP = 12;        // max processors
constexpr int NS = 10;        // max slots
constexpr int NSTR = 4;       // max input streams per query
constexpr int NFA_B = 64;     // lanes per workgroup
constexpr int NFA_CA = 4;           // attributes of the current event held in registers (Lane::cached)

enum { K_STREAM = 0, K_COUNT = 1, K_LOGICAL = 2, K_ABSENT = 3 };
// Feature mask of a lowered table: the lane interpreter is instantiated per mask so that the processor
// kinds and modes a query never uses are compiled out (smaller code, fewer registers and spills).
enum { FM_ABS = 1, FM_LOG = 2, FM_CNT = 4, FM_SEQ = 8, FM_PAT = 16, FM_WITHIN = 32, FM_ALL = 63 };
constexpr int NTQ = 64;       // distinct-run slots of one Scheduler queue per lane (run-length: repeats of the
                              // tail deadline only bump its count)

struct NProc {
  int8_t kind, stateId, isStart, withinEvery;
  int8_t thisLast, partner, isAnd, hasNext;
  int8_t nextPre, nextEveryPre, callbackPre, partnerPost;
  int16_t filter;
  int8_t absLog;     // K_LOGICAL element that is `not S[f] [for T]` (AbsentLogicalPreStateProcessor)
  int8_t absIdx;     // index in absOrder (the Scheduler's listener rank), -1 if no scheduler
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
  int8_t partitioned;      // pre-states live in PartitionSyncStateHolder (canDestroy drops them)
};

struct NCols {
  const uint8_t* col[NSTR][12];
  int32_t w[NSTR][12];
  const uint8_t* nul[NSTR];   // [row * na + attr] null flags (nullptr: the stream never carried a null)
  int32_t na[NSTR];
};

#define SG_AS3 __attribute__((address_space(3)))
// pointer into the lane pools: LDS (ds_* instructions) when the pools are staged there, else global
template <class T, bool IL> struct PoolPtr { using type = T*; };
template <class T> struct PoolPtr<T, true> { using type = SG_AS3 T*; };
template <class T, bool IL> using pptr = typename PoolPtr<T, IL>::type;
using RF = SG_AS3 int64_t*;   // the interpreter's register file (always LDS)

template <bool IL>
struct NStateT {         // SoA pools, element x of lane l at [x * L + l]
  int64_t L;
  int32_t se_cap, nd_cap, list_cap;
  int32_t ns = NS, np = NP;       // slots per StateEvent, processors (the LDS copy is sized to the query)
  pptr<int32_t, IL> se_slot;      // [se_cap * NS]
  pptr<int64_t, IL> se_ts;        // [se_cap]
  pptr<int8_t, IL> se_type;       // [se_cap]
  pptr<int32_t, IL> se_ref;       // [se_cap]
  pptr<int32_t, IL> se_free;      // [se_cap] free stack
  pptr<int32_t, IL> se_top;       // [1]
  pptr<int32_t, IL> nd_ev;        // [nd_cap]
  pptr<int32_t, IL> nd_next;
  pptr<int32_t, IL> nd_ref;
  pptr<int32_t, IL> nd_free;
  pptr<int32_t, IL> nd_top;
  pptr<int32_t, IL> pend;         // [NP * list_cap]
  pptr<int32_t, IL> npend;        // [NP]
  pptr<int32_t, IL> nev;          // [NP * list_cap]
  pptr<int32_t, IL> nnev;         // [NP]
  pptr<uint32_t, IL> flags;       // [NP] bit0 stateChanged, bit1 initialized, bit2 success, bit3 startStateReset, bit4 returned(post)
  pptr<int32_t, IL> created;      // [1]
  pptr<int32_t, IL> err;          // [1]
  pptr<int32_t, IL> ret;          // [list_cap] StateEvents returned by one processAndReturn (selected after the walk)
  pptr<int64_t, IL> lst;          // [NP] absent: lastScheduledTime; logical absent: lastArrivalTime
  int32_t nq;            // Scheduler queues per lane (absent processors, >= 1)
  pptr<int64_t, IL> tq;           // [nq * NTQ] the Scheduler's toNotifyQueue (FIFO, Scheduler.java:332), a ring of
  pptr<int32_t, IL> tqc;          // [nq * NTQ]   runs (deadline, multiplicity)
  pptr<int32_t, IL> ntq;          // [nq] runs queued
  pptr<int32_t, IL> tqh;          // [nq] ring head
};
using NState = NStateT<false>;
using NStateL = NStateT<true>;

// Scheduler bookkeeping of partitioned absent queries (see NfaExec::flush): every firing is logged so
// the host can find instances that share a deadline at one tick (SchedulerState.compareTo == 0 keeps
// only one per deadline, Scheduler.java:77-97); in exact mode every notifyAt is logged too, for the
// host's replay of the key -> SchedulerState HashMap whose iteration order picks the one that fires.
struct FireRec {
  int32_t tau;           // tick
  int32_t lane;
  int64_t head;          // the deadline the instance was collected under (toNotifyQueue.peek())
  int8_t sched;          // absOrder index
  int8_t empty_after;    // queue empty after the firing (the state is dropped at returnAllStates)
  int16_t pad;
  int32_t task;          // speculative task that logged it (-1: a run from the true state)
};
struct OpRec {           // one Scheduler.notifyAt, ordered (x, phase, tau, firing sched, head, sub)
  int32_t x;             // event index the op precedes (tick phase) or belongs to (event phase)
  int32_t tau;           // tick (tick phase), else -1
  int64_t head;          // firing head deadline (tick phase)
  int32_t sub;
  int32_t lane;
  int8_t phase;          // 0 = inside a tick's onTimeChange, 1 = event processing
  int8_t kfire;          // scheduler firing (tick phase)
  int8_t ktarget;        // scheduler notified
  int8_t pad[5];
};

// One CSR entry's event packed lane-major (k_nfa_pack, NfaExec::run_lanes): everything nfa_run_lane reads per
// event, so that a lane streams its events from consecutive 64-B records instead of chasing lane_ev -> rank /
// stream / row / ts / skip -> columns through scattered sectors of the arrival-ordered arrays (a single-lane wave
// fetched a whole sector per 4-B field).
struct NEvRec {
  int64_t ts;
  int64_t v[NFA_CA];         // the first NFA_CA attributes (Lane::prefetch_attrs), 0 past the stream's arity
  int32_t x;                 // event index
  int32_t rank;              // arrival rank
  int32_t row;               // row in its stream's columns
  int32_t tub;               // tick_ub[rank - tub0] (-1: no index, or the rank outside it)
  int8_t stream;
  int8_t cok;                // the stream never carried a null: v[] is the attribute values
  uint16_t skip;             // ev_skip
  int32_t pad;
};
static_assert(sizeof(NEvRec) == 64, "one record per 64-B sector");

struct NArgs {
  const int64_t* ev_ts;
  const int8_t* ev_stream;   // local stream index per event
  const int32_t* ev_row;     // row in that stream's columns
  const int32_t* ev_rank;    // position of each event in arrival order (seq, then push order): the
                             // order ticks and records are placed in (chained inputs arrive out of
                             // array order)
  const int32_t* lane_off;   // CSR over lanes of this flush
  const int32_t* lane_ev;
  const int32_t* lane_id;    // pool lane of CSR entry
  int32_t nl;
  // Scheduler ticks: lane_ev entries < 0 are ticks -(k+1)
  const int64_t* tick_now;   // [k] app clock the tick moved to
  const int32_t* tick_ev;    // [k] index of the next event (records fired by the tick sort before it)
  int32_t ntick;             // ticks of this flush (absent queries)
  int32_t tick_base;         // absolute index of tick 0 in rec_tick (0: records keep launch-relative ticks)
  // tick indexes (k_nfa_tick_index; null: binary search): tick_ub[x - tub0] = first tick whose next event
  // is after arrival rank x, tick_lb[t - tlb0] = first tick whose clock reaches t (dense over the ticks'
  // clock range).  They replace two binary searches over all ticks per event and per due deadline.
  const int32_t* tick_ub;
  int64_t tub0, ntub;
  const int32_t* tick_lb;
  int64_t tlb0, ntlb;
  int64_t start_now;         // app clock at start (partitionCreated of absent start states)
  const int64_t* ev_now;     // app clock each event is processed at (partitionCreated of a new key)
  // partitioned absent scheduling
  const int32_t* def_off;    // per CSR lane: deferred (tick, scheduler) firings [def_off[q], def_off[q+1])
  const int64_t* def_key;    // tick << 8 | absOrder index, ascending
  FireRec* fire;
  uint32_t* nfire;
  int64_t fire_cap;
  OpRec* ops;                // exact mode only (else null)
  uint32_t* nops;
  int64_t ops_cap;
  // output
  int64_t* rec_ts;           // output event timestamp (StateEvent ts)
  int32_t* rec_tick;         // tick that fired the record, -1 for event-driven ones
  int64_t* rec_dl;           // tick records: the firing instance's head deadline (TreeMultimap key)
  int8_t* rec_sched;         // tick records: absOrder index of the firing Scheduler
  uint64_t* rec_key;
  int32_t* rec_lane;         // pool lane (partition instance) of the record
  int64_t* rec_val;
  uint8_t* rec_nul;
  uint32_t* nrec;
  int64_t rec_cap;
  int32_t* rec_task;         // speculative segments: task of each record (-1: a task run from the true state)
  unsigned long long* probe; // SG_NFA_PROBE builds: wall-clock ticks per phase, summed over lanes (else null)
  // per event: bit k set when processor nexts[stream][k] takes the event and its filter, which reads only the
  // event itself, fails -- its processAndReturn would change nothing (k_nfa_prefilter); null: none skipped
  const uint16_t* ev_skip;
  const NEvRec* lane_rec;    // per CSR entry (parallel to lane_ev): the packed events (null: read through lane_ev)
  // 1: one lane per wavefront (few instances: NfaExec::launch_lanes).  Every thread of the wave runs the lane's
  // state machine redundantly on the same data (uniform control flow, one LDS pool); the wave's threads split the
  // list-parallel steps (within expiry: one __ballot per 64 entries and a popc-rank compaction) and the pool
  // staging, and the wave's first thread alone bumps the shared counters and writes records and logs.
  int32_t wide;
  int32_t pad_wide;
};

// Speculative time segments (NfaExec::run_spec).  A key whose timeline is long is cut into segments run in
// parallel; segment g > 0 starts from a freshly created instance, replays the H events before its segment
// without emitting (warm-up), and records its state there and at its end in canonical form.  Its records are
// kept only if the state after the warm-up equals the state segment g-1 ended with (then every later event
// is processed exactly as the sequential run would: the lane interpreter is deterministic in its state and
// the events); otherwise the key is re-run from its last verified state.
constexpr int SG_CANON = 384;    // ints of one canonical state (a longer state never verifies: re-run)
struct NSpec {
  const int32_t* w0;         // per task: first lane_ev entry of its warm-up (== e0 without one)
  const int32_t* e0;         // first entry whose records are emitted
  const int32_t* e1;         // end
  const int32_t* pool;       // >= 0: lane of the key's own pools (g); < 0: scratch lane -(x + 1) of gs (fresh)
  const uint8_t* tail;       // the key's last segment: it also runs the Scheduler ticks after its last event
  NState gs;
  int32_t* canon;            // [task][2][SG_CANON + 1]: length, then the state (after warm-up, at the end)
  int32_t* cmap;             // [task][2 * se_cap + nd_cap] scratch for the renaming (the larger caps)
  int32_t ntask;
  int32_t q0;                // first task of this launch (key tasks and scratch tasks launch separately)
  int32_t cmap_stride;
  int32_t blocked;           // gs is laid out in blocks of 64 lanes (nfa_block_view): one wave's pools are contiguous
  int32_t pad_blocked;
};

// Lane block b of a pool set laid out in blocks of 64 lanes (NfaExec::carve, blocked): every array [block][element][64]
// instead of [element][lane], so that the pools of the 64 lanes one wave runs are one contiguous region (a few pages)
// instead of each element of each lane in a different page of a flat array L lanes wide.  The view is an NState of
// L = 64 whose arrays start at the block; arrays of one element per lane (tops, created, err) coincide in both layouts.
__host__ __device__ inline NState nfa_block_view(const NState& g, int64_t b) {
  NState v = g;
  v.L = 64;
  const int64_t o = b * 64;
  v.se_slot = g.se_slot + o * g.se_cap * NS; v.se_ts = g.se_ts + o * g.se_cap; v.se_type = g.se_type + o * g.se_cap;
  v.se_ref = g.se_ref + o * g.se_cap; v.se_free = g.se_free + o * g.se_cap; v.se_top = g.se_top + o;
  v.nd_ev = g.nd_ev + o * g.nd_cap; v.nd_next = g.nd_next + o * g.nd_cap; v.nd_ref = g.nd_ref + o * g.nd_cap;
  v.nd_free = g.nd_free + o * g.nd_cap; v.nd_top = g.nd_top + o;
  v.pend = g.pend + o * NP * g.list_cap; v.npend = g.npend + o * NP; v.nev = g.nev + o * NP * g.list_cap;
  v.nnev = g.nnev + o * NP; v.flags = g.flags + o * NP; v.created = g.created + o; v.err = g.err + o;
  v.ret = g.ret + o * g.list_cap; v.lst = g.lst + o * NP;
  v.tq = g.tq + o * g.nq * NTQ; v.tqc = g.tqc + o * g.nq * NTQ; v.ntq = g.ntq + o * g.nq; v.tqh = g.tqh + o * g.nq;
  return v;
}

enum { F_CHANGED = 1, F_INIT = 2, F_SUCCESS = 4, F_RESET = 8, F_RET = 16, F_INACTIVE = 32 };
enum { E_SE = 1, E_ND = 2, E_LIST = 4, E_REC = 8, E_LOG = 16, E_SPIN = 32, E_TQ = 64, E_RET = 128 };
constexpr int MAX_DRAIN = 1 << 20;   // timer events one instance may drain at one tick before failing

// Table policy of the ahead-of-time interpreter: the table, the bytecode and the column table are read from LDS at
// every step.  The run-time compiled kernels (nfa_rtc.cpp) pass a generated policy instead: `Tab` is an empty struct
// whose static constexpr members mirror NTable (so every table read folds), and `pred` / `val` are straight-line
// functions generated from the query's bytecode.
// a stream index known at compile time (the compiled kernels' per-stream event bodies)
template <int V> struct SIc { constexpr operator int() const { return V; } };

struct LdsTab {
  static constexpr bool compiled = false;
  using Tab = const SG_AS3 NTable&;
  template <class LD> __device__ static bool pred(int, const LD&) { return true; }
  template <class LD> __device__ static void val(int, const LD&, int64_t&, bool&) {}
};

// SG_UNROLL: loops over the table's processor lists, fully unrolled in the compiled kernels (constant bounds there:
// every processor index becomes a constant, so register-resident per-processor state is never indexed dynamically)
#ifdef SG_RTC
#define SG_UNROLL _Pragma("unroll")
#else
#define SG_UNROLL
#endif

// kRtcRegs: the compiled kernels keep each processor's list lengths and flags in registers (Lane::regs_load); the
// generator recompiles with SG_RTC_NOREG (kept in the pools) when a kernel would index them dynamically (scratch)
#if defined(SG_RTC) && !defined(SG_RTC_NOREG)
constexpr bool kRtcRegs = true;
#else
constexpr bool kRtcRegs = false;
#endif

// SG_LI: methods the compiled kernels inline into one straight-line body (no calls, no frame in scratch)
#ifdef SG_RTC
#define SG_LI __device__ __attribute__((always_inline))
#else
#define SG_LI __device__
#endif

template <bool IL, int FM, class TP = LdsTab>
struct Lane {
  typename TP::Tab t;
  const NStateT<IL> s;
  const SG_AS3 NCols& c;
  const NArgs& a;
  const SG_AS3 Prog* progs;
  int64_t l;
  int32_t cur_ev;
  int32_t holder;
  int32_t sub;
  int32_t tick;        // tick being processed (-1: an event)
  int64_t now;         // app clock (TimestampGenerator.currentTime)
  int32_t fsched;      // tick phase: absOrder index of the Scheduler firing (-1 outside)
  int64_t fhead;       // tick phase: head deadline it fires under
  mutable int32_t opsub;  // notifyAt counter (exact-mode op log)
  int32_t q;           // CSR lane (deferral list)
  int32_t dpos;        // next deferral entry
  bool mute = false;   // speculative warm-up: events are processed, records are not written
  int rfs = NFA_B;     // stride of the LDS register file (lanes of the workgroup)
  int32_t task = -1;   // speculative task of the records (-1: not speculative)
  bool wide = false;   // one lane per wavefront (NArgs::wide): every thread of the wave runs this lane
  int32_t wl = 0;      // the thread's index in its wavefront (wide mode)
  mutable int64_t nd_h = INT64_MIN;   // next_deadline() cache (INT64_MIN: stale)
  mutable int32_t nd_k = -1;          // run_ticks: first tick reaching nd_h (-1: stale), and its next event
  mutable int32_t nd_tev = 0;
#ifdef SG_NFA_PROBE
  unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // ticks, expire, update, process, loads, events
#define SG_PROBE(k, stmt) do { const unsigned long long t0_ = wall_clock64(); stmt; pt[k] += wall_clock64() - t0_; } while (0)
#else
#define SG_PROBE(k, stmt) do { stmt; } while (0)
#endif
  // the event being processed: its first NFA_CA attributes, loaded one step ahead of their use (nfa_run_lane)
  int32_t cx = -1;
  bool cok = false;
  int64_t cv0 = 0, cv1 = 0, cv2 = 0, cv3 = 0;
  SG_LI bool cached(int ev, int attr, int64_t& v) const {
    if (ev != cx || !cok || attr >= NFA_CA) return false;
    v = attr == 0 ? cv0 : attr == 1 ? cv1 : attr == 2 ? cv2 : cv3;
    return true;
  }
  // issue the loads of event x's first attributes (stream st, row): no wait here, the first read waits
  SG_LI void prefetch_attrs(int x, int st, int row) {
    cx = x;
    cok = !c.nul[st];
    const int na = c.na[st];
    auto ld = [&](int k) -> int64_t {
      if (k >= na) return 0;
      const uint8_t* col = c.col[st][k];
      return c.w[st][k] == 8 ? ((const int64_t*)col)[row] : (int64_t)((const int32_t*)col)[row];
    };
    cv0 = ld(0); cv1 = ld(1); cv2 = ld(2); cv3 = ld(3);
  }


  // compile-time feature mask (FM_*): kinds and modes the query's table never uses fold away
  SG_LI bool seq() const {
    if constexpr ((FM & FM_SEQ) && (FM & FM_PAT)) return t.seq != 0;
    else return (FM & FM_SEQ) != 0;
  }
  template <class PR> SG_LI static bool isA(const PR& P) { return (FM & FM_ABS) && P.kind == K_ABSENT; }
  template <class PR> SG_LI static bool isL(const PR& P) { return (FM & FM_LOG) && P.kind == K_LOGICAL; }
  template <class PR> SG_LI static bool isC(const PR& P) { return (FM & FM_CNT) && P.kind == K_COUNT; }
  template <class PR> SG_LI static bool aLog(const PR& P) { return (FM & FM_ABS) && (FM & FM_LOG) && P.absLog; }
  SG_LI int32_t ntick() const { return (FM & FM_ABS) ? a.ntick : 0; }

  SG_LI auto& SS(int se, int k) const { return s.se_slot[((int64_t)se * s.ns + k) * s.L + l]; }
  SG_LI auto& STS(int se) const { return s.se_ts[(int64_t)se * s.L + l]; }
  SG_LI auto& STY(int se) const { return s.se_type[(int64_t)se * s.L + l]; }
  SG_LI auto& SREF(int se) const { return s.se_ref[(int64_t)se * s.L + l]; }
  SG_LI auto& NEV(int nd) const { return s.nd_ev[(int64_t)nd * s.L + l]; }
  SG_LI auto& NNX(int nd) const { return s.nd_next[(int64_t)nd * s.L + l]; }
  SG_LI auto& NREF(int nd) const { return s.nd_ref[(int64_t)nd * s.L + l]; }
  SG_LI auto& PEND(int p, int k) const { return s.pend[((int64_t)p * s.list_cap + k) * s.L + l]; }
  // The compiled kernels keep each processor's list lengths and flags in registers for the whole lane (every index
  // is a constant there): loaded from the pools before the lane runs, stored back after (regs_load / regs_store)
  mutable int32_t r_npend[NP] = {}, r_nnew[NP] = {};
  mutable uint32_t r_fl[NP] = {};
  SG_LI void regs_load() const {
    if constexpr (TP::compiled && kRtcRegs) {
#pragma unroll
      for (int p = 0; p < TP::Tab::nproc; p++) {
        r_npend[p] = s.npend[(int64_t)p * s.L + l];
        r_nnew[p] = s.nnev[(int64_t)p * s.L + l];
        r_fl[p] = s.flags[(int64_t)p * s.L + l];
      }
    }
  }
  SG_LI void regs_store() const {
    if constexpr (TP::compiled && kRtcRegs) {
#pragma unroll
      for (int p = 0; p < TP::Tab::nproc; p++) {
        s.npend[(int64_t)p * s.L + l] = r_npend[p];
        s.nnev[(int64_t)p * s.L + l] = r_nnew[p];
        s.flags[(int64_t)p * s.L + l] = r_fl[p];
      }
    }
  }
  SG_LI auto& NPEND(int p) const {
    if constexpr (TP::compiled && kRtcRegs) return r_npend[p];
    else return s.npend[(int64_t)p * s.L + l];
  }
  SG_LI auto& NEW(int p, int k) const { return s.nev[((int64_t)p * s.list_cap + k) * s.L + l]; }
  SG_LI auto& NNEW(int p) const {
    if constexpr (TP::compiled && kRtcRegs) return r_nnew[p];
    else return s.nnev[(int64_t)p * s.L + l];
  }
  SG_LI auto& FL(int p) const {
    if constexpr (TP::compiled && kRtcRegs) return r_fl[p];
    else return s.flags[(int64_t)p * s.L + l];
  }
  SG_LI auto& LST(int p) const { return s.lst[(int64_t)p * s.L + l]; }
  // Scheduler queue of absent processor p (ring of (deadline, count) runs, index absIdx)
  SG_LI auto& TQ(int ai, int k) const { return s.tq[((int64_t)ai * NTQ + k) * s.L + l]; }
  SG_LI auto& TQC(int ai, int k) const { return s.tqc[((int64_t)ai * NTQ + k) * s.L + l]; }
  SG_LI auto& NTQA(int ai) const { return s.ntq[(int64_t)ai * s.L + l]; }
  SG_LI auto& TQH(int ai) const { return s.tqh[(int64_t)ai * s.L + l]; }
  SG_LI bool q_empty(int p) const { return NTQA(t.p[p].absIdx) == 0; }
  SG_LI int64_t q_head(int p) const { const int ai = t.p[p].absIdx; return TQ(ai, TQH(ai)); }
  SG_LI void q_pop(int p) const {
    nd_h = INT64_MIN; nd_k = -1;
    const int ai = t.p[p].absIdx, h = TQH(ai);
    if (--TQC(ai, h) > 0) return;
    TQH(ai) = (h + 1) % NTQ;
    NTQA(ai)--;
  }
  // Scheduler.notifyAt (:113-126): append to the FIFO toNotifyQueue
  SG_LI void notify_at(int p, int64_t t2) const {
    nd_h = INT64_MIN; nd_k = -1;
    const int ai = t.p[p].absIdx;
    const int n = NTQA(ai);
    const int tail = (TQH(ai) + n - 1) % NTQ;
    if (n > 0 && TQ(ai, tail) == t2) TQC(ai, tail)++;
    else {
      if (n >= NTQ) { fail(E_TQ); return; }
      const int slot = (TQH(ai) + n) % NTQ;
      TQ(ai, slot) = t2;
      TQC(ai, slot) = 1;
      NTQA(ai) = n + 1;
    }
    if (a.ops) {                     // exact mode: PartitionSyncStateHolder.getState -> computeIfAbsent
      uint32_t k = bump(a.nops);
      if ((int64_t)k >= a.ops_cap) { fail(E_LOG); return; }
      OpRec r;
      r.x = cur_ev; r.tau = tick; r.head = fhead; r.sub = opsub++; r.lane = a.lane_id[q];
      r.phase = tick >= 0 ? 0 : 1; r.kfire = (int8_t)fsched; r.ktarget = t.p[p].absIdx;
      for (int z = 0; z < 5; z++) r.pad[z] = 0;
      if (writer()) a.ops[k] = r;
    }
  }
  // a shared counter bumped once per lane (wide mode: by the wave's first thread, the old value broadcast)
  SG_LI uint32_t bump(uint32_t* p) const {
    if (!wide) return atomicAdd(p, 1u);
    uint32_t k = 0;
    if (wl == 0) k = atomicAdd(p, 1u);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)k);
  }
  // the thread that writes the lane's records and logs (every thread of a narrow wave is its own lane)
  SG_LI bool writer() const { return !wide || wl == 0; }
  SG_LI bool flag(int p, uint32_t f) const { return (FL(p) & f) != 0; }
  SG_LI void setf(int p, uint32_t f, bool v) const { if (v) FL(p) |= f; else FL(p) &= ~f; }
  SG_LI void fail(int e) const {
    s.err[l] |= e;
    atomicOr(a.nrec + 3, (uint32_t)e);   // (the exact sweep reads this word instead of every lane's flags)
  }
  SG_LI bool bad() const { return s.err[l] != 0; }

  // ---- node (StreamEvent) pool ----
  SG_LI int nd_alloc(int ev) const {
    auto& top = s.nd_top[l];
    if (top <= 0) { fail(E_ND); return -1; }
    int nd = s.nd_free[(int64_t)(--top) * s.L + l];
    NEV(nd) = ev; NNX(nd) = -1; NREF(nd) = 0;
    return nd;
  }
  SG_LI void nd_inc(int nd) const { if (nd >= 0) NREF(nd)++; }
  SG_LI void nd_dec(int nd) const {
    while (nd >= 0) {
      if (--NREF(nd) > 0) return;
      int nx = NNX(nd);
      auto& top = s.nd_top[l];
      s.nd_free[(int64_t)(top++) * s.L + l] = nd;
      nd = nx;          // the freed node's `next` reference goes away too
    }
  }
  // a node whose event index is -1 is StreamEventFactory.newInstance(): timestamp -1, null attributes
  SG_LI int64_t nd_ts(int nd) const { const int ev = NEV(nd); return ev < 0 ? -1 : a.ev_ts[ev]; }

  // ---- StateEvent pool ----
  SG_LI int se_alloc() const {
    auto& top = s.se_top[l];
    if (top <= 0) { fail(E_SE); return -1; }
    int se = s.se_free[(int64_t)(--top) * s.L + l];
    for (int k = 0; k < t.nslots; k++) SS(se, k) = -1;
    STS(se) = -1; STY(se) = 0; SREF(se) = 0;
    return se;
  }
  SG_LI void se_inc(int se) const { SREF(se)++; }
  SG_LI void se_dec(int se) const {
    if (--SREF(se) > 0) return;
    for (int k = 0; k < t.nslots; k++) { nd_dec(SS(se, k)); SS(se, k) = -1; }
    auto& top = s.se_top[l];
    s.se_free[(int64_t)(top++) * s.L + l] = se;
  }
  SG_LI void set_slot(int se, int k, int nd) const {   // StateEvent.setEvent
    int old = SS(se, k);
    nd_inc(nd);
    SS(se, k) = nd;
    nd_dec(old);
  }
  SG_LI int clone(int se) const {                       // StateEventCloner.copyStateEvent (shallow)
    int c2 = se_alloc();
    if (c2 < 0) return -1;
    for (int k = 0; k < t.nslots; k++) { int nd = SS(se, k); nd_inc(nd); SS(c2, k) = nd; }
    STS(c2) = STS(se); STY(c2) = STY(se);
    return c2;
  }

  // ---- lists ----
  SG_LI void push_new(int p, int se) const {
    auto& n = NNEW(p);
    if (n >= s.list_cap) { fail(E_LIST); return; }
    NEW(p, n++) = se;
    se_inc(se);
  }
  SG_LI void clear_new(int p) const {
    for (int k = 0; k < NNEW(p); k++) se_dec(NEW(p, k));
    NNEW(p) = 0;
  }
  SG_LI void clear_pend(int p) const {
    for (int k = 0; k < NPEND(p); k++) se_dec(PEND(p, k));
    NPEND(p) = 0;
  }
  // updateState: stable sort newAndEvery by ts (-1 last), append to pending
  SG_LI void move_new_to_pending(int p) const {
    int n = NNEW(p);
    if (n == 0) return;
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
    auto& np = NPEND(p);
    if (np + n > s.list_cap) { fail(E_LIST); return; }
    for (int k = 0; k < n; k++) PEND(p, np++) = NEW(p, k);   // references move
    NNEW(p) = 0;
  }

  // ---- chains (StateEvent.getStreamEvent(int[]) :138-182) ----
  SG_LI int chain_at(int head, int idx) const {
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
    SG_LI bool load(int code, int attr, int64_t& v) const {
      int slot = code >> 4, chain = (code & 15) - 8;
      int nd = ln->chain_at(ln->SS(se, slot), chain);
      if (nd < 0) return false;
      int ev = ln->NEV(nd);
      if (ev < 0) return false;
      if (ln->cached(ev, attr, v)) return true;
      int st = ln->t.slotStream[slot];
      int row = ln->a.ev_row[ev];
      if (ln->c.nul[st] && ln->c.nul[st][(int64_t)row * ln->c.na[st] + attr]) return false;
      const uint8_t* col = ln->c.col[st][attr];
      v = ln->c.w[st][attr] == 8 ? ((const int64_t*)col)[row] : (int64_t)((const int32_t*)col)[row];
      return true;
    }
  };

  SG_LI bool filter_ok(int p, int se, RF rf) const {
    int f = t.p[p].filter;
    if (f < 0) return true;
    Ld ld{this, se};
    if constexpr (TP::compiled) return TP::pred(f, ld);
    else return run_pred(progs[f], ld, rf, rfs);
  }

  // ---- processors (mirrors oracle/siddhi_oracle.cpp Pre / Post) ----
  SG_LI void init(int p) const {
    const auto& P = t.p[p];
    if (P.isStart && (!flag(p, F_INIT) || P.nextEveryPre >= 0 ||
                      (seq() && P.nextPre >= 0 && isA(t.p[P.nextPre])))) {
      int se = se_alloc();
      if (se < 0) return;
      se_inc(se);
      add_state(p, se);
      se_dec(se);
      setf(p, F_INIT, true);
    }
  }

  // addState; a count state with minCount 0 passes the event on at once (CountPreStateProcessor.addState
  // :126-134 -> CountPostStateProcessor.minCountReached :67-79 -> the next state's addState).  That
  // recursion is unrolled: the chain of next states is walked in a loop, and the addEveryState calls
  // each level makes after its nested addState returns run afterwards, innermost first.
  SG_LI void add_state(int p, int se) const {
    int deferred[NP];
    int nd = 0;
    // (bounded by NP: the min-0 chain visits each processor at most once; a bound the compiled kernels unroll, so
    // that every p below is a constant there)
    SG_UNROLL
    for (int it = 0; it < NP; it++) {
      const auto& P = t.p[p];
      if (isA(P)) {            // AbsentStreamPreStateProcessor.addState (:78-100)
        if (!flag(p, F_INACTIVE)) {
          if (seq()) clear_new(p);
          push_new(p, se);
          if (!P.isStart) { LST(p) = STS(se) + t.waiting[p]; notify_at(p, LST(p)); }
        }
        break;
      }
      if (isL(P)) {          // LogicalPreStateProcessor.addState (:43-62)
        if (aLog(P) && flag(p, F_INACTIVE)) break;   // AbsentLogicalPreStateProcessor.addState (:78-99)
        if (P.isStart || seq()) {
          if (NNEW(p) == 0) push_new(p, se);
          if (NNEW(P.partner) == 0) push_new(P.partner, se);
        } else {
          push_new(p, se);
          push_new(P.partner, se);
        }
        if (aLog(P) && !P.isStart && t.waiting[p] != -1) {
          notify_at(p, STS(se) + t.waiting[p]);
          if (aLog(t.p[P.partner])) notify_at(P.partner, STS(se) + t.waiting[P.partner]);
        }
        break;
      }
      if (seq()) { if (NNEW(p) == 0) push_new(p, se); }
      else push_new(p, se);
      if (!(isC(P) && P.minCount == 0 && SS(se, P.stateId) < 0)) break;
      // min_count_reached(p, se), with its nested addState continued by the loop
      if (P.hasNext) { setf(p, F_CHANGED, true); setf(p, F_RET, true); }
      if (P.nextEveryPre >= 0 && nd < NP) deferred[nd++] = P.nextEveryPre;
      if (P.nextPre < 0) break;
      p = P.nextPre;
    }
    SG_UNROLL
    for (int k = NP - 1; k >= 0; k--)
      if (k < nd) add_every_state(deferred[k], se);
  }

  SG_LI void add_every_state(int p, int se) const {
    const auto& P = t.p[p];
    int c2 = clone(se);
    if (c2 < 0) return;
    STY(c2) = 0;
    if (aLog(P)) {                    // AbsentLogicalPreStateProcessor.addEveryState (:101-121)
      const int own = SS(c2, P.stateId);
      if (own >= 0) STS(c2) = nd_ts(own);
      set_slot(c2, P.stateId, -1);
      set_slot(c2, t.p[P.partner].stateId, -1);
      se_inc(c2);
      push_new(p, c2);
      push_new(P.partner, c2);
      se_dec(c2);
      return;
    }
    for (int k = P.stateId; k < t.nslots; k++) set_slot(c2, k, -1);
    se_inc(c2);
    push_new(p, c2);
    if (isL(P)) {
      set_slot(c2, t.p[P.partner].stateId, -1);
      push_new(P.partner, c2);
    }
    if (isA(P)) { LST(p) = STS(se) + t.waiting[p]; notify_at(p, LST(p)); }
    se_dec(c2);
  }

  SG_LI void reset_state(int p) const {
    const auto& P = t.p[p];
    if (isL(P)) {
      if (!P.isAnd || NPEND(p) == NPEND(P.partner)) {
        clear_pend(p);
        clear_pend(P.partner);
        if (P.isStart && NNEW(p) == 0) {
          if (seq() && P.nextEveryPre < 0 && P.nextPre >= 0 && NPEND(P.nextPre) != 0) return;
          init(p);
        }
      }
      return;
    }
    clear_pend(p);
    // AbsentStreamPreStateProcessor.resetState (:124-145) re-inits a start state without looking at
    // newAndEvery (StreamPreStateProcessor.resetState :287-305 requires it empty)
    if (P.isStart && (NNEW(p) == 0 || isA(P))) {
      if (seq() && P.nextEveryPre < 0 && P.nextPre >= 0 && NPEND(P.nextPre) != 0) return;
      init(p);
    }
  }

  SG_LI void update_state(int p) const {
    const auto& P = t.p[p];
    if (isC(P) && flag(p, F_RESET)) { setf(p, F_RESET, false); init(p); }
    move_new_to_pending(p);
    if (isL(P)) move_new_to_pending(P.partner);
  }

  SG_LI bool is_expired(int se, int64_t ts) const {
    if (!(FM & FM_WITHIN) || t.within < 0) return false;
    SG_UNROLL
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

  // ---- within expiry (StreamPreStateProcessor.expireEvents :325-361) ----
  // The pending list loses its expired prefix (the reference's walk stops at the first live entry); newAndEvery loses
  // every expired entry.  Expiry is evaluated as a bit mask over a chunk of entries -- in wide mode one __ballot of
  // is_expired across the wavefront, the 64 entries' slot -> node -> timestamp chains loaded in parallel; in narrow
  // mode (a wave of 64 instances) a per-thread mask over 32 entries, its loads independent of each other -- and the
  // survivors move to their popc-rank positions (wide: every thread moves its own entry).  Only the removals run one
  // by one, in list order: their refcount drops and the EXPIRED typing, whose last newly typed entry feeds withinEvery.
  SG_LI void expire_one(int se, int& expired) const {
    if (STY(se) != 1) { STY(se) = 1; if (expired >= 0) se_dec(expired); expired = se; se_inc(se); }
    se_dec(se);
  }
  // expired entries [base, base + cnt) of processor p's pending (pl) or newAndEvery list: bit j for entry base + j;
  // wide mode also returns the thread's own entry (base + wl) in v
  SG_LI uint64_t expired_mask(int p, bool pl, int base, int cnt, int64_t ts, int& v) const {
    if (wide) {
      const bool in = wl < cnt;
      v = in ? (pl ? PEND(p, base + wl) : NEW(p, base + wl)) : -1;
      return (uint64_t)__ballot(in && is_expired(v, ts));
    }
    uint64_t m = 0;
    for (int j = 0; j < cnt; j++) m |= (uint64_t)is_expired(pl ? PEND(p, base + j) : NEW(p, base + j), ts) << j;
    return m;
  }

  SG_LI void expire_events(int p, int64_t ts) const {
    if (!(FM & FM_WITHIN) || t.within < 0) return;            // no `within`: nothing ever expires
    const int ch = wide ? 64 : 32;
    int expired = -1;
    const int n = NPEND(p);
    int r = 0;                                                // the expired prefix of pending
    for (int base = 0; base < n; base += ch) {
      const int cnt = min(ch, n - base);
      int v = -1;
      const uint64_t live = ~expired_mask(p, true, base, cnt, ts, v);
      const int run = live ? min(cnt, (int)__builtin_ctzll(live)) : cnt;
      for (int j = 0; j < run; j++) expire_one(PEND(p, base + j), expired);
      r += run;
      if (run < cnt) break;
    }
    if (r) {
      const int keep = n - r;
      if (wide) {
        for (int base = 0; base < keep; base += 64) {        // each thread moves one survivor (reads before writes)
          const int k = base + wl;
          const int v = k < keep ? PEND(p, k + r) : 0;
          if (k < keep) PEND(p, k) = v;
        }
      } else {
        for (int k = 0; k < keep; k++) PEND(p, k) = PEND(p, k + r);
      }
      NPEND(p) = keep;
    }
    const int m = NNEW(p);
    int w = 0;
    for (int base = 0; base < m; base += ch) {
      const int cnt = min(ch, m - base);
      int v = -1;
      const uint64_t em = expired_mask(p, false, base, cnt, ts, v);
      for (uint64_t b = em; b; b &= b - 1) expire_one(NEW(p, base + (int)__builtin_ctzll(b)), expired);
      const uint64_t live = ~em & (cnt == 64 ? ~0ull : ((1ull << cnt) - 1));
      if (wide) {                                             // survivors to w + their rank among the chunk's survivors
        if ((live >> wl) & 1) NEW(p, w + __popcll(live & ((1ull << wl) - 1))) = v;
      } else {
        int wp = w;                                           // ascending: a move never overwrites an unread survivor
        for (uint64_t b = live; b; b &= b - 1) NEW(p, wp++) = NEW(p, base + (int)__builtin_ctzll(b));
      }
      w += __popcll(live);
    }
    NNEW(p) = w;
    if (expired >= 0) {
      int we = t.p[p].withinEvery;
      if (we >= 0) { add_every_state(we, expired); update_state(we); }
      se_dec(expired);
    }
  }

  SG_LI void count_start_state_reset(int p) const {     // CountPreStateProcessor.startStateReset
    // the reference re-invokes startStateReset on countPost.thisStatePreProcessor (itself) when its own
    // post carries a callback; setting the flag once is the observable effect
    setf(p, F_RESET, true);
  }

  SG_LI void stream_post(int p, int se) const {         // StreamPostStateProcessor.process (:64-83)
    const auto& P = t.p[p];
    setf(p, F_CHANGED, true);
    STS(se) = nd_ts(SS(se, P.stateId));
    if (P.hasNext) setf(p, F_RET, true);
    if (P.nextPre >= 0) add_state(P.nextPre, se);
    if (P.nextEveryPre >= 0) add_every_state(P.nextEveryPre, se);
    if (P.callbackPre >= 0) count_start_state_reset(P.callbackPre);
  }

  SG_LI void min_count_reached(int p, int se) const {   // CountPostStateProcessor (:67-79)
    const auto& P = t.p[p];
    if (P.hasNext) { setf(p, F_CHANGED, true); setf(p, F_RET, true); }
    if (P.nextPre >= 0) add_state(P.nextPre, se);
    if (P.nextEveryPre >= 0) add_every_state(P.nextEveryPre, se);
  }

  SG_LI void post_process(int p, int se) const {
    const auto& P = t.p[p];
    if (isA(P)) {                                 // AbsentStreamPostStateProcessor.process (:36-56)
      setf(p, F_CHANGED, true);
      const int64_t ts = nd_ts(SS(se, P.stateId));
      STS(se) = ts;
      setf(p, F_RET, true);
      if (P.isStart && P.nextEveryPre == p) add_every_state(p, se);
      LST(p) = ts + t.waiting[p];                            // updateLastArrivalTime
      notify_at(p, LST(p));
      return;
    }
    if (isC(P)) {                                  // CountPostStateProcessor.process (:39-65)
      int e = SS(se, P.stateId);
      int n = 1;
      while (NNX(e) >= 0) { n++; e = NNX(e); }
      setf(p, F_SUCCESS, true);
      STS(se) = nd_ts(e);
      if (n >= P.minCount) {
        if (seq()) {
          if (P.nextPre >= 0) add_state(P.nextPre, se);
          if (n != P.maxCount) add_state(p, se);
        } else if (n == P.minCount) {
          min_count_reached(p, se);
        }
        if (n == P.maxCount) setf(p, F_CHANGED, true);
      }
      return;
    }
    if (isL(P) && aLog(P)) {                    // AbsentLogicalPostStateProcessor.process (:36-47)
      setf(p, F_CHANGED, true);
      setf(p, F_RET, true);
      LST(p) = nd_ts(SS(se, P.stateId));                     // updateLastArrivalTime: lastArrivalTime
      return;
    }
    if (isL(P)) {                                // LogicalPostStateProcessor.process (:59-87)
      if (P.isAnd) {
        const bool go = aLog(t.p[P.partner]) ? partner_can_proceed(P.partner, se)
                                              : SS(se, t.p[P.partner].stateId) >= 0;
        if (go) stream_post(p, se);
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

  // AbsentLogicalPreStateProcessor.partnerCanProceed (:371-399) of absent-logical processor p
  SG_LI bool partner_can_proceed(int p, int se) const {
    const auto& P = t.p[p];
    if (seq() && P.nextEveryPre < 0 && LST(p) > 0) return false;
    if (t.waiting[p] == -1) {
      if (P.nextEveryPre < 0) return SS(se, P.stateId) < 0;
      if (LST(p) > 0) { LST(p) = 0; init(p); return false; }
      return true;
    }
    return SS(se, P.stateId) >= 0;
  }

  SG_LI void process_chain(int p, int se, RF rf) const {
    setf(p, F_CHANGED, false);
    if (filter_ok(p, se, rf)) post_process(p, se);
  }

  SG_LI void emit(int se, RF rf) const {
    if (mute) return;
    uint32_t k = bump(a.nrec);
    if ((int64_t)k >= a.rec_cap) { fail(E_REC); return; }
    const bool wr = writer();
    // order: trigger event, then tick records (holder field 0) before the event's holders (1 + k)
    const uint32_t hf = tick >= 0 ? 0u : (uint32_t)((holder + 1) & 15);
    const int64_t sts = STS(se);
    const int32_t lid = a.lane_id[q];
    if (wr) {
      a.rec_key[k] = ((uint64_t)(uint32_t)cur_ev << 24) | ((uint64_t)hf << 20) | (uint64_t)(sub & 0xfffff);
      a.rec_ts[k] = sts;
      a.rec_lane[k] = lid;
      a.rec_tick[k] = tick >= 0 ? tick + a.tick_base : -1;
      a.rec_dl[k] = fhead;
      a.rec_sched[k] = (int8_t)fsched;
      if (a.rec_task) a.rec_task[k] = task;
    }
    Ld ld{this, se};
    for (int q = 0; q < t.nsel; q++) {
      int64_t v = 0;
      bool isnull = false;
      if constexpr (TP::compiled) TP::val(t.nproc + q, ld, v, isnull);
      else run(progs[t.nproc + q], ld, v, isnull, rf, rfs);
      if (wr) {
        a.rec_val[(int64_t)k * t.nsel + q] = v;
        a.rec_nul[(int64_t)k * t.nsel + q] = isnull;
      }
    }
  }

  // processAndReturn (StreamPreStateProcessor :363-403 / Count :53-95 / Logical :128-165);
  // matches are projected immediately (QuerySelector.process on the returned StateEvent)
  SG_LI void process_and_return(int p, int ev, RF rf) {
    const auto& P = t.p[p];
    const int last = P.thisLast;
    int nret = 0;
    if (isA(P) && flag(p, F_INACTIVE)) return;   // AbsentStreamPreStateProcessor.processAndReturn
    if (aLog(P)) { absent_logical_arrival(p, ev, rf); return; }
    int n = NPEND(p), w = 0;
    for (int r = 0; r < n; r++) {
      if (bad()) { NPEND(p) = w; return; }
      int se = PEND(p, r);
      if (isC(P)) {
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
          if (seq()) removed = true;
        }
        if (removed) se_dec(se);
        else PEND(p, w++) = se;
        se_dec(se);
        continue;
      }
      if (isL(P) && !P.isAnd && SS(se, t.p[P.partner].stateId) >= 0) {
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
        if (!isA(P)) ret_push(se, nret);     // an absent state returns nothing on arrivals
      }
      if (flag(p, F_CHANGED)) {
        se_dec(se);                                    // removed from pending
      } else {
        set_slot(se, P.stateId, -1);
        if (seq()) {
          if (isA(P)) PEND(p, w++) = se;   // removeOnNoStateChange is false for absent
          else se_dec(se);
          if ((P.kind == K_STREAM || isA(P)) && P.callbackPre >= 0) count_start_state_reset(P.callbackPre);
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

  SG_LI void ret_push(int se, int& nret) const {
    if (nret >= s.list_cap) { fail(E_RET); return; }
    s.ret[(int64_t)(nret++) * s.L + l] = se;
    se_inc(se);
  }

  // AbsentStreamPreStateProcessor.process(TIMER chunk) (:150-227) for deadline `ct`
  SG_LI void absent_timer(int p, int64_t ct, RF rf) {
    const auto& P = t.p[p];
    // partitioned: the pre-state is dropped whenever its lists are empty and it is not an initialised
    // start state (StreamPreState.canDestroy :444-448 via PartitionSyncStateHolder.returnState), so a
    // non-start absent state reads a fresh lastScheduledTime (0) here
    if (t.partitioned && !P.isStart && NPEND(p) == 0 && NNEW(p) == 0) LST(p) = 0;
    if (flag(p, F_INACTIVE)) return;
    bool initialize = P.isStart && NNEW(p) == 0 && NPEND(p) == 0;
    if (initialize && seq() && P.nextEveryPre < 0 && LST(p) > 0) initialize = false;
    if (initialize) {
      int se = se_alloc();
      if (se < 0) return;
      se_inc(se);
      add_state(p, se);
      se_dec(se);
    } else if (seq() && NNEW(p) != 0) {
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


  // AbsentLogicalPreStateProcessor.processAndReturn (:313-369): returns nothing; an arrival that passes
  // the filter records lastArrivalTime and drops the candidate
  SG_LI void absent_logical_arrival(int p, int ev, RF rf) {
    const auto& P = t.p[p];
    if (flag(p, F_INACTIVE)) return;
    const int last = P.thisLast;
    const int pid = t.p[P.partner].stateId;
    int n = NPEND(p), w = 0;
    for (int r = 0; r < n; r++) {
      if (bad()) { NPEND(p) = w; return; }
      int se = PEND(p, r);
      if (!P.isAnd && SS(se, pid) >= 0) { se_dec(se); continue; }
      const int cur = SS(se, P.stateId);
      nd_inc(cur);                                   // held while the slot is swapped
      int nd = nd_alloc(ev);
      if (nd < 0) return;
      set_slot(se, P.stateId, nd);
      se_inc(se);
      process_chain(p, se, rf);
      if (t.waiting[p] != -1 || (seq() && P.isAnd && P.nextEveryPre >= 0)) set_slot(se, P.stateId, cur);
      bool removed = false;
      if (flag(last, F_RET)) {
        setf(last, F_RET, false);
        removed = true;
        if (seq()) {                                 // partner pending: LinkedList.remove(Object)
          const int pp = P.partner;
          const int m = NPEND(pp);
          for (int k = 0; k < m; k++)
            if (PEND(pp, k) == se) {
              for (int z = k + 1; z < m; z++) PEND(pp, z - 1) = PEND(pp, z);
              NPEND(pp) = m - 1;
              se_dec(se);
              break;
            }
        }
      }
      if (!flag(p, F_CHANGED)) {
        set_slot(se, P.stateId, cur);
        if (seq()) removed = true;
      }
      nd_dec(cur);
      if (removed) se_dec(se);
      else PEND(p, w++) = se;
      se_dec(se);
    }
    NPEND(p) = w;
  }

  // AbsentLogicalPreStateProcessor.sendEvent (:270-292)
  SG_LI void send_absent_logical(int p, int se, RF rf) {
    const auto& P = t.p[p];
    if (P.hasNext) { emit(se, rf); sub++; }
    if (P.nextPre >= 0) add_state(P.nextPre, se);
    if (P.nextEveryPre >= 0) add_every_state(P.nextEveryPre, se);
    else if (P.isStart) {
      setf(p, F_INACTIVE, true);
      if (!P.isAnd && aLog(t.p[P.partner])) setf(P.partner, F_INACTIVE, true);
    }
    if (P.callbackPre >= 0) count_start_state_reset(P.callbackPre);
  }

  // StateEvent.addEvent(stateId, streamEventFactory.newInstance())
  SG_LI void add_empty_event(int se, int k) const {
    int nd = nd_alloc(-1);
    if (nd < 0) return;
    int h = SS(se, k);
    if (h < 0) set_slot(se, k, nd);
    else { while (NNX(h) >= 0) h = NNX(h); NNX(h) = nd; nd_inc(nd); }
  }

  // AbsentLogicalPreStateProcessor.process(TIMER chunk) (:124-227) for deadline `ct`
  SG_LI void absent_logical_timer(int p, int64_t ct, RF rf) {
    const auto& P = t.p[p];
    if (flag(p, F_INACTIVE)) return;
    bool notProcessed = true;
    if (ct >= LST(p) + t.waiting[p]) {
      if (P.isStart && seq() && NNEW(p) == 0 && NPEND(p) == 0) {
        int se = se_alloc();
        if (se < 0) return;
        se_inc(se);
        add_state(p, se);
        se_dec(se);
      } else if (seq() && NNEW(p) != 0) {
        reset_state(p);
      }
      update_state(p);
      const int pid = t.p[P.partner].stateId;
      int expired = -1;
      int nret = 0;
      int n = NPEND(p), w = 0;
      for (int r = 0; r < n; r++) {
        int se = PEND(p, r);
        if (is_expired(se, ct)) {
          if (expired >= 0) se_dec(expired);
          expired = se;                              // the reference keeps the last one
          continue;                                  // (reference moves from pending to `expired`)
        }
        const int own = SS(se, P.stateId);
        const bool passed = own < 0 ? ct >= STS(se) + t.waiting[p] : ct >= nd_ts(own) + t.waiting[p];
        if (passed) {
          const bool partnerSet = SS(se, pid) >= 0;
          if (!P.isAnd && !partnerSet) { add_empty_event(se, P.stateId); ret_push(se, nret); }
          else if (P.isAnd && partnerSet) ret_push(se, nret);
          else if (P.isAnd && !partnerSet) add_empty_event(se, P.stateId);
          se_dec(se);
          continue;
        }
        PEND(p, w++) = se;
      }
      NPEND(p) = w;
      if (expired >= 0) {
        if (P.withinEvery >= 0) { add_every_state(P.withinEvery, expired); update_state(P.withinEvery); }
        se_dec(expired);
      }
      notProcessed = nret == 0;
      for (int k = 0; k < nret; k++) {
        int se = s.ret[(int64_t)k * s.L + l];
        STS(se) = ct;
        send_absent_logical(p, se, rf);
        se_dec(se);
      }
      LST(p) = 0;
    }
    if (P.nextEveryPre >= 0 || (notProcessed && P.isStart)) {
      const int64_t nb = LST(p) == 0 ? now + t.waiting[p] : LST(p) + t.waiting[p];
      notify_at(p, nb);
    }
  }

  // Scheduler.onTimeChange (:74-104) seen from this instance: per Scheduler in listener order, if the
  // FIFO head is due the instance is collected under that head and drains every due head
  // (sendTimerEvents :171-210).  A (tick, scheduler) the host deferred (another instance won the
  // shared deadline) is skipped: the instance is collected again at the next tick.
  SG_LI void fire_timers(RF rf) {
    SG_UNROLL
    for (int k = 0; k < t.nabs; k++) {
      const int p = t.absOrder[k];
      if (q_empty(p) || q_head(p) > now) continue;
      if (a.def_key) {
        const int64_t dk = ((int64_t)tick << 8) | k;
        const int de = a.def_off[q + 1];
        while (dpos < de && a.def_key[dpos] < dk) dpos++;
        if (dpos < de && a.def_key[dpos] == dk) { dpos++; continue; }
      }
      const int64_t head = q_head(p);
      fsched = k;
      fhead = head;
      int spins = 0;
      while (!q_empty(p) && q_head(p) - now <= 0) {
        // the reference would drain forever if every timer re-armed at or before the clock; the lane
        // fails instead of spinning (SG_E_CAPACITY)
        if (++spins > MAX_DRAIN) { fail(E_SPIN); return; }
        const int64_t tt = q_head(p);
        q_pop(p);
        if (aLog(t.p[p])) absent_logical_timer(p, tt, rf);
        else absent_timer(p, tt, rf);
        if (bad()) return;
      }
      fsched = -1;
      if (a.fire && !mute) {
        uint32_t f = bump(a.nfire);
        if ((int64_t)f >= a.fire_cap) { fail(E_LOG); return; }
        FireRec r;
        r.tau = tick; r.lane = a.lane_id[q]; r.head = head; r.sched = (int8_t)k;
        r.empty_after = q_empty(p); r.pad = 0; r.task = task;
        if (writer()) a.fire[f] = r;
      }
    }
  }

  SG_LI void on_tick(int k, RF rf) {
    now = a.tick_now[k];
    tick = k;
    cur_ev = a.tick_ev[k];
    sub = 0;
    fire_timers(rf);
    tick = -1;
  }

  // earliest FIFO head over the absent processors (INT64_MAX if none); cached in a register until a queue
  // changes (notify_at / q_pop), since run_ticks asks at every event and the queues rarely move
  SG_LI int64_t next_deadline() const {
    if (nd_h != INT64_MIN) return nd_h;
    int64_t h = INT64_MAX;
    SG_UNROLL
    for (int k = 0; k < t.nabs; k++) {
      const int p = t.absOrder[k];
      if (!q_empty(p) && q_head(p) < h) h = q_head(p);
    }
    nd_h = h;
    return h;
  }

  // first tick >= tk whose next event comes after arrival rank x (tick_ev is non-decreasing)
  SG_LI int tick_after(int tk, int32_t x) const {
    if (a.tick_ub && (int64_t)x >= a.tub0 && (int64_t)x - a.tub0 < a.ntub) return max(tk, a.tick_ub[x - a.tub0]);
    int lo = tk, hi = ntick();
    while (lo < hi) { const int mid = (lo + hi) >> 1; if (a.tick_ev[mid] > x) hi = mid; else lo = mid + 1; }
    return lo;
  }
  // first tick >= tk whose clock reaches h (tick clocks are non-decreasing)
  SG_LI int tick_at(int tk, int64_t h) const {
    if (a.tick_lb) {
      const int k = h <= a.tlb0 ? 0 : h - a.tlb0 >= a.ntlb ? ntick() : a.tick_lb[h - a.tlb0];
      return max(tk, k);
    }
    int lo = tk, hi = ntick();
    while (lo < hi) { const int mid = (lo + hi) >> 1; if (a.tick_now[mid] >= h) hi = mid; else lo = mid + 1; }
    return lo;
  }

  // run every tick in [tk, ntick) that precedes event `x` and finds a due head; returns the new cursor
  SG_LI int run_ticks(int tk, int32_t x, RF rf) {
    while (tk < ntick() && !bad()) {
      const int64_t h = next_deadline();
      if (h == INT64_MAX) break;
      // the first tick whose clock reaches h and its next event, cached with h (tick clocks do not decrease, so
      // tick_at(tk, h) = max(tk, tick_at(0, h)))
      if (nd_k < 0) { nd_k = tick_at(0, h); nd_tev = nd_k < ntick() ? a.tick_ev[nd_k] : INT32_MAX; }
      const int lo = max(tk, nd_k);
      if (lo >= ntick() || (lo == nd_k ? nd_tev : a.tick_ev[lo]) > x) break;
      on_tick(lo, rf);
      tk = lo + 1;
    }
    return tk;
  }

  // PartitionRuntime.initPartition / App.start: inner.init(), then partitionCreated of absent start
  // states (AbsentStreamPreStateProcessor :296-310, AbsentLogicalPreStateProcessor :387-404)
  SG_LI void create(int64_t at, RF rf) {
    (void)rf;
    SG_UNROLL
    for (int k = 0; k < t.ninit; k++) init(t.initOrder[k]);
    SG_UNROLL
    for (int k = 0; k < t.nabs; k++) {
      const int p = t.absOrder[k];
      if (t.p[p].isStart && t.waiting[p] != -1 && !flag(p, F_INACTIVE)) {
        if (aLog(t.p[p])) { notify_at(p, at + t.waiting[p]); continue; }
        LST(p) = at + t.waiting[p];
        notify_at(p, LST(p));
      }
    }
  }

  // The lane's state in canonical form (StateEvent and chain-node ids renamed by first appearance): per
  // processor its live flags, lastScheduledTime and the pending / new-and-every lists, then every StateEvent
  // reached (ts, type, each slot's chain of nodes with their events).  Two states with equal forms behave
  // identically on every later event.  Returns the length, -1 if it exceeds cap or the lane failed.
  SG_LI int canon(int32_t* out, int cap, int32_t* cm) const {
    if (bad()) return -1;
    int32_t* cse = cm;                      // raw StateEvent -> canonical
    int32_t* inv = cm + s.se_cap;           // canonical -> raw
    int32_t* cnd = cm + 2 * s.se_cap;       // raw node -> canonical
    for (int k = 0; k < s.se_cap; k++) cse[k] = -1;
    for (int k = 0; k < s.nd_cap; k++) cnd[k] = -1;
    int pos = 0, nse = 0, nnd = 0;
    bool over = false;
    auto put = [&](int32_t v) { if (pos < cap) out[pos++] = v; else over = true; };
    auto id = [&](int se) { if (cse[se] < 0) { cse[se] = nse; inv[nse++] = se; } return cse[se]; };
    put(s.created[l]);
    if constexpr ((FM & FM_ABS) != 0)
      SG_UNROLL
      for (int ai = 0; ai < t.nabs; ai++) {         // the Scheduler queues: runs (deadline, multiplicity) from the head
        const int nq_ = NTQA(ai);
        put(nq_);
        for (int k = 0; k < nq_; k++) {
          const int slot = (TQH(ai) + k) % NTQ;
          const int64_t d = TQ(ai, slot);
          put((int32_t)d); put((int32_t)(d >> 32)); put(TQC(ai, slot));
        }
      }
    // (from the pools: the compiled kernels' register copies are stored first, regs_store)
    regs_store();
    for (int p = 0; p < t.nproc; p++) {
      const int64_t x = (int64_t)p * s.L + l;
      // (stateChanged and the count post's success flag are written before every read -- process_chain and
      // process_and_return clear them per partial -- so their values between events are dead and not compared)
      put((int32_t)(s.flags[x] & ~(uint32_t)(F_CHANGED | F_SUCCESS)));
      const int64_t ls = LST(p);
      put((int32_t)ls); put((int32_t)(ls >> 32));
      const int np_ = s.npend[x], nn_ = s.nnev[x];
      put(np_);
      for (int k = 0; k < np_; k++) put(id(PEND(p, k)));
      put(nn_);
      for (int k = 0; k < nn_; k++) put(id(NEW(p, k)));
    }
    for (int c = 0; c < nse && !over; c++) {
      const int se = inv[c];
      const int64_t ts = STS(se);
      put((int32_t)ts); put((int32_t)(ts >> 32)); put(STY(se));
      for (int k = 0; k < t.nslots; k++) {
        for (int nd = SS(se, k); nd >= 0 && !over; nd = NNX(nd)) {
          if (cnd[nd] >= 0) { put(cnd[nd]); break; }     // a shared chain: the rest was written already
          cnd[nd] = nnd++;
          put(-2); put(NEV(nd));
        }
        put(-1);
      }
    }
    return over ? -1 : pos;
  }

  SG_LI void on_event(int ev, RF rf) {
    on_event(ev, a.ev_stream[ev], a.ev_ts[ev], a.ev_rank[ev], rf, a.ev_skip ? a.ev_skip[ev] : 0u);
  }
  SG_LI void on_event(int ev, int st, int64_t ts, int32_t rank, RF rf, uint32_t skip) {
    if constexpr (TP::compiled) {
      // the compiled kernels branch on the stream once, so that every processor index below is a constant
      using CT = typename TP::Tab;
      if constexpr (CT::nstreams > 0) if (st == 0) { on_event_s(ev, SIc<0>{}, ts, rank, rf, skip); return; }
      if constexpr (CT::nstreams > 1) if (st == 1) { on_event_s(ev, SIc<1>{}, ts, rank, rf, skip); return; }
      if constexpr (CT::nstreams > 2) if (st == 2) { on_event_s(ev, SIc<2>{}, ts, rank, rf, skip); return; }
      if constexpr (CT::nstreams > 3) if (st == 3) { on_event_s(ev, SIc<3>{}, ts, rank, rf, skip); return; }
    } else {
      on_event_s(ev, st, ts, rank, rf, skip);
    }
  }
  template <class STI>
  SG_LI void on_event_s(int ev, STI st, int64_t ts, int32_t rank, RF rf, uint32_t skip) {
    cur_ev = rank;
    sub = 0;
    SG_PROBE(1, SG_UNROLL for (int k = 0; k < t.nall; k++) expire_events(t.allPre[k], ts));
    SG_PROBE(2,
    if (seq()) {
      SG_UNROLL
      for (int k = 0; k < t.nreset; k++) reset_state(t.resetOrder[k]);
      SG_UNROLL
      for (int k = 0; k < t.nupdate; k++) update_state(t.updateOrder[k]);
    } else if (t.multi[st]) {
      SG_UNROLL
      for (int k = 0; k < t.nfor[st]; k++) update_state(t.forStream[st][k]);
    } else if (t.nfor[st] > 0) {
      update_state(t.forStream[st][0]);
    });
    SG_PROBE(3,
    if (t.multi[st]) {
      SG_UNROLL
      for (int k = t.nnext[st] - 1; k >= 0; k--) {
        if ((skip >> k) & 1u) continue;
        holder = k;
        sub = 0;
        process_and_return(t.nexts[st][k], ev, rf);
      }
    } else if (!(skip & 1u)) {
      holder = 0;
      process_and_return(t.nexts[st][0], ev, rf);
    });
  }
};

// Per-lane pool layout in LDS: every array of NState for the workgroup's lanes, struct-of-arrays with
// stride = lanes per workgroup (consecutive lanes, consecutive words).  A lane is a chain of dependent
// pool accesses; served from LDS instead of HBM/L2 each step costs ~100 cycles instead of ~1-2 us.
struct NLds {
  size_t off[24];
  int32_t ns = NS, np = NP;      // slots and processors the lane pools are sized for
  size_t bytes;          // lane pools (0: pools stay in global memory)
  size_t prog_off;       // bytecode programs (every program the lanes interpret) and the column table
  size_t cols_off;
  size_t rf_off;         // the interpreter's register file: MAX_REG x lanes int64, lane-minor
  size_t total;
  int32_t nprog;
  __host__ void finish(int np, int lanes) {
    nprog = np;
    prog_off = al(bytes);
    cols_off = al(prog_off + (size_t)np * sizeof(Prog));
    rf_off = al(cols_off + sizeof(NCols));
    total = rf_off + (size_t)MAX_REG * lanes * sizeof(int64_t);
  }
  __host__ __device__ static size_t al(size_t x) { return (x + 7) & ~(size_t)7; }
  __host__ __device__ void build(int se_cap, int nd_cap, int list_cap, int nq, int lw, int ns_, int np_) {
    const size_t w = (size_t)lw;
    ns = ns_; np = np_;
    const size_t sz[24] = {
        (size_t)se_cap * ns * 4, (size_t)se_cap * 8, (size_t)se_cap, (size_t)se_cap * 4, (size_t)se_cap * 4, 4,
        (size_t)nd_cap * 4, (size_t)nd_cap * 4, (size_t)nd_cap * 4, (size_t)nd_cap * 4, 4,
        (size_t)np * list_cap * 4, (size_t)np * 4, (size_t)np * list_cap * 4, (size_t)np * 4, (size_t)np * 4,
        4, 4, (size_t)list_cap * 4, (size_t)np * 8, (size_t)nq * NTQ * 8, (size_t)nq * 4, (size_t)nq * NTQ * 4,
        (size_t)nq * 4};
    size_t o = 0;
    for (int k = 0; k < 24; k++) { off[k] = o; o += al(sz[k] * w); }
    bytes = o;
  }
};

__device__ inline NStateL nfa_lds_state(unsigned char* base_g, const NLds& lay, const NState& g, int lw) {
  SG_AS3 unsigned char* base = (SG_AS3 unsigned char*)base_g;
  NStateL s;
  s.L = lw; s.se_cap = g.se_cap; s.nd_cap = g.nd_cap; s.list_cap = g.list_cap; s.nq = g.nq;
  s.ns = lay.ns; s.np = lay.np;
  s.se_slot = (SG_AS3 int32_t*)(base + lay.off[0]); s.se_ts = (SG_AS3 int64_t*)(base + lay.off[1]);
  s.se_type = (SG_AS3 int8_t*)(base + lay.off[2]); s.se_ref = (SG_AS3 int32_t*)(base + lay.off[3]);
  s.se_free = (SG_AS3 int32_t*)(base + lay.off[4]); s.se_top = (SG_AS3 int32_t*)(base + lay.off[5]);
  s.nd_ev = (SG_AS3 int32_t*)(base + lay.off[6]); s.nd_next = (SG_AS3 int32_t*)(base + lay.off[7]);
  s.nd_ref = (SG_AS3 int32_t*)(base + lay.off[8]); s.nd_free = (SG_AS3 int32_t*)(base + lay.off[9]);
  s.nd_top = (SG_AS3 int32_t*)(base + lay.off[10]); s.pend = (SG_AS3 int32_t*)(base + lay.off[11]);
  s.npend = (SG_AS3 int32_t*)(base + lay.off[12]); s.nev = (SG_AS3 int32_t*)(base + lay.off[13]);
  s.nnev = (SG_AS3 int32_t*)(base + lay.off[14]); s.flags = (SG_AS3 uint32_t*)(base + lay.off[15]);
  s.created = (SG_AS3 int32_t*)(base + lay.off[16]); s.err = (SG_AS3 int32_t*)(base + lay.off[17]);
  s.ret = (SG_AS3 int32_t*)(base + lay.off[18]); s.lst = (SG_AS3 int64_t*)(base + lay.off[19]);
  s.tq = (SG_AS3 int64_t*)(base + lay.off[20]); s.ntq = (SG_AS3 int32_t*)(base + lay.off[21]);
  s.tqc = (SG_AS3 int32_t*)(base + lay.off[22]); s.tqh = (SG_AS3 int32_t*)(base + lay.off[23]);
  return s;
}

// copy one lane's pools between the global SoA (lane gl of g.L) and the LDS SoA (lane tl of d.L); elements
// x0, x0 + dx, ... of every array (wide mode: the wave's threads split the copy, x0 = wl, dx = 64)
template <bool IN>
__device__ inline void nfa_lane_copy(const NState& g, int64_t gl, const NStateL& d, int tl, int x0 = 0, int dx = 1) {
  auto cp = [&](auto* gp, auto* dp, int64_t n) {
    for (int64_t x = x0; x < n; x += dx) {
      if (IN) dp[x * d.L + tl] = gp[x * g.L + gl];
      else gp[x * g.L + gl] = dp[x * d.L + tl];
    }
  };
  for (int64_t z = x0; z < (int64_t)g.se_cap * d.ns; z += dx) {
    const int64_t se = z / d.ns, k = z - se * d.ns;
    const int64_t xg = (se * g.ns + k) * g.L + gl, xd = (se * d.ns + k) * d.L + tl;
    if (IN) d.se_slot[xd] = g.se_slot[xg];
    else g.se_slot[xg] = d.se_slot[xd];
  }
  cp(g.se_ts, d.se_ts, g.se_cap); cp(g.se_type, d.se_type, g.se_cap);
  cp(g.se_ref, d.se_ref, g.se_cap); cp(g.se_free, d.se_free, g.se_cap); cp(g.se_top, d.se_top, 1);
  cp(g.nd_ev, d.nd_ev, g.nd_cap); cp(g.nd_next, d.nd_next, g.nd_cap); cp(g.nd_ref, d.nd_ref, g.nd_cap);
  cp(g.nd_free, d.nd_free, g.nd_cap); cp(g.nd_top, d.nd_top, 1);
  cp(g.pend, d.pend, (int64_t)d.np * g.list_cap); cp(g.npend, d.npend, d.np);
  cp(g.nev, d.nev, (int64_t)d.np * g.list_cap); cp(g.nnev, d.nnev, d.np); cp(g.flags, d.flags, d.np);
  cp(g.created, d.created, 1); cp(g.err, d.err, 1); cp(g.lst, d.lst, d.np);
  cp(g.tq, d.tq, (int64_t)g.nq * NTQ); cp(g.ntq, d.ntq, g.nq);
  cp(g.tqc, d.tqc, (int64_t)g.nq * NTQ); cp(g.tqh, d.tqh, g.nq);
}

// one lane's pools as k_nfa_pool_init leaves them (an instance that was never created); elements k0, k0 + dk, ...
template <class ST>
__device__ inline void nfa_pool_init_one(const ST& s, int64_t l, int k0 = 0, int dk = 1) {
  for (int k = k0; k < s.se_cap; k += dk) s.se_free[(int64_t)k * s.L + l] = s.se_cap - 1 - k;
  for (int k = k0; k < s.nd_cap; k += dk) s.nd_free[(int64_t)k * s.L + l] = s.nd_cap - 1 - k;
  for (int p = k0; p < s.np; p += dk) {
    s.npend[(int64_t)p * s.L + l] = 0; s.nnev[(int64_t)p * s.L + l] = 0; s.flags[(int64_t)p * s.L + l] = 0;
    s.lst[(int64_t)p * s.L + l] = 0;
  }
  for (int k = k0; k < s.nq; k += dk) { s.ntq[(int64_t)k * s.L + l] = 0; s.tqh[(int64_t)k * s.L + l] = 0; }
  if (k0 == 0) {
    s.se_top[l] = s.se_cap;
    s.nd_top[l] = s.nd_cap;
    s.created[l] = 0;
    s.err[l] = 0;
  }
}

template <class LN>
SG_LI void nfa_run_lane(LN& ln, const NArgs& a, int q, RF myrf, const NSpec* sp = nullptr) {
  const auto& s = ln.s;
  int w0, e0, e1;
  if (sp) { w0 = sp->w0[q]; e0 = sp->e0[q]; e1 = sp->e1[q]; ln.task = q; }
  else { e0 = a.lane_off[q]; e1 = a.lane_off[q + 1]; w0 = e0; }
  int32_t* cw = sp ? sp->canon + (size_t)q * 2 * (SG_CANON + 1) : nullptr;
  int32_t* cm = sp ? sp->cmap + (size_t)q * sp->cmap_stride : nullptr;
  int tk = 0;
  if (!s.created[ln.l]) {
    // first event of the partition key: PartitionRuntimeImpl.initPartition -> innerStateRuntime.init(),
    // at the app clock of that event, after the ticks that precede it (unpartitioned: App.start)
    s.created[ln.l] = 1;
    if (a.ev_now && w0 < e1) {
      const int x = a.ev_rank[a.lane_ev[w0]];
      ln.cur_ev = x;
      tk = a.ntick ? ln.tick_after(0, x) : 0;
      ln.create(a.ev_now[a.lane_ev[w0]], myrf);
    } else {
      ln.create(a.start_now, myrf);
    }
  }
  ln.mute = w0 < e0;
  if (sp && w0 < e0) cw[0] = -1;          // (a lane that fails in its warm-up never verifies)
  // Per event: its fields come from the packed records (NEvRec, the next record loaded while the current one runs),
  // or without them from a three-step load pipeline over lane_ev (a lane is one chain of dependent steps, so every
  // load it waits for is exposed: event e + 2's index, e + 1's arrival rank / stream / clock / row, and e's
  // attributes and tick cursor are issued before event e runs).  One on_event call site either way.
  const bool packed = a.lane_rec != nullptr;
  const int el = e1 - 1;
  NEvRec rn;
  int xa = 0, xb = 0, ra = 0, sa = 0, wa = 0;
  uint32_t ka = 0;                       // the event's prefilter mask (NArgs::ev_skip), loaded with the rest
  int64_t ta = 0;
  if (w0 < e1) {
    if (packed) {
      rn = a.lane_rec[w0];
    } else {
      xa = a.lane_ev[w0];
      xb = a.lane_ev[min(w0 + 1, el)];
      ra = a.ev_rank[xa]; sa = a.ev_stream[xa]; wa = a.ev_row[xa]; ta = a.ev_ts[xa];
      ka = a.ev_skip ? a.ev_skip[xa] : 0u;
    }
  }
  for (int e = w0; e < e1; e++) {
    int x, st, rank, ub;
    int64_t ts;
    uint32_t skip;
    if (packed) {
      const NEvRec rc = rn;
      if (e + 1 < e1) rn = a.lane_rec[e + 1];
      x = rc.x; st = rc.stream; rank = rc.rank; ts = rc.ts; skip = rc.skip; ub = rc.tub;
      ln.cx = rc.x;
      ln.cok = rc.cok != 0;
      ln.cv0 = rc.v[0]; ln.cv1 = rc.v[1]; ln.cv2 = rc.v[2]; ln.cv3 = rc.v[3];
    } else {
      const int xc = a.lane_ev[min(e + 2, el)];
      const int rb = a.ev_rank[xb], sb = a.ev_stream[xb], wb = a.ev_row[xb];
      const uint32_t kb = a.ev_skip ? a.ev_skip[xb] : 0u;
      const int64_t tb = a.ev_ts[xb];
      ln.prefetch_attrs(xa, sa, wa);
      const int64_t ro = (int64_t)ra - a.tub0;
      ub = ln.ntick() && a.tick_ub && ro >= 0 && ro < a.ntub ? a.tick_ub[ro] : -1;
      x = xa; st = sa; rank = ra; ts = ta; skip = ka;
      xa = xb; xb = xc; ra = rb; sa = sb; wa = wb; ta = tb; ka = kb;
    }
    if (e == e0 && w0 < e0) {              // end of the warm-up: the state the segment starts from
      cw[0] = ln.canon(cw + 1, SG_CANON, cm);
      ln.mute = false;
    }
    if (ln.bad()) break;
    if (ln.ntick()) {
#ifdef SG_NFA_PROBE
      { const unsigned long long t0_ = wall_clock64(); tk = ln.run_ticks(tk, rank, myrf); ln.pt[0] += wall_clock64() - t0_; }
#else
      tk = ln.run_ticks(tk, rank, myrf);
#endif
      tk = ub >= 0 ? max(tk, ub) : ln.tick_after(tk, rank);   // ticks that precede the event are past after it
    }
    ln.on_event(x, st, ts, rank, myrf, skip);
#ifdef SG_NFA_PROBE
    ln.pt[5]++;
#endif
  }
#ifdef SG_NFA_PROBE
  if (a.probe && ln.writer()) for (int k = 0; k < 6; k++) atomicAdd(&a.probe[k], ln.pt[k]);
#endif
  ln.cx = -1;
  if (sp) {
    // the end state is taken before the ticks that follow the last event: the next segment runs those
    cw[SG_CANON + 1] = ln.canon(cw + SG_CANON + 2, SG_CANON, cm);
    if (sp->tail[q] && ln.ntick() && !ln.bad()) ln.run_ticks(tk, INT32_MAX, myrf);
    return;
  }
  if (ln.ntick() && !ln.bad()) ln.run_ticks(tk, INT32_MAX, myrf);
}

static_assert(sizeof(NTable) % 4 == 0 && sizeof(Prog) % 4 == 0 && sizeof(NCols) % 4 == 0, "LDS copies by words");

// One lane per partition instance.  With `lay.bytes` > 0 the workgroup's lanes run on LDS copies of
// their pools (copied in at the start, back at the end).  t3 / c3 / p3: the table, column table and bytecode
// (LDS copies for the interpreter; the compiled kernels pass their constexpr table and no bytecode).
// Narrow mode: thread = lane, blockDim.x lanes per workgroup.  Wide mode (a.wide): one lane per workgroup of one
// wavefront, every thread running it (NArgs::wide); the staging copies are split over the wave.
template <int FM, class TP>
__device__ __forceinline__ void nfa_lanes_run(const NArgs& a, const NState& g, const NLds& lay, const NSpec* spec,
                                              typename TP::Tab t3, const SG_AS3 NCols& c3, const SG_AS3 Prog* p3,
                                              unsigned char* nfa_dyn) {
  const bool wide = a.wide != 0;
  const int lpw = wide ? 1 : (int)blockDim.x;            // lanes per workgroup
  const int lw = wide ? 0 : (int)threadIdx.x;            // this thread's lane in the workgroup
  const int wl = wide ? (int)(threadIdx.x & 63) : 0;     // its thread in the wave (wide)
  const int qi = blockIdx.x * lpw + lw;
  if (qi >= a.nl) return;
  const int q = spec ? qi + spec->q0 : qi;
  // the pools the lane runs on: the instance's own (lane_id), or for a speculative segment a scratch lane
  // that starts as a never-created instance
  int64_t gl = spec ? (spec->pool[q] < 0 ? (int64_t)(-spec->pool[q] - 1) : (int64_t)spec->pool[q]) : a.lane_id[q];
  // blocked scratch pools (a launch of scratch tasks only, workgroups of a power of two <= 64 lanes, scratch lane =
  // task index - q0: a workgroup's lanes lie in one block, so the block and its view are uniform)
  const bool blk = spec && spec->blocked;
  const NState pg = blk ? nfa_block_view(spec->gs, (int64_t)__builtin_amdgcn_readfirstlane((int)(gl >> 6)))
                        : (spec && spec->pool[q] < 0) ? spec->gs : g;
  if (blk) gl &= 63;
  const bool fresh = spec && spec->pool[q] < 0;
  RF rf3 = (RF)((int64_t*)(nfa_dyn + lay.rf_off) + lw);
  const int x0 = wide ? wl : 0, dx = wide ? 64 : 1;
  if (lay.bytes > 0) {                   // pools staged in LDS: ds_* accesses
    const NStateL s = nfa_lds_state(nfa_dyn, lay, pg, lpw);
    const int l = lw;
    if (fresh) nfa_pool_init_one(s, l, x0, dx);
    else nfa_lane_copy<true>(pg, gl, s, l, x0, dx);
    if (wide) __syncthreads();           // (one wave per workgroup: every thread reads what the others staged)
    Lane<true, FM, TP> ln{t3, s, c3, a, p3, l, 0, 0, 0, -1, a.start_now, -1, 0, 0, q, 0};
    ln.rfs = lpw;
    ln.wide = wide;
    ln.wl = wl;
    if (a.def_key) ln.dpos = a.def_off[q];
    ln.regs_load();
    nfa_run_lane(ln, a, q, rf3, spec);
    ln.regs_store();
    if (wide) __syncthreads();
    nfa_lane_copy<false>(pg, gl, s, l, x0, dx);
  } else {
    if (fresh) {
      nfa_pool_init_one(pg, gl, x0, dx);
      if (wide) __syncthreads();         // (global pools: the barrier also orders the threads' stores)
    }
    Lane<false, FM, TP> ln{t3, pg, c3, a, p3, gl, 0, 0, 0, -1, a.start_now, -1, 0, 0, q, 0};
    ln.rfs = lpw;
    ln.wide = wide;
    ln.wl = wl;
    if (a.def_key) ln.dpos = a.def_off[q];
    ln.regs_load();
    nfa_run_lane(ln, a, q, rf3, spec);
    ln.regs_store();
  }
}

#ifndef SG_RTC
// The interpreter: one kernel per feature mask, every query's table, bytecode and columns copied into LDS.
template <int FM>
__global__ void __launch_bounds__(NFA_B) k_nfa_lanes(NArgs a, NState g, NLds lay, const NTable* __restrict__ tab,
                                                     const NCols* __restrict__ cols, const Prog* __restrict__ progs,
                                                     const NSpec* __restrict__ spec) {
  __shared__ NTable st;
  extern __shared__ __align__(16) unsigned char nfa_dyn[];
  // the table, the bytecode and the column table are read at every step of the interpreter: LDS copies
  for (int k = threadIdx.x; k < (int)(sizeof(NTable) / 4); k += blockDim.x) ((int32_t*)&st)[k] = ((const int32_t*)tab)[k];
  Prog* lprogs = (Prog*)(nfa_dyn + lay.prog_off);
  for (int k = threadIdx.x; k < (int)(lay.nprog * sizeof(Prog) / 4); k += blockDim.x)
    ((int32_t*)lprogs)[k] = ((const int32_t*)progs)[k];
  NCols* lcols = (NCols*)(nfa_dyn + lay.cols_off);
  for (int k = threadIdx.x; k < (int)(sizeof(NCols) / 4); k += blockDim.x) ((int32_t*)lcols)[k] = ((const int32_t*)cols)[k];
  __syncthreads();
  nfa_lanes_run<FM, LdsTab>(a, g, lay, spec, *(const SG_AS3 NTable*)&st, *(const SG_AS3 NCols*)lcols,
                            (const SG_AS3 Prog*)lprogs, nfa_dyn);
}
#endif

}  // namespace sg
