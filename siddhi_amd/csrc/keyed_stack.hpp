// keyed_stack.hpp — streaming stack matcher + trigger-order pass for SG_PATH_KEYED_FOLLOWED_BY (config 4).
//
// Reference semantics (per partition key, PartitionStreamReceiver.java:82-282): inside a key's instance
// `every e1=S[f1] -> e2=S[f2] within W` completes the partial of start i at
//   m(i) = min{ j > i : k_j = k_i, ts_j - ts_i <= W, x_j OP x_i }
// (StreamPreStateProcessor.processAndReturn :363-403 with expireEvents :325-361), and the records of one
// trigger j are emitted together, in ascending i (MultiProcessStreamReceiver.ReturnEventHolder :306-316),
// callbacks in arrival order of j.
//
// For OP in {>, >=, <, <=} the open starts of one key form a stack: a trigger completes exactly the top run
// of starts it satisfies (a start below an unsatisfied one holds a value at least as hard to satisfy), the
// starts left are never satisfied by it, and the newest start goes on top.  Expiry is lazy: the first node
// from the top older than W ends the walk and every node below it is older still.  So one pass over a
// key's events in arrival order decides every m(i) with one stack step per start -- no key sort, no
// per-start forward walk.
//
//   k_ks_match   one wavefront per task = (bucket b, time group g): the bucket's entries whose events lie in
//                the group's super-tiles, replayed from the first entry within W before them (the halo:
//                it rebuilds the stacks exactly, nothing older can still be completed).  64 entries per
//                round; lanes of one round that share a key run in arrival order (ballot-matched ranks
//                as levels).  Stacks are linked nodes in an LDS ring of R nodes addressed by allocation
//                ordinal (a reference older than R allocations is a node that died before its slot was
//                reused; reusing the slot of a live node flags the task for a rerun with a larger ring).
//                Records {j, i, projections} go to the task's slice of a temp array in (j, i) order, and
//                the task notes, for every order group h of its time group, how many records precede it.
//   k_ks_order   one workgroup per order group h (KS_HQ consecutive trigger indices): the 1024-ish pieces
//                (one per bucket) of its records are counting-sorted by j (a trigger's records are one run of
//                one piece, already in ascending i) and written densely at the group's exclusive base:
//                the output is the reference's callback order, in HBM.
//
// HBM per event: entries read once (+ the halo share), records written to the temp and moved once.
#pragma once
#include "keyed_tiles.hpp"

namespace sg {

constexpr int KS_HQB = 14;                     // log2 trigger indices per order group
constexpr int KS_HQ = 1 << KS_HQB;
constexpr uint32_t KS_NONE = 0xffffffffu;      // no node
constexpr uint32_t KS_POPPED = 0x80000000u;    // node ts word: completed (or never allocated)
constexpr uint32_t KS_POPTAG = 0x80000000u;    // node link word after completion: KS_POPTAG | round
constexpr int KS_ORDER_NT = 1024;
constexpr int KS_R = 1024, KS_KS = 4;          // first launch: ring nodes, completions staged per lane
constexpr int KS_R2 = 2048, KS_KS2 = 32;       // rerun of the flagged tasks

struct KsArgs {
  const void* ent;            // bucketed entries (KtE12 or 16-B logical form)
  const uint32_t* tbase;      // [P * nst] exclusive scan of the bucket histogram: first position of (b, st)
  const uint32_t* bstart;     // [P + 1]
  int64_t n, lo;              // events; [0, lo) are carried starts (never triggers)
  int32_t nst, pb, spg;       // super-tiles, log2 buckets, super-tiles per time group
  int32_t ngroups, hpg;       // time groups; order groups per time group (spg * KT_ST / KS_HQ)
  uint32_t w32;               // within (ms, saturated to 31 bits)
  uint32_t ts_last_rel;       // last timestamp of the flush, relative
  int32_t* rec;               // temp records, `stride` words each, task slice = its entry positions
  int32_t stride;
  uint32_t* offs;             // [G][hpg + 1][P]: records of task (b, g) before order group h
  int32_t* carry;
  uint32_t* ncarry;
  uint32_t* nflag;            // [0] tasks flagged for a rerun, [1] a rerun overflowed too
  uint32_t* flist;            // flagged task ids (g * P + b)
  int32_t exp;                // measurement-only bits (SG_KS_EXP): 1 no record stores, 2 no offs stores
  int32_t nproj;
  int32_t src[FB_MAXP];
  int32_t w[FB_MAXP];
  const uint8_t* col[FB_MAXP];
};

__device__ __forceinline__ uint32_t ks_ts(uint4 e) { return e.y & 0x7fffffffu; }

// inclusive wave scan (64 lanes)
__device__ __forceinline__ uint32_t ks_wave_incl(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

// Task (b, g) of workgroup w.  First launch: blockIdx -> XCD x = blockIdx % 8 takes the buckets
// [x P/8, (x+1) P/8) in time-group-major order, so a bucket's halo (the previous group's tail) was read on
// the same XCD and every XCD writes whole lines of the offs rows.
__device__ __forceinline__ void ks_task(const KsArgs& a, uint32_t& b, uint32_t& g) {
  const uint32_t P = 1u << a.pb;
  const uint32_t t = blockIdx.x;
  if (P >= 8) {
    const uint32_t per = P / 8, x = t & 7, q = t >> 3;
    b = x * per + q % per;
    g = q / per;
  } else {
    b = t & (P - 1);
    g = t >> a.pb;
  }
}

constexpr int KS_RING = 128;                   // LDS record ring per task (records await their store)

template <int R, int KS, int NLK>
struct KsLds {
  uint4 nd[R];                  // node: {ts_rel | KS_POPPED, x, event index, below ordinal | KS_POPTAG|round}
  uint32_t top[NLK];            // per local key: ordinal of its top node (KS_NONE)
  uint2 stage[64 * KS];         // per lane: {event index, x} of the starts it completed this round (top first)
  uint4 ring[KS_RING];          // 4-word records of the task, in (j, i) order, not yet stored
};

// raw entry as loaded (decoded where it is used, so the wait for a prefetched entry sits at its use)
template <bool E12> struct KsRaw { using T = uint4; };
template <> struct KsRaw<true> { using T = KtE12; };
template <bool E12>
__device__ __forceinline__ typename KsRaw<E12>::T ks_load(const void* ent, uint32_t i) {
  if constexpr (E12) return ((const KtE12*)ent)[i];
  else return ((const uint4*)ent)[i];
}
template <bool E12>
__device__ __forceinline__ uint4 ks_decode(const typename KsRaw<E12>::T& r) {
  if constexpr (E12) return make_uint4(r.idx, (r.y & 0x80000000u) | ((r.y >> KT_LB) & 0x1fffffu), r.x, r.y & (KT_NL - 1));
  else return r;
}

// VEC: 4-word records whose projections are the start's key, the start's x or the trigger's x (built from
// registers and LDS, stored through the ring); otherwise records of any width with column gathers
template <int OP, class V, bool E12, bool VEC, int LB, int R, int KS>
__device__ void ks_match_task(const KsArgs& a, const uint32_t b, const uint32_t g, KsLds<R, KS, (1 << LB)>& sm,
                              const bool rerun) {
  const int lane = threadIdx.x;
  const uint64_t ltm = (1ull << lane) - 1;
  const uint32_t P = 1u << a.pb;
  if (g >= (uint32_t)a.ngroups) return;
  const int64_t stb = (int64_t)b * a.nst;
  const int32_t st0 = (int32_t)g * a.spg, st1 = st0 + a.spg;
  const uint32_t P0 = a.tbase[stb + st0];
  const uint32_t P1 = st1 < a.nst ? a.tbase[stb + st1] : a.bstart[b + 1];
  const bool last = st1 >= a.nst;
  const int64_t grow = (int64_t)g * (a.hpg + 1);
  auto offs_at = [&](int h) -> uint32_t* { return a.offs + (grow + h) * P + b; };
  if (P0 == P1 && !last) {                                   // nothing to match, nothing to carry
    for (int h = lane; h <= a.hpg; h += 64) *offs_at(h) = 0u;
    return;
  }
  // rows are written where the task's entries cross into a group; a row no entry reaches keeps KS_NONE and
  // reads as the next row (a rerun starts from clean rows)
  if (rerun)
    for (int h = lane; h <= a.hpg; h += 64) *offs_at(h) = KS_NONE;
  // the halo: the first entry of the bucket within W of the task's first trigger (of the flush's last
  // timestamp for an empty last task), by a 64-ary search over the non-decreasing bucketed timestamps
  const uint32_t B0 = a.bstart[b];
  const uint32_t tref = P0 < P1 ? ks_ts(kt_get<E12>(a.ent, P0)) : a.ts_last_rel;
  uint32_t lo = B0, hi = P0;
  while (hi - lo > 64) {
    const uint32_t step = (hi - lo + 63) / 64;
    const uint32_t q = lo + (uint32_t)lane * step;
    const bool pred = q < hi && tref - ks_ts(kt_get<E12>(a.ent, q)) <= a.w32;
    const uint64_t bm = __ballot(pred);
    if (bm & 1ull) { hi = lo; break; }
    if (!bm) { lo = lo + ((hi - 1 - lo) / step) * step + 1; continue; }   // past the last sample below hi
    const int f = __ffsll((long long)bm) - 1;
    const uint32_t nlo = lo + (uint32_t)(f - 1) * step + 1, nhi = lo + (uint32_t)f * step;
    lo = nlo;
    hi = nhi;
  }
  {
    const uint32_t q = lo + (uint32_t)lane;
    const bool pred = q < hi && tref - ks_ts(kt_get<E12>(a.ent, q)) <= a.w32;
    const uint64_t bm = __ballot(pred);
    lo = bm ? lo + (uint32_t)(__ffsll((long long)bm) - 1) : hi;
  }
  const uint32_t H0 = lo;
  for (int s = lane; s < R; s += 64) sm.nd[s] = make_uint4(KS_POPPED, 0u, 0u, KS_POPTAG | 0x7fffffffu);
  for (int k = lane; k < (1 << LB); k += 64) sm.top[k] = KS_NONE;
  __syncthreads();
  const uint32_t cap = P1 - P0;
  const int64_t g0 = (int64_t)st0 * KT_ST;                   // first event index of the time group
  const int ps0 = a.src[0], ps1 = a.src[1];
  const uint32_t keyhi = b;                                   // key = lk << pb | b
  uint32_t cur = 0, running = 0, flushed = 0;
  int hh_last = -1;
  bool ovf = false;
  const uint32_t Pm = P1 > 0 ? P1 - 1 : 0;
  // entries two rounds ahead are in flight (every round issues exactly one record store and one offs store,
  // so the wait for them never waits for the stores)
  // one round: the 64 entries from `base` (their raw form `er`); true when the task overflowed
  auto run_round = [&](const typename KsRaw<E12>::T& er, const uint32_t base, const uint32_t round) -> bool {
    const uint32_t p = base + (uint32_t)lane;
    const bool valid = p < P1;
    const uint4 e = ks_decode<E12>(er);
    const uint32_t lk = e.w, tsr = ks_ts(e), xb = e.z, idx = e.x;
    const bool task = valid && p >= P0;
    const bool trig = task && (int64_t)idx >= a.lo;
    const V x = kt_val<V>(xb);
    bool push = valid && (e.y >> 31);
    if constexpr (std::is_floating_point<V>::value) push = push && x == x;   // a NaN start is never completed
    // same-key lanes of the round run in arrival order: level = rank among the round's lanes of its key
    const uint64_t peers = kt_match_peers<LB>(lk, valid);
    const int level = __popcll(peers & ltm);
    uint32_t c = 0;
    for (int L = 0; __ballot(valid && level >= L); L++) {
      const bool act = valid && level == L;
      uint32_t o = KS_NONE;
      if (act) {
        o = sm.top[lk];
        while (true) {
          if (o == KS_NONE || cur - o >= (uint32_t)R) { o = KS_NONE; break; }   // died before its slot was reused
          const uint32_t s = o & (R - 1);
          const uint4 nt = sm.nd[s];
          if (tsr - nt.x > a.w32) { o = KS_NONE; break; }                      // expired: so is all below
          if (!cmpv<OP, V>(x, kt_val<V>(nt.y))) break;                          // nor anything below
          if (trig) {
            if (c < (uint32_t)KS) sm.stage[lane * KS + c] = make_uint2(nt.z, nt.y);
            c++;
          }
          sm.nd[s] = make_uint4(nt.x | KS_POPPED, nt.y, nt.z, KS_POPTAG | round);
          o = nt.w;
        }
      }
      const bool pl = act && push;
      const uint64_t pm = __ballot(pl);
      if (pl) {
        const uint32_t my = cur + (uint32_t)__popcll(pm & ltm);
        const uint32_t s = my & (R - 1);
        const uint4 old = sm.nd[s];
        // the slot's previous node must be dead: completed in an earlier round (its record data is no
        // longer needed) or expired
        const bool dead = (old.x & KS_POPPED) ? old.w != (KS_POPTAG | round) : tsr - old.x > a.w32;
        ovf |= !dead;
        sm.nd[s] = make_uint4(tsr, xb, idx, o);
        sm.top[lk] = my;
      } else if (act) {
        sm.top[lk] = o;
      }
      cur += (uint32_t)__popcll(pm);
    }
    // records, in (j, i) order: lanes in arrival order, a lane's completions reversed (bottom-most first).
    // The lane-order prefix of c from bit-sliced ballots (no cross-lane LDS traffic); c > KS overflows anyway
    ovf |= c > (uint32_t)KS;
    constexpr int CB = KS < 8 ? 3 : KS < 16 ? 4 : KS < 32 ? 5 : 6;   // bits of c <= KS (larger c overflows)
    const uint32_t cc = min(c, (uint32_t)KS);
    uint32_t excl = 0, tot = 0;
#pragma unroll
    for (int bit = 0; bit < CB; bit++) {
      const uint64_t bm = __ballot((cc >> bit) & 1u);
      excl += (uint32_t)__popcll(bm & ltm) << bit;
      tot += (uint32_t)__popcll(bm) << bit;
    }
    ovf |= running + tot > cap;
    if (__any(ovf)) return true;
    if constexpr (VEC) {
      // the ring: records enter in order; one store per lane per round drains up to 64 of them
      if (running + tot - flushed > (uint32_t)KS_RING) {
        // a burst beyond the ring (rare): drain it first, then wait, so the common path's count holds
        while (flushed < running) {
          const uint32_t m = min(64u, running - flushed);
          if ((uint32_t)lane < m)
            *(uint4*)(a.rec + (int64_t)(P0 + flushed + lane) * 4) = sm.ring[(flushed + lane) & (KS_RING - 1)];
          flushed += m;
        }
        __builtin_amdgcn_s_waitcnt(0);
        if (tot > (uint32_t)KS_RING) { ovf = true; return true; }
      }
      for (uint32_t k = 0; k < c; k++) {
        const uint2 st = sm.stage[lane * KS + (c - 1 - k)];
        const uint32_t kv = (lk << a.pb) | keyhi;
        const uint32_t v0 = ps0 == KT_KEY ? kv : ps0 == KT_XI ? st.y : xb;
        const uint32_t v1 = ps1 == KT_KEY ? kv : ps1 == KT_XI ? st.y : xb;
        sm.ring[(running + excl + k) & (KS_RING - 1)] = make_uint4(idx, st.x, v0, v1);
      }
      const uint32_t m = min(64u, running + tot - flushed);
      if ((uint32_t)lane < m && !(a.exp & 1))
        *(uint4*)(a.rec + (int64_t)(P0 + flushed + lane) * 4) = sm.ring[(flushed + lane) & (KS_RING - 1)];
      flushed += m;
    } else {
      for (uint32_t k = 0; k < c; k++) {
        const uint2 st = sm.stage[lane * KS + (c - 1 - k)];
        const uint32_t ig = st.x, xi = st.y;
        int32_t* rp = a.rec + (int64_t)(P0 + running + excl + k) * a.stride;
        rp[0] = (int32_t)idx;
        rp[1] = (int32_t)ig;
        int wo = 2;
        for (int cc = 0; cc < a.nproj; cc++) {
          int64_t val;
          switch (a.src[cc]) {
            case KT_KEY: val = (int32_t)((lk << a.pb) | b); break;
            case KT_XI: val = (int32_t)xi; break;
            case KT_XJ: val = (int32_t)xb; break;
            default: {
              const int64_t gi = a.src[cc] == KT_COL_I ? ig : idx;
              val = a.w[cc] == 2 ? ((const int64_t*)a.col[cc])[gi] : (int64_t)((const int32_t*)a.col[cc])[gi];
            }
          }
          rp[wo] = (int32_t)val;
          if (a.w[cc] == 2) rp[wo + 1] = (int32_t)(val >> 32);
          wo += a.w[cc];
        }
      }
    }
    // order-group boundaries: the first lane of the task's entries in a group writes that group's row (the
    // records of this task before it); rows of groups no entry reaches stay KS_NONE.  Groups are monotone
    // over the round's task lanes and few per round: one ballot per group present
    const uint64_t tm = __ballot(task);
    if (tm) {
      const int hv = task ? (int)((int64_t)idx - g0 < 0 ? 0 : ((int64_t)idx - g0) >> KS_HQB) : -1;
      const int hfirst = __builtin_amdgcn_readlane(hv, __ffsll((long long)tm) - 1);
      const int hlast = __builtin_amdgcn_readlane(hv, 63 - __clzll((long long)tm));
      for (int h = hfirst; h <= hlast; h++) {
        const uint64_t gm = __ballot(task && hv == h);
        if (gm && h > hh_last && h < a.hpg && lane == __ffsll((long long)gm) - 1 && !(a.exp & 2))
          *offs_at(h) = running + excl;
      }
      hh_last = max(hh_last, min(hlast, a.hpg - 1));
    }
    running += tot;
    return false;
  };
  // two register sets for the entries in flight (rounds unrolled by two), so a loaded set is consumed where
  // it was loaded into: no copy at the loop latch waits for the newest load (and the stores before it)
  typename KsRaw<E12>::T ea = ks_load<E12>(a.ent, min(H0 + (uint32_t)lane, Pm));
  typename KsRaw<E12>::T eb = ks_load<E12>(a.ent, min(H0 + 64u + (uint32_t)lane, Pm));
  for (uint32_t base = H0, round = 0; base < P1; base += 128, round += 2) {
    if (run_round(ea, base, round)) break;
    ea = ks_load<E12>(a.ent, min(base + 128u + (uint32_t)lane, Pm));
    if (base + 64 >= P1) break;
    if (run_round(eb, base + 64, round + 1)) break;
    eb = ks_load<E12>(a.ent, min(base + 192u + (uint32_t)lane, Pm));
  }
  if (__any(ovf)) {
    if (lane == 0) {
      if (rerun) atomicOr(a.nflag + 1, 1u);                   // the rerun's larger ring overflowed too
      else a.flist[atomicAdd(a.nflag, 1u)] = (g << a.pb) | b;
    }
    return;
  }
  if constexpr (VEC)
    for (; flushed < running; flushed += 64)
      if (flushed + lane < running)
        *(uint4*)(a.rec + (int64_t)(P0 + flushed + lane) * 4) = sm.ring[(flushed + lane) & (KS_RING - 1)];
  for (int h = hh_last + 1 + lane; h <= a.hpg; h += 64) *offs_at(h) = running;
  if (last) {
    // the bucket's open starts at the flush's end (not completed, not expired at its last timestamp)
    // carry into the next flush
    for (int s = lane; s < R; s += 64) {
      const uint4 nt = sm.nd[s];
      if (!(nt.x & KS_POPPED) && a.ts_last_rel - nt.x <= a.w32) a.carry[atomicAdd(a.ncarry, 1u)] = (int32_t)nt.z;
    }
  }
}

// LB: local-key bits per bucket (the key table); the ring holds 2^LB nodes (a bucket's starts in one
// `within` window at the mean rate fit it)
template <int OP, class V, bool E12, bool VEC, int LB>
__global__ void __launch_bounds__(64) k_ks_match(KsArgs a) {
  __shared__ KsLds<(1 << LB), KS_KS, (1 << LB)> sm;
  uint32_t b, g;
  ks_task(a, b, g);
  ks_match_task<OP, V, E12, VEC, LB, (1 << LB), KS_KS>(a, b, g, sm, false);
}

// the tasks the first launch flagged, with a larger ring and more completions per trigger (a grid that
// walks the device-side list: no host round trip)
template <int OP, class V, bool E12, bool VEC, int LB>
__global__ void __launch_bounds__(64) k_ks_rerun(KsArgs a) {
  __shared__ KsLds<KS_R2, KS_KS2, (1 << LB)> sm;
  const uint32_t nt = *(volatile const uint32_t*)a.nflag;
  for (uint32_t k = blockIdx.x; k < nt; k += gridDim.x) {
    const uint32_t t = a.flist[k];
    ks_match_task<OP, V, E12, VEC, LB, KS_R2, KS_KS2>(a, t & ((1u << a.pb) - 1), t >> a.pb, sm, true);
    __syncthreads();
  }
}

// Row h of task (b, g) in the offs table; a KS_NONE row (no entry of the task in group h) reads as the next
// row (row hpg is always written)
__device__ __forceinline__ uint32_t ks_row(const KsArgs& a, int64_t g, int h, int b) {
  const int64_t P = 1 << a.pb;
  const uint32_t* p = a.offs + ((int64_t)g * (a.hpg + 1) + h) * P + b;
  uint32_t v = *p;
  while (v == KS_NONE && h < a.hpg) { h++; p += P; v = *p; }
  return v;
}

// records per order group h: sum over buckets of the task's offsets at h + 1 minus those at h
__global__ void __launch_bounds__(256) k_ks_order_count(KsArgs a, uint32_t* __restrict__ tot) {
  __shared__ uint32_t red[4];
  if (a.nflag[1]) return;                                     // the flush goes to the tile matcher
  const int h = blockIdx.x, g = h / a.hpg, hh = h - g * a.hpg;
  const int P = 1 << a.pb;
  uint32_t s = 0;
  for (int b = threadIdx.x; b < P; b += 256) s += ks_row(a, g, hh + 1, b) - ks_row(a, g, hh, b);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) tot[h] = red[0] + red[1] + red[2] + red[3];
}

constexpr int KS_ORDER_RPT = 8;                 // records per thread held in registers (4-word records)
constexpr int KS_ORDER_CAP = KS_ORDER_RPT * KS_ORDER_NT;

// One order group h: trigger indices [j0, j0 + KS_HQ).  Its records are one piece per bucket (the task's
// records with j in the group, already in (j, i) order).  Counting sort by j: a trigger's records are one
// run of one piece, so a record's place is its trigger's exclusive count plus its rank in that run.  Records
// are read once (consecutive threads, consecutive records of a piece) and kept in registers; groups with more
// than KS_ORDER_CAP records (or wider records) stream them twice.
// LDS (dynamic): hist[KS_HQ] u32 | pp[P + 1] u32 | sb[P] u32 | kk[KS_ORDER_CAP] u16
__global__ void __launch_bounds__(KS_ORDER_NT) k_ks_order(KsArgs a, const uint32_t* __restrict__ hbase,
                                                         int32_t* __restrict__ out) {
  extern __shared__ uint32_t ks_dyn[];
  __shared__ uint32_t wsum[KS_ORDER_NT / 64];
  if (a.nflag[1]) return;
  const int h = blockIdx.x, g = h / a.hpg, hh = h - g * a.hpg;
  const int P = 1 << a.pb;
  uint32_t* hist = ks_dyn;
  uint32_t* pp = hist + KS_HQ;
  uint32_t* sb = pp + P + 1;
  uint16_t* kk = (uint16_t*)(sb + P);
  const int t = threadIdx.x;
  for (int b = t; b < P; b += KS_ORDER_NT) {
    const uint32_t o0 = ks_row(a, g, hh, b);
    pp[b] = ks_row(a, g, hh + 1, b) - o0;
    sb[b] = a.tbase[(int64_t)b * a.nst + (int64_t)g * a.spg] + o0;
  }
  for (int k = t; k < KS_HQ; k += KS_ORDER_NT) hist[k] = 0;
  __syncthreads();
  const uint32_t total = kt_block_scan<KS_ORDER_NT>(pp, P, wsum);
  if (t == 0) pp[P] = total;
  __syncthreads();
  if (total == 0) return;
  const int64_t j0 = (int64_t)g * a.spg * KT_ST + (int64_t)hh * KS_HQ;
  const int S = a.stride;
  const int64_t ob = hbase[h];
  auto piece = [&](uint32_t r) -> int {        // last b with pp[b] <= r
    int lo = 0, hi = P - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pp[mid] <= r) lo = mid; else hi = mid - 1;
    }
    return lo;
  };
  if (S == 4 && total <= (uint32_t)KS_ORDER_CAP) {
    uint4 rv[KS_ORDER_RPT];
    uint16_t rb[KS_ORDER_RPT];
#pragma unroll
    for (int u = 0; u < KS_ORDER_RPT; u++) {
      const uint32_t r = (uint32_t)(t + u * KS_ORDER_NT);
      if (r < total) {
        const int b = piece(r);
        rb[u] = (uint16_t)b;
        rv[u] = *(const uint4*)(a.rec + ((int64_t)sb[b] + (r - pp[b])) * 4);
      }
    }
#pragma unroll
    for (int u = 0; u < KS_ORDER_RPT; u++) {
      const uint32_t r = (uint32_t)(t + u * KS_ORDER_NT);
      if (r < total) {
        const uint32_t key = (uint32_t)((int64_t)(int32_t)rv[u].x - j0);
        kk[r] = (uint16_t)key;
        atomicAdd(&hist[key], 1u);
      }
    }
    __syncthreads();
    kt_block_scan<KS_ORDER_NT>(hist, KS_HQ, wsum);
#pragma unroll
    for (int u = 0; u < KS_ORDER_RPT; u++) {
      const uint32_t r = (uint32_t)(t + u * KS_ORDER_NT);
      if (r < total) {
        const uint32_t key = kk[r], r0 = pp[rb[u]];
        uint32_t q = r;
        while (q > r0 && kk[q - 1] == key) q--;
        *(uint4*)(out + (ob + hist[key] + (r - q)) * 4) = rv[u];
      }
    }
    return;
  }
  // streaming form: any record width, any group size
  for (uint32_t r = t; r < total; r += KS_ORDER_NT) {
    const int b = piece(r);
    atomicAdd(&hist[(uint32_t)((int64_t)a.rec[((int64_t)sb[b] + (r - pp[b])) * S] - j0)], 1u);
  }
  __syncthreads();
  kt_block_scan<KS_ORDER_NT>(hist, KS_HQ, wsum);
  for (uint32_t r = t; r < total; r += KS_ORDER_NT) {
    const int b = piece(r);
    const int64_t src = (int64_t)sb[b] + (r - pp[b]);
    const int32_t j = a.rec[src * S];
    uint32_t rank = 0;
    for (int64_t q = src - 1; q >= (int64_t)sb[b] && a.rec[q * S] == j; q--) rank++;
    int32_t* dst = out + (ob + hist[(uint32_t)((int64_t)j - j0)] + rank) * S;
    for (int w = 0; w < S; w++) dst[w] = a.rec[src * S + w];
  }
}

inline size_t ks_order_lds(int P) { return ((size_t)KS_HQ + 2 * (size_t)P + 1) * 4 + (size_t)KS_ORDER_CAP * 2; }

}  // namespace sg
