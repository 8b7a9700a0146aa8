// keyed_chunks.hpp — chunk-sorted pipeline for SG_PATH_KEYED_FOLLOWED_BY (config 4, the bench path).
//
// Same closed form as keyed_tiles.hpp (PartitionStreamReceiver.java:82-282 routes each event to its key's
// instance; inside an instance `every e1=S[f1] -> e2=S[f2] within W` completes the partial of start i at
// m(i) = min{ j > i : k_j = k_i, ts_j - ts_i <= W, f2(i, j) }, emitted at j in ascending i --
// StreamPreStateProcessor.java:363-403, StreamPostStateProcessor.java:64-83), with a different HBM layout:
//
//   k_kc_sort    one workgroup per chunk of KC_C consecutive events: the chunk is counting-sorted by key bucket
//                b = key & (P-1) in LDS (stable: ballot-matched ranks + per-(wave, bucket) counters) and written
//                back CONTIGUOUSLY as 8-B entries, with one u16 row of bucket offsets per chunk.  Every store is
//                a whole line: no partial-line write amplification, and no global histogram pass.
//   k_kc_slices  time slices of KC_SPC chunks; each slice's back-halo starts at the first chunk that can hold an
//                event within W of the slice's first event (binary search over chunk end timestamps).
//   k_kc_match   one workgroup per (slice, bucket) tile, dealt XCD-contiguously (an XCD takes one eighth of the
//                buckets of a slice, so the tiles in flight on it read neighbouring runs of the same chunk lines
//                through its L2): the bucket's run of every chunk in [halo, slice end) is gathered into LDS, then
//                key-run sorted and walked as in k_kt_match (forward walks to m(i), per-trigger record counts,
//                records in (j, i) order).  Records go to a bump-allocated region per tile {offset, count}, and the
//                tile writes the order rows of the groups of its slice as one contiguous u16 run (keyed_order.hpp,
//                chunk mode).
//
// 8-B entry {x, y}: y = ts8 << 24 | start << 23 | chunk-local index << 10 | local key (key >> pb, 10 bits).
// ts8 = ts - (the chunk's first ts): a chunk spanning KC_TSPAN (256) ms or more sets the `wide` flag (the flush
// falls back to keyed_tiles.hpp).  The global index of an entry is chunk * KC_C + its chunk-local index.
//
// Algorithmic HBM bytes per event: input 16 B read once; 8-B entry written and read (1 + halo share) times;
// 0.5 B of bucket offsets; records 16 B per match written once, then moved once by the order pass.
#pragma once
#include <hip/hip_runtime.h>

#include "fb_shape.hpp"
#include "keyed_tiles.hpp"

namespace sg {

constexpr int KC_C = 8192;                  // events per chunk
constexpr int KC_CB = 13;                   // log2 KC_C (chunk-local index bits)
constexpr int KC_NT = 1024;                 // k_kc_sort threads (8 events each)
constexpr int KC_NCH = 1024;                // max chunks a matcher tile gathers (halo + slice)
constexpr int KC_TSB = 32 - 10 - KC_CB - 1; // bits of a chunk-relative timestamp (ts8)
constexpr int KC_TSPAN = 1 << KC_TSB;       // a chunk's timestamps must span less than this

struct KcArgs {
  // input columns
  const int64_t* ts;
  const uint32_t* keycol;
  const uint32_t* xcol;
  int32_t f1kind, f1op, f1t, f1w;
  const uint8_t* f1col;
  int64_t f1c;
  int64_t n, ts0, within, ts_last_rel;
  int32_t pb;                 // log2 buckets
  int64_t nchunks;
  // sorted chunks
  uint2* ent;                 // [nchunks * KC_C] entries, chunk-major, bucket-sorted inside a chunk
  uint16_t* off;              // [nchunks][P] chunk-local first entry of bucket b
  int64_t* cts0;              // [nchunks] first timestamp of each chunk
  uint32_t* flags;            // [0] carried starts, [1] overflow, [2] unsorted, [3] wide chunk
  // slices
  int32_t spc;                // chunks per slice (a multiple of KS_HQ / KC_C: slices hold whole order groups)
  int64_t nslices;
  int32_t* shalo;             // [nslices] first halo chunk
  // matcher outputs
  int32_t* rec;
  int32_t stride;
  uint32_t rcap;              // record slots available (the host reserves LC per tile: tile W's region starts at W * LC)
  uint2* tdir;                // [nslices * P] {first record slot, records} per tile (s * P + b)
  int32_t* carry;
  uint16_t* rows16;           // [nslices * P][gps] order rows (keyed_order.hpp, chunk mode): tile (s, b)'s first
                              // record with trigger index >= (s * gps + g) << hqb, relative to its tdir slot
  int32_t gps;                // order groups per slice (spc * KC_C >> hqb)
  int32_t hqb;                // log2 trigger indices per order group
  // projection
  int32_t nproj;
  int32_t src[FB_MAXP];
  int32_t w[FB_MAXP];
  const uint8_t* col[FB_MAXP];
  int32_t vec_rec;
  int32_t atomic_rank;        // ranks by LDS atomics (default; SG_KC_PEER_RANK: by ballot-matched peers)
  int32_t exp;                // measurement-only bits (SG_KC_EXP, wrong results): 1 matcher stops after the gather,
                              // 2 tiles dealt in plain (slice, bucket) order
  int64_t* dbg;               // phase timestamps (wall_clock64) of the first dbg_n matcher tiles, KC_NPROBE per tile
  int32_t dbg_n;
};
constexpr int KC_NPROBE = 12;

template <int F1W>
__device__ __forceinline__ void kc_load(const KcArgs& a, int64_t e, KtRaw<F1W>& r) {
  r.ts = a.ts[e];
  r.key = a.keycol[e];
  r.x = a.xcol[e];
  if constexpr (F1W == 8) r.f1 = ((const int64_t*)a.f1col)[e];
  else if constexpr (F1W == 4) r.f1 = ((const int32_t*)a.f1col)[e];
  else r.f1 = 0;
}

// LDS (dynamic, sized by P): hist[NW][P] u16, and the stage[KC_C] uint2 over it (every thread takes its entries'
// places from hist before the stage is written): max(64 KB, 2 NW P bytes)
inline size_t kc_sort_lds(int P, int nt) {
  return std::max((size_t)P * (nt / 64) * 2, (size_t)KC_C * 8) + KC_C / 8;   // + the bucket-start bitmap
}

template <int F1W, int NT = KC_NT>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(8))) k_kc_sort(KcArgs a) {
  extern __shared__ uint32_t kc_dyn[];
  __shared__ uint32_t wsum[NT / 64];
  constexpr int NW = NT / 64, RPW = KC_C / NT, QW = KC_C / NW;
  const int P = 1 << a.pb;
  const uint32_t mask = (uint32_t)P - 1;
  uint16_t* hist = (uint16_t*)kc_dyn;
  uint2* stage = (uint2*)kc_dyn;
  uint32_t* bstart = kc_dyn + max(P * NW / 2, KC_C * 2);   // [KC_C / 32]: positions where some bucket starts
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t c = blockIdx.x, e0 = c * KC_C;
  const int nc = (int)min<int64_t>(KC_C, a.n - e0);
  const int64_t tsc = a.ts[e0];
  KtRaw<F1W> r[RPW];
#pragma unroll
  for (int k = 0; k < RPW; k++) kc_load<F1W>(a, e0 + min(w * QW + k * 64 + lane, nc - 1), r[k]);
  for (int k = t; k < P * NW / 2; k += NT) kc_dyn[k] = 0;
  for (int k = t; k < KC_C / 32; k += NT) bstart[k] = 0;
  // non-decreasing timestamps (each event against its predecessor) and the chunk's span (9-bit ts8); the
  // predecessor comes by a DPP wave shift (lane 0: the previous round's lane 63, by readlane)
  {
    const int64_t q0 = e0 + w * QW;
    const int64_t tprev = a.ts[q0 > 0 ? q0 - 1 : 0];
    bool bad = false, wide = false;
    auto wave_shr1 = [](int64_t x) -> int64_t {        // lane i gets lane i - 1's value (lane 0: 0)
      const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, 0x138, 0xf, 0xf, true);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), 0x138, 0xf, 0xf, true);
      return (int64_t)((uint64_t)hi << 32 | lo);
    };
    auto lane63 = [](int64_t x) -> int64_t {
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63);
      return (int64_t)((uint64_t)hi << 32 | lo);
    };
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      const int64_t up = wave_shr1(r[k].ts);
      const int64_t last = k ? lane63(r[k - 1].ts) : tprev;
      const bool v = w * QW + k * 64 + lane < nc;
      bad |= v && r[k].ts < (lane ? up : last);
      wide |= v && r[k].ts - tsc >= KC_TSPAN;
    }
    if (__any(bad) && lane == 0) atomicOr(a.flags + 2, 1u);
    if (__any(wide) && lane == 0) atomicOr(a.flags + 3, 1u);
  }
  uint32_t bk[RPW];
  uint2 v[RPW];
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    const int q = w * QW + k * 64 + lane;
    bk[k] = r[k].key & mask;
    const bool st = F1W == 0 || cmp(a.f1op, a.f1t, r[k].f1v(), a.f1c);
    const uint32_t ts8 = (uint32_t)(r[k].ts - tsc) & (KC_TSPAN - 1);
    v[k] = make_uint2(r[k].x, (ts8 << (32 - KC_TSB)) | (st ? 1u << (10 + KC_CB) : 0u) | ((uint32_t)q << 10) |
                                  (r[k].key >> a.pb));
  }
  __syncthreads();
  // bk[k] becomes bucket | rank << 16, then the entry's place in the sorted chunk (one register per entry)
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    const bool valid = w * QW + k * 64 + lane < nc;
    const int h = w * P + (int)bk[k];
    if (a.atomic_rank) {          // an LDS atomic per entry (lane-ordered: the sorted runs are checked below)
      uint32_t old = 0;
      if (valid) old = atomicAdd((uint32_t*)hist + (h >> 1), 1u << (16 * (h & 1)));
      bk[k] |= ((old >> (16 * (h & 1))) & 0xffffu) << 16;
      continue;
    }
    const uint64_t peers = kt_match_peers_n(bk[k], valid, a.pb);
    const uint64_t below = peers & ((1ull << lane) - 1);
    const uint32_t hb = valid ? hist[h] : 0u;
    if (valid && below == 0) hist[h] = (uint16_t)(hb + __popcll(peers));
    bk[k] |= (hb + __popcll(below)) << 16;
  }
  __syncthreads();
  kt_scan_kw<NT, NW>(hist, P, wsum);        // (bucket, wave) order: hist[b] (wave 0) = bucket b's first entry
#pragma unroll
  for (int k = 0; k < RPW; k++) bk[k] = (uint32_t)hist[w * P + (int)(bk[k] & 0xffffu)] + (bk[k] >> 16);
  for (int b = t; b < P; b += NT) {
    const uint32_t h0 = hist[b];
    a.off[c * P + b] = (uint16_t)h0;
    if (a.atomic_rank && h0 < KC_C) atomicOr(bstart + (h0 >> 5), 1u << (h0 & 31));
  }
  if (t == 0) a.cts0[c] = tsc;
  __syncthreads();                          // hist is dead: the stage is written over it
#pragma unroll
  for (int k = 0; k < RPW; k++)
    if (w * QW + k * 64 + lane < nc) stage[bk[k]] = v[k];
  __syncthreads();
  // the sorted chunk leaves as one contiguous run: 16-B stores of entry pairs by consecutive lanes
  uint4* dst = (uint4*)(a.ent + e0);
  const uint4* sp = (const uint4*)stage;
  for (int l = t; l < nc / 2; l += NT) dst[l] = sp[l];
  if ((nc & 1) && t == 0) a.ent[e0 + nc - 1] = stage[nc - 1];
  if (a.atomic_rank) {
    // atomic ranks are stable only if the LDS serves a wave's same-address atomics in lane order: inside a bucket's
    // run the chunk-local indices must increase, or the flush goes to keyed_tiles.hpp
    bool bad = false;
    for (int l = 1 + t; l < nc; l += NT) {
      const uint32_t q1 = (stage[l].y >> 10) & (KC_C - 1), q0 = (stage[l - 1].y >> 10) & (KC_C - 1);
      bad |= q1 <= q0 && !((bstart[l >> 5] >> (l & 31)) & 1u);
    }
    if (bad) atomicOr(a.flags + 1, 1u);
  }
}

// first halo chunk of each slice: the first chunk whose last timestamp is within W of the slice's first event
__global__ void k_kc_slices(KcArgs a) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.nslices) return;
  const int64_t cb = s * a.spc;
  const int64_t tf = a.ts[cb * KC_C];
  auto tlast = [&](int64_t c) { return a.ts[min<int64_t>(a.n, (c + 1) * KC_C) - 1]; };
  int64_t lo = 0, hi = cb;                         // first c in [0, cb] with tlast(c) >= tf - W (cb if none)
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (tlast(mid) >= tf - a.within) hi = mid; else lo = mid + 1;
  }
  a.shalo[s] = (int32_t)lo;
}

// Matcher LDS: T = trigger capacity of a tile, LC = entry capacity (triggers + back-halo), NL = local keys.
template <int T, int LC, int NT, int NL>
struct KcMatchLds {
  static constexpr int L = LC;
  static constexpr int NW = NT / 64;
  union {
    uint16_t hist[NW * NL];             // [wave][key] counts -> key-run positions
    uint32_t rl[T];                     // record slot -> key-run positions: start | trigger << 16
    struct {
      uint32_t cts[KC_NCH];             // gather: each chunk's first timestamp, relative to the flush's
      uint16_t cpos[KC_NCH];            // gather: each chunk's first tile position (an overflowing tile is caught
                                        // by the scan's 32-bit total before any position is used)
      uint16_t co[KC_NCH];              // gather: the bucket's first entry inside each chunk
    };
  };
  union {
    struct {
      uint2 tx[L];                      // key-run order: {ts_rel | start << 31, x}
      uint32_t rr[L];                   // the position's local (arrival) position | its key run's end << 16
                                        // (then its global index)
    };
    struct {
      uint2 se[L];                      // gather: the raw entries in arrival order
      uint16_t sc[L];                   // gather: each entry's chunk (relative to the tile's first)
    };
  };
  uint16_t tc[T];                       // per-trigger record counts -> offsets (two u16 per word)
  uint32_t hdr[2];                      // record base, carry candidates
};

template <int OP, class V, int T, int LC, int NT, int NLB, int WPE>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE))) k_kc_match(KcArgs a) {
  constexpr int NL = 1 << NLB;
  using S = KcMatchLds<T, LC, NT, NL>;
  constexpr int L = S::L, NW = S::NW, RPW = (L + NT - 1) / NT;
  __shared__ S sm;
  __shared__ uint32_t wsum[NW];
  const uint32_t P = 1u << a.pb, g = blockIdx.x;
  uint32_t s, b;
#define KC_PROBE(i) \
  do { if (a.dbg && (int)g < a.dbg_n && threadIdx.x == 0) a.dbg[(int64_t)g * KC_NPROBE + (i)] = (int64_t)wall_clock64(); } while (0)
  KC_PROBE(0);
  if (P >= 8 && !(a.exp & 2)) {                   // XCD x = g % 8 takes buckets [x P/8, (x + 1) P/8) of a slice
    const uint32_t per = P >> 3, r = g >> 3;
    b = (g & 7) * per + r % per;
    s = r / per;
  } else {
    s = g / P;
    b = g % P;
  }
  if (s >= (uint32_t)a.nslices) return;
  const uint32_t W = s * P + b;
  const int64_t cb = (int64_t)s * a.spc, ce = min<int64_t>(cb + a.spc, a.nchunks), ch = a.shalo[s];
  const int nchk = (int)(ce - ch);
  const bool last = s + 1 == (uint32_t)a.nslices;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (nchk > KC_NCH) {                            // a back-halo of too many chunks: keyed_tiles.hpp takes the flush
    if (t == 0) atomicOr(a.flags + 1, 1u);
    return;
  }
  // gather: the bucket's run of each chunk, in chunk order (arrival order)
  // (unconditional loads: the last bucket's end is selected after the load, and cts needs only the low word)
  for (int i = t; i < nchk; i += NT) {
    const int64_t c = ch + i;
    const uint32_t o0 = a.off[c * P + b];
    const uint32_t o1n = a.off[c * P + min(b + 1, P - 1)];
    const uint32_t ct = ((const uint32_t*)a.cts0)[2 * c];
    const uint32_t o1 = b + 1 < P ? o1n : (uint32_t)min<int64_t>(KC_C, a.n - c * KC_C);
    sm.cpos[i] = (uint16_t)(o1 - o0);
    sm.co[i] = (uint16_t)o0;
    sm.cts[i] = ct - (uint32_t)a.ts0;
  }
  __syncthreads();
  KC_PROBE(1);
  const uint32_t Ln = kt_block_scan<NT>(sm.cpos, nchk, wsum);
  KC_PROBE(2);
  const int toff = (int)sm.cpos[cb - ch];         // first trigger position (the slice's first chunk)
  const int ntrig = (int)Ln - toff;
  if (Ln > (uint32_t)L || ntrig > T) {
    if (t == 0) atomicOr(a.flags + 1, 1u);
    return;
  }
  // the tile's record region: a fixed LC slots per tile (records <= starts <= Ln <= LC), so no tile waits on a
  // global cursor (a bump allocator's returning atomic on one address held every tile's gather behind its vmcnt)
  if (t == 0) sm.hdr[0] = W * (uint32_t)L;
  {
    // groups of KC_G lanes copy one chunk's run each (lane l: entries l, l + KC_G, ...): the loads of a wave's
    // KC_RU rounds are issued back to back, with no dependence between them
    // Only the loaded entries are held across the round (run bounds are read from LDS again when they land), and
    // every load is unconditional at a clamped in-bounds address (a load under a branch is merged with the
    // branch's default at the join, where the compiler then waits for it).
    constexpr int KC_G = 8, NG = NT / KC_G, KC_RU = (KC_NCH + NG - 1) / NG > 8 ? 8 : (KC_NCH + NG - 1) / NG;
    const int gi = t / KC_G, gl = t % KC_G;
    const int64_t emax = a.nchunks * KC_C - 1;
    auto run = [&](int i, uint32_t& p0, uint32_t& len) {
      p0 = sm.cpos[i];
      len = (i + 1 < nchk ? (uint32_t)sm.cpos[i + 1] : Ln) - p0;
    };
    for (int i0 = 0; i0 < nchk; i0 += NG * KC_RU) {
      uint32_t ex[KC_RU], ey[KC_RU];
#pragma unroll
      for (int u = 0; u < KC_RU; u++) {
        const int i = min(i0 + u * NG + gi, nchk - 1);
        uint32_t p0, len;
        run(i, p0, len);
        const uint2 e = a.ent[min<int64_t>((ch + i) * KC_C + sm.co[i] + min((uint32_t)gl, len ? len - 1 : 0u), emax)];
        ex[u] = e.x;
        ey[u] = e.y;
      }
#pragma unroll
      for (int u = 0; u < KC_RU; u++) {
        const int i = i0 + u * NG + gi;
        if (i >= nchk) continue;
        uint32_t p0, len;
        run(i, p0, len);
        if ((uint32_t)gl < len) { sm.se[p0 + gl] = make_uint2(ex[u], ey[u]); sm.sc[p0 + gl] = (uint16_t)i; }
        for (uint32_t r = gl + KC_G; r < len; r += KC_G) {           // a run longer than the group (rare)
          sm.se[p0 + r] = a.ent[(ch + i) * KC_C + sm.co[i] + r];
          sm.sc[p0 + r] = (uint16_t)i;
        }
      }
    }
  }
  __syncthreads();
  KC_PROBE(3);
  const int64_t hs0 = (cb * KC_C) >> a.hqb;      // the slice's first order group
  uint16_t* rows = a.rows16 + (int64_t)W * a.gps;
  const uint32_t w32 = (uint32_t)min<int64_t>(a.within, 0x7fffffff);
  const int Lni = (int)Ln;
  const int CW = ((Lni + NW * 64 - 1) / (NW * 64)) * 64;
  const int p0 = w * CW;
  uint4 v[RPW];                                   // logical entries {global index, ts_rel | start << 31, x, local key}
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    const int p = min(p0 + k * 64 + lane, max(Lni - 1, 0));
    const uint2 e = sm.se[p];
    const uint32_t cc = sm.sc[p];
    const uint32_t gi = (uint32_t)((ch + cc) * KC_C + ((e.y >> 10) & (KC_C - 1)));
    const uint32_t tsr = sm.cts[cc] + (e.y >> (32 - KC_TSB));
    v[k] = make_uint4(gi, tsr | ((e.y >> (10 + KC_CB)) & 1u) << 31, e.x, e.y & (NL - 1));
  }
  __syncthreads();                                // cpos / cts and se / sc are dead from here
  KC_PROBE(4);
  if (a.exp & 1) { if (a.dbg) { KC_PROBE(11); } return; }
  if (Lni == 0) {
    if (t == 0) a.tdir[W] = make_uint2(0u, 0u);
    for (int g = t; g < a.gps; g += NT) rows[g] = 0;
    return;
  }
  for (int k = t; k < NL * NW / 2; k += NT) ((uint32_t*)sm.hist)[k] = 0;
  for (int k = t; k < T / 2; k += NT) ((uint32_t*)sm.tc)[k] = 0;
  __syncthreads();
  uint16_t rk[RPW];
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    const int p = p0 + k * 64 + lane;
    const bool valid = p < min(p0 + CW, Lni);
    if (k * 64 >= CW) { rk[k] = 0; continue; }   // wave-uniform
    const uint32_t key = v[k].w;
    const int hidx = w * NL + (int)(key & (NL - 1));
    if (a.atomic_rank) {                          // an LDS atomic per entry: its return is the rank (stable: checked below)
      uint32_t old = 0;
      if (valid) old = atomicAdd((uint32_t*)sm.hist + (hidx >> 1), 1u << (16 * (hidx & 1)));
      rk[k] = (uint16_t)(old >> (16 * (hidx & 1)));
      continue;
    }
    const uint64_t peers = kt_match_peers<NLB>(key, valid);
    const uint64_t below = peers & ((1ull << lane) - 1);
    const uint32_t hb = valid ? sm.hist[hidx] : 0u;
    if (valid && below == 0) sm.hist[hidx] = (uint16_t)(hb + __popcll(peers));
    rk[k] = (uint16_t)(hb + __popcll(below));
  }
  __syncthreads();
  KC_PROBE(5);
  kt_scan_kw<NT, NW>(sm.hist, NL, wsum);
  KC_PROBE(6);
  uint32_t dq[RPW], gk[RPW];                      // after the place: key-run position | local key << 16, global index
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    const int p = p0 + k * 64 + lane;
    dq[k] = 0xffffffffu;
    gk[k] = v[k].x;
    if (k * 64 < CW && p < min(p0 + CW, Lni)) {
      const int key = (int)v[k].w;
      const int q = sm.hist[w * NL + key] + rk[k];
      dq[k] = (uint32_t)q | (uint32_t)key << 16;
      sm.tx[q] = make_uint2(v[k].y, v[k].z);
      sm.rr[q] = (uint32_t)p | ((key + 1 < NL ? (uint32_t)sm.hist[key + 1] : (uint32_t)Lni) << 16);
    }
  }
  __syncthreads();
  KC_PROBE(7);
  // forward walks: every start walks its key run to m(i), the first later entry within W with x_m OP x_i; the
  // record belongs to this tile when m is one of its triggers (fm = m | rank << 12 | m's trigger index << 19);
  // fm = KC_CARRY: the slice is the flush's last and the start is still open at its end (carried)
  constexpr uint32_t KC_CARRY = 0xfffffffeu;
  uint32_t fm[RPW];                               // m | rank << 12 | trigger index << 19 (rank saturates at 127:
                                                  // more than KT_MAXREC records for a trigger overflow the tile)
  {
    uint2 ti[RPW], tn[RPW];
    int re[RPW];
    bool unstable = false;
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      const int q = min(t + k * NT, Lni - 1);
      ti[k] = sm.tx[q];
      const uint32_t rq = sm.rr[q];
      re[k] = (int)(rq >> 16);
      tn[k] = sm.tx[min(q + 1, Lni - 1)];
      fm[k] = 0xffffffffu;
      // atomic ranks rely on the LDS serving a wave's same-address atomics in lane order: a key run whose arrival
      // positions do not increase sends the flush to keyed_tiles.hpp instead of matching out of order
      if (a.atomic_rank && q + 1 < re[k]) unstable |= (sm.rr[q + 1] & 0xffffu) <= (rq & 0xffffu);
    }
    if (unstable) atomicOr(a.flags + 1, 1u);
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      if (k * NT >= Lni) break;                                    // uniform
      const int q = t + k * NT;
      const bool st = q < Lni && (ti[k].x >> 31);
      const uint32_t tsi = ti[k].x & 0x7fffffffu;
      const V xi = kt_val<V>(ti[k].y);
      int r = q + 1, m = -1;
      bool act = st && r < re[k], expired = false;
      uint2 tr = tn[k];
      while (act) {
        if ((tr.x & 0x7fffffffu) - tsi > w32) { expired = true; act = false; }
        else if (cmpv<OP, V>(kt_val<V>(tr.y), xi)) { m = r; act = false; }
        else if (++r >= re[k]) act = false;
        else tr = sm.tx[r];
      }
      if (m >= 0) {
        const int lj = (int)(sm.rr[m] & 0xffffu) - toff;
        if (lj >= 0) fm[k] = (uint32_t)m | min(kt_tc_add(sm.tc, lj, 1u), 127u) << 12 | (uint32_t)lj << 19;
      } else if (last && st && !expired && (uint32_t)a.ts_last_rel - tsi <= w32) {
        fm[k] = KC_CARRY;
      }
    }
  }
  __syncthreads();
  KC_PROBE(8);
  // the walks are done: each owner deposits its entry's global index over the run bounds and its local key over
  // the timestamp half of tx (x stays), so the record writes and carries read only LDS
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    if (dq[k] != 0xffffffffu) {
      sm.rr[dq[k] & 0xffffu] = gk[k];
      sm.tx[dq[k] & 0xffffu].x = dq[k] >> 16;
    }
  }
  const uint32_t nrec = kt_scan16<NT, T>(sm.tc, wsum);             // (its barriers order the deposits)
  if (nrec > (uint32_t)T) {
    if (t == 0) atomicOr(a.flags + 1, 1u);
    return;
  }
  if (t == 0) {
    a.tdir[W] = make_uint2(sm.hdr[0], nrec);
    if (nrec) atomicAdd(a.flags + 5, nrec);       // the matcher's own record count: the host checks the order pass's
  }
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    if (fm[k] == KC_CARRY) a.carry[atomicAdd(a.flags, 1u)] = (int32_t)sm.rr[t + k * NT];
    else if (fm[k] != 0xffffffffu) {
      const uint32_t m = fm[k] & 0xfffu, rank = (fm[k] >> 12) & 0x7fu;
      sm.rl[sm.tc[fm[k] >> 19] + rank] = (uint32_t)(t + k * NT) | (m << 16);
    }
  }
  __syncthreads();
  const uint32_t base = sm.hdr[0];
  if ((uint64_t)base + Ln > a.rcap) {             // (a guard: the host reserves LC slots per tile)
    if (t == 0) atomicOr(a.flags + 1, 1u);
    return;
  }
  // each trigger sorts its (few) slots by start position (arrival order inside the key run): records in ascending
  // i; more than KT_MAXREC records for one trigger (a long falling run) send the flush to another pipeline
  {
    bool sat = false;
    static_assert(T % NT == 0, "whole rounds of triggers");
#pragma unroll
    for (int u = 0; u < T / NT; u++) {            // (unrolled: the count reads of every round issue together)
      const int lj = t + u * NT;
      if (lj >= ntrig) continue;
      const uint32_t o = sm.tc[lj];
      const uint32_t cnt = (lj + 1 < T ? (uint32_t)sm.tc[lj + 1] : nrec) - o;
      if (cnt < 2) continue;
      if (cnt > KT_MAXREC) { sat = true; continue; }
      for (uint32_t x = 1; x < cnt; x++) {
        const uint32_t v0 = sm.rl[o + x];
        uint32_t y = x;
        while (y > 0 && sm.rl[o + y - 1] > v0) { sm.rl[o + y] = sm.rl[o + y - 1]; y--; }
        sm.rl[o + y] = v0;
      }
    }
    if (sat) atomicOr(a.flags + 1, 1u);
  }
  __syncthreads();
  KC_PROBE(9);
  // records whose projections all come from the tile (key, x_i, x_j): no global loads, so the stores of
  // successive records are not serialised behind a wait for a possible load
  const bool from_tile = a.vec_rec && a.stride == 4 && a.nproj == 2 && a.src[0] <= KT_XJ && a.src[1] <= KT_XJ;
  if (from_tile) {
    for (uint32_t r = t; r < nrec; r += NT) {
      const uint32_t pr = sm.rl[r];
      const int q = (int)(pr & 0xffffu), m = (int)(pr >> 16);
      const uint2 ti = sm.tx[q];
      const uint32_t xj = sm.tx[m].y, ig = sm.rr[q], jg = sm.rr[m];
      auto pj = [&](int c) -> uint32_t {
        return a.src[c] == KT_KEY ? (ti.x << a.pb) | b : a.src[c] == KT_XI ? ti.y : xj;
      };
      *(uint4*)(a.rec + (int64_t)(base + r) * 4) = make_uint4(jg, ig, pj(0), pj(1));
    }
  }
  for (uint32_t r = from_tile ? nrec : t; r < nrec; r += NT) {
    const uint32_t pr = sm.rl[r];
    const int q = (int)(pr & 0xffffu), m = (int)(pr >> 16);
    const uint2 ti = sm.tx[q];                                      // {local key, x} of the start
    const uint32_t ig = sm.rr[q], jg = sm.rr[m];
    int32_t* rp = a.rec + (int64_t)(base + r) * a.stride;
    auto proj = [&](int c) -> int64_t {
      switch (a.src[c]) {
        case KT_KEY: return (int32_t)((ti.x << a.pb) | b);
        case KT_XI: return (int32_t)ti.y;
        case KT_XJ: return (int32_t)sm.tx[m].y;
        default: {
          const int64_t gi = a.src[c] == KT_COL_I ? ig : jg;
          return a.w[c] == 2 ? ((const int64_t*)a.col[c])[gi] : (int64_t)((const int32_t*)a.col[c])[gi];
        }
      }
    };
    if (a.vec_rec && a.stride == 4 && a.nproj == 2) {
      *(uint4*)rp = make_uint4(jg, ig, (uint32_t)proj(0), (uint32_t)proj(1));
    } else {
      rp[0] = (int32_t)jg;
      rp[1] = (int32_t)ig;
      int wo = 2;
      for (int c = 0; c < a.nproj; c++) {
        const int64_t val = proj(c);
        rp[wo] = (int32_t)val;
        if (a.w[c] == 2) rp[wo + 1] = (int32_t)(val >> 32);
        wo += a.w[c];
      }
    }
  }
  // order rows of the slice's groups: row g = the first record with trigger index >= (hs0 + g) << hqb (records are
  // in (j, i) order), so record r writes the rows of the groups after its predecessor's, up to its own; the rows
  // after the last record's group hold nrec
  {
    auto grp = [&](uint32_t r) { return (int)(((int64_t)sm.rr[sm.rl[r] >> 16] >> a.hqb) - hs0); };
    for (uint32_t r = t; r < nrec; r += NT) {
      const int g1 = grp(r), g0 = r ? grp(r - 1) : -1;
      for (int g = g0 + 1; g <= g1; g++) rows[g] = (uint16_t)r;
    }
    const int gl = nrec ? grp(nrec - 1) : -1;
    for (int g = gl + 1 + t; g < a.gps; g += NT) rows[g] = (uint16_t)nrec;
  }
  if (a.dbg) { __syncthreads(); KC_PROBE(11); }
#undef KC_PROBE
}

}  // namespace sg
