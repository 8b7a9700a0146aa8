// keyed_tiles.hpp — bucketed-tile pipeline for SG_PATH_KEYED_FOLLOWED_BY (config 4, the bench path).
//
// Same closed form as keyed_fb.hip (PartitionStreamReceiver.java:82-282 routes each event to its
// key's instance; inside an instance `every e1=S[f1] -> e2=S[f2] within W` completes the partial of
// start i at m(i) = min{ j > i : k_j = k_i, ts_j - ts_i <= W, f2(i, j) }, emitted at j in ascending
// i — StreamPreStateProcessor.java:363-403, StreamPostStateProcessor.java:64-83), computed without a
// global sort:
//
//   k_kt_hist     per super-tile (KT_ST events) histogram of key buckets b = key & (P-1)
//   scan          exclusive scan of the [bucket][super-tile] counts -> stable scatter bases
//   k_kt_buckets  bucket starts + tile prefix; k_kt_tdesc: bucket-major tile table with exact back-halos
//   k_kt_scatter  stable partition by bucket: 16-B entries {idx, ts_rel|start<<31, x, lkey}.  Inside
//                 a bucket entries stay in arrival order, so every key's events are in time order.
//   k_kt_match    one workgroup per (bucket, tile of T triggers).  The tile plus its back-halo (the
//                 bucket's entries with ts >= ts_first - W, at most KT_H) is staged in LDS, counting-
//                 sorted by local key (lkey = key >> log2 P, < 2^KT_LB), and every start walks its
//                 key run forward to m(i).  A trigger j of the tile then walks back over its key run
//                 (only entries within W can have m = j) and writes its records in ascending i.
//
// HBM layout of the output: records {j, i, projection words} grouped per tile, in (j, i) order inside
// a tile; tiles of a bucket are placed in its own region by a per-bucket cursor and listed in a tile
// directory {offset, count}.  The reference's global order (ascending j, then i) is the merge by j of
// the tiles, decoded in one linear pass over the key column (KeyedFollowedByExec::materialise_tiled).
//
// Fallbacks (never silently wrong): a back-halo longer than KT_H sets the overflow flag and the flush
// is re-run by the packed sort pipeline; shapes outside the fast atom (or >2^(KT_LB+12) key values,
// no `within`, carried starts) use the sort pipelines from the start.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "fb_shape.hpp"

namespace sg {

constexpr int KT_NT = 512;          // threads per workgroup (8 waves): partition kernels
constexpr int KM_NT = 1024;         // threads per workgroup (16 waves): matcher
constexpr int KT_LB = 10;           // local-key bits per bucket
constexpr int KT_NL = 1 << KT_LB;   // local keys per bucket
constexpr int KT_MAXPB = 12;        // at most 4096 buckets
constexpr int KT_ST = 65536;        // scatter super-tile (events per workgroup)
constexpr int KT_H = 2048;          // max back-halo entries (matcher tiles: T = 2048 or 4096 triggers)
constexpr uint32_t KT_MAXREC = 64;  // records per trigger in one matcher tile (more: overflow fallback)

__device__ __forceinline__ uint32_t kt_wave_scan(uint32_t x) { return sg_wave_scan(x); }

// exclusive scan in place of n values in LDS (thread t owns a contiguous run); returns the total
template <int NT, class T>
__device__ __forceinline__ uint32_t kt_block_scan(T* a, int n, uint32_t* wsum) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int ipt = (n + NT - 1) / NT, b0 = min(t * ipt, n), b1 = min(b0 + ipt, n);
  uint32_t loc = 0;
  for (int k = b0; k < b1; k++) loc += a[k];
  const uint32_t inc = kt_wave_scan(loc);
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; k++) {
    const uint32_t v = wsum[k];
    base += k < w ? v : 0;
    tot += v;
  }
  uint32_t run = base + inc - loc;
  for (int k = b0; k < b1; k++) {
    const uint32_t v = a[k];
    a[k] = (T)run;
    run += v;
  }
  __syncthreads();
  return tot;
}

// Stable in-wave rank of a local key among the lanes of one round: `peers` = lanes holding the same
// key, by ballot matching one bit at a time.  x is all-ones where the lane's bit is 0, so `bb ^ x`
// keeps the lanes that agree with this lane on the bit (two 3-input bit ops per bit on gfx950).
template <int NB>
__device__ __forceinline__ uint64_t kt_match_peers(uint32_t key, bool valid) {
  const uint64_t vb = __ballot(valid);
  uint32_t plo = (uint32_t)vb, phi = (uint32_t)(vb >> 32);
  const uint32_t nk = ~key;
#pragma unroll
  for (int bt = 0; bt < NB; bt++) {
    const uint32_t x = (uint32_t)((int32_t)(nk << (31 - bt)) >> 31);
    const uint64_t bb = __ballot(x == 0u);
    plo &= (uint32_t)bb ^ x;
    phi &= (uint32_t)(bb >> 32) ^ x;
  }
  return ((uint64_t)phi << 32) | plo;
}

__device__ __forceinline__ uint64_t kt_match_peers_n(uint32_t key, bool valid, int nb) {
  const uint64_t vb = __ballot(valid);
  uint32_t plo = (uint32_t)vb, phi = (uint32_t)(vb >> 32);
  const uint32_t nk = ~key;
  for (int bt = 0; bt < nb; bt++) {
    const uint32_t x = (uint32_t)((int32_t)(nk << (31 - bt)) >> 31);
    const uint64_t bb = __ballot(x == 0u);
    plo &= (uint32_t)bb ^ x;
    phi &= (uint32_t)(bb >> 32) ^ x;
  }
  return ((uint64_t)phi << 32) | plo;
}

// exclusive scan, in (key, wave) order, of counters laid out [wave][key] (nk keys); thread t owns a
// contiguous key range, so lanes read consecutive keys (conflict-free) -- returns the total
template <int NT, int NW>
__device__ __forceinline__ uint32_t kt_scan_kw(uint16_t* h, int nk, uint32_t* wsum) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int kpt = (nk + NT - 1) / NT, k0 = min(t * kpt, nk), k1 = min(k0 + kpt, nk);
  uint32_t loc = 0;
  for (int k = k0; k < k1; k++) {
#pragma unroll
    for (int v = 0; v < NW; v++) loc += h[v * nk + k];
  }
  const uint32_t inc = kt_wave_scan(loc);
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; k++) {
    const uint32_t v = wsum[k];
    base += k < w ? v : 0;
    tot += v;
  }
  uint32_t run = base + inc - loc;
  for (int k = k0; k < k1; k++) {
#pragma unroll
    for (int v = 0; v < NW; v++) {
      const uint32_t c = h[v * nk + k];
      h[v * nk + k] = (uint16_t)run;
      run += c;
    }
  }
  __syncthreads();
  return tot;
}

struct KtArgs {
  // input columns
  const int64_t* ts;
  const uint32_t* keycol;
  const uint32_t* xcol;
  int32_t f1kind, f1op, f1t, f1w;
  const uint8_t* f1col;
  int64_t f1c;
  int64_t n, ts0, within;
  int64_t lo;                 // events [0, lo) are carried starts of earlier flushes: never triggers
  int32_t pb;                 // log2 buckets
  int32_t tile_t;             // triggers per matcher tile
  int32_t vec_rec;            // write 4-word records with one 16-B store
  int64_t* dbg;               // phase timestamps (wall_clock64) of the first dbg_n matcher tiles, 8 per tile
  int32_t dbg_n;
  int32_t exp;                // measurement-only bits (SG_KT_EXP): 1 scatter stores to the dummy slot
  int32_t nst;                // super-tiles
  int32_t ent12;              // entries are 12 B (KtE12): relative timestamps fit 21 bits
  // partition
  uint32_t* hist;             // [P * nst] counts -> exclusive bases
  uint4* ent;                 // [n + 1] bucketed entries (+ the scatter's dummy slot)
  // tiles
  int64_t ntiles_max;         // tile-table slots (an upper bound: n / T + P + 1)
  uint32_t* bstart;           // [P + 1] bucket start (entries)
  uint32_t* tprefix;          // [P + 1] exclusive prefix of tiles per bucket
  uint4* tdesc;               // [ntiles_max] {bucket, first trigger, end, halo start} (x = 0xffffffff: none)
  // matcher outputs
  int32_t* rec;               // records, `stride` int32 words each
  int32_t stride;
  uint32_t* bcur;             // [P] per-bucket record totals (start at bstart)
  uint2* tdir;                // [ntiles_max] {offset, count}
  int32_t* carry;
  uint32_t* ncarry;
  uint32_t* overflow;
  uint32_t* unsorted;         // set when the timestamps go backwards (device-resident input is unchecked)
  int64_t ts_last_rel;
  // projection
  int32_t nproj;
  int32_t src[FB_MAXP];
  int32_t w[FB_MAXP];
  const uint8_t* col[FB_MAXP];
  // trigger-order groups (k_kt_order): rows [nh + 1][P] of {record slot, tile} -- the slot of the first record
  // of the bucket whose trigger index is >= h << 14, inside that tile's records; each group boundary is
  // written by the one tile of the bucket whose trigger range reaches it (null: not ordered on the device)
  uint2* toffs;
  int64_t nh;
  int32_t xcd_tiles;          // matcher grid is XCD-contiguous over the tile table (kt_xcd_index)
};

// XCD-contiguous index of workgroup g in a grid of 8 * ceil(n / 8): XCD g % 8 takes [x * per, (x + 1) * per)
__device__ __forceinline__ uint32_t kt_xcd_index(uint32_t g, uint32_t n) {
  const uint32_t per = (n + 7) / 8;
  return (g & 7) * per + (g >> 3);
}

constexpr int KT_HQB = 14;                  // log2 trigger indices per order group (= keyed_stack.hpp KS_HQB)

// The order-group rows this tile is responsible for: groups h whose first trigger index h << KT_HQB lies after
// the previous tile's last trigger of the bucket (every group from 0 for the bucket's first tile) and at or
// before this tile's last trigger (every remaining group for the bucket's last tile).  off(h) = records of the
// tile with j < h << KT_HQB, by binary search over the tile's records (ascending j); jrec(r) = j of record r.
// A row holds the absolute slot base + off(h) and the tile, so the order pass reads a piece that stays in one
// tile without the tile directory.
template <class JRec>
__device__ void kt_write_toffs(const KtArgs& a, uint32_t b, uint32_t w, uint32_t base, int64_t jprev, int64_t jlast,
                               bool last, uint32_t nrec, JRec&& jrec) {
  const int64_t P = (int64_t)1 << a.pb;
  const int64_t hlo = jprev < a.lo ? 0 : (jprev >> KT_HQB) + 1;
  const int64_t hhi = last ? a.nh : min<int64_t>(a.nh, jlast >> KT_HQB);
  for (int64_t h = hlo + threadIdx.x; h <= hhi; h += blockDim.x) {
    const int64_t hs = h << KT_HQB;
    uint32_t l = 0, r = nrec;
    while (l < r) {
      const uint32_t m = (l + r) >> 1;
      if ((int64_t)jrec(m) < hs) l = m + 1; else r = m;
    }
    a.toffs[h * P + b] = make_uint2(base + l, w);
  }
}

// Entry formats.  16 B: {idx, ts_rel | start << 31, x, local key}.  12 B (when the flush's relative
// timestamps fit 21 bits, e.g. 35 minutes of milliseconds): {idx, start << 31 | ts_rel << 10 | local key, x}
// -- a quarter less scatter write and matcher read traffic.  kt_put / kt_get convert from / to the 16-B
// logical form; the array is addressed in entries of the format's size.
struct KtE12 {
  uint32_t idx, y, x;
};
template <bool E12>
__device__ __forceinline__ void kt_put(void* ent, int64_t i, uint4 v) {
  if constexpr (E12) {
    KtE12 e;
    e.idx = v.x;
    e.y = (v.y & 0x80000000u) | ((v.y & 0x1fffffu) << KT_LB) | v.w;
    e.x = v.z;
    ((KtE12*)ent)[i] = e;
  } else {
    ((uint4*)ent)[i] = v;
  }
}
template <bool E12>
__device__ __forceinline__ uint4 kt_get(const void* ent, int64_t i) {
  if constexpr (E12) {
    const KtE12 e = ((const KtE12*)ent)[i];
    return make_uint4(e.idx, (e.y & 0x80000000u) | ((e.y >> KT_LB) & 0x1fffffu), e.x, e.y & (KT_NL - 1));
  } else {
    return ((const uint4*)ent)[i];
  }
}

__global__ void __launch_bounds__(KT_NT) k_kt_hist(KtArgs a) {
  __shared__ uint32_t h[1 << KT_MAXPB];
  const int P = 1 << a.pb;
  for (int b = threadIdx.x; b < P; b += KT_NT) h[b] = 0;
  __syncthreads();
  const int64_t e0 = (int64_t)blockIdx.x * KT_ST, e1 = min<int64_t>(e0 + KT_ST, a.n);
  const uint32_t mask = (uint32_t)P - 1;
  // 16-B loads (4 keys per lane, super-tiles are 16-B aligned: KT_ST % 4 == 0), 4 loads in flight per lane
  const bool al16 = ((uintptr_t)a.keycol & 15) == 0;                // caller-owned column: check
  const int64_t v1 = al16 ? e0 + ((e1 - e0) & ~(int64_t)(4 * 4 * KT_NT - 1)) : e0;
  for (int64_t e = e0 + 4 * threadIdx.x; e < v1; e += 4 * 4 * KT_NT) {
    uint4 k[4];
#pragma unroll
    for (int u = 0; u < 4; u++) k[u] = *(const uint4*)(a.keycol + e + (int64_t)u * 4 * KT_NT);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      atomicAdd(&h[k[u].x & mask], 1u);
      atomicAdd(&h[k[u].y & mask], 1u);
      atomicAdd(&h[k[u].z & mask], 1u);
      atomicAdd(&h[k[u].w & mask], 1u);
    }
  }
  for (int64_t e = v1 + threadIdx.x; e < e1; e += KT_NT) atomicAdd(&h[a.keycol[e] & mask], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < P; b += KT_NT) a.hist[(int64_t)b * a.nst + blockIdx.x] = h[b];
}

// bucket starts, per-bucket record cursors and the exclusive prefix of tiles per bucket (one workgroup)
__global__ void __launch_bounds__(KT_NT) k_kt_buckets(KtArgs a) {
  __shared__ uint32_t tc[1 << KT_MAXPB];
  __shared__ uint32_t wsum[KT_NT / 64];
  const int P = 1 << a.pb;
  for (int b = threadIdx.x; b < P; b += KT_NT) {
    const uint32_t s0 = a.hist[(int64_t)b * a.nst];
    const uint32_t s1 = b + 1 < P ? a.hist[(int64_t)(b + 1) * a.nst] : (uint32_t)a.n;
    a.bstart[b] = s0;
    a.bcur[b] = s0;
    tc[b] = (s1 - s0 + a.tile_t - 1) / a.tile_t;
  }
  if (threadIdx.x == 0) a.bstart[P] = (uint32_t)a.n;
  __syncthreads();
  const uint32_t total = kt_block_scan<KT_NT>(tc, P, wsum);
  for (int b = threadIdx.x; b < P; b += KT_NT) a.tprefix[b] = tc[b];
  if (threadIdx.x == 0) a.tprefix[P] = total;
}

// matcher tile table, bucket-major (consecutive workgroups take consecutive tiles of a bucket, so a tile's
// back-halo is the L2-resident tail of the previous one; a tile-major order measured 40 % slower).  Entry
// w: {bucket, first trigger, end, first halo entry} (bucket-relative; x = 0xffffffff: no such tile).  The
// back-halo is exact: the first entry within W of the tile's first trigger, by binary search over the
// (non-decreasing) timestamps of the KT_H entries before it.  A window reaching further back than KT_H
// entries raises the overflow flag (the flush is re-run by the sort pipeline).
__global__ void __launch_bounds__(KT_NT) k_kt_tdesc(KtArgs a) {
  const int64_t w = (int64_t)blockIdx.x * KT_NT + threadIdx.x;
  if (w >= a.ntiles_max) return;
  const int P = 1 << a.pb;
  if (w >= a.tprefix[P]) { a.tdesc[w] = make_uint4(0xffffffffu, 0, 0, 0); return; }
  int lo = 0, hi = P - 1;                       // last b with tprefix[b] <= w (the non-empty one)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (a.tprefix[mid] <= (uint32_t)w) lo = mid; else hi = mid - 1;
  }
  const uint32_t b = (uint32_t)lo, tile = (uint32_t)w - a.tprefix[lo];
  const uint32_t B0 = a.bstart[b], nb = a.bstart[b + 1] - B0;
  uint32_t s = tile * (uint32_t)a.tile_t;
  const uint32_t e = min(s + (uint32_t)a.tile_t, nb);
  auto tsat = [&](uint32_t p) {
    return a.ent12 ? (int64_t)((((const KtE12*)a.ent)[B0 + p].y >> KT_LB) & 0x1fffffu)
                   : (int64_t)(a.ent[B0 + p].y & 0x7fffffffu);
  };
  auto idxat = [&](uint32_t p) { return a.ent12 ? ((const KtE12*)a.ent)[B0 + p].idx : a.ent[B0 + p].x; };
  if (a.lo > 0 && idxat(s) < (uint64_t)a.lo) {
    // carried starts lead the bucket (arrival order): the tile's triggers begin at the first new event
    uint32_t l = s, h = e;
    while (l < h) {
      const uint32_t mid = (l + h) >> 1;
      if (idxat(mid) < (uint64_t)a.lo) l = mid + 1; else h = mid;
    }
    s = l;
    if (s == e && e != nb) { a.tdesc[w] = make_uint4(0xffffffffu, 0, 0, 0); return; }   // no trigger, not last
  }
  // the back-halo reaches W before the first trigger (a trigger-less last tile: before the flush's last
  // timestamp, for the starts it carries on)
  const int64_t tsf = s < e ? tsat(s) : a.ts_last_rel;
  uint32_t l = s > KT_H ? s - KT_H : 0, h = s;    // first p in [l, s] with tsf - ts_p <= W
  if (l > 0 && tsf - tsat(l - 1) <= a.within) atomicOr(a.overflow, 1u);
  while (l < h) {
    const uint32_t mid = (l + h) >> 1;
    if (tsf - tsat(mid) <= a.within) h = mid; else l = mid + 1;
  }
  a.tdesc[w] = make_uint4(b, s, e, l);
}

__device__ __forceinline__ bool kt_start(const KtArgs& a, int64_t e) {
  if (a.f1kind != 1) return true;
  const int64_t v = a.f1w == 8 ? ((const int64_t*)a.f1col)[e] : (int64_t)((const int32_t*)a.f1col)[e];
  return cmp(a.f1op, a.f1t, v, a.f1c);
}

// one event's columns in registers; F1W = bytes of the start filter's column (0: no filter, 1: the
// filter compares the x column itself, 4 / 8: a column of its own)
template <int F1W>
struct KtRaw {
  int64_t ts;
  uint32_t key, x;
  std::conditional_t<F1W == 8, int64_t, int32_t> f1;
  __device__ __forceinline__ int64_t f1v() const {
    if constexpr (F1W == 1) return (int64_t)(int32_t)x;
    else return (int64_t)f1;
  }
};

// unconditional loads (callers clamp e): a branch around a load makes hipcc wait for it at once
template <int F1W>
__device__ __forceinline__ void kt_load(const KtArgs& a, int64_t e, KtRaw<F1W>& r) {
  r.ts = a.ts[e];
  r.key = a.keycol[e];
  r.x = a.xcol[e];
  if constexpr (F1W == 8) r.f1 = ((const int64_t*)a.f1col)[e];
  else if constexpr (F1W == 4) r.f1 = ((const int32_t*)a.f1col)[e];
  else r.f1 = 0;
}

// Stable partition of one super-tile, KT_C events at a time, straight from registers: wave w owns the
// chunk positions [w*KT_C/NW, (w+1)*KT_C/NW) in rounds of 64; a lane's rank among the round's lanes of its
// bucket comes from ballot matching on the bucket bits, its rank against earlier rounds from a per-(bucket,
// wave) counter, and a scan of those counters gives every entry its place behind the bucket cursor.  The
// next chunk's columns are loaded into registers while the current one is ranked and stored.
// LDS (dynamic, sized by P): hist[NW][P] u16 | cur[P] u32 | stage_e[KT_C] 12 B | stage_d[KT_C] u32
template <int KT_C, int F1W, int NT = KT_NT, bool E12 = false>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) k_kt_scatter(KtArgs a) {
  extern __shared__ uint32_t kt_dyn[];
  __shared__ uint32_t wsum[NT / 64];
  constexpr int NW = NT / 64, RPW = KT_C / NT;
  const int P = 1 << a.pb;
  uint16_t* hist = (uint16_t*)kt_dyn;
  uint32_t* cur = kt_dyn + (P * NW + 1) / 2;
  KtE12* stage_e = (KtE12*)(cur + P);                       // [KT_C] (12-B entries only)
  uint32_t* stage_d = (uint32_t*)(stage_e + KT_C);          // [KT_C] destinations
  const uint32_t mask = (uint32_t)P - 1;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int b = t; b < P; b += NT) cur[b] = a.hist[(int64_t)b * a.nst + blockIdx.x];
  const int64_t e0 = (int64_t)blockIdx.x * KT_ST, e1 = min<int64_t>(e0 + KT_ST, a.n);
  // chunks in pairs with two register sets (A: even chunks, B: odd), so the next chunk's loads are
  // never copied at the loop latch, and unconditional stores (lanes past the end write the dummy slot
  // ent[n]): hipcc's wait counts then only make a chunk wait for its own columns, not for stores
  KtRaw<F1W> ra[RPW], rb[RPW];
#pragma unroll
  for (int k = 0; k < RPW; k++) kt_load<F1W>(a, min<int64_t>(e0 + w * (KT_C / NW) + k * 64 + lane, e1 - 1), ra[k]);
  auto chunk = [&](const KtRaw<F1W> (&r)[RPW], KtRaw<F1W> (&rn)[RPW], int64_t c0) {
    const int nc = (int)max<int64_t>(0, min<int64_t>(KT_C, e1 - c0));
    for (int k = t; k < P * NW / 2; k += NT) ((uint32_t*)hist)[k] = 0;
    uint4 v[RPW];
    uint32_t bk[RPW];
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      const int q = w * (KT_C / NW) + k * 64 + lane;
      bk[k] = r[k].key & mask;
      const bool st = F1W == 0 || cmp(a.f1op, a.f1t, r[k].f1v(), a.f1c);
      v[k] = make_uint4((uint32_t)(c0 + q), (uint32_t)(r[k].ts - a.ts0) | (st ? 0x80000000u : 0u), r[k].x,
                        r[k].key >> a.pb);
    }
    {
      // non-decreasing timestamps (the relative encoding and the halos rely on it): each event against
      // its predecessor -- the lane below, the previous round's last lane, or the wave range's predecessor
      const int64_t q0 = c0 + w * (KT_C / NW);
      const int64_t tprev = a.ts[q0 > 0 ? q0 - 1 : 0];
      bool bad = false;
#pragma unroll
      for (int k = 0; k < RPW; k++) {
        const int64_t up = __shfl_up(r[k].ts, 1, 64);
        const int64_t last = k ? __shfl(r[k - 1].ts, 63, 64) : tprev;
        bad |= w * (KT_C / NW) + k * 64 + lane < nc && r[k].ts < (lane ? up : last);
      }
      if (__any(bad) && lane == 0) atomicOr(a.unsorted, 1u);
    }
#pragma unroll
    for (int k = 0; k < RPW; k++)                   // prefetch the next chunk
      kt_load<F1W>(a, min<int64_t>(c0 + KT_C + w * (KT_C / NW) + k * 64 + lane, e1 - 1), rn[k]);
    __syncthreads();
    uint16_t rk[RPW];
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      const bool valid = w * (KT_C / NW) + k * 64 + lane < nc;
      const uint64_t peers = kt_match_peers_n(bk[k], valid, a.pb);
      const uint64_t below = peers & ((1ull << lane) - 1);
      const int h = w * P + (int)bk[k];
      const uint32_t hb = valid ? hist[h] : 0u;
      if (valid && below == 0) hist[h] = (uint16_t)(hb + __popcll(peers));
      rk[k] = (uint16_t)(hb + __popcll(below));
    }
    __syncthreads();
    kt_scan_kw<NT, NW>(hist, P, wsum);   // -> chunk-local bucket-run offsets, (bucket, wave) order
    if (E12 && !(a.exp & 1024)) {
      // 12-B entries are staged in LDS in chunk-sorted (bucket, arrival) order with their destinations,
      // then stored by consecutive lanes: a bucket's run of the chunk leaves as one contiguous piece
#pragma unroll
      for (int k = 0; k < RPW; k++) {
        const bool valid = w * (KT_C / NW) + k * 64 + lane < nc;
        if (!valid) continue;
        const uint32_t b = bk[k];
        const int loc = hist[w * P + b] + rk[k];
        const uint4 e = v[k];
        stage_e[loc] = KtE12{e.x, (e.y & 0x80000000u) | ((e.y & 0x1fffffu) << KT_LB) | e.w, e.z};
        stage_d[loc] = cur[b] - hist[b] + (uint32_t)loc;
      }
      __syncthreads();
      for (int l = t; l < nc; l += NT) ((KtE12*)a.ent)[stage_d[l]] = stage_e[l];
    } else {
#pragma unroll
      for (int k = 0; k < RPW; k++) {
        const bool valid = w * (KT_C / NW) + k * 64 + lane < nc;
        const uint32_t b = bk[k];
        const int64_t dst = valid && !(a.exp & 1) ? (int64_t)cur[b] + (hist[w * P + b] - hist[b]) + rk[k] : a.n;
        kt_put<E12>(a.ent, dst, v[k]);
      }
    }
    __syncthreads();
    for (int b = t; b < P; b += NT) cur[b] += (b + 1 < P ? hist[b + 1] : (uint32_t)nc) - hist[b];
    __syncthreads();
  };
  for (int64_t c0 = e0; c0 < e1; c0 += 2 * KT_C) {
    chunk(ra, rb, c0);
    chunk(rb, ra, c0 + KT_C);                       // past the end: no valid lanes
  }
}

inline size_t kt_scatter_lds(int NT, int P, int chunk) {
  return (size_t)P * (NT / 64) * 2 + 4 + (size_t)P * 4 + (size_t)chunk * 16;
}

enum KtSrc { KT_KEY = 0, KT_XI, KT_XJ, KT_COL_I, KT_COL_J };

template <class V>
__device__ __forceinline__ V kt_val(uint32_t b) {
  V v;
  __builtin_memcpy(&v, &b, 4);
  return v;
}

__device__ __forceinline__ uint32_t kt_tc_add(uint16_t* tc, int c, uint32_t v) {
  const uint32_t old = atomicAdd((uint32_t*)tc + (c >> 1), (c & 1) ? (v << 16) : v);
  return (c & 1) ? (old >> 16) : (old & 0xffffu);
}

// Trigger-centric form of m(i) = min{ j > i : same key, ts_j - ts_i <= W, x_j OP x_i }: trigger j
// completes start i iff x_j OP x_i, ts_j - ts_i <= W, and no event r strictly between them (same key) has
// x_r OP x_i.  Walking back from j over its key run, that last condition reduces per OP to a summary of
// the events passed so far: their max (GT, GE) or min (LT, LE) over the non-NaN values, whether one equals
// x_j (EQ), or whether they all hold one value (NE); each summary also says when no earlier start can
// qualify.  Returns the count; every record found is appended to `found` as start | j << PB | its index
// among j's records, nearest start first (saturating), << 2 PB  (PB = bits of a tile position).
// (tj = tx[q], rs = its run's first position and tr1 = tx[q - 1] come preloaded: the caller issues those
// LDS reads for all of its positions at once)
// EMIT = 0: the count pass of the two-walk matcher (no writes); EMIT = 1: its second walk, which writes
// each record straight to its final slot rl[last - c] (c = discovery index, nearest start first) so a
// trigger's records run in ascending i; EMIT = 2: the single-walk form (discovery list through an LDS
// atomic counter).
template <int OP, class V, int PB, int EMIT = 2>
__device__ __forceinline__ uint32_t kt_back(const uint2* tx, int q, uint2 tj, int rs, uint2 tr1, uint32_t w32,
                                            uint32_t* found, uint32_t* nfound, uint32_t cap) {
  constexpr uint32_t CIM = (1u << (32 - 2 * PB)) - 1;
  const uint32_t tsj = tj.x & 0x7fffffffu;
  const V xj = kt_val<V>(tj.y);
  if constexpr (OP != C_NE && OP != C_EQ) {
    if (xj != xj) return 0;                     // NaN trigger: no order comparison holds
  }
  V ext = xj;                                   // summary of the events between (valid when any)
  bool any = false, uni = true;
  uint32_t c = 0;
  for (int r = q - 1; r >= rs; r--) {
    const uint2 tr = r == q - 1 ? tr1 : tx[r];
    if (tsj - (tr.x & 0x7fffffffu) > w32) break;
    const V xr = kt_val<V>(tr.y);
    bool qual, stop;
    if constexpr (OP == C_GT || OP == C_GE || OP == C_LT || OP == C_LE) {
      qual = cmpv<OP, V>(xj, xr) && (!any || !cmpv<OP, V>(ext, xr));
      if (xr == xr) {
        if constexpr (OP == C_GT || OP == C_GE) ext = any ? (xr > ext ? xr : ext) : xr;
        else ext = any ? (xr < ext ? xr : ext) : xr;
        any = true;
      }
      if constexpr (OP == C_GT || OP == C_GE) stop = any && ext >= xj;
      else stop = any && ext <= xj;
    } else if constexpr (OP == C_EQ) {
      qual = xr == xj;
      stop = qual;
    } else {                                      // NE: every event between must equal x_i
      qual = xj != xr && (!any || (uni && xr == ext));
      if (!any) { ext = xr; any = true; }
      else uni = uni && xr == ext;
      stop = !uni || !(xj != ext);
    }
    if (qual && (tr.x >> 31)) {
      if constexpr (EMIT == 2) {
        const uint32_t slot = atomicAdd(nfound, 1u);
        if (slot < cap) found[slot] = (uint32_t)r | ((uint32_t)q << PB) | (min(c, CIM) << (2 * PB));
      } else if constexpr (EMIT == 1) {
        found[cap - c] = (uint32_t)r | ((uint32_t)q << 16);   // cap = the trigger's last slot
      }
      c++;
    }
    if (stop) break;
  }
  return c;
}

// Wave-uniform form of kt_back (EMIT = 2) for one position per lane: the whole wave steps its lanes'
// walks together, so a record's slot comes from a ballot over the wave's private list (`wcnt`, uniform)
// instead of an LDS atomic: one LDS round trip per step (the {ts, x} pair as one 8-B read).  Records past
// `cap` are counted but not stored (the caller turns that into the overflow fallback).
template <int OP, class V, int PB>
__device__ __forceinline__ uint32_t kt_back_w(const uint2* tx, bool act, int q, uint2 tj, int rs, uint2 tr1,
                                              uint32_t w32, uint32_t* found, uint32_t& wcnt, uint32_t cap) {
  constexpr uint32_t CIM = (1u << (32 - 2 * PB)) - 1;
  const uint32_t tsj = tj.x & 0x7fffffffu;
  const V xj = kt_val<V>(tj.y);
  if constexpr (OP != C_NE && OP != C_EQ) act = act && xj == xj;   // NaN trigger: no order comparison holds
  V ext = xj;
  bool any = false, uni = true;
  uint32_t c = 0;
  int r = q - 1;
  act = act && r >= rs;
  uint2 tr = tr1;
  const uint64_t lt = (1ull << (threadIdx.x & 63)) - 1;
  while (__ballot(act)) {
    bool rec = false;
    if (act) {
      if (tsj - (tr.x & 0x7fffffffu) > w32) {
        act = false;
      } else {
        const V xr = kt_val<V>(tr.y);
        bool qual, stop;
        if constexpr (OP == C_GT || OP == C_GE || OP == C_LT || OP == C_LE) {
          qual = cmpv<OP, V>(xj, xr) && (!any || !cmpv<OP, V>(ext, xr));
          if (xr == xr) {
            if constexpr (OP == C_GT || OP == C_GE) ext = any ? (xr > ext ? xr : ext) : xr;
            else ext = any ? (xr < ext ? xr : ext) : xr;
            any = true;
          }
          if constexpr (OP == C_GT || OP == C_GE) stop = any && ext >= xj;
          else stop = any && ext <= xj;
        } else if constexpr (OP == C_EQ) {
          qual = xr == xj;
          stop = qual;
        } else {
          qual = xj != xr && (!any || (uni && xr == ext));
          if (!any) { ext = xr; any = true; }
          else uni = uni && xr == ext;
          stop = !uni || !(xj != ext);
        }
        rec = qual && (tr.x >> 31);
        if (stop) act = false;
      }
    }
    const uint64_t bm = __ballot(rec);
    if (rec) {
      const uint32_t slot = wcnt + (uint32_t)__popcll(bm & lt);
      if (slot < cap) found[slot] = (uint32_t)r | ((uint32_t)q << PB) | (min(c, CIM) << (2 * PB));
      c++;
    }
    wcnt += (uint32_t)__popcll(bm);
    if (act) {
      r--;
      if (r < rs) act = false;
      else tr = tx[r];
    }
  }
  return c;
}

// ---- matcher: one workgroup per (bucket, tile), one lane per key-run position --------------------
// Tile = bucket b's triggers [s, e) plus the back-halo [hs, s) (its entries within W of the first
// trigger).  Phases (barrier-separated, NT = 512 threads = 8 waves):
//   rank   wave w owns local positions [w*CW, (w+1)*CW) in rounds of 64; a lane's stable rank among its
//          key's entries = ballot-matched lower peers of the round + the per-(wave, key) counter
//   scan   exclusive scan of the [wave][key] counters in (key, wave) order -> key-run positions
//   place  ts, x, local position and run end scattered to key-run order: each local key's events are
//          contiguous and in arrival order
//   walk   every start walks its run forward to m(i) (first j with ts_j - ts_i <= W and f2); each
//          trigger of this tile counts its records
//   slot   counts -> offsets (records in trigger order); a start's rank among the starts completed by the
//          same trigger (those of its run before it with the same m, all within W) gives its record
//          slot, and the slot list (LDS, over the dead counters) names the start of every record
//   write  dense: consecutive lanes write consecutive records {j, i, projections} (coalesced 16-B stores)
template <int T, int H, int NT>
struct KtMatchLds {
  static constexpr int L = T + H;
  static constexpr int NW = NT / 64;
  union {
    uint16_t hist[NW * KT_NL];          // [wave][key] counts -> key-run positions
    struct {
      uint32_t rl[T];                   // record slot -> key-run positions: start | trigger << 16
      uint32_t found[T];                // records in discovery order (kt_back)
    };
  };
  uint2 tx[L];                          // key-run order: {ts_rel | start << 31, x} (one read per walk step)
  uint32_t rr[L];                       // the position's key run: first position | end << 16
  uint16_t lp[L];                       // local (arrival) position
  uint16_t tc[T];                       // per-trigger record counts -> offsets (two u16 per word)
  uint32_t wc[NW];                      // records found by each wave (its private part of `found`)
};

// exclusive scan in place of N u16 counters, 4 per thread read and written as one 8-B word
template <int NT, int N>
__device__ __forceinline__ uint32_t kt_scan16(uint16_t* a, uint32_t* wsum) {
  static_assert(N == 4 * NT, "four counters per thread");
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint2 c = ((const uint2*)a)[t];
  const uint32_t c0 = c.x & 0xffffu, c1 = c.x >> 16, c2 = c.y & 0xffffu, c3 = c.y >> 16;
  const uint32_t loc = c0 + c1 + c2 + c3;
  const uint32_t inc = kt_wave_scan(loc);
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; k++) {
    const uint32_t v = wsum[k];
    base += k < w ? v : 0;
    tot += v;
  }
  const uint32_t r0 = base + inc - loc, r1 = r0 + c0, r2 = r1 + c1, r3 = r2 + c2;
  ((uint2*)a)[t] = make_uint2((r0 & 0xffffu) | (r1 << 16), (r2 & 0xffffu) | (r3 << 16));
  __syncthreads();
  return tot;
}

template <int OP, class V, int T, int H, int NT, bool E12 = false, bool TWO = false, bool FWD = true>
__global__ void __launch_bounds__(NT) k_kt_match(KtArgs a) {
  using S = KtMatchLds<T, H, NT>;
  constexpr int L = S::L, NW = S::NW, RPW = (L + NT - 1) / NT;
  constexpr int PB = L > 4096 ? 13 : 12;                          // bits of a tile position
  __shared__ S sm;
  __shared__ uint32_t wsum[NW];
  __shared__ uint32_t nfound;
#define KT_PROBE(i) \
  do { if (a.dbg && (int)blockIdx.x < a.dbg_n && threadIdx.x == 0) a.dbg[blockIdx.x * 8 + (i)] = (int64_t)wall_clock64(); } while (0)
  KT_PROBE(0);
  // workgroups are dealt to the 8 XCDs round-robin; with xcd_tiles each XCD takes one contiguous eighth of the
  // (bucket-major) tile table, so a tile's back-halo -- the previous tile's tail -- was read through its own L2
  const uint32_t W = a.xcd_tiles ? kt_xcd_index(blockIdx.x, (uint32_t)a.ntiles_max) : blockIdx.x;
  if (W >= (uint32_t)a.ntiles_max) return;
  const uint4 d = a.tdesc[W];
  if (d.x == 0xffffffffu) {
    if (a.toffs && threadIdx.x == 0) a.tdir[W] = make_uint2(0u, 0u);   // no records (carried starts only)
    return;
  }
  const uint32_t b = d.x;
  const uint32_t B0 = a.bstart[b];
  const int s = (int)d.y, e = (int)d.z, hs = (int)d.w;
  const int Ln = e - hs, toff = s - hs, tend = e - hs;
  // triggers of the previous tile of the bucket end at position s - 1 (a carried start there: none)
  const int64_t jprev = a.toffs && s > 0 ? (int64_t)kt_get<E12>(a.ent, (int64_t)B0 + s - 1).x : -1;
  if (Ln <= 0) {                                  // a trigger-less last tile with nothing left open
    if (threadIdx.x == 0) a.tdir[W] = make_uint2(B0 + (uint32_t)s, 0u);
    if (a.toffs) kt_write_toffs(a, b, W, B0 + (uint32_t)s, jprev, -1, true, 0u, [](uint32_t) { return (uint32_t)0; });
    return;
  }
  const bool last = e == (int)(a.bstart[b + 1] - B0);
  const uint32_t w32 = (uint32_t)min<int64_t>(a.within, 0x7fffffff);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int CW = ((Ln + NW * 64 - 1) / (NW * 64)) * 64;
  const int p0 = w * CW;
  const int64_t eb = (int64_t)B0 + hs;            // the tile: halo + triggers, bucket-relative positions
  uint4 v[RPW];
#pragma unroll
  for (int k = 0; k < RPW; k++) v[k] = kt_get<E12>(a.ent, eb + min(p0 + k * 64 + lane, Ln - 1));
  for (int k = t; k < KT_NL * NW / 2; k += NT) ((uint32_t*)sm.hist)[k] = 0;
  for (int k = t; k < T / 2; k += NT) ((uint32_t*)sm.tc)[k] = 0;
  __syncthreads();
  KT_PROBE(1);
  uint16_t rk[RPW];
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    const int p = p0 + k * 64 + lane;
    const bool valid = p < min(p0 + CW, Ln);
    if (k * 64 >= CW) { rk[k] = 0; continue; }   // wave-uniform
    const uint32_t key = v[k].w;
    const uint64_t peers = kt_match_peers<KT_LB>(key, valid);
    const uint64_t below = peers & ((1ull << lane) - 1);
    const int hidx = w * KT_NL + (int)(key & (KT_NL - 1));
    const uint32_t hb = valid ? sm.hist[hidx] : 0u;
    if (valid && below == 0) sm.hist[hidx] = (uint16_t)(hb + __popcll(peers));
    rk[k] = (uint16_t)(hb + __popcll(below));
  }
  __syncthreads();
  KT_PROBE(2);
  kt_scan_kw<NT, NW>(sm.hist, KT_NL, wsum);
  KT_PROBE(3);
  uint16_t qk[RPW];                                                // key-run position of each owned entry
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    const int p = p0 + k * 64 + lane;
    qk[k] = 0xffffu;
    if (k * 64 < CW && p < min(p0 + CW, Ln)) {
      const int key = (int)v[k].w;
      const int q = sm.hist[w * KT_NL + key] + rk[k];
      qk[k] = (uint16_t)q;
      sm.tx[q] = make_uint2(v[k].y, v[k].z);
      sm.lp[q] = (uint16_t)p;
      sm.rr[q] = (uint32_t)sm.hist[key] | ((key + 1 < KT_NL ? (uint32_t)sm.hist[key + 1] : (uint32_t)Ln) << 16);
    }
  }
  __syncthreads();
  KT_PROBE(4);
  // count: every trigger of the tile walks back over its key run (within W) and counts the starts it
  // completes (kt_back); halo positions never walk
  if (t == 0) nfound = 0;
  __syncthreads();                                                 // hist is dead: its space holds the lists
  bool shared_list = false;
  // forward form (FWD): every start walks forward over its key run to m(i) = the first later entry within W
  // with x_m OP x_i; a record belongs to this tile when m is one of its triggers.  Its rank among the
  // trigger's records comes from a u16 LDS counter (arbitrary order; the trigger's slots are sorted by i
  // after the scan).  fm = m | rank << 16 (0xffffffff: no record here), fj = m's trigger index in the tile.
  uint32_t fm[RPW];
  uint16_t fj[RPW];
  if constexpr (FWD) {
    uint2 ti[RPW], tn[RPW];
    int re[RPW];
#pragma unroll
    for (int k = 0; k < RPW; k++) {               // all LDS reads of the walks' first step, back to back
      const int q = min(t + k * NT, Ln - 1);
      ti[k] = sm.tx[q];
      re[k] = (int)(sm.rr[q] >> 16);
      tn[k] = sm.tx[min(q + 1, Ln - 1)];
      fm[k] = 0xffffffffu;
      fj[k] = 0;
    }
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      if (k * NT >= Ln) break;                                     // uniform
      const int q = t + k * NT;
      const bool st = q < Ln && (ti[k].x >> 31);
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
        const int lj = (int)sm.lp[m] - toff;
        if (lj >= 0 && lj < tend - toff) {
          fj[k] = (uint16_t)lj;
          fm[k] = (uint32_t)m | (kt_tc_add(sm.tc, lj, 1u) << 16);
        }
      } else if (last && st && !expired && (uint32_t)a.ts_last_rel - tsi <= w32) {
        // the bucket's last tile: a start with no completing entry up to the flush's end, not expired at
        // its last timestamp, carries into the next flush
        a.carry[atomicAdd(a.ncarry, 1u)] = (int32_t)kt_get<E12>(a.ent, eb + sm.lp[q]).x;
      }
    }
  } else {
    int lq[RPW], rs[RPW];
    uint2 tj[RPW], t1[RPW];
#pragma unroll
    for (int k = 0; k < RPW; k++) {               // all LDS reads of the walks' first step, back to back
      const int q = min(t + k * NT, Ln - 1);
      lq[k] = sm.lp[q];
      tj[k] = sm.tx[q];
      rs[k] = (int)(sm.rr[q] & 0xffffu);
      t1[k] = sm.tx[max(q - 1, 0)];
    }
    if constexpr (TWO) {
#pragma unroll
      for (int k = 0; k < RPW; k++) {
        const int q = t + k * NT;
        if (q < Ln && lq[k] >= toff && lq[k] < tend)
          sm.tc[lq[k] - toff] = (uint16_t)kt_back<OP, V, PB, 0>(sm.tx, q, tj[k], rs[k], t1[k], w32, nullptr, nullptr, 0);
      }
    } else {
      // each wave appends to its own T / NW slots of `found`; its count stays wave-uniform
      uint32_t wcnt = 0;
#pragma unroll
      for (int k = 0; k < RPW; k++) {
        const int q = t + k * NT;
        const bool act = q < Ln && lq[k] >= toff && lq[k] < tend;
        if (k * NT >= Ln) break;                                     // uniform
        const uint32_t c = kt_back_w<OP, V, PB>(sm.tx, act, q, tj[k], rs[k], t1[k], w32, sm.found + w * (T / NW),
                                                wcnt, T / NW);
        if (act) sm.tc[lq[k] - toff] = (uint16_t)c;
      }
      if (lane == 0) sm.wc[w] = wcnt;
      __syncthreads();
#pragma unroll
      for (int k = 0; k < NW; k++) shared_list |= sm.wc[k] > (uint32_t)(T / NW);
      if (shared_list) {
        // a wave found more records than its slots (skewed keys): redo the walks into one shared list
#pragma unroll
        for (int k = 0; k < RPW; k++) {
          const int q = t + k * NT;
          if (q < Ln && lq[k] >= toff && lq[k] < tend)
            kt_back<OP, V, PB>(sm.tx, q, tj[k], rs[k], t1[k], w32, sm.found, &nfound, T);
        }
      }
    }
  }
  // the bucket's last tile: starts still open at its end (no trigger after them within W, not expired at
  // the flush's last timestamp) carry into the next flush
  if (!FWD && last) {
    for (int q = t; q < Ln; q += NT) {
      const uint2 tq = sm.tx[q];
      if (!(tq.x >> 31)) continue;
      const uint32_t tsi = tq.x & 0x7fffffffu;
      if ((uint32_t)a.ts_last_rel - tsi > w32) continue;
      const int end = (int)(sm.rr[q] >> 16);
      bool open = true;
      for (int r = q + 1; r < end && open; r++) {
        const uint2 tr = sm.tx[r];
        if ((tr.x & 0x7fffffffu) - tsi > w32) break;
        open = !cmpv<OP, V>(kt_val<V>(tr.y), kt_val<V>(tq.y));
      }
      if (open) a.carry[atomicAdd(a.ncarry, 1u)] = (int32_t)kt_get<E12>(a.ent, eb + sm.lp[q]).x;
    }
  }
  __syncthreads();
  uint32_t nrec = 0;
  if constexpr (TWO && !FWD) {
    // counts -> offsets, then the second walk writes every record to its slot (no LDS atomics)
    nrec = kt_scan16<NT, T>(sm.tc, wsum);
    if (nrec <= (uint32_t)(e - s)) {
      for (int k = 0; k < RPW; k++) {
        const int q = t + k * NT;
        if (q >= Ln) break;
        const int lj = sm.lp[q] - toff;
        if (lj < 0 || lj >= tend - toff) continue;
        const uint32_t off = sm.tc[lj];
        const uint32_t cnt = (lj + 1 < T ? (uint32_t)sm.tc[lj + 1] : nrec) - off;
        if (cnt == 0) continue;
        kt_back<OP, V, PB, 1>(sm.tx, q, sm.tx[q], (int)(sm.rr[q] & 0xffffu), sm.tx[max(q - 1, 0)], w32, sm.rl,
                              nullptr, off + cnt - 1);
      }
    }
    __syncthreads();
  }
  // the walks are done: each owner deposits its entry's global index over the run bounds (rr) and its
  // local key over the timestamp half of tx (x stays), so the record writes read only LDS
#pragma unroll
  for (int k = 0; k < RPW; k++) {
    if (qk[k] != 0xffffu) {
      sm.rr[qk[k]] = v[k].x;
      sm.tx[qk[k]].x = v[k].w;
    }
  }
  KT_PROBE(5);
  if constexpr (!TWO || FWD) nrec = kt_scan16<NT, T>(sm.tc, wsum);
  const uint32_t base = B0 + (uint32_t)s;
  const bool fits = nrec <= (uint32_t)(e - s);
  if (t == 0) {
    if (!fits) atomicOr(a.overflow, 1u);
    else if (nrec) atomicAdd(&a.bcur[b], nrec);
    a.tdir[W] = make_uint2(base, nrec);
  }
  if (!fits) return;
  // place each found record at its slot: offset of its trigger + (count - 1 - its index), so a trigger's
  // records run in ascending i.  Indices saturate (255, or 63 for 4096-trigger tiles): a trigger with more
  // records (a long falling run) makes the flush overflow to the sort pipeline
  if constexpr (FWD) {
    // slot = the trigger's offset + rank; then each trigger sorts its (few) slots by start position, which
    // inside one key run is arrival order: a trigger's records run in ascending i.  More than KT_MAXREC
    // records for one trigger (a long falling run) send the flush to the sort pipeline.
#pragma unroll
    for (int k = 0; k < RPW; k++) {
      if (fm[k] != 0xffffffffu) {
        const uint32_t m = fm[k] & 0xffffu, rank = fm[k] >> 16;
        sm.rl[sm.tc[fj[k]] + rank] = (uint32_t)(t + k * NT) | (m << 16);
      }
    }
    __syncthreads();
    bool sat = false;
    for (int lj = t; lj < tend - toff; lj += NT) {
      const uint32_t off = sm.tc[lj];
      const uint32_t cnt = (lj + 1 < T ? (uint32_t)sm.tc[lj + 1] : nrec) - off;
      if (cnt < 2) continue;
      if (cnt > KT_MAXREC) { sat = true; continue; }
      for (uint32_t x = 1; x < cnt; x++) {                         // insertion sort (same m: by value)
        const uint32_t v0 = sm.rl[off + x];
        uint32_t y = x;
        while (y > 0 && sm.rl[off + y - 1] > v0) { sm.rl[off + y] = sm.rl[off + y - 1]; y--; }
        sm.rl[off + y] = v0;
      }
    }
    if (sat) atomicOr(a.overflow, 1u);
    __syncthreads();
  } else if constexpr (!TWO) {
    constexpr uint32_t PM = (1u << PB) - 1, CIM = (1u << (32 - 2 * PB)) - 1;
    // this wave's own list, or (after a redo) the shared one
    const uint32_t* fl = shared_list ? sm.found : sm.found + w * (T / NW);
    const uint32_t r0 = shared_list ? t : lane, rstep = shared_list ? NT : 64;
    const uint32_t nl = shared_list ? nrec : sm.wc[w];
    bool sat = false;
    for (uint32_t r = r0; r < nl; r += rstep) {
      const uint32_t f = fl[r];
      const uint32_t q = f & PM, j = (f >> PB) & PM, ci = f >> (2 * PB);
      const int lj = sm.lp[j] - toff;
      const uint32_t off = sm.tc[lj];
      const uint32_t cnt = (lj + 1 < T ? (uint32_t)sm.tc[lj + 1] : nrec) - off;
      sat |= cnt > CIM;
      sm.rl[off + cnt - 1 - min(ci, cnt - 1)] = q | (j << 16);
    }
    if (sat) atomicOr(a.overflow, 1u);
    __syncthreads();
  }
  KT_PROBE(6);
  // write: dense, consecutive lanes -> consecutive records
  for (uint32_t r = t; r < nrec; r += NT) {
    const uint32_t pr = sm.rl[r];
    const int q = (int)(pr & 0xffffu), m = (int)(pr >> 16);
    const uint2 ti = sm.tx[q];                                      // {local key, x} of the start
    const uint32_t ig = sm.rr[q], jg = sm.rr[m];                    // global indices of start and trigger
    const uint32_t lk = ti.x;
    int32_t* rp = a.rec + (int64_t)(base + r) * a.stride;
    auto proj = [&](int c) -> int64_t {
      switch (a.src[c]) {
        case KT_KEY: return (int32_t)((lk << a.pb) | b);
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
  if (a.toffs) {
    // records are in (j, i) order: j of record r is the trigger's global index (rr, deposited above)
    const int64_t jlast = s < e ? (int64_t)kt_get<E12>(a.ent, (int64_t)B0 + e - 1).x : -1;
    kt_write_toffs(a, b, W, base, jprev, jlast, last, nrec,
                   [&](uint32_t r) { return sm.rr[sm.rl[r] >> 16]; });
  }
  if (a.dbg) { __syncthreads(); KT_PROBE(7); }
#undef KT_PROBE
}

}  // namespace sg
