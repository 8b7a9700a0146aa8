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
//   k_kt_buckets  bucket starts + per-bucket tile prefix; k_kt_tdesc: tile table (bucket, tile) for the matcher grid
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

// exclusive scan in place of n values in LDS (thread t owns a contiguous run); returns the total
template <int NT, class T>
__device__ __forceinline__ uint32_t kt_block_scan(T* a, int n, uint32_t* wsum) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int ipt = (n + NT - 1) / NT, b0 = min(t * ipt, n), b1 = min(b0 + ipt, n);
  uint32_t loc = 0;
  for (int k = b0; k < b1; k++) loc += a[k];
  uint32_t inc = loc;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d, 64);
    if (lane >= d) inc += o;
  }
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

struct KtArgs {
  // input columns
  const int64_t* ts;
  const uint32_t* keycol;
  const uint32_t* xcol;
  int32_t f1kind, f1op, f1t, f1w;
  const uint8_t* f1col;
  int64_t f1c;
  int64_t n, ts0, within;
  int32_t pb;                 // log2 buckets
  int32_t tile_t;             // triggers per matcher tile
  int32_t nst;                // super-tiles
  // partition
  uint32_t* hist;             // [P * nst] counts -> exclusive bases
  uint4* ent;                 // [n] bucketed entries
  // tiles
  int32_t ntiles_max;
  uint32_t* bstart;           // [P + 1] bucket start (entries)
  uint32_t* tprefix;          // [P + 1] exclusive prefix of tiles per bucket
  uint32_t* tdesc;            // [ntiles_max] (bucket << 20 | tile)  (0xffffffff = none)
  // matcher outputs
  int32_t* rec;               // records, `stride` int32 words each
  int32_t stride;
  uint32_t* bcur;             // [P] per-bucket record cursors (start at bstart)
  uint2* tdir;                // [ntiles_max] {offset, count}
  int32_t* carry;
  uint32_t* ncarry;
  uint32_t* overflow;
  int64_t ts_last_rel;
  // projection
  int32_t nproj;
  int32_t src[FB_MAXP];
  int32_t w[FB_MAXP];
  const uint8_t* col[FB_MAXP];
};

__global__ void __launch_bounds__(KT_NT) k_kt_hist(KtArgs a) {
  __shared__ uint32_t h[1 << KT_MAXPB];
  const int P = 1 << a.pb;
  for (int b = threadIdx.x; b < P; b += KT_NT) h[b] = 0;
  __syncthreads();
  const int64_t e0 = (int64_t)blockIdx.x * KT_ST, e1 = min<int64_t>(e0 + KT_ST, a.n);
  const uint32_t mask = (uint32_t)P - 1;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += KT_NT) atomicAdd(&h[a.keycol[e] & mask], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < P; b += KT_NT) a.hist[(int64_t)b * a.nst + blockIdx.x] = h[b];
}

// bucket starts, per-bucket record cursors and the exclusive tile prefix (one workgroup)
__global__ void __launch_bounds__(KT_NT) k_kt_buckets(KtArgs a) {
  __shared__ uint32_t tc[1 << KT_MAXPB];
  __shared__ uint32_t wsum[KT_NT / 64];
  const int P = 1 << a.pb;
  for (int b = threadIdx.x; b < (1 << KT_MAXPB); b += KT_NT) {
    uint32_t c = 0;
    if (b < P) {
      const uint32_t s0 = a.hist[(int64_t)b * a.nst];
      const uint32_t s1 = b + 1 < P ? a.hist[(int64_t)(b + 1) * a.nst] : (uint32_t)a.n;
      a.bstart[b] = s0;
      a.bcur[b] = s0;
      c = (s1 - s0 + a.tile_t - 1) / a.tile_t;
    }
    tc[b] = c;
  }
  if (threadIdx.x == 0) a.bstart[P] = (uint32_t)a.n;
  __syncthreads();
  const uint32_t total = kt_block_scan<KT_NT>(tc, P, wsum);
  for (int b = threadIdx.x; b < P; b += KT_NT) a.tprefix[b] = tc[b];
  if (threadIdx.x == 0) a.tprefix[P] = total;
}

// matcher tile table: tile w -> (bucket << 20 | tile in bucket), by binary search of the tile prefix
__global__ void __launch_bounds__(KT_NT) k_kt_tdesc(KtArgs a) {
  const int64_t w = (int64_t)blockIdx.x * KT_NT + threadIdx.x;
  if (w >= a.ntiles_max) return;
  const int P = 1 << a.pb;
  const uint32_t total = a.tprefix[P];
  if (w >= total) { a.tdesc[w] = 0xffffffffu; return; }
  int lo = 0, hi = P - 1;                       // last b with tprefix[b] <= w
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (a.tprefix[mid] <= (uint32_t)w) lo = mid; else hi = mid - 1;
  }
  a.tdesc[w] = ((uint32_t)lo << 20) | ((uint32_t)w - a.tprefix[lo]);
}

__device__ __forceinline__ bool kt_start(const KtArgs& a, int64_t e) {
  if (a.f1kind != 1) return true;
  const int64_t v = a.f1w == 8 ? ((const int64_t*)a.f1col)[e] : (int64_t)((const int32_t*)a.f1col)[e];
  return cmp(a.f1op, a.f1t, v, a.f1c);
}

struct KtRaw {
  int64_t ts, f1;
  uint32_t key, x;
};

__device__ __forceinline__ void kt_load(const KtArgs& a, int64_t e, KtRaw& r) {
  r.ts = a.ts[e];
  r.key = a.keycol[e];
  r.x = a.xcol[e];
  if (a.f1kind == 1) r.f1 = a.f1w == 8 ? ((const int64_t*)a.f1col)[e] : (int64_t)((const int32_t*)a.f1col)[e];
}

// Stable partition of one super-tile, C events at a time; the next chunk's columns are loaded into
// registers while the current one is ranked and written.  LDS (dynamic, sized by P):
//   stage[KT_C] uint4 | sbk[KT_C] u16 | cnt[P] | cst[P] | cur[P]
template <int KT_C>
__global__ void __launch_bounds__(KT_NT) k_kt_scatter(KtArgs a) {
  extern __shared__ uint4 kt_dyn[];
  __shared__ uint32_t wsum[KT_NT / 64];
  constexpr int EPT = KT_C / KT_NT;
  const int P = 1 << a.pb;
  uint4* stage = kt_dyn;
  uint16_t* sbk = (uint16_t*)(stage + KT_C);
  uint32_t* cnt = (uint32_t*)(sbk + KT_C);
  uint32_t* cst = cnt + P;
  uint32_t* cur = cst + P;
  const uint32_t mask = (uint32_t)P - 1;
  for (int b = threadIdx.x; b < P; b += KT_NT) {
    cur[b] = a.hist[(int64_t)b * a.nst + blockIdx.x];
    cnt[b] = 0;
  }
  const int64_t e0 = (int64_t)blockIdx.x * KT_ST, e1 = min<int64_t>(e0 + KT_ST, a.n);
  KtRaw r[EPT];
#pragma unroll
  for (int k = 0; k < EPT; k++) {
    const int64_t e = e0 + k * KT_NT + threadIdx.x;
    if (e < e1) kt_load(a, e, r[k]);
  }
  __syncthreads();
  for (int64_t c0 = e0; c0 < e1; c0 += KT_C) {
    const int nc = (int)min<int64_t>(KT_C, e1 - c0);
    uint4 v[EPT];
    uint32_t bk[EPT], rk[EPT];
#pragma unroll
    for (int k = 0; k < EPT; k++) {
      const int q = k * KT_NT + threadIdx.x;
      if (q < nc) {
        bk[k] = r[k].key & mask;
        const bool st = a.f1kind != 1 || cmp(a.f1op, a.f1t, r[k].f1, a.f1c);
        v[k] = make_uint4((uint32_t)(c0 + q), (uint32_t)(r[k].ts - a.ts0) | (st ? 0x80000000u : 0u), r[k].x,
                          r[k].key >> a.pb);
        rk[k] = atomicAdd(&cnt[bk[k]], 1u);
      }
    }
    // prefetch the next chunk
#pragma unroll
    for (int k = 0; k < EPT; k++) {
      const int64_t e = c0 + KT_C + k * KT_NT + threadIdx.x;
      if (e < e1) kt_load(a, e, r[k]);
    }
    __syncthreads();
    kt_block_scan<KT_NT>(cnt, P, wsum);     // cnt -> chunk-local bucket starts
#pragma unroll
    for (int k = 0; k < EPT; k++) {
      const int q = k * KT_NT + threadIdx.x;
      if (q < nc) {
        const uint32_t p = cnt[bk[k]] + rk[k];
        stage[p] = v[k];
        sbk[p] = (uint16_t)bk[k];
      }
    }
    for (int b = threadIdx.x; b < P; b += KT_NT) cst[b] = cnt[b];
    __syncthreads();
    // restore arrival order inside each bucket run (runs are ~KT_C/P entries; LDS atomics are unordered)
    for (int b = threadIdx.x; b < P; b += KT_NT) {
      const uint32_t s0 = cst[b], s1 = b + 1 < P ? cst[b + 1] : (uint32_t)nc;
      for (uint32_t p = s0 + 1; p < s1; p++) {
        const uint4 x = stage[p];
        uint32_t q = p;
        while (q > s0 && stage[q - 1].x > x.x) { stage[q] = stage[q - 1]; q--; }
        stage[q] = x;
      }
    }
    __syncthreads();
    for (int p = threadIdx.x; p < nc; p += KT_NT) {
      const uint32_t b = sbk[p];
      a.ent[cur[b] + (p - cst[b])] = stage[p];
    }
    __syncthreads();
    for (int b = threadIdx.x; b < P; b += KT_NT) {
      const uint32_t s1 = b + 1 < P ? cst[b + 1] : (uint32_t)nc;
      cur[b] += s1 - cst[b];
      cnt[b] = 0;
    }
    __syncthreads();
  }
}

inline size_t kt_scatter_lds(int C, int P) { return (size_t)C * 18 + (size_t)P * 12; }

enum KtSrc { KT_KEY = 0, KT_XI, KT_XJ, KT_COL_I, KT_COL_J };

// Transitive compares (> < >= <=) on values without NaN: the open starts of one key are monotone in x
// (a later start that beats an earlier one would have completed it), so a trigger completes exactly a
// top segment of the stack of open starts, and expiry pops the bottom.
template <int OP>
constexpr bool kt_stackable() { return OP == C_GT || OP == C_LT || OP == C_GE || OP == C_LE; }

template <class V>
__device__ __forceinline__ bool kt_isnan(uint32_t b) {
  if constexpr (std::is_same<V, float>::value) return (b & 0x7fffffffu) > 0x7f800000u;
  else return false;
}

template <class V>
__device__ __forceinline__ V kt_val(uint32_t b) {
  V v;
  __builtin_memcpy(&v, &b, 4);
  return v;
}

// LDS image of one matcher tile
template <int T, int L>
struct KtTile {
  uint32_t ts[L];        // ts_rel | start << 31
  uint32_t x[L];
  uint32_t idx[L];       // global event index
  uint16_t sp[L];        // sorted position -> local position (key runs in arrival order)
  uint16_t stk[L];       // per key run: stack of open starts (local positions)
  uint16_t tc[T];        // per-trigger record counts -> offsets (two u16 per word, LDS atomics)
  uint32_t cnt[KT_NL];   // local-key bins -> run starts
};

template <int OP, class V, int T, int L>
__device__ __forceinline__ void kt_emit(const KtArgs& a, KtTile<T, L>& S, uint32_t bucket, uint32_t key, int j,
                                        int i, uint32_t pos) {
  int32_t* rp = a.rec + (int64_t)pos * a.stride;
  const uint32_t jg = S.idx[j], ig = S.idx[i];
  rp[0] = (int32_t)jg;
  rp[1] = (int32_t)ig;
  int wo = 2;
  for (int c = 0; c < a.nproj; c++) {
    int64_t v;
    switch (a.src[c]) {
      case KT_KEY: v = (int32_t)((key << a.pb) | bucket); break;
      case KT_XI: v = (int32_t)S.x[i]; break;
      case KT_XJ: v = (int32_t)S.x[j]; break;
      default: {
        const int64_t g = a.src[c] == KT_COL_I ? ig : jg;
        v = a.w[c] == 2 ? ((const int64_t*)a.col[c])[g] : (int64_t)((const int32_t*)a.col[c])[g];
      }
    }
    rp[wo] = (int32_t)v;
    if (a.w[c] == 2) rp[wo + 1] = (int32_t)(v >> 32);
    wo += a.w[c];
  }
}

__device__ __forceinline__ uint32_t kt_tc_get(const uint16_t* tc, int c) { return tc[c]; }
__device__ __forceinline__ uint32_t kt_tc_add(uint16_t* tc, int c, uint32_t v) {
  const uint32_t old = atomicAdd((uint32_t*)tc + (c >> 1), (c & 1) ? (v << 16) : v);
  return (c & 1) ? (old >> 16) : (old & 0xffffu);
}

// One key run [s0, s1) of sorted positions, by one lane.  PASS 0 counts the records of the tile's
// triggers, PASS 1 writes them at the scanned offsets (ascending i per trigger) and carries the starts
// left open at the end of the bucket.
template <int PASS, int OP, class V, int T, int L>
__device__ void kt_run(const KtArgs& a, KtTile<T, L>& S, uint32_t bucket, uint32_t key, int s0, int s1, int toff,
                       int tend, bool last, uint32_t base) {
  bool walk = !kt_stackable<OP>();
  if (!walk && std::is_same<V, float>::value)
    for (int r = s0; r < s1; r++) walk |= kt_isnan<V>(S.x[S.sp[r]]);
  if (!walk) {
    int bot = s0, top = s0;                      // stack of open starts in S.stk[bot, top)
    for (int r = s0; r < s1; r++) {
      const int j = S.sp[r];
      const uint32_t tj = S.ts[j];
      const int64_t tsj = tj & 0x7fffffffu;
      const V xj = kt_val<V>(S.x[j]);
      while (bot < top && tsj - (int64_t)(S.ts[S.stk[bot]] & 0x7fffffffu) > a.within) bot++;
      int nt = top;
      while (nt > bot && cmpv<OP, V>(xj, kt_val<V>(S.x[S.stk[nt - 1]]))) nt--;
      if (nt < top && j >= toff && j < tend) {
        if (PASS == 0) kt_tc_add(S.tc, j - toff, (uint32_t)(top - nt));
        else {
          const uint32_t o = base + kt_tc_get(S.tc, j - toff);
          for (int k = nt; k < top; k++) kt_emit<OP, V>(a, S, bucket, key, j, S.stk[k], o + (k - nt));
        }
      }
      top = nt;
      if (tj >> 31) S.stk[top++] = (uint16_t)j;
    }
    if (PASS == 1 && last)
      for (int k = bot; k < top; k++) {
        const int i = S.stk[k];
        if (a.ts_last_rel - (int64_t)(S.ts[i] & 0x7fffffffu) <= a.within)
          a.carry[atomicAdd(a.ncarry, 1u)] = (int32_t)S.idx[i];
      }
    return;
  }
  // general compare (or NaN in the run): every start walks forward to m(i)
  for (int r = s0; r < s1; r++) {
    const int i = S.sp[r];
    const uint32_t ti = S.ts[i];
    if (!(ti >> 31)) continue;
    const int64_t tsi = ti & 0x7fffffffu;
    const V yi = kt_val<V>(S.x[i]);
    int m = -1;
    bool open = true;
    for (int q = r + 1; q < s1; q++) {
      const int j = S.sp[q];
      if ((int64_t)(S.ts[j] & 0x7fffffffu) - tsi > a.within) { open = false; break; }
      if (cmpv<OP, V>(kt_val<V>(S.x[j]), yi)) { m = j; open = false; break; }
    }
    if (m >= toff && m < tend) {
      const uint32_t p = kt_tc_add(S.tc, m - toff, 1u);   // starts arrive in ascending i
      if (PASS == 1) kt_emit<OP, V>(a, S, bucket, key, m, i, base + p);
    } else if (PASS == 1 && open && last && a.ts_last_rel - tsi <= a.within) {
      a.carry[atomicAdd(a.ncarry, 1u)] = (int32_t)S.idx[i];
    }
  }
}

template <int OP, class V, int T, int H, int NT>
__global__ void __launch_bounds__(NT) k_kt_match(KtArgs a) {
  constexpr int L = T + H;
  constexpr int EPT = (L + NT - 1) / NT;
  __shared__ KtTile<T, L> S;
  __shared__ uint32_t wsum[NT / 64];
  __shared__ int32_t s_hs;
  __shared__ uint32_t s_base;
  const uint32_t td = a.tdesc[blockIdx.x];
  if (td == 0xffffffffu) return;
  const uint32_t b = td >> 20, tile = td & 0xfffff;
  const int64_t B0 = a.bstart[b], nb = (int64_t)a.bstart[b + 1] - B0;
  const int64_t s = (int64_t)tile * T, e = min<int64_t>(s + T, nb);
  const uint4* ent = a.ent + B0;
  const int t = threadIdx.x;
  // back-halo: probe every (H/64)th entry behind the tile (one wave), keep those within W of the first trigger
  constexpr int PS = H / 64;
  if (t < 64) {
    const uint32_t tsf = ent[s].y & 0x7fffffffu;
    const int64_t p = s - PS * (int64_t)(t + 1);
    bool in = false;
    if (p >= 0) in = (int64_t)tsf - (int64_t)(ent[p].y & 0x7fffffffu) <= a.within;
    // timestamps are non-decreasing, so the probes inside W are a prefix
    const int k = __popcll(__ballot(in));
    if (t == 0) {
      // probe k is the first outside W (or before the bucket): nothing before it is inside
      int64_t hs = max<int64_t>(0, s - PS * (int64_t)(k + 1) + 1);
      if (k == 64) { atomicOr(a.overflow, 1u); hs = -1; }   // the window may reach beyond H entries
      s_hs = (int32_t)hs;
    }
  }
  for (int k = t; k < KT_NL; k += NT) S.cnt[k] = 0;
  for (int k = t; k < T; k += NT) S.tc[k] = 0;
  __syncthreads();
  if (s_hs < 0) return;
  const int64_t hs = max<int64_t>(s_hs, s - H);
  const int Ln = (int)(e - hs), toff = (int)(s - hs), tend = (int)(e - hs);
  // stage: all loads in flight at once, then LDS stores + local-key histogram (unordered ranks)
  uint4 v[EPT];
  uint32_t rk[EPT];
#pragma unroll
  for (int k = 0; k < EPT; k++) {
    const int p = k * NT + t;
    if (p < Ln) v[k] = ent[hs + p];
  }
#pragma unroll
  for (int k = 0; k < EPT; k++) {
    const int p = k * NT + t;
    if (p < Ln) {
      S.ts[p] = v[k].y;
      S.x[p] = v[k].z;
      S.idx[p] = v[k].x;
      rk[k] = atomicAdd(&S.cnt[v[k].w], 1u);
    }
  }
  __syncthreads();
  kt_block_scan<NT>(S.cnt, KT_NL, wsum);
#pragma unroll
  for (int k = 0; k < EPT; k++) {
    const int p = k * NT + t;
    if (p < Ln) S.sp[S.cnt[v[k].w] + rk[k]] = (uint16_t)p;
  }
  __syncthreads();
  const bool last = e == nb;
  // pass 0: one lane per key run: arrival order inside the run, then record counts
  for (int k = t; k < KT_NL; k += NT) {
    const int s0 = S.cnt[k], s1 = k + 1 < KT_NL ? S.cnt[k + 1] : Ln;
    for (int p = s0 + 1; p < s1; p++) {
      const uint16_t x = S.sp[p];
      int q = p;
      while (q > s0 && S.sp[q - 1] > x) { S.sp[q] = S.sp[q - 1]; q--; }
      S.sp[q] = x;
    }
    kt_run<0, OP, V>(a, S, b, (uint32_t)k, s0, s1, toff, tend, last, 0u);
  }
  __syncthreads();
  const uint32_t nrec = kt_block_scan<NT>(S.tc, T, wsum);
  if (t == 0) {
    s_base = nrec ? atomicAdd(&a.bcur[b], nrec) : 0u;
    a.tdir[blockIdx.x] = make_uint2(s_base, nrec);
  }
  __syncthreads();
  if (nrec == 0 && !last) return;
  const uint32_t base = s_base;
  // pass 1: the same runs again, writing the records (and the carry at the end of the bucket)
  for (int k = t; k < KT_NL; k += NT) {
    const int s0 = S.cnt[k], s1 = k + 1 < KT_NL ? S.cnt[k + 1] : Ln;
    kt_run<1, OP, V>(a, S, b, (uint32_t)k, s0, s1, toff, tend, last, base);
  }
}

}  // namespace sg
