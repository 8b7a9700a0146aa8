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
  uint4* tdesc;               // [ntiles_max] {bucket, first trigger, end, halo start} (x = 0xffffffff: none)
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

// matcher tile table: tile w -> {bucket, first trigger, end, first halo entry} (bucket-relative).  The
// back-halo is exact: the first entry within W of the tile's first trigger, found by binary search over
// the (non-decreasing) timestamps of the KT_H entries before it.  A window reaching further back than KT_H
// entries raises the overflow flag (the flush is re-run by the sort pipeline).
__global__ void __launch_bounds__(KT_NT) k_kt_tdesc(KtArgs a) {
  const int64_t w = (int64_t)blockIdx.x * KT_NT + threadIdx.x;
  if (w >= a.ntiles_max) return;
  const int P = 1 << a.pb;
  const uint32_t total = a.tprefix[P];
  if (w >= total) { a.tdesc[w] = make_uint4(0xffffffffu, 0, 0, 0); return; }
  int lo = 0, hi = P - 1;                       // last b with tprefix[b] <= w
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (a.tprefix[mid] <= (uint32_t)w) lo = mid; else hi = mid - 1;
  }
  const uint32_t b = (uint32_t)lo, tile = (uint32_t)w - a.tprefix[lo];
  const uint32_t B0 = a.bstart[b], nb = a.bstart[b + 1] - B0;
  const uint32_t s = tile * (uint32_t)a.tile_t, e = min(s + (uint32_t)a.tile_t, nb);
  const uint4* ent = a.ent + B0;
  const int64_t tsf = ent[s].y & 0x7fffffffu;
  uint32_t l = s > KT_H ? s - KT_H : 0, h = s;    // first p in [l, s] with tsf - ts_p <= W
  if (l > 0 && tsf - (int64_t)(ent[l - 1].y & 0x7fffffffu) <= a.within) atomicOr(a.overflow, 1u);
  while (l < h) {
    const uint32_t mid = (l + h) >> 1;
    if (tsf - (int64_t)(ent[mid].y & 0x7fffffffu) <= a.within) h = mid; else l = mid + 1;
  }
  a.tdesc[w] = make_uint4(b, s, e, l);
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

// unconditional loads (callers clamp e): a branch around a load makes hipcc wait for it at once
template <int F1W>
__device__ __forceinline__ void kt_load(const KtArgs& a, int64_t e, KtRaw& r) {
  r.ts = a.ts[e];
  r.key = a.keycol[e];
  r.x = a.xcol[e];
  if constexpr (F1W == 8) r.f1 = ((const int64_t*)a.f1col)[e];
  else if constexpr (F1W == 4) r.f1 = (int64_t)((const int32_t*)a.f1col)[e];
  else r.f1 = 0;
}

// Stable partition of one super-tile, C events at a time; the next chunk's columns are loaded into
// registers while the current one is ranked and written.  LDS (dynamic, sized by P):
//   stage[KT_C] uint4 | sbk[KT_C] u16 | cnt[P] | cst[P] | cur[P]
template <int KT_C, int F1W>
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
  for (int k = 0; k < EPT; k++) kt_load<F1W>(a, min<int64_t>(e0 + k * KT_NT + threadIdx.x, e1 - 1), r[k]);
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
        const bool st = F1W == 0 || cmp(a.f1op, a.f1t, r[k].f1, a.f1c);
        v[k] = make_uint4((uint32_t)(c0 + q), (uint32_t)(r[k].ts - a.ts0) | (st ? 0x80000000u : 0u), r[k].x,
                          r[k].key >> a.pb);
        rk[k] = atomicAdd(&cnt[bk[k]], 1u);
      }
    }
    // prefetch the next chunk
#pragma unroll
    for (int k = 0; k < EPT; k++) kt_load<F1W>(a, min<int64_t>(c0 + KT_C + k * KT_NT + threadIdx.x, e1 - 1), r[k]);
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

template <class V>
__device__ __forceinline__ V kt_val(uint32_t b) {
  V v;
  __builtin_memcpy(&v, &b, 4);
  return v;
}

constexpr uint16_t KT_NONE = 0xffff, KT_OPEN = 0xfffe;

// Matcher tile (bucket b, triggers [s, e) + back-halo [hs, s)).  Each lane owns the local positions
// p = k*NT + t and keeps their entries in registers; LDS holds ts, x, the key-run order (sp, rp) and m.
//   stage     entries -> LDS, local-key histogram (LDS atomics), scan, placement; lane-per-key insertion
//             sort restores arrival order inside each key run (runs are ~(T+H)/2^KT_LB entries)
//   forward   every start walks its key run forward: first j within W with f2 -> m(i); per-trigger counts
//   scan      per-trigger offsets; one atomic per tile reserves the records in the bucket's region
//   rank      a start's rank among the starts completed by the same trigger (backward walk, bounded by W)
//   write     start lanes write {i, e1 projections}, trigger lanes write {j, e2 projections}
template <int OP, class V, int T, int H, int NT>
__global__ void __launch_bounds__(NT) k_kt_match(KtArgs a) {
  constexpr int L = T + H;
  constexpr int EPT = (L + NT - 1) / NT;
  __shared__ uint32_t s_ts[L];          // ts_rel | start << 31
  __shared__ uint32_t s_x[L];
  __shared__ uint16_t s_sp[L];          // sorted position -> local position
  __shared__ uint16_t s_rp[L];          // local position -> sorted position
  __shared__ uint16_t s_m[L];           // local position of m(i), KT_NONE / KT_OPEN
  __shared__ uint16_t s_tc[T];          // per-trigger record counts -> offsets (two u16 per word)
  __shared__ uint32_t s_cnt[KT_NL];     // local-key bins -> run starts
  __shared__ uint32_t wsum[NT / 64];
  __shared__ uint32_t s_base;
  const uint4 d = a.tdesc[blockIdx.x];
  if (d.x == 0xffffffffu) return;
  const uint32_t b = d.x;
  const uint4* ent = a.ent + a.bstart[b];
  const int64_t s = d.y, e = d.z, hs = d.w;
  const int Ln = (int)(e - hs), toff = (int)(s - hs), tend = (int)(e - hs);
  const int t = threadIdx.x;
  const bool last = e == (int64_t)(a.bstart[b + 1] - a.bstart[b]);
  // stage: every load in flight at once (clamped, unconditional)
  uint4 v[EPT];
#pragma unroll
  for (int k = 0; k < EPT; k++) v[k] = ent[hs + min(k * NT + t, Ln - 1)];
  for (int k = t; k < KT_NL; k += NT) s_cnt[k] = 0;
  for (int k = t; k < T / 2; k += NT) ((uint32_t*)s_tc)[k] = 0;
  __syncthreads();
  uint32_t rk[EPT];
#pragma unroll
  for (int k = 0; k < EPT; k++) {
    const int p = k * NT + t;
    if (p < Ln) {
      s_ts[p] = v[k].y;
      s_x[p] = v[k].z;
      rk[k] = atomicAdd(&s_cnt[v[k].w], 1u);
    }
  }
  __syncthreads();
  kt_block_scan<NT>(s_cnt, KT_NL, wsum);
#pragma unroll
  for (int k = 0; k < EPT; k++) {
    const int p = k * NT + t;
    if (p < Ln) s_sp[s_cnt[v[k].w] + rk[k]] = (uint16_t)p;
  }
  __syncthreads();
  for (int k = t; k < KT_NL; k += NT) {
    const int s0 = s_cnt[k], s1 = k + 1 < KT_NL ? s_cnt[k + 1] : Ln;
    for (int p = s0 + 1; p < s1; p++) {
      const uint16_t x = s_sp[p];
      int q = p;
      while (q > s0 && s_sp[q - 1] > x) { s_sp[q] = s_sp[q - 1]; q--; }
      s_sp[q] = x;
    }
  }
  __syncthreads();
  for (int q = t; q < Ln; q += NT) s_rp[s_sp[q]] = (uint16_t)q;
  __syncthreads();
  // forward: m(i) for the starts this lane owns
  uint16_t mr[EPT];
#pragma unroll
  for (int k = 0; k < EPT; k++) {
    const int p = k * NT + t;
    mr[k] = KT_NONE;
    if (p < Ln && (v[k].y >> 31)) {
      const int64_t tsi = v[k].y & 0x7fffffffu;
      const V yi = kt_val<V>(v[k].z);
      const int q = s_rp[p];
      const int send = v[k].w + 1 < KT_NL ? (int)s_cnt[v[k].w + 1] : Ln;
      uint16_t m = KT_OPEN;
      for (int r = q + 1; r < send; r++) {
        const int j = s_sp[r];
        if ((int64_t)(s_ts[j] & 0x7fffffffu) - tsi > a.within) { m = KT_NONE; break; }
        if (cmpv<OP, V>(kt_val<V>(s_x[j]), yi)) { m = (uint16_t)j; break; }
      }
      if (m < KT_OPEN && m >= toff) atomicAdd((uint32_t*)s_tc + ((m - toff) >> 1), ((m - toff) & 1) ? 0x10000u : 1u);
      mr[k] = m;
    }
    if (p < Ln) s_m[p] = mr[k];
  }
  __syncthreads();
  const uint32_t nrec = kt_block_scan<NT>(s_tc, T, wsum);
  if (t == 0) {
    const uint32_t base = nrec ? atomicAdd(&a.bcur[b], nrec) : 0u;   // in flight during the rank walks
    s_base = base;
    a.tdir[blockIdx.x] = make_uint2(base, nrec);
  }
  // rank: starts i' < i of the same key with m(i') = m(i); all lie within W before m(i)
  uint16_t rr[EPT];
#pragma unroll
  for (int k = 0; k < EPT; k++) {
    const int p = k * NT + t;
    rr[k] = 0;
    if (p < Ln && mr[k] < KT_OPEN && mr[k] >= toff) {
      const int q = s_rp[p], sb = s_cnt[v[k].w];
      const int64_t tsj = s_ts[mr[k]] & 0x7fffffffu;
      uint16_t c = 0;
      for (int r = q - 1; r >= sb; r--) {
        const int i = s_sp[r];
        if (tsj - (int64_t)(s_ts[i] & 0x7fffffffu) > a.within) break;
        c += s_m[i] == mr[k];
      }
      rr[k] = c;
    }
  }
  __syncthreads();
  const uint32_t base = s_base;
  const uint32_t key0 = 0;
  (void)key0;
#pragma unroll
  for (int k = 0; k < EPT; k++) {
    const int p = k * NT + t;
    if (p >= Ln) continue;
    const uint32_t key = (v[k].w << a.pb) | b;
    // as a start: {i, e1 projections}
    if (mr[k] < KT_OPEN && mr[k] >= toff) {
      int32_t* rp = a.rec + (int64_t)(base + s_tc[mr[k] - toff] + rr[k]) * a.stride;
      rp[1] = (int32_t)v[k].x;
      int wo = 2;
      for (int c = 0; c < a.nproj; c++) {
        const int src = a.src[c];
        if (src == KT_KEY || src == KT_XI || src == KT_COL_I) {
          int64_t val;
          if (src == KT_KEY) val = (int32_t)key;
          else if (src == KT_XI) val = (int32_t)v[k].z;
          else val = a.w[c] == 2 ? ((const int64_t*)a.col[c])[v[k].x] : (int64_t)((const int32_t*)a.col[c])[v[k].x];
          rp[wo] = (int32_t)val;
          if (a.w[c] == 2) rp[wo + 1] = (int32_t)(val >> 32);
        }
        wo += a.w[c];
      }
    } else if (mr[k] == KT_OPEN && last && a.ts_last_rel - (int64_t)(v[k].y & 0x7fffffffu) <= a.within) {
      a.carry[atomicAdd(a.ncarry, 1u)] = (int32_t)v[k].x;   // open at the end of the bucket
    }
    // as a trigger: {j, e2 projections} of each of its records
    if (p >= toff && p < tend) {
      const uint32_t o0 = s_tc[p - toff], o1 = p - toff + 1 < T ? s_tc[p - toff + 1] : nrec;
      for (uint32_t o = o0; o < o1; o++) {
        int32_t* rp = a.rec + (int64_t)(base + o) * a.stride;
        rp[0] = (int32_t)v[k].x;
        int wo = 2;
        for (int c = 0; c < a.nproj; c++) {
          const int src = a.src[c];
          if (src == KT_XJ || src == KT_COL_J) {
            int64_t val;
            if (src == KT_XJ) val = (int32_t)v[k].z;
            else val = a.w[c] == 2 ? ((const int64_t*)a.col[c])[v[k].x] : (int64_t)((const int32_t*)a.col[c])[v[k].x];
            rp[wo] = (int32_t)val;
            if (a.w[c] == 2) rp[wo + 1] = (int32_t)(val >> 32);
          }
          wo += a.w[c];
        }
      }
    }
  }
}

}  // namespace sg
