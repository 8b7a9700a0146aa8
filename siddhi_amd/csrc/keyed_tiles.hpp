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
//   k_kt_match    one workgroup per (bucket, tile of KT_T triggers).  The tile plus its back-halo (the
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

constexpr int KT_NT = 512;          // threads per workgroup (8 waves)
constexpr int KT_LB = 10;           // local-key bits per bucket
constexpr int KT_NL = 1 << KT_LB;   // local keys per bucket
constexpr int KT_MAXPB = 12;        // at most 4096 buckets
constexpr int KT_C = 4096;          // scatter chunk (events staged in LDS)
constexpr int KT_ST = 65536;        // scatter super-tile (events per workgroup)
constexpr int KT_T = 4096;          // triggers per matcher tile
constexpr int KT_H = 2048;          // max back-halo entries
constexpr int KT_L = KT_T + KT_H;   // max staged entries
constexpr uint16_t KT_NONE = 0xffff, KT_OPEN = 0xfffe;

// exclusive scan in place of n = IPT * KT_NT values in LDS (thread t owns [t*IPT, (t+1)*IPT)); returns the total
template <int IPT, class T>
__device__ __forceinline__ uint32_t kt_block_scan(T* a, uint32_t* wsum) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t loc = 0;
#pragma unroll
  for (int k = 0; k < IPT; k++) loc += a[t * IPT + k];
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
  for (int k = 0; k < KT_NT / 64; k++) {
    const uint32_t v = wsum[k];
    base += k < w ? v : 0;
    tot += v;
  }
  uint32_t run = base + inc - loc;
#pragma unroll
  for (int k = 0; k < IPT; k++) {
    const uint32_t v = a[t * IPT + k];
    a[t * IPT + k] = (T)run;
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
  constexpr int IPT = (1 << KT_MAXPB) / KT_NT;
  for (int b = threadIdx.x; b < (1 << KT_MAXPB); b += KT_NT) {
    uint32_t c = 0;
    if (b < P) {
      const uint32_t s0 = a.hist[(int64_t)b * a.nst];
      const uint32_t s1 = b + 1 < P ? a.hist[(int64_t)(b + 1) * a.nst] : (uint32_t)a.n;
      a.bstart[b] = s0;
      a.bcur[b] = s0;
      c = (s1 - s0 + KT_T - 1) / KT_T;
    }
    tc[b] = c;
  }
  if (threadIdx.x == 0) a.bstart[P] = (uint32_t)a.n;
  __syncthreads();
  const uint32_t total = kt_block_scan<IPT>(tc, wsum);
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

// Stable partition of one super-tile, KT_C events at a time.
__global__ void __launch_bounds__(KT_NT) k_kt_scatter(KtArgs a) {
  __shared__ uint4 stage[KT_C];
  __shared__ uint16_t sbk[KT_C];
  __shared__ uint32_t cnt[1 << KT_MAXPB];
  __shared__ uint32_t cst[1 << KT_MAXPB];
  __shared__ uint32_t cur[1 << KT_MAXPB];
  __shared__ uint32_t wsum[KT_NT / 64];
  constexpr int IPT = (1 << KT_MAXPB) / KT_NT;
  constexpr int EPT = KT_C / KT_NT;
  const int P = 1 << a.pb;
  const uint32_t mask = (uint32_t)P - 1;
  for (int b = threadIdx.x; b < (1 << KT_MAXPB); b += KT_NT) {
    cur[b] = b < P ? a.hist[(int64_t)b * a.nst + blockIdx.x] : 0;
    cnt[b] = 0;
  }
  __syncthreads();
  const int64_t e0 = (int64_t)blockIdx.x * KT_ST, e1 = min<int64_t>(e0 + KT_ST, a.n);
  for (int64_t c0 = e0; c0 < e1; c0 += KT_C) {
    const int nc = (int)min<int64_t>(KT_C, e1 - c0);
    uint4 v[EPT];
    uint32_t bk[EPT], rk[EPT];
#pragma unroll
    for (int k = 0; k < EPT; k++) {
      const int q = k * KT_NT + threadIdx.x;
      if (q < nc) {
        const int64_t e = c0 + q;
        const uint32_t key = a.keycol[e];
        bk[k] = key & mask;
        const int64_t tr = a.ts[e] - a.ts0;
        v[k] = make_uint4((uint32_t)e, (uint32_t)tr | (kt_start(a, e) ? 0x80000000u : 0u), a.xcol[e], key >> a.pb);
        rk[k] = atomicAdd(&cnt[bk[k]], 1u);
      }
    }
    __syncthreads();
    kt_block_scan<IPT>(cnt, wsum);          // cnt -> chunk-local bucket starts (counts recovered below)
    // cst keeps the starts; cnt is rebuilt as counts from the start differences
#pragma unroll
    for (int k = 0; k < EPT; k++) {
      const int q = k * KT_NT + threadIdx.x;
      if (q < nc) {
        const uint32_t p = cnt[bk[k]] + rk[k];
        stage[p] = v[k];
        sbk[p] = (uint16_t)bk[k];
      }
    }
    for (int b = threadIdx.x; b < (1 << KT_MAXPB); b += KT_NT) cst[b] = cnt[b];
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

enum KtSrc { KT_KEY = 0, KT_XI, KT_XJ, KT_COL_I, KT_COL_J };

template <int OP, class V>
__global__ void __launch_bounds__(KT_NT) k_kt_match(KtArgs a) {
  __shared__ uint32_t s_ts[KT_L];       // ts_rel | start << 31
  __shared__ uint32_t s_x[KT_L];
  __shared__ uint16_t s_lk[KT_L];
  __shared__ uint16_t s_sp[KT_L];       // sorted position -> local position
  __shared__ uint16_t s_m[KT_L];        // local position of m(i), KT_NONE / KT_OPEN
  __shared__ uint16_t s_tc[KT_T];       // per-trigger record counts -> offsets
  __shared__ uint32_t s_cnt[KT_NL];
  __shared__ uint32_t wsum[KT_NT / 64];
  __shared__ int32_t s_hs;
  __shared__ uint32_t s_base;
  const uint32_t td = a.tdesc[blockIdx.x];
  if (td == 0xffffffffu) return;
  const uint32_t b = td >> 20, tile = td & 0xfffff;
  const int64_t B0 = a.bstart[b], nb = (int64_t)a.bstart[b + 1] - B0;
  const int64_t s = (int64_t)tile * KT_T, e = min<int64_t>(s + KT_T, nb);
  const uint4* ent = a.ent + B0;
  const int t = threadIdx.x;
  // back-halo: probe every 32nd entry behind the tile (one wave), keep those within W of the first trigger
  if (t < 64) {
    const uint32_t tsf = ent[s].y & 0x7fffffffu;
    const int64_t p = s - 32 * (int64_t)(t + 1);
    bool in = false;
    if (p >= 0) in = (int64_t)tsf - (int64_t)(ent[p].y & 0x7fffffffu) <= a.within;
    const unsigned long long bal = __ballot(in);
    // probes are monotone in p (timestamps are non-decreasing): count how many stay inside W
    const int k = __popcll(bal);
    if (t == 0) {
      // probe k (at s - 32(k+1)) is the first outside W or before the bucket: nothing before it is inside
      int64_t hs = max<int64_t>(0, s - 32 * (int64_t)(k + 1) + 1);
      if (k == 64) { atomicOr(a.overflow, 1u); hs = -1; }   // the window may reach beyond KT_H entries
      s_hs = (int32_t)hs;
    }
  }
  for (int k = t; k < KT_NL; k += KT_NT) s_cnt[k] = 0;
  for (int k = t; k < KT_T; k += KT_NT) s_tc[k] = 0;
  __syncthreads();
  if (s_hs < 0) return;
  const int64_t hs = max<int64_t>(s_hs, s - KT_H);
  const int L = (int)(e - hs), toff = (int)(s - hs), tend = (int)(e - hs);
  // stage + local-key histogram (unordered ranks)
  for (int p = t; p < L; p += KT_NT) {
    const uint4 v = ent[hs + p];
    s_ts[p] = v.y;
    s_x[p] = v.z;
    s_lk[p] = (uint16_t)v.w;
    s_m[p] = (uint16_t)atomicAdd(&s_cnt[v.w], 1u);   // rank, parked in s_m
  }
  __syncthreads();
  kt_block_scan<KT_NL / KT_NT>(s_cnt, wsum);
  for (int p = t; p < L; p += KT_NT) s_sp[s_cnt[s_lk[p]] + s_m[p]] = (uint16_t)p;
  __syncthreads();
  // arrival order inside each key run
  for (int k = t; k < KT_NL; k += KT_NT) {
    const uint32_t s0 = s_cnt[k], s1 = k + 1 < KT_NL ? s_cnt[k + 1] : (uint32_t)L;
    for (uint32_t p = s0 + 1; p < s1; p++) {
      const uint16_t x = s_sp[p];
      uint32_t q = p;
      while (q > s0 && s_sp[q - 1] > x) { s_sp[q] = s_sp[q - 1]; q--; }
      s_sp[q] = x;
    }
  }
  __syncthreads();
  // every start: forward walk over its key run
  for (int q = t; q < L; q += KT_NT) {
    const int i = s_sp[q];
    const uint32_t ti = s_ts[i];
    uint16_t m = KT_NONE;
    if (ti >> 31) {
      const uint16_t key = s_lk[i];
      const int64_t tsi = ti & 0x7fffffffu;
      uint32_t xb = s_x[i];
      V yi;
      __builtin_memcpy(&yi, &xb, 4);
      m = KT_OPEN;
      for (int r = q + 1; r < L; r++) {
        const int j = s_sp[r];
        if (s_lk[j] != key) break;
        if ((int64_t)(s_ts[j] & 0x7fffffffu) - tsi > a.within) { m = KT_NONE; break; }
        uint32_t xjb = s_x[j];
        V xj;
        __builtin_memcpy(&xj, &xjb, 4);
        if (cmpv<OP, V>(xj, yi)) { m = (uint16_t)j; break; }
      }
      // per-trigger record counts for the triggers of this tile (two u16 counters per LDS word)
      if (m < KT_OPEN && m >= toff) atomicAdd((uint32_t*)s_tc + ((m - toff) >> 1), ((m - toff) & 1) ? 0x10000u : 1u);
    }
    s_m[i] = m;
  }
  __syncthreads();
  const uint32_t nrec = kt_block_scan<KT_T / KT_NT>(s_tc, wsum);
  if (t == 0) {
    s_base = nrec ? atomicAdd(&a.bcur[b], nrec) : 0u;
    a.tdir[blockIdx.x] = make_uint2(s_base, nrec);
  }
  __syncthreads();
  const uint32_t base = s_base;
  // triggers: walk back over the key run, write records in ascending i
  if (nrec) {
    for (int q = t; q < L; q += KT_NT) {
      const int j = s_sp[q];
      if (j < toff || j >= tend) continue;
      const uint32_t o0 = s_tc[j - toff], o1 = j - toff + 1 < KT_T ? s_tc[j - toff + 1] : nrec;
      if (o1 == o0) continue;
      const uint16_t key = s_lk[j];
      const int64_t tsj = s_ts[j] & 0x7fffffffu;
      uint32_t w = o1;
      const int64_t jg = ent[hs + j].x;   // global index of j (entries are L2-hot)
      for (int r = q - 1; r >= 0 && w > o0; r--) {
        const int i = s_sp[r];
        if (s_lk[i] != key) break;
        if (tsj - (int64_t)(s_ts[i] & 0x7fffffffu) > a.within) break;
        if (s_m[i] != j) continue;
        w--;
        int32_t* rp = a.rec + (int64_t)(base + w) * a.stride;
        const int64_t ig = ent[hs + i].x;
        rp[0] = (int32_t)jg;
        rp[1] = (int32_t)ig;
        int wo = 2;
        for (int c = 0; c < a.nproj; c++) {
          int64_t v;
          switch (a.src[c]) {
            case KT_KEY: v = (int32_t)(((uint32_t)s_lk[i] << a.pb) | b); break;
            case KT_XI: v = (int32_t)s_x[i]; break;
            case KT_XJ: v = (int32_t)s_x[j]; break;
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
    }
  }
  // starts still open at the end of the bucket: carried to the next flush
  if (e == nb) {
    for (int i = t; i < L; i += KT_NT) {
      if (s_m[i] != KT_OPEN) continue;
      if (a.ts_last_rel - (int64_t)(s_ts[i] & 0x7fffffffu) > a.within) continue;   // can never complete
      a.carry[atomicAdd(a.ncarry, 1u)] = (int32_t)ent[hs + i].x;
    }
  }
}

}  // namespace sg
