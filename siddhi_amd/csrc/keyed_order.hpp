// keyed_order.hpp — trigger-order pass of the keyed followed-by pipeline (config 4, the bench path): the
// matcher's records, written per tile in (j, i) order, are moved into the reference's callback order
// (ascending trigger index j, then start i: MultiProcessStreamReceiver's ReturnEventHolder flush order,
// MultiProcessStreamReceiver.java:306-316, across the partition instances PartitionStreamReceiver.java:82-282
// feeds one event at a time).  One workgroup per order group h of KS_HQ consecutive trigger indices gathers the
// group's piece of every bucket (rows toffs[h][b] written by the matcher tiles) and counting-sorts it by j.
#pragma once
#include "keyed_tiles.hpp"

namespace sg {

constexpr int KS_HQB = 14;                       // log2 trigger indices per order group
constexpr int KS_HQ = 1 << KS_HQB;
constexpr uint32_t KS_NONE = 0xffffffffu;        // no record slot
constexpr int KS_ORDER_NT = 1024;
constexpr int KS_ORDER_RPT = 8;                  // records per thread held in registers (4-word records)
constexpr int KS_ORDER_CAP = KS_ORDER_RPT * KS_ORDER_NT;
// 16-B records: loaded as a native vector and held as four scalar words.  HIP's uint4 (a union of member views)
// is copied through a private-memory memcpy, which put every record of the fast forms in scratch behind a
// vmcnt(0) per load; an array of native vectors is promoted to one 32-word vector copied whole at every
// conditional assignment (600+ B of spills).  Scalar arrays split into registers.
typedef uint32_t ko_v4 __attribute__((ext_vector_type(4)));
struct KoRec {
  uint32_t x[KS_ORDER_RPT], y[KS_ORDER_RPT], z[KS_ORDER_RPT], w[KS_ORDER_RPT];
  __device__ __forceinline__ void load(int u, const int32_t* p) {
    const ko_v4 v = *(const ko_v4*)p;
    x[u] = v.x; y[u] = v.y; z[u] = v.z; w[u] = v.w;
  }
  __device__ __forceinline__ void clear(int u) { x[u] = y[u] = z[u] = w[u] = 0; }
  __device__ __forceinline__ ko_v4 get(int u) const { return ko_v4{x[u], y[u], z[u], w[u]}; }
};

// ---- trigger order for the bucketed-tile matcher (keyed_tiles.hpp k_kt_match with toffs) -------------
// Rows toffs[h][b] = {slot, tile}: the record slot of bucket b's first record with trigger index >= h << KS_HQB,
// inside `tile`'s records.  The records of bucket b for group h run from row h to row h + 1 across the bucket's
// consecutive tiles -- almost always inside one tile, where the piece is [slot(h), slot(h + 1)) and needs no
// tile directory read.  Each bucket's piece is already in (j, i) order; k_kt_order counting-sorts the group by j.
struct KtOrderArgs {
  const uint2* toffs;
  const uint2* tdir;          // per tile {first record slot, records}
  const uint32_t* flags;      // [1]: the matcher overflowed (the flush is re-run by another pipeline)
  const int32_t* rec;
  int32_t stride, pb;
  int64_t nh;
  int32_t xcd;                // groups dealt XCD-contiguously (kt_xcd_index): neighbouring groups share lines
  int32_t slice_tiles;        // tiles are time slices aligned to the order groups (keyed_chunks.hpp): a group's
                              // piece of a bucket never leaves the tile its row h names
  // chunk mode (keyed_chunks.hpp): the matcher tile (s, b) writes gps u16 rows rows16[(s * P + b) * gps + g], the
  // first of its records (relative to its tdir slot) with trigger index >= (s * gps + g) << KS_HQB -- one
  // contiguous run per tile instead of toffs' P-strided uint2 rows.  toffs is unused then.
  const uint16_t* rows16;
  int32_t gps;                // order groups per slice
};

// chunk mode: {first record slot, records} of group h's piece in bucket b (unconditional loads: the end row of a
// slice's last group is replaced by the tile's record count after the load, not instead of it)
__device__ __forceinline__ uint2 kto_piece16(const KtOrderArgs& a, int64_t h, int b) {
  const int64_t s = h / a.gps;
  const int gl = (int)(h - s * a.gps);
  const int64_t W = (s << a.pb) + b;
  const uint2 d = a.tdir[W];
  const uint16_t* r = a.rows16 + W * a.gps;
  const uint32_t st = r[gl], en1 = r[min(gl + 1, a.gps - 1)];
  const uint32_t en = gl + 1 < a.gps ? en1 : d.y;
  return make_uint2(d.x + st, en - st);
}

__device__ __forceinline__ uint32_t kto_len(const KtOrderArgs& a, uint2 r0, uint2 r1) {
  if (r0.y == 0xffffffffu) return 0;          // a bucket without events: no tile wrote its rows
  if (r0.y == r1.y) return r1.x - r0.x;
  if (a.slice_tiles) {                         // the group ends its slice: the rest of row h's tile
    const uint2 d0 = a.tdir[r0.y];
    return d0.x + d0.y - r0.x;
  }
  const uint2 d0 = a.tdir[r0.y];
  uint32_t n = d0.x + d0.y - r0.x;             // the rest of r0's tile, the tiles between, r1's tile before r1
  for (uint32_t w = r0.y + 1; w < r1.y; w++) n += a.tdir[w].y;
  return n + (r1.x - a.tdir[r1.y].x);
}

// record slot of the k-th record of the piece starting at row r0
__device__ __forceinline__ int64_t kto_src(const KtOrderArgs& a, uint2 r0, uint32_t k) {
  uint32_t w = r0.y;
  uint2 d = a.tdir[w];
  uint32_t o = r0.x - d.x;
  while (o + k >= d.y) {          // past this tile's records: the next tile of the bucket
    k -= d.y - o;
    o = 0;
    d = a.tdir[++w];
  }
  return (int64_t)d.x + o + k;
}

__global__ void __launch_bounds__(256) k_kt_order_count(KtOrderArgs a, uint32_t* __restrict__ tot) {
  __shared__ uint32_t red[4];
  if (a.flags[1]) return;
  const int64_t h = a.xcd ? kt_xcd_index(blockIdx.x, (uint32_t)a.nh) : blockIdx.x;
  if (h >= a.nh) return;
  const int64_t P = (int64_t)1 << a.pb;
  uint32_t s = 0;
  if (a.rows16) {
#pragma unroll
    for (int u = 0; u < 2048 / 256; u++) {        // (P <= 2048: every row load of the group in flight at once)
      const int b = threadIdx.x + u * 256;
      const uint32_t len = kto_piece16(a, h, (int)min<int64_t>(b, P - 1)).y;
      s += b < P ? len : 0u;
    }
  }
  else
    for (int64_t b = threadIdx.x; b < P; b += 256) s += kto_len(a, a.toffs[h * P + b], a.toffs[(h + 1) * P + b]);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) tot[h] = red[0] + red[1] + red[2] + red[3];
}

// LDS (dynamic), 80 KB (two workgroups per CU): region A = 64 KB, then pp[P + 1] u32 | rw[P] uint2 (row h of
// each bucket) | pb[P] u32 (slot of the piece's first record, KS_NONE when the piece crosses tiles).
// Fast form (4-word records, at most KS_ORDER_CAP of them): A = hist[KS_HQ] u16 (counts, then offsets below
// KS_ORDER_CAP) | kk[KS_ORDER_CAP] u16 (trigger offset per record) | pm[KS_ORDER_CAP] u16 (piece per record);
// records are located through pm and pb (no search) and held in registers.  Streaming form: A = hist[KS_HQ]
// u32, records located by a search over pp and read twice.
// Chunk mode (rows16).  LDS (dynamic) 72 KB, two workgroups per CU: region A = 64 KB, then pp[P] u32 (each piece's
// first record in the group, then the slot delta of its records).  Fast form (4-word records, at most
// KS_ORDER_CAP): A = hist[KS_HQ] u16 | kk[KS_ORDER_CAP] u16 | pm[KS_ORDER_CAP] u16; streaming form: A = hist[KS_HQ]
// u32 and each record's piece found by a search over pp (its slot read from the rows again).
constexpr int KS_ORDER16_BPT = 2048 / KS_ORDER_NT;   // buckets per thread (P <= 2048)
__device__ __forceinline__ void kto_order16(const KtOrderArgs& a, int64_t h, const uint32_t* __restrict__ hbase,
                                            int32_t* __restrict__ out, uint32_t* ks_dyn, uint32_t* wsum) {
  const int P = 1 << a.pb;
  uint32_t* pp = ks_dyn + KS_HQ;
  const int t = threadIdx.x;
  uint32_t pbase[KS_ORDER16_BPT], plen[KS_ORDER16_BPT];
#pragma unroll
  for (int u = 0; u < KS_ORDER16_BPT; u++) {      // every bucket's row loads first (one round trip), then the stores
    const uint2 pc = kto_piece16(a, h, min(t + u * KS_ORDER_NT, P - 1));
    pbase[u] = pc.x;
    plen[u] = t + u * KS_ORDER_NT < P ? pc.y : 0u;
  }
#pragma unroll
  for (int u = 0; u < KS_ORDER16_BPT; u++)
    if (t + u * KS_ORDER_NT < P) pp[t + u * KS_ORDER_NT] = plen[u];
  __syncthreads();
  const uint32_t total = kt_block_scan<KS_ORDER_NT>(pp, P, wsum);
  __syncthreads();
  if (total == 0) return;
  const int64_t j0 = h << KS_HQB;
  const int S = a.stride;
  const int64_t ob = hbase[h];
  if (S == 4 && total <= (uint32_t)KS_ORDER_CAP) {
    uint16_t* hist = (uint16_t*)ks_dyn;
    uint16_t* kk = hist + KS_HQ;
    uint16_t* pm = kk + KS_ORDER_CAP;
    for (int k = t; k < KS_HQ / 2; k += KS_ORDER_NT) ((uint32_t*)hist)[k] = 0;
    uint32_t pfirst[KS_ORDER16_BPT];
#pragma unroll
    for (int u = 0; u < KS_ORDER16_BPT; u++) {            // record -> piece map
      const int b = t + u * KS_ORDER_NT;
      if (b < P) {
        pfirst[u] = pp[b];
        for (uint32_t r = pfirst[u], e = r + plen[u]; r < e; r++) pm[r] = (uint16_t)b;
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < KS_ORDER16_BPT; u++) {            // pp[b] becomes the slot delta of piece b's records
      const int b = t + u * KS_ORDER_NT;
      if (b < P) pp[b] = pbase[u] - pfirst[u];
    }
    __syncthreads();
    KoRec rv;
#pragma unroll
    for (int u = 0; u < KS_ORDER_RPT; u++) {
      const uint32_t r = (uint32_t)(t + u * KS_ORDER_NT);
      if (r < total) rv.load(u, a.rec + (int64_t)(pp[pm[r]] + r) * 4);
      else rv.clear(u);
    }
#pragma unroll
    for (int u = 0; u < KS_ORDER_RPT; u++) {
      const uint32_t r = (uint32_t)(t + u * KS_ORDER_NT);
      if (r < total) {
        const uint32_t key = (uint32_t)((int64_t)(int32_t)rv.x[u] - j0);
        kk[r] = (uint16_t)key;
        atomicAdd((uint32_t*)(hist + (key & ~1u)), 1u << (16 * (key & 1)));   // 16-bit bins in 32-bit words
      }
    }
    __syncthreads();
    kt_block_scan<KS_ORDER_NT>(hist, KS_HQ, wsum);
    __syncthreads();
    // a trigger's records are consecutive inside one piece (one bucket): its rank is the distance back to the first
    // record of the same trigger index
    uint32_t dst[KS_ORDER_RPT];
#pragma unroll
    for (int u = 0; u < KS_ORDER_RPT; u++) {
      const uint32_t r = (uint32_t)(t + u * KS_ORDER_NT);
      dst[u] = 0xffffffffu;
      if (r < total) {
        const uint32_t key = kk[r];
        uint32_t q = r;
        while (q > 0 && kk[q - 1] == key) q--;
        dst[u] = hist[key] + (r - q);
      }
    }
    __syncthreads();                                  // region A is free: it becomes the staging slice
    constexpr uint32_t SL = KS_HQ * 4 / 16;           // records per slice
    ko_v4* stage = (ko_v4*)ks_dyn;
    for (uint32_t c0 = 0; c0 < total; c0 += SL) {
#pragma unroll
      for (int u = 0; u < KS_ORDER_RPT; u++)
        if (dst[u] - c0 < SL) stage[dst[u] - c0] = rv.get(u);
      __syncthreads();
      const uint32_t m = min(SL, total - c0);
      for (uint32_t k = t; k < m; k += KS_ORDER_NT) *(ko_v4*)(out + (ob + c0 + k) * 4) = stage[k];
      __syncthreads();
    }
    return;
  }
  // streaming form: any record width, any group size
  uint32_t* hist = ks_dyn;
  for (int k = t; k < KS_HQ; k += KS_ORDER_NT) hist[k] = 0;
  __syncthreads();
  auto piece = [&](uint32_t r) -> int {        // last b with pp[b] <= r and a non-empty piece
    int lo = 0, hi = P - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pp[mid] <= r) lo = mid; else hi = mid - 1;
    }
    return lo;
  };
  auto src = [&](uint32_t r) -> int64_t {
    const int b = piece(r);
    return (int64_t)kto_piece16(a, h, b).x + (r - pp[b]);
  };
  for (uint32_t r = t; r < total; r += KS_ORDER_NT)
    atomicAdd(&hist[(uint32_t)((int64_t)a.rec[src(r) * S] - j0)], 1u);
  __syncthreads();
  kt_block_scan<KS_ORDER_NT>(hist, KS_HQ, wsum);
  __syncthreads();
  for (uint32_t r = t; r < total; r += KS_ORDER_NT) {
    const int64_t sr = src(r);
    const int32_t j = a.rec[sr * S];
    uint32_t rank = 0;
    while (rank < r && a.rec[src(r - rank - 1) * S] == j) rank++;
    int32_t* d = out + (ob + hist[(uint32_t)((int64_t)j - j0)] + rank) * S;
    for (int w = 0; w < S; w++) d[w] = a.rec[sr * S + w];
  }
}

__global__ void __launch_bounds__(KS_ORDER_NT) k_kt_order(KtOrderArgs a, const uint32_t* __restrict__ hbase,
                                                         int32_t* __restrict__ out) {
  extern __shared__ uint32_t ks_dyn[];
  __shared__ uint32_t wsum[KS_ORDER_NT / 64];
  if (a.flags[1]) return;
  const int64_t h = a.xcd ? kt_xcd_index(blockIdx.x, (uint32_t)a.nh) : blockIdx.x;
  if (h >= a.nh) return;
  const int P = 1 << a.pb;
  uint32_t* pp = ks_dyn + KS_HQ;
  const int t = threadIdx.x;
  if (a.rows16) { kto_order16(a, h, hbase, out, ks_dyn, wsum); return; }
  uint2* rw = (uint2*)(pp + P + 1 + ((P + 1) & 1));
  uint32_t* pb = (uint32_t*)(rw + P);
  for (int b = t; b < P; b += KS_ORDER_NT) {
    const uint2 r0 = a.toffs[h * P + b], r1 = a.toffs[(h + 1) * P + b];
    rw[b] = r0;
    pp[b] = kto_len(a, r0, r1);
    // a piece inside one tile (the usual case): its records are consecutive slots from row h's
    pb[b] = r0.y != 0xffffffffu && (r1.y == r0.y || a.slice_tiles) ? r0.x : KS_NONE;
  }
  __syncthreads();
  const uint32_t total = kt_block_scan<KS_ORDER_NT>(pp, P, wsum);
  if (t == 0) pp[P] = total;
  __syncthreads();
  if (total == 0) return;
  const int64_t j0 = h << KS_HQB;
  const int S = a.stride;
  const int64_t ob = hbase[h];
  if (S == 4 && total <= (uint32_t)KS_ORDER_CAP) {
    uint16_t* hist = (uint16_t*)ks_dyn;
    uint16_t* kk = hist + KS_HQ;
    uint16_t* pm = kk + KS_ORDER_CAP;
    for (int k = t; k < KS_HQ / 2; k += KS_ORDER_NT) ((uint32_t*)hist)[k] = 0;
    // record -> piece map: each piece writes its index over its records' positions
    for (int b = t; b < P; b += KS_ORDER_NT)
      for (uint32_t r = pp[b], e = pp[b + 1]; r < e; r++) pm[r] = (uint16_t)b;
    __syncthreads();
    KoRec rv;
#pragma unroll
    for (int u = 0; u < KS_ORDER_RPT; u++) {
      const uint32_t r = (uint32_t)(t + u * KS_ORDER_NT);
      if (r < total) {
        const int b = pm[r];
        const uint32_t base = pb[b];
        const int64_t src = base != KS_NONE ? (int64_t)base + (r - pp[b]) : kto_src(a, rw[b], r - pp[b]);
        rv.load(u, a.rec + src * 4);
      } else {
        rv.clear(u);
      }
    }
#pragma unroll
    for (int u = 0; u < KS_ORDER_RPT; u++) {
      const uint32_t r = (uint32_t)(t + u * KS_ORDER_NT);
      if (r < total) {
        const uint32_t key = (uint32_t)((int64_t)(int32_t)rv.x[u] - j0);
        kk[r] = (uint16_t)key;
        atomicAdd((uint32_t*)(hist + (key & ~1u)), 1u << (16 * (key & 1)));   // 16-bit bins in 32-bit words
      }
    }
    __syncthreads();
    kt_block_scan<KS_ORDER_NT>(hist, KS_HQ, wsum);
    __syncthreads();
    // each record's place in the group, then the group leaves through LDS in 64-KB slices, so consecutive lanes
    // store consecutive records (whole lines) instead of scattering 16-B stores over the group's range
    uint32_t dst[KS_ORDER_RPT];
#pragma unroll
    for (int u = 0; u < KS_ORDER_RPT; u++) {
      const uint32_t r = (uint32_t)(t + u * KS_ORDER_NT);
      dst[u] = 0xffffffffu;
      if (r < total) {
        const uint32_t key = kk[r], r0 = pp[pm[r]];
        uint32_t q = r;
        while (q > r0 && kk[q - 1] == key) q--;
        dst[u] = hist[key] + (r - q);
      }
    }
    __syncthreads();                                  // region A is free: it becomes the staging slice
    constexpr uint32_t SL = KS_HQ * 4 / 16;           // records per slice
    ko_v4* stage = (ko_v4*)ks_dyn;
    for (uint32_t c0 = 0; c0 < total; c0 += SL) {
#pragma unroll
      for (int u = 0; u < KS_ORDER_RPT; u++)
        if (dst[u] - c0 < SL) stage[dst[u] - c0] = rv.get(u);
      __syncthreads();
      const uint32_t m = min(SL, total - c0);
      for (uint32_t k = t; k < m; k += KS_ORDER_NT) *(ko_v4*)(out + (ob + c0 + k) * 4) = stage[k];
      __syncthreads();
    }
    return;
  }
  // streaming form: any record width, any group size (a trigger's records sit in one tile, contiguous)
  uint32_t* hist = ks_dyn;
  for (int k = t; k < KS_HQ; k += KS_ORDER_NT) hist[k] = 0;
  __syncthreads();
  auto piece = [&](uint32_t r) -> int {        // last b with pp[b] <= r
    int lo = 0, hi = P - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pp[mid] <= r) lo = mid; else hi = mid - 1;
    }
    return lo;
  };
  for (uint32_t r = t; r < total; r += KS_ORDER_NT) {
    const int b = piece(r);
    atomicAdd(&hist[(uint32_t)((int64_t)a.rec[kto_src(a, rw[b], r - pp[b]) * S] - j0)], 1u);
  }
  __syncthreads();
  kt_block_scan<KS_ORDER_NT>(hist, KS_HQ, wsum);
  __syncthreads();
  for (uint32_t r = t; r < total; r += KS_ORDER_NT) {
    const int b = piece(r);
    const uint32_t k = r - pp[b];
    const int64_t src = kto_src(a, rw[b], k);
    const int32_t j = a.rec[src * S];
    uint32_t rank = 0;
    while (rank < k && a.rec[kto_src(a, rw[b], k - rank - 1) * S] == j) rank++;
    int32_t* dst = out + (ob + hist[(uint32_t)((int64_t)j - j0)] + rank) * S;
    for (int w = 0; w < S; w++) dst[w] = a.rec[src * S + w];
  }
}

inline size_t kt_order16_lds(int P) { return (size_t)KS_HQ * 4 + (size_t)P * 4; }

inline size_t kt_order_lds(int P) {
  return (size_t)KS_HQ * 4 + ((size_t)P + 2) * 4 + (size_t)P * 8 + (size_t)P * 4;
}

}  // namespace sg
