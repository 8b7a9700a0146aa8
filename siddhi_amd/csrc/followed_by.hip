// followed_by.hip — execution path SG_PATH_FOLLOWED_BY.
//
// Query shape:  from every e1=A[f1] -> e2=B[f2(e1,e2)] (within W)?  select <projection of e1/e2>
//
// Reference semantics (restated, see oracle/siddhi_oracle.cpp for the object-level version):
//   * e1's pre-processor always holds one empty partial (every re-seeds it through
//     StreamPostStateProcessor.process -> addEveryState, StreamPreStateProcessor.java:229-247),
//     so a partial is created for event i iff i is an A event and f1(i) holds.
//   * the partial becomes visible to e2 at the next arrival (newAndEvery -> pending in
//     updateState, :307-323); e2 is processed before e1 for the same event (reverse order,
//     PatternMultiProcessStreamReceiver.java:29-39), so candidates are j > i.
//   * before each arrival j the partial expires iff |ts_i - ts_j| > W (isExpired :118-129, strict);
//     with non-decreasing timestamps the head-`break` in expireEvents (:340-341) removes exactly
//     the expired prefix, so expiry is the closed form  ts_j - ts_i > W.
//   * the first B event j with f2(i, j) completes the match and removes the partial (stateChanged).
//   => m(i) = min{ j > i : j in B, ts_j - ts_i <= W, f2(i,j) }, emitted at j, and all matches
//      completing at the same j are emitted in pending-list order = ascending i.
//   * callback grouping: when A == B the stream has a PatternMultiProcessStreamReceiver and every
//     (event, processor) pair gets one ReturnEventHolder -> one QueryCallback per distinct j
//     (MultiProcessStreamReceiver.java:216-241); when A != B, B's receiver is a
//     PatternSingleProcessStreamReceiver and every match is its own callback (:48-73).
//
// Kernels (gfx950):
//   k_fb_tile<OP,V>   the hot path (single stream, f2 = `e2.x OP e1.y`).  One 512-thread workgroup
//                     owns a tile of T trigger events [J0, J0+T) and stages ts/x/y of
//                     [J0-H, J0+T) in LDS (coalesced 8/4-byte loads).  Every start in that region is
//                     scanned forward in LDS: phase 1 gives each lane S1 steps; the unresolved starts
//                     are compacted into an LDS queue and re-spread over all lanes (phase 2), so the
//                     heavy tail of long scans does not serialise whole waves.  Matches landing in
//                     the tile are bucketed by j with LDS atomics + a block scan, each bucket is
//                     ordered by i, and records + select-list columns are written contiguously.
//                     A start still open at the end of the last tile covering it (a "long-range"
//                     start, scan > H events) goes to an overflow list.
//   k_fb_list_atom    long-range / carried starts: forward scan in HBM from a resume index.
//   k_fb_scan         generic predicates (bytecode interpreter, LDS register file) and two-stream
//                     queries: one lane per start.
//   radix sort        (j, i) order of the list-path matches (few), merged before the tile records
//                     of the same j (their i are smaller by construction).
// Non-decreasing timestamps are required (checked at push); otherwise SG_E_UNSUPPORTED.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>

#include "fb_shape.hpp"
#include "runtime.hpp"
#include "snapshot.hpp"

namespace sg {

constexpr int FB_MAXC = 12;
constexpr int TILE_B = 512;       // threads per tile workgroup
constexpr int TILE_S1 = 8;        // phase-1 scan steps per start (r06b: 32 -> 4.22 ms, 16 -> 3.67, 8 -> 3.67, 4 -> 4.17 per 100M)
constexpr int GEN_B = 256;        // threads per workgroup of the list / generic kernels

struct FBCols {
  const uint8_t* a[FB_MAXC];
  const uint8_t* b[FB_MAXC];
  int32_t aw[FB_MAXC];
  int32_t bw[FB_MAXC];
};

struct FBLoader {
  const FBCols* c;
  int64_t i, j;
  __device__ __forceinline__ bool load(int slot, int attr, int64_t& v) const {
    const uint8_t* col = slot == 0 ? c->a[attr] : c->b[attr];
    int w = slot == 0 ? c->aw[attr] : c->bw[attr];
    int64_t idx = slot == 0 ? i : j;
    if (w == 8) v = ((const int64_t*)col)[idx];
    else v = (int64_t)((const int32_t*)col)[idx];
    return true;
  }
};


// ------------------------------------------------------------------------------------------------
// Generic scan (bytecode predicates): new starts [new_lo, n) and/or an (i, resume) list.
struct FBScanArgs {
  const int64_t* ts;
  const uint8_t* tag;     // bit0 = A event, bit1 = B event (nullptr: every event is both)
  int64_t n;
  int64_t within;         // -1: no within
  int64_t new_lo;         // first new start index (n: list only)
  int64_t start_end;      // events at or past this index start no partial (halo, sg_set_halo)
  int32_t n_list;
  const int32_t* list_i;
  const int32_t* list_j;
  uint64_t* keys;
  uint32_t* nkeys;
  int32_t* npend_i;
  int32_t* npend_j;
  uint32_t* nnpend;
};

__global__ void __launch_bounds__(GEN_B) k_fb_scan(FBScanArgs a, const FBCols* __restrict__ cols,
                                                    const Prog* __restrict__ progs) {
  __shared__ int64_t rf[MAX_REG * GEN_B];
  int64_t* myrf = rf + threadIdx.x;
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t i, j0;
  FBLoader ld{cols, 0, 0};
  if (t < a.n_list) {
    i = a.list_i[t];
    j0 = a.list_j[t];
  } else {
    i = a.new_lo + (t - a.n_list);
    if (i >= a.n || i >= a.start_end) return;
    if (a.tag && !(a.tag[i] & 1)) return;
    ld.i = i;
    if (!run_pred(progs[0], ld, myrf, GEN_B)) return;
    j0 = i + 1;
  }
  ld.i = i;
  const int64_t tsi = a.ts[i];
  for (int64_t j = j0; j < a.n; j++) {
    if (a.within >= 0 && a.ts[j] - tsi > a.within) return;   // expired before j
    if (a.tag && !(a.tag[j] & 2)) continue;
    ld.j = j;
    if (run_pred(progs[1], ld, myrf, GEN_B)) {
      uint32_t k = atomicAdd(a.nkeys, 1u);
      a.keys[k] = ((uint64_t)j << 32) | (uint64_t)i;
      return;
    }
  }
  uint32_t k = atomicAdd(a.nnpend, 1u);
  a.npend_i[k] = (int32_t)i;
  a.npend_j[k] = (int32_t)a.n;
}

// Long-range / carried starts for the atom fast path: (i, resume) list, scan in HBM.
template <int OP, class V>
__global__ void __launch_bounds__(GEN_B) k_fb_list_atom(FBScanArgs a, const V* __restrict__ x,
                                                         const V* __restrict__ y) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.n_list) return;
  const int64_t i = a.list_i[t];
  const V yi = y[i];
  const int64_t tsi = a.ts[i];
  for (int64_t j = a.list_j[t]; j < a.n; j++) {
    if (a.within >= 0 && a.ts[j] - tsi > a.within) return;
    if (cmpv<OP, V>(x[j], yi)) {
      uint32_t k = atomicAdd(a.nkeys, 1u);
      a.keys[k] = ((uint64_t)j << 32) | (uint64_t)i;
      return;
    }
  }
  uint32_t k = atomicAdd(a.nnpend, 1u);
  a.npend_i[k] = (int32_t)i;
  a.npend_j[k] = (int32_t)a.n;
}

// ------------------------------------------------------------------------------------------------
// The tile kernel.
struct TileArgs {
  const int64_t* ts;
  const uint8_t* x;        // e2-side column of the f2 atom
  const uint8_t* y;        // e1-side column
  int32_t same_xy;
  int64_t n;
  int64_t j_lo;            // first trigger index of this flush (starts < j_lo belong to the list path)
  int64_t start_end;       // events at or past this index start no partial (halo, sg_set_halo)
  int64_t within;
  int32_t T, H;
  int32_t s1;              // phase-1 steps per start (lane per start) before the start joins the phase-2 queue
  // f1: 0 = always, 1 = atom `col OP const` (typed), 2 = precomputed start flags
  int32_t f1kind, f1op, f1t, f1w;
  const uint8_t* f1col;
  int64_t f1c;
  const uint8_t* f1flags;
  // outputs
  int32_t* seg_j;          // ntiles * cap
  int32_t* seg_i;          // optional (generic projection)
  int32_t cap;
  int32_t nproj;
  const uint8_t* pcol[FB_MAXP];   // plain-variable projection: source column
  int32_t pslot[FB_MAXP];         // 0 = e1 (i), 1 = e2 (j)
  int32_t pw[FB_MAXP];
  uint8_t* pout[FB_MAXP];         // ntiles * cap values of width pw
  int32_t* tile_cnt;
  int32_t* ovf_i;
  int32_t* ovf_j;
  uint32_t* n_ovf;
  uint32_t* unsorted;      // set when the staged timestamps go backwards
};

__device__ __forceinline__ bool f1_atom(const TileArgs& a, int64_t g) {
  int64_t v = a.f1w == 8 ? ((const int64_t*)a.f1col)[g] : (int64_t)((const int32_t*)a.f1col)[g];
  return cmp(a.f1op, a.f1t, v, a.f1c);
}

// block-wide exclusive scan of cnt[0..T) in place; returns the total (all threads)
__device__ int block_exclusive_scan(int32_t* cnt, int T, int32_t* wave_tot) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int per = (T + TILE_B - 1) / TILE_B;
  const int beg = tid * per, end = min(T, beg + per);
  int s = 0;
  for (int k = beg; k < end; k++) s += cnt[k];
  const int incl = (int)sg_wave_scan((uint32_t)s);
  if (lane == 63) wave_tot[wid] = incl;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int w = 0; w < TILE_B / 64; w++) { int v = wave_tot[w]; wave_tot[w] = acc; acc += v; }
    wave_tot[TILE_B / 64] = acc;
  }
  __syncthreads();
  int run = wave_tot[wid] + incl - s;
  for (int k = beg; k < end; k++) { int c = cnt[k]; cnt[k] = run; run += c; }
  __syncthreads();
  return wave_tot[TILE_B / 64];
}

template <int OP, class V>
__global__ void __launch_bounds__(TILE_B) k_fb_tile(TileArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int T = a.T, H = a.H, R = T + H;
  const int tid = threadIdx.x;
  int64_t* s_ts = (int64_t*)smem;
  V* s_x = (V*)(s_ts + R);
  V* s_y = a.same_xy ? s_x : s_x + R;
  int32_t* s_m = (int32_t*)(a.same_xy ? s_x + R : s_x + 2 * R);
  int32_t* s_scr = s_m + R;             // T + R ints: queue (scan) / cnt + out (emit)
  int32_t* s_misc = s_scr + T + R;      // 16 ints: queue length, wave totals
  const int64_t J0 = a.j_lo + (int64_t)blockIdx.x * T;
  const int64_t J1 = min(J0 + (int64_t)T, a.n);
  const int64_t R0 = max(a.j_lo, J0 - H);
  const int nr = (int)(J1 - R0);
  const int jo = (int)(J0 - R0);        // local index of the first trigger of the tile
  const int64_t W = a.within;
  if (tid == 0) s_misc[0] = 0;
  // ---- stage the region ----
  for (int k = tid; k < nr; k += TILE_B) {
    const int64_t g = R0 + k;
    s_ts[k] = a.ts[g];
    s_x[k] = ((const V*)a.x)[g];
    if (!a.same_xy) s_y[k] = ((const V*)a.y)[g];
    bool st = g < a.start_end && (a.f1kind == 0 ? true : (a.f1kind == 1 ? f1_atom(a, g) : a.f1flags[g] != 0));
    s_m[k] = st ? -3 : -1;
  }
  __syncthreads();
  {  // non-decreasing timestamps (consecutive tiles overlap by the halo, so every pair is seen)
    bool bad = false;
    for (int k = tid + 1; k < nr; k += TILE_B) bad |= s_ts[k] < s_ts[k - 1];
    if (__any(bad) && (tid & 63) == 0) atomicOr(a.unsorted, 1u);
  }
  // ---- phase 1: one lane per start, S1 steps, LDS reads issued 4 at a time ----
  for (int k = tid; k < nr; k += TILE_B) {
    if (s_m[k] != -3) continue;
    const V yk = s_y[k];
    const int64_t t0 = s_ts[k];
    const int lim = min(nr, k + 1 + a.s1);
    int res = -3, j = k + 1;
    while (j < lim && res == -3) {
      V xv[4];
      int64_t tv[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int jj = min(j + u, nr - 1);
        xv[u] = s_x[jj];
        tv[u] = s_ts[jj];
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (res != -3 || j >= lim) break;
        if (W >= 0 && tv[u] - t0 > W) res = -1;            // expired before event j
        else if (cmpv<OP, V>(xv[u], yk)) res = j;         // first match
        else j++;
      }
    }
    if (res == -3) {
      if (j >= nr) res = -2;
      else { int q = atomicAdd(&s_misc[0], 1); s_scr[q] = (k << 16) | j; }
    }
    s_m[k] = res;
  }
  __syncthreads();
  // ---- phase 2: the compacted tail, one queue entry per wave, 64 candidates per step ----
  // Queue entries are dealt to waves statically with wave-uniform (SGPR) indices: a lane-0 atomic
  // broadcast by a shuffle lets the compiler split the loop per lane and never reconverge.  A wave takes
  // PQ entries at a time and issues their first 64-candidate blocks together (their LDS reads overlap); an
  // entry still open after its first block continues alone (a run of 64 non-matching candidates is rare).
  {
    constexpr int PQ = 4;
    const int qn = __builtin_amdgcn_readfirstlane(s_misc[0]);
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int q0 = wid * PQ; q0 < qn; q0 += (TILE_B / 64) * PQ) {
      int kq[PQ], jq[PQ];
      V yq[PQ], xq[PQ];
      int64_t tq[PQ], tj[PQ];
#pragma unroll
      for (int u = 0; u < PQ; u++) {
        const int e = s_scr[min(q0 + u, qn - 1)];
        kq[u] = e >> 16;
        jq[u] = e & 0xffff;
      }
#pragma unroll
      for (int u = 0; u < PQ; u++) {
        yq[u] = s_y[kq[u]];
        tq[u] = s_ts[kq[u]];
        const int j = min(jq[u] + lane, nr - 1);
        xq[u] = s_x[j];
        tj[u] = s_ts[j];
      }
#pragma unroll
      for (int u = 0; u < PQ; u++) {
        if (q0 + u >= qn) break;                        // (uniform)
        int res = -2;
        bool open = true;
        {
          const int j = jq[u] + lane;
          const bool in = j < nr;
          const bool ex = in && W >= 0 && tj[u] - tq[u] > W;
          const bool hit = in && !ex && cmpv<OP, V>(xq[u], yq[u]);
          const unsigned long long me = __ballot(ex), mh = __ballot(hit);
          if (me | mh) {
            const int fe = me ? __ffsll(me) - 1 : 64;
            const int fh = mh ? __ffsll(mh) - 1 : 64;
            res = fh < fe ? jq[u] + fh : -1;
            open = false;
          }
        }
        for (int jb = jq[u] + 64; open && jb < nr; jb += 64) {
          const int j = jb + lane;
          const bool in = j < nr;
          const bool ex = in && W >= 0 && s_ts[j] - tq[u] > W;
          const bool hit = in && !ex && cmpv<OP, V>(s_x[j], yq[u]);
          const unsigned long long me = __ballot(ex), mh = __ballot(hit);
          if (me | mh) {
            const int fe = me ? __ffsll(me) - 1 : 64;
            const int fh = mh ? __ffsll(mh) - 1 : 64;
            res = fh < fe ? jb + fh : -1;
            open = false;
          }
        }
        if (lane == 0) s_m[kq[u]] = res;
      }
    }
  }
  __syncthreads();
  // ---- overflow: open starts not covered by the next tile's region ----
  const bool last = J1 >= a.n;
  for (int k = tid; k < nr; k += TILE_B) {
    if (s_m[k] != -2) continue;
    const int64_t g = R0 + k;
    bool flag;
    int64_t resume = J1;
    if (last) flag = true;                               // carried to the next flush
    else if (g < J1 - H) flag = (W < 0) || (a.ts[J1] - s_ts[k] <= W);
    else flag = false;                                   // the next tile re-scans it
    if (flag) {
      uint32_t o = atomicAdd(a.n_ovf, 1u);
      a.ovf_i[o] = (int32_t)g;
      a.ovf_j[o] = (int32_t)resume;
    }
  }
  // ---- bucket matches by trigger j (reference emission order: ascending j, then ascending i) ----
  int32_t* cnt = s_scr;
  int32_t* outb = s_scr + T;
  for (int k = tid; k < T; k += TILE_B) cnt[k] = 0;
  __syncthreads();
  for (int k = tid; k < nr; k += TILE_B) {
    int m = s_m[k];
    if (m >= jo) atomicAdd(&cnt[m - jo], 1);
  }
  __syncthreads();
  const int total = block_exclusive_scan(cnt, T, s_misc + 1);
  for (int k = tid; k < nr; k += TILE_B) {
    int m = s_m[k];
    if (m >= jo) {
      int pos = atomicAdd(&cnt[m - jo], 1);
      outb[pos] = ((m - jo) << 13) | k;
    }
  }
  __syncthreads();
  // after placement cnt[jl] = end of bucket jl; bucket jl = [cnt[jl-1], cnt[jl])
  for (int jl = tid; jl < T; jl += TILE_B) {
    int beg = jl == 0 ? 0 : cnt[jl - 1], end = cnt[jl];
    for (int p = beg + 1; p < end; p++) {          // insertion sort by i (buckets are tiny)
      int v = outb[p], q = p - 1;
      while (q >= beg && outb[q] > v) { outb[q + 1] = outb[q]; q--; }
      outb[q + 1] = v;
    }
  }
  __syncthreads();
  // ---- emit records and the plain-variable projection ----
  const int64_t base = (int64_t)blockIdx.x * a.cap;
  for (int p = tid; p < total; p += TILE_B) {
    const int rec = outb[p];
    const int64_t j = J0 + (rec >> 13);
    const int64_t i = R0 + (rec & 8191);
    a.seg_j[base + p] = (int32_t)j;
    if (a.seg_i) a.seg_i[base + p] = (int32_t)i;
    for (int c = 0; c < a.nproj; c++) {
      const int64_t src = a.pslot[c] == 0 ? i : j;
      if (a.pw[c] == 8) ((int64_t*)a.pout[c])[base + p] = ((const int64_t*)a.pcol[c])[src];
      else ((int32_t*)a.pout[c])[base + p] = ((const int32_t*)a.pcol[c])[src];
    }
  }
  if (tid == 0) a.tile_cnt[blockIdx.x] = total;
}

// ------------------------------------------------------------------------------------------------
// Compaction of the per-tile segments into one dense array (materialisation only).
__global__ void __launch_bounds__(256) k_fb_compact(const int32_t* __restrict__ tile_cnt,
                                                     const int64_t* __restrict__ tile_off, int32_t cap,
                                                     const int32_t* __restrict__ seg, int32_t* __restrict__ dst) {
  const int t = blockIdx.x;
  const int c = tile_cnt[t];
  const int64_t o = tile_off[t];
  for (int p = threadIdx.x; p < c; p += blockDim.x) dst[o + p] = seg[(int64_t)t * cap + p];
}

// select-list evaluation for (j, i) pairs (generic projection / list-path records)
struct FBProjArgs {
  const int32_t* j;
  const int32_t* i;
  const uint64_t* keys;    // alternatively packed (j << 32 | i)
  int64_t m;
  int32_t nout;
  int64_t* out_raw;        // m * nout
  uint8_t* out_null;       // m * nout
};

__global__ void __launch_bounds__(GEN_B) k_fb_project(FBProjArgs a, const FBCols* __restrict__ cols,
                                                       const Prog* __restrict__ sel) {
  __shared__ int64_t rf[MAX_REG * GEN_B];
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.m) return;
  int64_t j, i;
  if (a.keys) { uint64_t key = a.keys[k]; j = (int64_t)(key >> 32); i = (int64_t)(key & 0xffffffffu); }
  else { j = a.j[k]; i = a.i[k]; }
  FBLoader ld{cols, i, j};
  for (int c = 0; c < a.nout; c++) {
    int64_t v = 0;
    bool isnull = false;
    run(sel[c], ld, v, isnull, rf + threadIdx.x, GEN_B);
    a.out_raw[k * a.nout + c] = v;
    a.out_null[k * a.nout + c] = isnull;
  }
}

// ------------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------------
struct FollowedByExec : Exec {
  int sA = -1, sB = -1;
  bool same = false;
  int64_t within = -1;
  Prog progs[2];
  std::vector<Prog> sel;
  FastPath fp;
  int tileT = 2048, tileH = 512;
  // event buffer (device)
  int64_t n = 0;
  DBuf<int64_t> ts;
  DBuf<uint8_t> tag;
  std::vector<DCol> colA, colB;
  const int64_t* ext_ts = nullptr;               // adopted device input (push_device)
  std::vector<const void*> ext_cols;
  std::vector<int64_t> h_seq;                    // host mirror: arrival seq per buffered event
  int64_t last_ts = INT64_MIN;
  int64_t examined = 0;                          // trigger/start indices [0, examined) done
  int64_t start_end = INT64_MAX;                 // halo: events at or past this index start nothing
  DBuf<int32_t> pend_i, pend_j, npend_i, npend_j;
  int32_t n_pend = 0;
  DBuf<uint64_t> keys, keys_sorted;
  DBuf<uint32_t> counters;
  DBuf<uint8_t> sort_tmp;
  DBuf<FBCols> d_cols;
  DBuf<Prog> d_progs, d_sel;
  // tile outputs
  DBuf<int32_t> seg_j, seg_i, tile_cnt, dense_j, dense_i;
  std::vector<DBuf<uint8_t>> seg_p;
  DBuf<int64_t> tile_off;
  DBuf<int64_t> out_raw;
  DBuf<uint8_t> out_null;
  int64_t ntiles_last = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;

  ~FollowedByExec() override {
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
  }

  int arity(int s) const { return (int)app->streams[s].types.size(); }
  const int64_t* d_ts() const { return ext_ts ? ext_ts : ts.p; }
  const uint8_t* colptr(int slot, int c) const {
    if (ext_ts) return (const uint8_t*)ext_cols[c];
    const std::vector<DCol>& v = (slot == 0 || same) ? colA : colB;
    return v[c].b.p;
  }

  void ensure_cap(int64_t need, hipStream_t s) {
    if (ext_ts) throw Error(-2, "cannot append host events after device-resident ingest");
    ts.reserve(need, true, s, n);
    if (!same) tag.reserve(need, true, s, n);
    for (auto& c : colA) c.b.reserve(need * c.w, true, s, n * c.w);
    for (auto& c : colB) c.b.reserve(need * c.w, true, s, n * c.w);
  }

  void push(const HostBatch& b) override {
    if (b.stream != sA && b.stream != sB) return;
    for (int64_t k = 0; k < b.n; k++) {
      if (b.ts[k] < last_ts)
        throw Error(-2, "followed-by path needs non-decreasing event timestamps (got " + std::to_string(b.ts[k]) +
                            " after " + std::to_string(last_ts) + ")");
      last_ts = b.ts[k];
    }
    hipStream_t s = app->stream;
    ensure_cap(n + b.n, s);
    SG_HIP(hipMemcpyAsync(ts.p + n, b.ts.data(), b.n * 8, hipMemcpyHostToDevice, s));
    std::vector<uint8_t> tv;
    if (!same) {
      tv.assign(b.n, (uint8_t)((b.stream == sA ? 1 : 0) | (b.stream == sB ? 2 : 0)));
      SG_HIP(hipMemcpyAsync(tag.p + n, tv.data(), b.n, hipMemcpyHostToDevice, s));
    }
    std::vector<DCol>& cols = (b.stream == sA) ? colA : colB;
    for (size_t k = 0; k < cols.size(); k++)
      SG_HIP(hipMemcpyAsync(cols[k].b.p + n * cols[k].w, b.cols[k].data(), b.n * cols[k].w, hipMemcpyHostToDevice, s));
    SG_HIP(hipStreamSynchronize(s));
    for (int64_t k = 0; k < b.n; k++) h_seq.push_back(b.seqs.empty() ? b.seq0 + k : b.seqs[k]);
    n += b.n;
  }

  void push_device(int stream, int64_t cnt, const int64_t* dts, const void* const* dcols, int batch,
                   hipStream_t s) override {
    (void)batch; (void)s;
    if (!same || stream != sA) throw Error(-2, "device ingest supports single-stream followed-by queries");
    if (n != 0 || ext_ts) throw Error(-2, "device ingest adopts one resident batch per runtime (sg_reset first)");
    ext_ts = dts;
    ext_cols.assign(dcols, dcols + arity(sA));
    n = cnt;
    h_seq.clear();
  }

  void set_halo(int stream, int64_t n_halo) override {
    if (!same || stream != sA) throw Error(-2, "halo events need a single-stream followed-by query");
    if (n_halo > n) throw Error(-1, "halo longer than the events pushed");
    start_end = n - n_halo;
  }

  void reset() override {
    start_end = INT64_MAX;
    n = 0; examined = 0; n_pend = 0; ext_ts = nullptr; ext_cols.clear();
    h_seq.clear(); last_ts = INT64_MIN; last_matches = 0;
  }

  void upload_tables(hipStream_t s) {
    FBCols hc;
    std::memset(&hc, 0, sizeof(hc));
    for (int k = 0; k < arity(sA); k++) { hc.a[k] = colptr(0, k); hc.aw[k] = tsize(app->streams[sA].types[k]); }
    for (int k = 0; k < arity(sB); k++) { hc.b[k] = colptr(1, k); hc.bw[k] = tsize(app->streams[sB].types[k]); }
    d_cols.reserve(1);
    SG_HIP(hipMemcpyAsync(d_cols.p, &hc, sizeof(hc), hipMemcpyHostToDevice, s));
    d_progs.reserve(2);
    SG_HIP(hipMemcpyAsync(d_progs.p, progs, sizeof(progs), hipMemcpyHostToDevice, s));
    if (!sel.empty()) {
      d_sel.reserve(sel.size());
      SG_HIP(hipMemcpyAsync(d_sel.p, sel.data(), sel.size() * sizeof(Prog), hipMemcpyHostToDevice, s));
    }
  }

  template <int OP, class V>
  void launch_tile(TileArgs& ta, int64_t ntiles, size_t lds, hipStream_t s) {
    auto fn = k_fb_tile<OP, V>;
    SG_HIP(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(fn, dim3((unsigned)ntiles), dim3(TILE_B), lds, s, ta);
  }
  template <int OP, class V>
  void launch_list(FBScanArgs& a, hipStream_t s) {
    hipLaunchKernelGGL((k_fb_list_atom<OP, V>), dim3((unsigned)((a.n_list + GEN_B - 1) / GEN_B)), dim3(GEN_B), 0, s,
                       a, (const V*)colptr(1, fp.xcol), (const V*)colptr(0, fp.ycol));
  }
  template <class V>
  void dispatch_op(bool tile, TileArgs* ta, FBScanArgs* la, int64_t ntiles, size_t lds, hipStream_t s) {
    switch (fp.op) {
#define SG_OPCASE(o)                                                   \
      case o:                                                          \
        if (tile) launch_tile<o, V>(*ta, ntiles, lds, s);              \
        else launch_list<o, V>(*la, s);                                \
        break;
      SG_OPCASE(C_GT) SG_OPCASE(C_LT) SG_OPCASE(C_GE) SG_OPCASE(C_LE) SG_OPCASE(C_EQ) SG_OPCASE(C_NE)
#undef SG_OPCASE
    }
  }
  void dispatch(bool tile, TileArgs* ta, FBScanArgs* la, int64_t ntiles, size_t lds, hipStream_t s) {
    switch (fp.t) {
      case T_FLOAT: dispatch_op<float>(tile, ta, la, ntiles, lds, s); break;
      case T_DOUBLE: dispatch_op<double>(tile, ta, la, ntiles, lds, s); break;
      case T_LONG: dispatch_op<int64_t>(tile, ta, la, ntiles, lds, s); break;
      default: dispatch_op<int32_t>(tile, ta, la, ntiles, lds, s); break;
    }
  }

  void flush(std::vector<Callback>& out, bool materialise, hipStream_t s) override;
  void materialise_records(std::vector<Callback>& out, int64_t mt, int64_t ml, hipStream_t s);

  // Compaction (host ingest, no halo): after a flush every pending start resumes at the next new event,
  // so only the pending starts' rows are read again.  The buffer becomes those rows in arrival order
  // (an event between a pending start and its future trigger that was dropped cannot satisfy f2 for it,
  // or the start would not be pending) and memory follows the open partials.
  DBuf<uint8_t> cmp_tmp;
  DBuf<int64_t> cmp_idx;
  DBuf<uint32_t> ts_bad;
  int64_t buffered() const override { return n; }
  void compact(hipStream_t s) {
    if (ext_ts || n == 0 || start_end != INT64_MAX) return;
    std::vector<int32_t> c((size_t)n_pend);
    if (n_pend) {
      SG_HIP(hipMemcpyAsync(c.data(), pend_i.p, (size_t)n_pend * 4, hipMemcpyDeviceToHost, s));
      SG_HIP(hipStreamSynchronize(s));
    }
    std::sort(c.begin(), c.end());
    std::vector<int64_t> idx(c.begin(), c.end());
    const int64_t m = (int64_t)idx.size();
    if (m) {
      cmp_idx.reserve((size_t)m, false);
      SG_HIP(hipMemcpyAsync(cmp_idx.p, idx.data(), (size_t)m * 8, hipMemcpyHostToDevice, s));
      compact_rows(ts.p, cmp_idx.p, m, cmp_tmp, s);
      if (!same) compact_rows(tag.p, cmp_idx.p, m, cmp_tmp, s);
      for (auto& col : colA) compact_col(col.b.p, col.w, cmp_idx.p, m, cmp_tmp, s);
      for (auto& col : colB) compact_col(col.b.p, col.w, cmp_idx.p, m, cmp_tmp, s);
      std::vector<int32_t> pi((size_t)m), pj((size_t)m, (int32_t)m);
      for (int64_t k = 0; k < m; k++) pi[(size_t)k] = (int32_t)k;
      SG_HIP(hipMemcpyAsync(pend_i.p, pi.data(), (size_t)m * 4, hipMemcpyHostToDevice, s));
      SG_HIP(hipMemcpyAsync(pend_j.p, pj.data(), (size_t)m * 4, hipMemcpyHostToDevice, s));
      SG_HIP(hipStreamSynchronize(s));
    }
    if (!h_seq.empty()) h_seq = gather_host(h_seq, idx);
    n = examined = m;
  }

  // sg_snapshot / sg_restore: e2's pending StateEvents of `every e1 -> e2` (StreamPreStateProcessor.
  // StreamPreState.snapshot, :451-469), i.e. the pending starts -- after the flush sg_snapshot runs,
  // the compacted buffer's rows with (start, next trigger) pairs, their columns, tags and arrival seqs.
  bool can_snapshot() const override { return true; }
  void snapshot(SnapWriter& w, hipStream_t s) override {
    if (ext_ts) throw Error(-2, "snapshot after device-resident ingest is not supported (the input is the caller's)");
    if (start_end != INT64_MAX) throw Error(-2, "snapshot of a multi-GPU halo split is not supported");
    if (examined != n) throw Error(-5, "followed-by snapshot needs a flushed buffer");
    w.pod(n); w.pod(n_pend); w.pod(last_ts);
    w.dev(ts, (size_t)n, s);
    if (!same) w.dev(tag, (size_t)n, s);
    for (auto& c : colA) w.dev(c.b, (size_t)(n * c.w), s);
    if (!same) for (auto& c : colB) w.dev(c.b, (size_t)(n * c.w), s);
    w.dev(pend_i, (size_t)n_pend, s);
    w.dev(pend_j, (size_t)n_pend, s);
    w.vec(h_seq);
  }
  void restore(SnapReader& r, hipStream_t s) override {
    reset();
    const int64_t nn = r.pod<int64_t>();
    const int32_t np = r.pod<int32_t>();
    const int64_t lts = r.pod<int64_t>();
    if (nn < 0 || np < 0 || nn >= (int64_t)INT32_MAX) throw Error(-1, "snapshot counts out of range");
    auto want = [](size_t got, int64_t need, const char* what) {
      if ((int64_t)got != need) throw Error(-1, std::string("snapshot ") + what + " size does not match its count");
    };
    want(r.dev(ts, s), nn, "event timestamps");
    if (!same) want(r.dev(tag, s), nn, "event tags");
    for (auto& c : colA) want(r.dev(c.b, s), nn * c.w, "column");
    if (!same) for (auto& c : colB) want(r.dev(c.b, s), nn * c.w, "column");
    want(r.dev(pend_i, s), np, "pending starts");
    want(r.dev(pend_j, s), np, "pending triggers");
    r.vec(h_seq);
    if (!h_seq.empty() && (int64_t)h_seq.size() != nn) throw Error(-1, "snapshot arrival seqs do not match the events");
    n = examined = nn; n_pend = np; last_ts = lts;
  }
};

void FollowedByExec::flush(std::vector<Callback>& out, bool materialise, hipStream_t s) {
  last_matches = 0;
  kernel_ms.clear();
  const int64_t new_lo = examined;
  if (n - new_lo + n_pend <= 0) return;
  if (n >= (int64_t)INT32_MAX) throw Error(-2, "followed-by buffer exceeds 2^31 events");
  upload_tables(s);
  if (!ev0) { SG_HIP(hipEventCreate(&ev0)); SG_HIP(hipEventCreate(&ev1)); }
  counters.reserve(4);
  SG_HIP(hipMemsetAsync(counters.p, 0, 4 * sizeof(uint32_t), s));
  const bool generic = !(fp.ok && same);
  const bool tile = !generic && n > new_lo;
  if (ext_ts && !tile) check_ts_order(ext_ts, n, ts_bad, s, "followed-by");
  int64_t ntiles = 0;
  int64_t mt = 0;                     // tile-path matches
  int32_t n_list = n_pend;            // list-path starts: carried + overflow
  float ms = 0;
  if (tile) {
    const int vw = tsize(fp.t);
    const int T = tileT, H = tileH;
    const int R = T + H;
    ntiles = (n - new_lo + T - 1) / T;
    const int cap = R;
    seg_j.reserve((size_t)ntiles * cap);
    if (!fp.plain_proj) seg_i.reserve((size_t)ntiles * cap);
    seg_p.resize(fp.pslot.size());
    for (size_t c = 0; c < fp.pslot.size(); c++) {
      int w = tsize(app->streams[sA].types[fp.pcol[c]]);
      seg_p[c].reserve((size_t)ntiles * cap * w);
    }
    tile_cnt.reserve(ntiles);
    pend_i.reserve(n_pend + (size_t)ntiles * R + 1, true, s, n_pend);   // keep the carried starts
    pend_j.reserve(n_pend + (size_t)ntiles * R + 1, true, s, n_pend);
    TileArgs ta;
    std::memset(&ta, 0, sizeof(ta));
    ta.ts = d_ts();
    ta.x = colptr(1, fp.xcol);
    ta.y = colptr(0, fp.ycol);
    ta.same_xy = fp.xcol == fp.ycol;
    ta.n = n;
    ta.j_lo = new_lo;
    ta.start_end = start_end;
    ta.within = within;
    ta.T = T;
    ta.H = H;
    // phase-1 depth (tuning hook SG_FB_S1): a lane walks its start this many candidates, then the start joins the
    // wave-per-start ballot queue; a wave waits for its longest walk, and next-greater distances are heavy-tailed
    ta.s1 = getenv("SG_FB_S1") ? std::max(1, atoi(getenv("SG_FB_S1"))) : TILE_S1;
    ta.f1kind = fp.f1kind;
    ta.f1op = fp.f1op;
    ta.f1t = fp.f1t;
    if (fp.f1kind == 1) { ta.f1col = colptr(0, fp.f1col); ta.f1w = tsize(app->streams[sA].types[fp.f1col]); }
    ta.f1c = fp.f1c;
    ta.seg_j = seg_j.p;
    ta.seg_i = fp.plain_proj ? nullptr : seg_i.p;
    ta.cap = cap;
    ta.nproj = fp.plain_proj ? (int)fp.pslot.size() : 0;
    for (int c = 0; c < ta.nproj; c++) {
      ta.pcol[c] = colptr(fp.pslot[c], fp.pcol[c]);
      ta.pslot[c] = fp.pslot[c];
      ta.pw[c] = tsize(app->streams[sA].types[fp.pcol[c]]);
      ta.pout[c] = seg_p[c].p;
    }
    ta.tile_cnt = tile_cnt.p;
    // the overflow list is appended after the carried starts in pend_* (one list for the list path)
    ta.ovf_i = pend_i.p + n_pend;
    ta.ovf_j = pend_j.p + n_pend;
    ta.n_ovf = counters.p + 2;
    ta.unsorted = counters.p + 3;
    size_t lds = (size_t)R * 8 + (size_t)R * vw * (ta.same_xy ? 1 : 2) + (size_t)R * 4 + (size_t)(T + R) * 4 + 16 * 4;
    SG_HIP(hipEventRecord(ev0, s));
    dispatch(true, &ta, nullptr, ntiles, lds, s);
    SG_HIP(hipGetLastError());
    SG_HIP(hipEventRecord(ev1, s));
    uint32_t novf[2] = {0, 0};
    SG_HIP(hipMemcpyAsync(novf, counters.p + 2, 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    if (novf[1]) throw Error(-1, "followed-by: event timestamps go backwards (device-resident input must be "
                                 "non-decreasing, as sg_push enforces for host batches)");
    SG_HIP(hipEventElapsedTime(&ms, ev0, ev1));
    kernel_ms["k_fb_tile"] = ms;
    n_list += (int32_t)novf[0];
    ntiles_last = ntiles;
  }
  // list path (carried + overflow) or the whole generic path
  int64_t ml = 0;
  int64_t work = n_list + (generic ? (n - new_lo) : 0);
  if (work > 0) {
    keys.reserve(work);
    npend_i.reserve(work);
    npend_j.reserve(work);
    FBScanArgs a;
    a.ts = d_ts();
    a.tag = same ? nullptr : tag.p;
    a.n = n;
    a.within = within;
    a.new_lo = generic ? new_lo : n;
    a.start_end = start_end;
    a.n_list = n_list;
    a.list_i = pend_i.p;
    a.list_j = pend_j.p;
    a.keys = keys.p;
    a.nkeys = counters.p;
    a.npend_i = npend_i.p;
    a.npend_j = npend_j.p;
    a.nnpend = counters.p + 1;
    SG_HIP(hipEventRecord(ev0, s));
    if (!generic) dispatch(false, nullptr, &a, 0, 0, s);
    else hipLaunchKernelGGL(k_fb_scan, dim3((unsigned)((work + GEN_B - 1) / GEN_B)), dim3(GEN_B), 0, s, a, d_cols.p,
                            d_progs.p);
    SG_HIP(hipGetLastError());
    SG_HIP(hipEventRecord(ev1, s));
    uint32_t hcnt[2];
    SG_HIP(hipMemcpyAsync(hcnt, counters.p, sizeof(hcnt), hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    SG_HIP(hipEventElapsedTime(&ms, ev0, ev1));
    kernel_ms[generic ? "k_fb_scan" : "k_fb_list_atom"] = ms;
    ml = hcnt[0];
    std::swap(pend_i.p, npend_i.p); std::swap(pend_i.cap, npend_i.cap);
    std::swap(pend_j.p, npend_j.p); std::swap(pend_j.cap, npend_j.cap);
    n_pend = (int32_t)hcnt[1];
    if (ml > 0) {
      keys_sorted.reserve(ml);
      int end_bit = 32;
      while (end_bit < 64 && (1ull << (end_bit - 32)) <= (uint64_t)n) end_bit++;
      size_t tmp = 0;
      SG_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, keys.p, keys_sorted.p, (int)ml, 0, end_bit, s));
      sort_tmp.reserve(tmp);
      SG_HIP(hipcub::DeviceRadixSort::SortKeys(sort_tmp.p, tmp, keys.p, keys_sorted.p, (int)ml, 0, end_bit, s));
    }
  } else {
    n_pend = 0;
  }
  examined = n;
  // tile-path match count
  if (tile) {
    std::vector<int32_t> hc(ntiles);
    SG_HIP(hipMemcpyAsync(hc.data(), tile_cnt.p, ntiles * 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    for (auto c : hc) mt += c;
  }
  last_matches = mt + ml;
  if (materialise && (mt + ml) > 0) materialise_records(out, mt, ml, s);
  compact(s);
}

void FollowedByExec::materialise_records(std::vector<Callback>& out, int64_t mt, int64_t ml, hipStream_t s) {
  const int nout = (int)sel.size();
  std::vector<int32_t> tj(mt), ti;
  std::vector<std::vector<uint8_t>> tcols;
  std::vector<int64_t> traw, lraw;
  std::vector<uint8_t> tnul, lnul;
  if (mt > 0) {
    // dense compaction of the tile segments
    std::vector<int32_t> hc(ntiles_last);
    SG_HIP(hipMemcpyAsync(hc.data(), tile_cnt.p, ntiles_last * 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    std::vector<int64_t> ho(ntiles_last);
    int64_t acc = 0;
    for (int64_t t = 0; t < ntiles_last; t++) { ho[t] = acc; acc += hc[t]; }
    tile_off.reserve(ntiles_last);
    SG_HIP(hipMemcpyAsync(tile_off.p, ho.data(), ntiles_last * 8, hipMemcpyHostToDevice, s));
    const int cap = tileT + tileH;
    dense_j.reserve(mt);
    hipLaunchKernelGGL(k_fb_compact, dim3((unsigned)ntiles_last), dim3(256), 0, s, tile_cnt.p, tile_off.p, cap,
                       seg_j.p, dense_j.p);
    SG_HIP(hipMemcpyAsync(tj.data(), dense_j.p, mt * 4, hipMemcpyDeviceToHost, s));
    if (fp.plain_proj) {
      tcols.resize(fp.pslot.size());
      for (size_t c = 0; c < fp.pslot.size(); c++) {
        // compaction of a w-byte column through 4-byte lanes (w = 4 or 8)
        int w = tsize(app->streams[sA].types[fp.pcol[c]]);
        tcols[c].resize((size_t)mt * w);
        if (w == 4) {
          dense_i.reserve(mt);
          hipLaunchKernelGGL(k_fb_compact, dim3((unsigned)ntiles_last), dim3(256), 0, s, tile_cnt.p, tile_off.p, cap,
                             (const int32_t*)seg_p[c].p, dense_i.p);
          SG_HIP(hipMemcpyAsync(tcols[c].data(), dense_i.p, mt * 4, hipMemcpyDeviceToHost, s));
          SG_HIP(hipStreamSynchronize(s));
        } else {
          std::vector<int64_t> all((size_t)ntiles_last * cap);
          SG_HIP(hipMemcpyAsync(all.data(), seg_p[c].p, all.size() * 8, hipMemcpyDeviceToHost, s));
          SG_HIP(hipStreamSynchronize(s));
          int64_t* dst = (int64_t*)tcols[c].data();
          for (int64_t t = 0; t < ntiles_last; t++)
            std::memcpy(dst + ho[t], all.data() + t * cap, (size_t)hc[t] * 8);
        }
      }
    } else {
      ti.resize(mt);
      dense_i.reserve(mt);
      hipLaunchKernelGGL(k_fb_compact, dim3((unsigned)ntiles_last), dim3(256), 0, s, tile_cnt.p, tile_off.p, cap,
                         seg_i.p, dense_i.p);
      // generic projection over the dense (j, i) pairs
      out_raw.reserve((size_t)mt * std::max(nout, 1));
      out_null.reserve((size_t)mt * std::max(nout, 1));
      FBProjArgs pa{dense_j.p, dense_i.p, nullptr, mt, nout, out_raw.p, out_null.p};
      hipLaunchKernelGGL(k_fb_project, dim3((unsigned)((mt + GEN_B - 1) / GEN_B)), dim3(GEN_B), 0, s, pa, d_cols.p,
                         d_sel.p);
      traw.resize((size_t)mt * nout);
      tnul.resize((size_t)mt * nout);
      if (nout) {
        SG_HIP(hipMemcpyAsync(traw.data(), out_raw.p, traw.size() * 8, hipMemcpyDeviceToHost, s));
        SG_HIP(hipMemcpyAsync(tnul.data(), out_null.p, tnul.size(), hipMemcpyDeviceToHost, s));
      }
    }
    SG_HIP(hipStreamSynchronize(s));
  }
  std::vector<uint64_t> lkeys(ml);
  if (ml > 0) {
    out_raw.reserve((size_t)ml * std::max(nout, 1));
    out_null.reserve((size_t)ml * std::max(nout, 1));
    FBProjArgs pa{nullptr, nullptr, keys_sorted.p, ml, nout, out_raw.p, out_null.p};
    hipLaunchKernelGGL(k_fb_project, dim3((unsigned)((ml + GEN_B - 1) / GEN_B)), dim3(GEN_B), 0, s, pa, d_cols.p,
                       d_sel.p);
    lraw.resize((size_t)ml * nout);
    lnul.resize((size_t)ml * nout);
    if (nout) {
      SG_HIP(hipMemcpyAsync(lraw.data(), out_raw.p, lraw.size() * 8, hipMemcpyDeviceToHost, s));
      SG_HIP(hipMemcpyAsync(lnul.data(), out_null.p, lnul.size(), hipMemcpyDeviceToHost, s));
    }
    SG_HIP(hipMemcpyAsync(lkeys.data(), keys_sorted.p, ml * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
  }
  std::vector<int64_t> hts(n);
  SG_HIP(hipMemcpyAsync(hts.data(), d_ts(), n * 8, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  // merge: for equal j the list-path records (smaller i) come first
  Callback* cur = nullptr;
  int64_t curj = -1;
  auto emit = [&](int64_t j, const int64_t* raw, const uint8_t* nul) {
    if (!same || cur == nullptr || j != curj) {
      out.emplace_back();
      cur = &out.back();
      cur->seq = h_seq.empty() ? j : h_seq[j];
      cur->order = qi;
      cur->kind = 0;
      cur->target = qi;
      curj = j;
    }
    OutEvent e;
    e.ts = hts[j];
    e.raw.assign(raw, raw + nout);
    e.nul.assign(nul, nul + nout);
    cur->ts = e.ts;
    cur->ev.push_back(std::move(e));
  };
  std::vector<int64_t> rowraw(nout);
  std::vector<uint8_t> rownul(nout, 0);
  int64_t a = 0, b = 0;
  while (a < ml || b < mt) {
    int64_t ja = a < ml ? (int64_t)(lkeys[a] >> 32) : INT64_MAX;
    int64_t jb = b < mt ? (int64_t)tj[b] : INT64_MAX;
    if (ja <= jb) {
      emit(ja, lraw.data() + a * nout, lnul.data() + a * nout);
      a++;
    } else {
      if (fp.plain_proj) {
        for (int c = 0; c < nout; c++) {
          Ty t = app->streams[sA].types[fp.pcol[c]];
          int w = tsize(t);
          int64_t v;
          if (w == 8) v = ((const int64_t*)tcols[c].data())[b];
          else {
            int32_t x = ((const int32_t*)tcols[c].data())[b];
            v = (t == T_FLOAT) ? (int64_t)(uint32_t)x : (int64_t)x;
          }
          rowraw[c] = v;
        }
        emit(jb, rowraw.data(), rownul.data());
      } else {
        emit(jb, traw.data() + b * nout, tnul.data() + b * nout);
      }
      b++;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Shape recognition: next(every(stream A [f1]), stream B [f2]), PATTERN, projection-only selector.
std::unique_ptr<Exec> make_followed_by(App& app, int qi, const J& q, std::string& why) {
  const J& in = q["input"];
  if (in["kind"].s != "state") { why = "not a state query"; return nullptr; }
  if (in["type"].s != "PATTERN") { why = "sequence"; return nullptr; }
  if (q.has("partition")) { why = "partitioned"; return nullptr; }
  const J& el = in["element"];
  if (el["k"].s != "next" || el["a"]["k"].s != "every" || el["a"]["e"]["k"].s != "stream" || el["b"]["k"].s != "stream") {
    why = "not `every e1 -> e2`";
    return nullptr;
  }
  const J& e1 = el["a"]["e"];
  const J& e2 = el["b"];
  if (e1["slot"].as_int() != 0 || e2["slot"].as_int() != 1) { why = "slot layout"; return nullptr; }
  const J& s = q["select"];
  if (s["group_by"].size() || !s["having"].null() || s["order_by"].size() || !s["limit"].null() || !s["offset"].null()) {
    why = "selector features";
    return nullptr;
  }
  const J& out = q["output"];
  if (out["events"].s != "current" && !out["events"].s.empty()) { why = "expired events output"; return nullptr; }
  std::function<bool(const J&)> has_agg = [&](const J& e) -> bool {
    if (e["op"].s == "agg" || e["op"].s == "multivar") return true;
    for (const char* c : {"a", "b"}) if (e.has(c) && has_agg(e[c])) return true;
    return false;
  };
  for (size_t k = 0; k < s["attrs"].size(); k++)
    if (has_agg(s["attrs"][k]["e"])) { why = "aggregator in select"; return nullptr; }
  auto ex = std::make_unique<FollowedByExec>();
  ex->app = &app;
  ex->qi = qi;
  ex->path = 1;
  ex->sA = app.stream_idx.at(e1["stream"].s);
  ex->sB = app.stream_idx.at(e2["stream"].s);
  ex->same = ex->sA == ex->sB;
  ex->within = in["within"].null() ? -1 : in["within"].as_int();
  auto intern = [&](const std::string& str) { return app.intern(str); };
  // chain index -1 (CURRENT) and 0 resolve to the slot's single event; anything else is null
  auto sm = [&](int slot, int chain) -> int {
    if (slot != 0 && slot != 1) return -1;
    if (chain != -1 && chain != 0) return -1;
    return slot;
  };
  // e1's own filter cannot see e2 (null) — map slot 1 to null there
  auto sm1 = [&](int slot, int chain) -> int { return slot == 0 ? sm(slot, chain) : -1; };
  try {
    compile_filters(ex->progs[0], e1["filters"], sm1, intern);
    compile_filters(ex->progs[1], e2["filters"], sm, intern);
    for (size_t k = 0; k < s["attrs"].size(); k++) {
      Prog p;
      compile_expr(p, s["attrs"][k]["e"], sm, intern);
      ex->sel.push_back(p);
    }
  } catch (CompileError& e) {
    why = e.what();
    return nullptr;
  }
  if (app.streams[ex->sA].types.size() > FB_MAXC || app.streams[ex->sB].types.size() > FB_MAXC) {
    why = "too many attributes";
    return nullptr;
  }
  ex->fp = recognise(app, ex->sA, ex->sB, e1, e2, s);
  if (ex->fp.ok && tsize(ex->fp.t) == 8) ex->tileH = 256;
  // test hook: smaller tiles / halos force the long-range (overflow) path
  if (const char* e = getenv("SG_FB_TILE_T")) ex->tileT = std::max(64, std::min(4096, atoi(e)));
  if (const char* e = getenv("SG_FB_TILE_H")) ex->tileH = std::max(1, std::min(ex->tileT, atoi(e)));
  for (Ty t : app.streams[ex->sA].types) { ex->colA.emplace_back(); ex->colA.back().w = tsize(t); }
  if (!ex->same)
    for (Ty t : app.streams[ex->sB].types) { ex->colB.emplace_back(); ex->colB.back().w = tsize(t); }
  ex->in_streams = {ex->sA};
  if (!ex->same) ex->in_streams.push_back(ex->sB);
  return ex;
}

}  // namespace sg
