// keyed_fb.hip — execution path SG_PATH_KEYED_FOLLOWED_BY.
//
// Query shape:  partition with (k of S) begin
//                 from every e1=S[f1] -> e2=S[f2(e1,e2)] (within W)? select <projection> insert into ...
//               end
//
// Reference semantics (restated; oracle/siddhi_oracle.cpp App::instance / QueryRT):
//   * PartitionStreamReceiver (CORE/partition/PartitionStreamReceiver.java:82-282) routes each event
//     to the instance of its key (ValuePartitionExecutor.execute :34-40); the first event of a key
//     creates the instance (PartitionRuntimeImpl.initPartition :346-402), whose `every` start state
//     holds an empty partial from init — so, as in followed_by.hip, a partial exists for every event
//     i with f1(i), and it only ever sees later events of the SAME key.
//   * Inside one instance the followed-by closed form holds (see followed_by.hip):
//       m(i) = min{ j > i : k_j = k_i, ts_j - ts_i <= W, f2(i, j) }
//     and, because expiry and matching of key k only happen on arrivals of key k, nothing else
//     changes.  Outputs are emitted at j; matches completing at the same j are in ascending i (all
//     of them belong to j's key).  Callbacks: one per distinct j (PatternMultiProcessStreamReceiver
//     holder per event), in arrival order of j.
//
// Device pipeline per flush (entries = starts carried from earlier flushes + the new events):
//   k_kf_entries   (key, index) pairs; carried starts first, so a stable sort keeps index order
//   radix sort     hipcub pairs sort on the key bits actually used (key segments in index order)
//   k_kf_scan      one lane per sorted entry: a start scans forward inside its key segment until
//                  expiry / first f2 match / segment end (-> carried); atomic per-trigger counts
//   exclusive scan per-trigger counts -> record offsets (records ordered by trigger j)
//   k_kf_place     scatter each match into its trigger's bucket
//   k_kf_order     one lane per trigger: insertion sort of the (tiny) bucket by i, fused plain-variable
//                  projection into HBM output columns
// Non-decreasing timestamps are required (checked at push); otherwise SG_E_UNSUPPORTED.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>

#include "fb_shape.hpp"
#include "keyed_chunks.hpp"
#include "keyed_order.hpp"
#include "keyed_tiles.hpp"
#include "runtime.hpp"
#include "snapshot.hpp"

namespace sg {

constexpr int KF_MAXC = 12;
constexpr int KF_B = 256;

struct KfCols {
  const uint8_t* c[KF_MAXC];
  int32_t w[KF_MAXC];
};

struct KfLoader {
  const KfCols* c;
  int64_t i, j;
  __device__ __forceinline__ bool load(int slot, int attr, int64_t& v) const {
    const int64_t idx = slot == 0 ? i : j;
    if (c->w[attr] == 8) v = ((const int64_t*)c->c[attr])[idx];
    else v = (int64_t)((const int32_t*)c->c[attr])[idx];
    return true;
  }
};

template <class K>
__global__ void __launch_bounds__(KF_B) k_kf_entries(const K* __restrict__ keycol, const int32_t* __restrict__ carried,
                                                     int64_t nc, int64_t lo, int64_t n, K* __restrict__ keys,
                                                     int32_t* __restrict__ idx) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nc + (n - lo)) return;
  const int64_t e = t < nc ? (int64_t)carried[t] : lo + (t - nc);
  keys[t] = keycol[e];
  idx[t] = (int32_t)e;
}

template <class K>
__global__ void __launch_bounds__(KF_B) k_kf_keybits(const K* __restrict__ keycol, int64_t lo, int64_t n,
                                                     unsigned long long* __restrict__ acc) {
  const int64_t t = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long v = t < n ? (unsigned long long)keycol[t] : 0ull;
  // wave-level OR, one atomic per wave
  for (int d = 32; d >= 1; d >>= 1) v |= __shfl_xor(v, d, 64);
  if ((threadIdx.x & 63) == 0 && v) atomicOr(acc, v);
}

struct KfScanArgs {
  const int64_t* ts;
  const void* skey;          // sorted keys (K)
  const int32_t* sidx;       // sorted event indices
  int64_t m;                 // entries
  int64_t lo, n;             // new events [lo, n)
  int64_t within;
  // atom fast path
  int32_t f1kind, f1op, f1t, f1w;
  const uint8_t* f1col;
  int64_t f1c;
  const uint8_t* x;          // e2.x
  const uint8_t* y;          // e1.y
  // outputs
  int32_t* mj;               // per entry: matched trigger or -1
  int32_t* cnt;              // [n - lo + 1] matches per trigger
  int32_t* carry;
  uint32_t* ncarry;
};

template <class K, class Pred>
__device__ __forceinline__ void kf_scan_one(const KfScanArgs& a, int64_t p, Pred&& f2) {
  const K* skey = (const K*)a.skey;
  const int64_t i = a.sidx[p];
  const K key = skey[p];
  const int64_t tsi = a.ts[i];
  for (int64_t q = p + 1; q < a.m; q++) {
    if (skey[q] != key) break;
    const int64_t j = a.sidx[q];
    if (j < a.lo) continue;                                    // carried entries are not candidates
    if (a.within >= 0 && a.ts[j] - tsi > a.within) { a.mj[p] = -1; return; }   // expired before j
    if (f2(i, j)) {
      a.mj[p] = (int32_t)j;
      atomicAdd(&a.cnt[j - a.lo], 1);
      return;
    }
  }
  a.mj[p] = -1;
  a.carry[atomicAdd(a.ncarry, 1u)] = (int32_t)i;               // still open: carried to the next flush
}

template <class K, int OP, class V>
__global__ void __launch_bounds__(KF_B) k_kf_scan_atom(KfScanArgs a) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.m) return;
  const int64_t i = a.sidx[p];
  if (i >= a.lo && a.f1kind == 1) {
    const int64_t v = a.f1w == 8 ? ((const int64_t*)a.f1col)[i] : (int64_t)((const int32_t*)a.f1col)[i];
    if (!cmp(a.f1op, a.f1t, v, a.f1c)) { a.mj[p] = -1; return; }
  }
  const V yi = ((const V*)a.y)[i];
  const V* x = (const V*)a.x;
  kf_scan_one<K>(a, p, [&](int64_t, int64_t j) { return cmpv<OP, V>(x[j], yi); });
}

template <class K>
__global__ void __launch_bounds__(KF_B) k_kf_scan_gen(KfScanArgs a, const KfCols* __restrict__ cols,
                                                      const Prog* __restrict__ progs) {
  __shared__ int64_t rf[MAX_REG * KF_B];
  int64_t* myrf = rf + threadIdx.x;
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.m) return;
  const int64_t i = a.sidx[p];
  KfLoader ld{cols, i, 0};
  if (i >= a.lo && !run_pred(progs[0], ld, myrf, KF_B)) { a.mj[p] = -1; return; }
  kf_scan_one<K>(a, p, [&](int64_t, int64_t j) {
    ld.j = j;
    return run_pred(progs[1], ld, myrf, KF_B);
  });
}

__global__ void __launch_bounds__(KF_B) k_kf_place(int64_t m, const int32_t* __restrict__ mj,
                                                   const int32_t* __restrict__ sidx, int64_t lo,
                                                   int32_t* __restrict__ fill, int32_t* __restrict__ rec_i) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= m) return;
  const int32_t j = mj[p];
  if (j < 0) return;
  const int32_t pos = atomicAdd(&fill[j - lo], 1);
  rec_i[pos] = sidx[p];
}

struct KfOrderArgs {
  const int32_t* off;        // [nn + 1]
  int64_t lo, nn;
  int32_t* rec_i;
  int32_t* rec_j;
  int32_t nproj;
  const uint8_t* pcol[FB_MAXP];
  int32_t pslot[FB_MAXP];
  int32_t pw[FB_MAXP];
  uint8_t* pout[FB_MAXP];
};

__global__ void __launch_bounds__(KF_B) k_kf_order(KfOrderArgs a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.nn) return;
  const int32_t beg = a.off[t], end = a.off[t + 1];
  if (beg == end) return;
  const int32_t j = (int32_t)(a.lo + t);
  for (int32_t p = beg + 1; p < end; p++) {
    const int32_t v = a.rec_i[p];
    int32_t q = p - 1;
    while (q >= beg && a.rec_i[q] > v) { a.rec_i[q + 1] = a.rec_i[q]; q--; }
    a.rec_i[q + 1] = v;
  }
  for (int32_t p = beg; p < end; p++) {
    const int32_t i = a.rec_i[p];
    a.rec_j[p] = j;
    for (int c = 0; c < a.nproj; c++) {
      const int64_t src = a.pslot[c] == 0 ? i : j;
      if (a.pw[c] == 8) ((int64_t*)a.pout[c])[p] = ((const int64_t*)a.pcol[c])[src];
      else ((int32_t*)a.pout[c])[p] = ((const int32_t*)a.pcol[c])[src];
    }
  }
}

// select-list programs over (i, j) records (generic projection)
__global__ void __launch_bounds__(KF_B) k_kf_project(int64_t nrec, const int32_t* __restrict__ rec_i,
                                                     const int32_t* __restrict__ rec_j, int32_t nout,
                                                     const KfCols* __restrict__ cols, const Prog* __restrict__ sel,
                                                     int64_t* __restrict__ out_raw, uint8_t* __restrict__ out_null) {
  __shared__ int64_t rf[MAX_REG * KF_B];
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrec) return;
  KfLoader ld{cols, rec_i[r], rec_j[r]};
  for (int c = 0; c < nout; c++) {
    int64_t v = 0;
    bool isnull = true;
    run(sel[c], ld, v, isnull, rf + threadIdx.x, KF_B);
    out_raw[r * nout + c] = v;
    out_null[r * nout + c] = isnull ? 1 : 0;
  }
}

// ---- packed variant (fast atom, 4-byte compare column, 32-bit keys): the sort carries the payload ----
// keys = key << 32 | event index (sorted on the key bits only: stable, so index order within a key),
// vals = start flag << 63 | (ts - ts_base) << 32 | x bits.  The scan then reads only coalesced sorted
// arrays; the only random accesses left are one atomic per match and the record scatter.
struct KpArgs {
  const int64_t* ts;
  const uint32_t* keycol;
  const uint32_t* xcol;
  int32_t f1kind, f1op, f1t, f1w;
  const uint8_t* f1col;
  int64_t f1c;
  const int32_t* carried;
  int64_t nc, lo, n, ts_base, within;
  uint64_t* keys;
  uint64_t* vals;
  // scan outputs
  int64_t m;
  int32_t* mj;
  uint32_t* mx;
  int32_t* rank;           // order of arrival of this start's match in its trigger's bucket
  int32_t* cnt;
  int32_t* carry;
  uint32_t* ncarry;
};

__global__ void __launch_bounds__(KF_B) k_kp_entries(KpArgs a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.nc + (a.n - a.lo)) return;
  const int64_t e = t < a.nc ? (int64_t)a.carried[t] : a.lo + (t - a.nc);
  bool start = true;
  if (e >= a.lo && a.f1kind == 1) {
    const int64_t v = a.f1w == 8 ? ((const int64_t*)a.f1col)[e] : (int64_t)((const int32_t*)a.f1col)[e];
    start = cmp(a.f1op, a.f1t, v, a.f1c);
  }
  int64_t tsr = 0;
  if (a.within >= 0) {
    tsr = a.ts[e] - a.ts_base;
    if (tsr < 0) { start = false; tsr = 0; }     // a carried start already expired for every new event
  }
  a.keys[t] = ((uint64_t)a.keycol[e] << 32) | (uint32_t)e;
  a.vals[t] = ((uint64_t)(start ? 1 : 0) << 63) | ((uint64_t)(tsr & 0x7fffffff) << 32) | a.xcol[e];
}

template <int OP, class V>
__global__ void __launch_bounds__(KF_B) k_kp_scan(KpArgs a) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.m) return;
  const uint64_t v = a.vals[p];
  a.mj[p] = -1;
  if (!(v >> 63)) return;
  const uint64_t k = a.keys[p];
  const uint32_t key = (uint32_t)(k >> 32);
  const int64_t i = (uint32_t)k;
  const int64_t tsi = (int64_t)((v >> 32) & 0x7fffffff);
  const uint32_t ybits = (uint32_t)v;
  V yi;
  __builtin_memcpy(&yi, &ybits, 4);
  for (int64_t q = p + 1; q < a.m; q++) {
    const uint64_t kq = a.keys[q];
    if ((uint32_t)(kq >> 32) != key) break;
    const int64_t j = (uint32_t)kq;
    if (j < a.lo) continue;                                  // carried entries are not candidates
    const uint64_t vq = a.vals[q];
    if (a.within >= 0 && (int64_t)((vq >> 32) & 0x7fffffff) - tsi > a.within) return;   // expired before j
    const uint32_t xb = (uint32_t)vq;
    V xj;
    __builtin_memcpy(&xj, &xb, 4);
    if (cmpv<OP, V>(xj, yi)) {
      a.mj[p] = (int32_t)j;
      a.mx[p] = xb;
      a.rank[p] = atomicAdd(&a.cnt[j - a.lo], 1);
      return;
    }
  }
  a.carry[atomicAdd(a.ncarry, 1u)] = (int32_t)i;
}

// projection sources of the packed records
enum KpSrc { KP_KEY = 0, KP_XI, KP_XJ, KP_COL_I, KP_COL_J };

struct KpPlaceArgs {
  int64_t m, lo, nn;
  const uint64_t* keys;
  const uint64_t* vals;
  const int32_t* mj;
  const uint32_t* mx;
  const int32_t* rank;
  const int32_t* off;
  int32_t* rec;            // AoS, `stride` int32 words: j, i, projection words
  int32_t stride;
  int32_t nproj;
  int32_t src[FB_MAXP];
  int32_t w[FB_MAXP];      // 1 or 2 words
  const uint8_t* col[FB_MAXP];
};

__global__ void __launch_bounds__(KF_B) k_kp_place(KpPlaceArgs a) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.m) return;
  const int32_t j = a.mj[p];
  if (j < 0) return;
  const uint64_t k = a.keys[p];
  const int32_t i = (int32_t)(uint32_t)k;
  const int32_t pos = a.off[j - a.lo] + a.rank[p];
  int32_t* r = a.rec + (int64_t)pos * a.stride;
  r[0] = j;
  r[1] = i;
  int wo = 2;
  for (int c = 0; c < a.nproj; c++) {
    int64_t v;
    switch (a.src[c]) {
      case KP_KEY: v = (int32_t)(uint32_t)(k >> 32); break;
      case KP_XI: v = (int32_t)(uint32_t)a.vals[p]; break;
      case KP_XJ: v = (int32_t)a.mx[p]; break;
      default: {
        const int64_t e = a.src[c] == KP_COL_I ? i : j;
        v = a.w[c] == 2 ? ((const int64_t*)a.col[c])[e] : (int64_t)((const int32_t*)a.col[c])[e];
      }
    }
    r[wo] = (int32_t)v;
    if (a.w[c] == 2) r[wo + 1] = (int32_t)(v >> 32);
    wo += a.w[c];
  }
}

// buckets with more than one start (several partials completed by the same trigger): order by i.
// (A single global list of such triggers, appended with one atomic counter, serialised the scan: r1.)
__global__ void __launch_bounds__(KF_B) k_kp_order(const int32_t* __restrict__ off, int64_t nn, int32_t* rec,
                                                   int32_t stride) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nn) return;
  const int32_t beg = off[t], end = off[t + 1];
  if (end - beg < 2) return;
  int32_t tmp[2 + 2 * FB_MAXP];
  for (int32_t p = beg + 1; p < end; p++) {
    for (int w = 0; w < stride; w++) tmp[w] = rec[(int64_t)p * stride + w];
    int32_t q = p - 1;
    while (q >= beg && rec[(int64_t)q * stride + 1] > tmp[1]) {
      for (int w = 0; w < stride; w++) rec[(int64_t)(q + 1) * stride + w] = rec[(int64_t)q * stride + w];
      q--;
    }
    for (int w = 0; w < stride; w++) rec[(int64_t)(q + 1) * stride + w] = tmp[w];
  }
}

// ------------------------------------------------------------------------------------------------
struct KeyedFollowedByExec : Exec {
  int st = -1;
  int kcol = -1;             // partition attribute
  Ty kty = T_INT;
  int64_t within = -1;
  Prog progs[2];
  std::vector<Prog> sel;
  FastPath fp;
  // event buffer
  int64_t n = 0, lo = 0;
  DBuf<int64_t> ts;
  std::vector<DCol> cols;
  const int64_t* ext_ts = nullptr;
  std::vector<const void*> ext_cols;
  std::vector<int64_t> h_seq;
  int64_t last_ts = INT64_MIN;
  // carried starts
  DBuf<int32_t> carry, ncarry_buf, new_carry;   // carried starts (double-buffered: no allocation per flush)
  int64_t n_carry = 0;
  // work buffers
  DBuf<uint8_t> keys_in, keys_out, sort_tmp;
  DBuf<int32_t> idx_in, idx_out, mj, cnt, off, rec_i, rec_j;
  DBuf<uint32_t> counters;
  DBuf<unsigned long long> keybits;
  std::vector<DBuf<uint8_t>> pout;
  DBuf<KfCols> d_cols;
  DBuf<Prog> d_progs, d_sel;
  DBuf<int64_t> out_raw;
  DBuf<uint8_t> out_null;
  int64_t nrec = 0;
  // packed variant
  DBuf<uint64_t> kp_keys_in, kp_keys_out, kp_vals_in, kp_vals_out;
  DBuf<uint32_t> kp_mx;
  DBuf<int32_t> kp_rank;
  DBuf<int32_t> kp_rec;
  int32_t kp_stride = 2;
  bool last_packed = false;
  // bucketed-tile variant (keyed_tiles.hpp)
  DBuf<uint32_t> kt_hist, kt_bstart, kt_tprefix, kt_bcur, kt_flags;
  DBuf<uint4> kt_tdesc;
  DBuf<uint4> kt_ent;
  DBuf<uint2> kt_tdir;
  int kt_pb = 0, kt_T = 2048;
  int64_t kt_ntiles = 0, kt_mgrid = 0;   // tile-table slots; matcher grid (XCD-rounded)
  bool last_tiled = false;
  hipEvent_t ev[8] = {};

  ~KeyedFollowedByExec() override {
    for (auto& e : ev) if (e) (void)hipEventDestroy(e);
  }

  int arity() const { return (int)app->streams[st].types.size(); }
  const int64_t* d_ts() const { return ext_ts ? ext_ts : ts.p; }
  const uint8_t* colptr(int c) const { return ext_ts ? (const uint8_t*)ext_cols[c] : cols[c].b.p; }
  int kw() const { return tsize(kty); }

  void push(const HostBatch& b) override {
    if (b.stream != st) return;
    if (ext_ts) throw Error(-2, "cannot append host events after device-resident ingest");
    for (int64_t k = 0; k < b.n; k++) {
      if (b.ts[k] < last_ts)
        throw Error(-2, "keyed followed-by path needs non-decreasing event timestamps (got " + std::to_string(b.ts[k]) +
                            " after " + std::to_string(last_ts) + ")");
      last_ts = b.ts[k];
    }
    if (n + b.n >= (int64_t)INT32_MAX) throw Error(-2, "keyed followed-by buffer exceeds 2^31 events");
    hipStream_t s = app->stream;
    ts.reserve(n + b.n, true, s, n);
    for (auto& c : cols) c.b.reserve((n + b.n) * c.w, true, s, n * c.w);
    SG_HIP(hipMemcpyAsync(ts.p + n, b.ts.data(), b.n * 8, hipMemcpyHostToDevice, s));
    for (size_t k = 0; k < cols.size(); k++)
      SG_HIP(hipMemcpyAsync(cols[k].b.p + n * cols[k].w, b.cols[k].data(), b.n * cols[k].w, hipMemcpyHostToDevice, s));
    SG_HIP(hipStreamSynchronize(s));
    for (int64_t k = 0; k < b.n; k++) h_seq.push_back(b.seqs.empty() ? b.seq0 + k : b.seqs[k]);
    n += b.n;
  }

  void push_device(int stream, int64_t cnt_, const int64_t* dts, const void* const* dcols, int batch,
                   hipStream_t s) override {
    (void)batch; (void)s;
    if (stream != st) throw Error(-2, "device ingest: stream is not the partitioned pattern stream");
    if (n != 0 || ext_ts) throw Error(-2, "device ingest adopts one resident batch per runtime (sg_reset first)");
    if (cnt_ >= (int64_t)INT32_MAX) throw Error(-2, "keyed followed-by buffer exceeds 2^31 events");
    ext_ts = dts;
    ext_cols.assign(dcols, dcols + arity());
    n = cnt_;
    h_seq.clear();
    ext_seq = nullptr;
  }
  void set_device_seq(const int64_t* d_seq) override { ext_seq = d_seq; }
  void fetch_seq(hipStream_t s) {
    if (!ext_seq || !h_seq.empty()) return;
    h_seq.resize(n);
    SG_HIP(hipMemcpyAsync(h_seq.data(), ext_seq, n * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
  }
  const int64_t* ext_seq = nullptr;   // device-resident global arrival seq (copied to h_seq when materialising)

  void reset() override {
    n = lo = 0; n_carry = 0; ext_ts = nullptr; ext_seq = nullptr; ext_cols.clear(); h_seq.clear(); last_ts = INT64_MIN;
    carry_prefix = false;
    last_matches = 0; nrec = 0;
  }

  void timed(int k, hipStream_t s) { SG_HIP(hipEventRecord(ev[k], s)); }

  template <class K>
  void run(hipStream_t s, bool materialise, std::vector<Callback>& out);
  template <class K, int OP, class V>
  void scan_atom(KfScanArgs& a, hipStream_t s) {
    hipLaunchKernelGGL((k_kf_scan_atom<K, OP, V>), dim3((unsigned)((a.m + KF_B - 1) / KF_B)), dim3(KF_B), 0, s, a);
  }
  template <class K, class V>
  void scan_op(KfScanArgs& a, hipStream_t s) {
    switch (fp.op) {
      case C_GT: scan_atom<K, C_GT, V>(a, s); break;
      case C_LT: scan_atom<K, C_LT, V>(a, s); break;
      case C_GE: scan_atom<K, C_GE, V>(a, s); break;
      case C_LE: scan_atom<K, C_LE, V>(a, s); break;
      case C_EQ: scan_atom<K, C_EQ, V>(a, s); break;
      default: scan_atom<K, C_NE, V>(a, s); break;
    }
  }
  template <class K>
  void scan(KfScanArgs& a, hipStream_t s) {
    if (!fp.ok) {
      hipLaunchKernelGGL(k_kf_scan_gen<K>, dim3((unsigned)((a.m + KF_B - 1) / KF_B)), dim3(KF_B), 0, s, a, d_cols.p,
                         d_progs.p);
      return;
    }
    switch (fp.t) {
      case T_FLOAT: scan_op<K, float>(a, s); break;
      case T_DOUBLE: scan_op<K, double>(a, s); break;
      case T_LONG: scan_op<K, int64_t>(a, s); break;
      default: scan_op<K, int32_t>(a, s); break;
    }
  }

  void flush(std::vector<Callback>& out, bool materialise, hipStream_t s) override {
    last_matches = 0;
    kernel_ms.clear();
    if (n - lo + n_carry <= 0 || n == lo) { return; }
    for (auto& e : ev) if (!e) SG_HIP(hipEventCreate(&e));
    last_chunked = chunked_ok() && run_chunked(s, materialise, out);
    last_tiled = !last_chunked && tiled_ok() && run_tiled(s, materialise, out);
    if (!last_chunked && !last_tiled) {
      if (ext_ts) check_ts_order(ext_ts, n, ts_bad, s, "keyed followed-by");
      last_packed = packed_ok() && run_packed(s, materialise, out);
      if (!last_packed) {
        if (kw() == 8) run<uint64_t>(s, materialise, out);
        else run<uint32_t>(s, materialise, out);
      }
    }
    compact(s);
  }

  // Compaction (host ingest): after a flush only the carried starts are read again -- every later
  // trigger is a new event, and a dropped event between a carried start i and its future trigger
  // cannot satisfy f2 for i within W (i would not be carried).  The buffer becomes the carried starts
  // in arrival order and the carry list its identity prefix [0, lo), so memory follows the open
  // partials, not the events ever pushed, and the tiled path keeps taking later flushes (positions
  // below lo are never triggers there).
  bool carry_prefix = false;        // carry == [0, n_carry) and lo == n_carry
  DBuf<uint32_t> ts_bad;
  DBuf<uint8_t> cmp_tmp;
  DBuf<int64_t> cmp_idx;
  int64_t buffered() const override { return n; }
  void compact(hipStream_t s) {
    if (ext_ts || n == 0) return;
    std::vector<int32_t> c((size_t)n_carry);
    if (n_carry) {
      SG_HIP(hipMemcpyAsync(c.data(), carry.p, (size_t)n_carry * 4, hipMemcpyDeviceToHost, s));
      SG_HIP(hipStreamSynchronize(s));
    }
    std::sort(c.begin(), c.end());
    std::vector<int64_t> idx(c.begin(), c.end());
    const int64_t m = (int64_t)idx.size();
    if (m) {
      cmp_idx.reserve((size_t)m, false);
      SG_HIP(hipMemcpyAsync(cmp_idx.p, idx.data(), (size_t)m * 8, hipMemcpyHostToDevice, s));
      compact_rows(ts.p, cmp_idx.p, m, cmp_tmp, s);
      for (auto& col : cols) compact_col(col.b.p, col.w, cmp_idx.p, m, cmp_tmp, s);
      std::vector<int32_t> id((size_t)m);
      for (int64_t k = 0; k < m; k++) id[(size_t)k] = (int32_t)k;
      SG_HIP(hipMemcpyAsync(carry.p, id.data(), (size_t)m * 4, hipMemcpyHostToDevice, s));
      SG_HIP(hipStreamSynchronize(s));
    }
    if (!h_seq.empty()) h_seq = gather_host(h_seq, idx);
    n = lo = m;
    carry_prefix = true;
  }

  // sg_snapshot / sg_restore.  The reference's state of `every e1 -> e2 within W` per partition key is
  // e2's pending StateEvents (StreamPreStateProcessor.StreamPreState.snapshot, :451-469: the pending
  // list with each StateEvent's e1 StreamEvent) -- here the carried starts, which after the flush
  // sg_snapshot runs are the compacted buffer's rows [0, n_carry) in arrival order (their timestamps,
  // columns and arrival seqs; the key of each is its partition key column).  The e1 start state itself
  // is stateless (`every` re-arms it), and rows past the carried starts do not exist after compaction.
  bool can_snapshot() const override { return true; }
  void snapshot(SnapWriter& w, hipStream_t s) override {
    if (ext_ts) throw Error(-2, "snapshot after device-resident ingest is not supported (the input is the caller's)");
    if (lo != n || (n && !carry_prefix)) throw Error(-5, "keyed followed-by snapshot needs a compacted buffer");
    w.pod(n); w.pod(n_carry); w.pod(last_ts);
    w.dev(ts, (size_t)n, s);
    w.pod<uint64_t>(cols.size());
    for (auto& c : cols) w.dev(c.b, (size_t)(n * c.w), s);
    w.dev(carry, (size_t)n_carry, s);
    w.vec(h_seq);
  }
  void restore(SnapReader& r, hipStream_t s) override {
    reset();
    const int64_t nn = r.pod<int64_t>(), nc = r.pod<int64_t>();
    const int64_t lts = r.pod<int64_t>();
    if (nn < 0 || nc < 0 || nc > nn || nn >= (int64_t)INT32_MAX) throw Error(-1, "snapshot counts out of range");
    auto want = [](size_t got, int64_t need, const char* what) {
      if ((int64_t)got != need) throw Error(-1, std::string("snapshot ") + what + " size does not match its count");
    };
    want(r.dev(ts, s), nn, "event timestamps");
    if (r.pod<uint64_t>() != cols.size()) throw Error(-1, "snapshot columns do not match the query");
    for (auto& c : cols) want(r.dev(c.b, s), nn * c.w, "column");
    want(r.dev(carry, s), nc, "carried starts");
    r.vec(h_seq);
    if (!h_seq.empty() && (int64_t)h_seq.size() != nn) throw Error(-1, "snapshot arrival seqs do not match the events");
    n = lo = nn; n_carry = nc; last_ts = lts; carry_prefix = true;
  }

  bool packed_ok() const {
    if (getenv("SG_KEYED_NO_PACK")) return false;   // test hook: force the general pipeline
    return fp.ok && fp.plain_proj && fp.xcol == fp.ycol && tsize(fp.t) == 4 && kw() == 4 && fp.f1kind <= 1 &&
           (int)fp.pslot.size() <= FB_MAXP;
  }
  bool tiled_ok() const {
    if (getenv("SG_KEYED_NO_TILES")) return false;   // test hook: force the sort pipelines
    return packed_ok() && within >= 0 && lo == n_carry && (lo == 0 || carry_prefix);
  }
  bool run_tiled(hipStream_t s, bool materialise, std::vector<Callback>& out);
  // chunk-sorted pipeline (keyed_chunks.hpp): a flush without carried starts from earlier flushes (the bench's
  // device-resident step); SG_KEYED_NO_CHUNKS keeps the bucketed tiles
  bool chunked_ok() const {
    if (getenv("SG_KEYED_NO_CHUNKS")) return false;
    return tiled_ok() && lo == 0 && n_carry == 0;
  }
  bool run_chunked(hipStream_t s, bool materialise, std::vector<Callback>& out);
  bool last_chunked = false;
  DBuf<uint2> kc_ent;
  DBuf<uint16_t> kc_off;
  DBuf<int64_t> kc_cts0;
  DBuf<int32_t> kc_shalo;
  DBuf<uint32_t> kc_flags;
  // matcher variants: small tiles (2304 entries with the back-halo, slices sized for 0.85 * 1536 triggers per bucket,
  // 9-bit local keys: 46 KB of LDS, three workgroups per CU) when the buckets are sparse enough, else large tiles
  // (4096 entries, slices for 0.85 * 2048 triggers, 10-bit keys, two per CU)
  bool kc_small = false;
  template <int OP, class V>
  void kc_match_launch(KcArgs& a, unsigned grid, hipStream_t s) {
    static const int wpe = getenv("SG_KC_WPE") ? atoi(getenv("SG_KC_WPE")) : 6;   // tuning hook
    if (kc_small && wpe == 8) hipLaunchKernelGGL((k_kc_match<OP, V, 2048, 2304, 512, 9, 8>), dim3(grid), dim3(512), 0, s, a);
    else if (kc_small && wpe == 6) hipLaunchKernelGGL((k_kc_match<OP, V, 2048, 2304, 512, 9, 6>), dim3(grid), dim3(512), 0, s, a);
    else if (kc_small) hipLaunchKernelGGL((k_kc_match<OP, V, 2048, 2304, 512, 9, 4>), dim3(grid), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((k_kc_match<OP, V, 2048, 4096, 512, 10, 4>), dim3(grid), dim3(512), 0, s, a);
  }
  template <class V>
  void kc_match_op(KcArgs& a, unsigned grid, hipStream_t s) {
    switch (fp.op) {
      case C_GT: kc_match_launch<C_GT, V>(a, grid, s); break;
      case C_LT: kc_match_launch<C_LT, V>(a, grid, s); break;
      case C_GE: kc_match_launch<C_GE, V>(a, grid, s); break;
      case C_LE: kc_match_launch<C_LE, V>(a, grid, s); break;
      case C_EQ: kc_match_launch<C_EQ, V>(a, grid, s); break;
      default: kc_match_launch<C_NE, V>(a, grid, s); break;
    }
  }
  bool kt_partition(hipStream_t s, KtArgs& a, int pb, int64_t ts_lo, int64_t ts_hi, int& stride);
  DBuf<uint32_t> ks_tot, ks_hbase;
  DBuf<uint2> kt_toffs;
  DBuf<uint16_t> kc_rows;
  DBuf<int32_t> ks_out;
  DBuf<int64_t> ks_ots;
  DBuf<int64_t> ko_ts, ko_raw, ko_cts, ko_crow, ko_cseq;           // columnar callbacks (materialise_ordered)
  DBuf<uint8_t> ko_first;
  DBuf<int32_t> ko_cfirst;
  void materialise_ordered(const int32_t* d_rec, int64_t total, std::vector<Callback>& out, hipStream_t s);
  void build_callbacks(const int32_t* recs, const int64_t* hts, int64_t total, std::vector<Callback>& out);
  template <int OP, class V>
  void kt_match_launch(KtArgs& a, hipStream_t s) {
    static const bool two = getenv("SG_KT_TWOWALK") != nullptr;   // tuning hook: the two-walk matcher
    static const bool back = getenv("SG_KT_BACKWALK") != nullptr; // tuning hook: trigger-centric back-walks
    if (a.ent12 && two)
      hipLaunchKernelGGL((k_kt_match<OP, V, 2048, KT_H, 512, true, true, false>), dim3((unsigned)kt_mgrid), dim3(512), 0, s, a);
    else if (a.ent12 && back)
      hipLaunchKernelGGL((k_kt_match<OP, V, 2048, KT_H, 512, true, false, false>), dim3((unsigned)kt_mgrid), dim3(512), 0, s, a);
    else if (a.ent12)
      hipLaunchKernelGGL((k_kt_match<OP, V, 2048, KT_H, 512, true>), dim3((unsigned)kt_mgrid), dim3(512), 0, s, a);
    else if (kt_T == 4096)
      hipLaunchKernelGGL((k_kt_match<OP, V, 4096, KT_H, 1024>), dim3((unsigned)kt_mgrid), dim3(1024), 0, s, a);
    else
      hipLaunchKernelGGL((k_kt_match<OP, V, 2048, KT_H, 512>), dim3((unsigned)kt_mgrid), dim3(512), 0, s, a);
  }
  template <class V>
  void kt_match_op(KtArgs& a, hipStream_t s) {
    switch (fp.op) {
      case C_GT: kt_match_launch<C_GT, V>(a, s); break;
      case C_LT: kt_match_launch<C_LT, V>(a, s); break;
      case C_GE: kt_match_launch<C_GE, V>(a, s); break;
      case C_LE: kt_match_launch<C_LE, V>(a, s); break;
      case C_EQ: kt_match_launch<C_EQ, V>(a, s); break;
      default: kt_match_launch<C_NE, V>(a, s); break;
    }
  }
  void materialise_tiled(std::vector<Callback>& out, hipStream_t s);
  int key_end_bit(hipStream_t s);
  bool run_packed(hipStream_t s, bool materialise, std::vector<Callback>& out);
  template <int OP, class V>
  void kp_scan_launch(KpArgs& a, hipStream_t s) {
    hipLaunchKernelGGL((k_kp_scan<OP, V>), dim3((unsigned)((a.m + KF_B - 1) / KF_B)), dim3(KF_B), 0, s, a);
  }
  template <class V>
  void kp_scan_op(KpArgs& a, hipStream_t s) {
    switch (fp.op) {
      case C_GT: kp_scan_launch<C_GT, V>(a, s); break;
      case C_LT: kp_scan_launch<C_LT, V>(a, s); break;
      case C_GE: kp_scan_launch<C_GE, V>(a, s); break;
      case C_LE: kp_scan_launch<C_LE, V>(a, s); break;
      case C_EQ: kp_scan_launch<C_EQ, V>(a, s); break;
      default: kp_scan_launch<C_NE, V>(a, s); break;
    }
  }

  void materialise_records(std::vector<Callback>& out, hipStream_t s);
  void materialise_packed(std::vector<Callback>& out, hipStream_t s);
};

template <class K>
void KeyedFollowedByExec::run(hipStream_t s, bool materialise, std::vector<Callback>& out) {
  const int64_t nn = n - lo;
  const int64_t m = n_carry + nn;
  // tables
  KfCols hc;
  std::memset(&hc, 0, sizeof(hc));
  for (int k = 0; k < arity(); k++) { hc.c[k] = colptr(k); hc.w[k] = tsize(app->streams[st].types[k]); }
  d_cols.reserve(1);
  SG_HIP(hipMemcpyAsync(d_cols.p, &hc, sizeof(hc), hipMemcpyHostToDevice, s));
  d_progs.reserve(2);
  SG_HIP(hipMemcpyAsync(d_progs.p, progs, sizeof(progs), hipMemcpyHostToDevice, s));
  if (!sel.empty()) {
    d_sel.reserve(sel.size());
    SG_HIP(hipMemcpyAsync(d_sel.p, sel.data(), sel.size() * sizeof(Prog), hipMemcpyHostToDevice, s));
  }
  const K* keycol = (const K*)colptr(kcol);
  const int end_bit = key_end_bit(s);
  keys_in.reserve(m * sizeof(K));
  keys_out.reserve(m * sizeof(K));
  idx_in.reserve(m);
  idx_out.reserve(m);
  mj.reserve(m);
  cnt.reserve(nn + 1);
  off.reserve(nn + 1);
  counters.reserve(4);
  SG_HIP(hipMemsetAsync(counters.p, 0, 16, s));
  SG_HIP(hipMemsetAsync(cnt.p, 0, (nn + 1) * 4, s));
  new_carry.reserve(std::max<int64_t>(m, 1));
  timed(0, s);
  hipLaunchKernelGGL(k_kf_entries<K>, dim3((unsigned)((m + KF_B - 1) / KF_B)), dim3(KF_B), 0, s, keycol, carry.p,
                     n_carry, lo, n, (K*)keys_in.p, idx_in.p);
  SG_HIP(hipGetLastError());
  timed(1, s);
  size_t tmp = 0;
  SG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const K*)keys_in.p, (K*)keys_out.p, idx_in.p, idx_out.p,
                                            (int)m, 0, end_bit, s));
  sort_tmp.reserve(tmp);
  SG_HIP(hipcub::DeviceRadixSort::SortPairs(sort_tmp.p, tmp, (const K*)keys_in.p, (K*)keys_out.p, idx_in.p, idx_out.p,
                                            (int)m, 0, end_bit, s));
  timed(2, s);
  KfScanArgs a;
  std::memset(&a, 0, sizeof(a));
  a.ts = d_ts(); a.skey = keys_out.p; a.sidx = idx_out.p; a.m = m; a.lo = lo; a.n = n; a.within = within;
  if (fp.ok) {
    a.f1kind = fp.f1kind; a.f1op = fp.f1op; a.f1t = fp.f1t; a.f1c = fp.f1c;
    if (fp.f1kind == 1) { a.f1col = colptr(fp.f1col); a.f1w = tsize(app->streams[st].types[fp.f1col]); }
    a.x = colptr(fp.xcol); a.y = colptr(fp.ycol);
  }
  a.mj = mj.p; a.cnt = cnt.p; a.carry = new_carry.p; a.ncarry = counters.p;
  scan<K>(a, s);
  SG_HIP(hipGetLastError());
  timed(3, s);
  size_t tmp2 = 0;
  SG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp2, cnt.p, off.p, (int)(nn + 1), s));
  if (tmp2 > sort_tmp.cap) sort_tmp.reserve(tmp2, false);
  SG_HIP(hipcub::DeviceScan::ExclusiveSum(sort_tmp.p, tmp2, cnt.p, off.p, (int)(nn + 1), s));
  int32_t total = 0;
  SG_HIP(hipMemcpyAsync(&total, off.p + nn, 4, hipMemcpyDeviceToHost, s));
  uint32_t nc = 0;
  SG_HIP(hipMemcpyAsync(&nc, counters.p, 4, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  rec_i.reserve(std::max(total, 1));
  rec_j.reserve(std::max(total, 1));
  // fill = copy of the offsets (cnt is free now)
  SG_HIP(hipMemcpyAsync(cnt.p, off.p, (nn + 1) * 4, hipMemcpyDeviceToDevice, s));
  timed(4, s);
  hipLaunchKernelGGL(k_kf_place, dim3((unsigned)((m + KF_B - 1) / KF_B)), dim3(KF_B), 0, s, m, mj.p, idx_out.p, lo,
                     cnt.p, rec_i.p);
  KfOrderArgs oa;
  std::memset(&oa, 0, sizeof(oa));
  oa.off = off.p; oa.lo = lo; oa.nn = nn; oa.rec_i = rec_i.p; oa.rec_j = rec_j.p;
  oa.nproj = fp.plain_proj ? (int)fp.pslot.size() : 0;
  pout.resize(oa.nproj);
  for (int c = 0; c < oa.nproj; c++) {
    oa.pcol[c] = colptr(fp.pcol[c]);
    oa.pslot[c] = fp.pslot[c];
    oa.pw[c] = tsize(app->streams[st].types[fp.pcol[c]]);
    pout[c].reserve((size_t)std::max(total, 1) * oa.pw[c]);
    oa.pout[c] = pout[c].p;
  }
  hipLaunchKernelGGL(k_kf_order, dim3((unsigned)((nn + KF_B - 1) / KF_B)), dim3(KF_B), 0, s, oa);
  SG_HIP(hipGetLastError());
  if (!fp.plain_proj && total > 0 && !sel.empty()) {
    out_raw.reserve((size_t)total * sel.size());
    out_null.reserve((size_t)total * sel.size());
    hipLaunchKernelGGL(k_kf_project, dim3((unsigned)((total + KF_B - 1) / KF_B)), dim3(KF_B), 0, s, (int64_t)total,
                       rec_i.p, rec_j.p, (int32_t)sel.size(), d_cols.p, d_sel.p, out_raw.p, out_null.p);
    SG_HIP(hipGetLastError());
  }
  timed(5, s);
  SG_HIP(hipStreamSynchronize(s));
  float ms = 0;
  SG_HIP(hipEventElapsedTime(&ms, ev[0], ev[1])); kernel_ms["k_kf_entries"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[1], ev[2])); kernel_ms["radix_sort"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[2], ev[3])); kernel_ms["k_kf_scan"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[4], ev[5])); kernel_ms["k_kf_place_order"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[0], ev[5])); kernel_ms["total"] = ms;
  // carried starts for the next flush
  std::swap(carry, new_carry);
  n_carry = nc;
  lo = n;
  nrec = total;
  last_matches = total;
  if (materialise && total > 0) materialise_records(out, s);
}


int KeyedFollowedByExec::key_end_bit(hipStream_t s) {
  // key bits actually used: string ids are bounded by the dictionary; other keys by an OR-reduction
  if (kty == T_STRING) {
    int b = 1;
    while (b < 32 && (1ull << b) < (unsigned long long)app->strings.size()) b++;
    return b;
  }
  keybits.reserve(1);
  SG_HIP(hipMemsetAsync(keybits.p, 0, 8, s));
  if (kw() == 8)
    hipLaunchKernelGGL(k_kf_keybits<uint64_t>, dim3((unsigned)((n + KF_B - 1) / KF_B)), dim3(KF_B), 0, s,
                       (const uint64_t*)colptr(kcol), (int64_t)0, n, keybits.p);
  else
    hipLaunchKernelGGL(k_kf_keybits<uint32_t>, dim3((unsigned)((n + KF_B - 1) / KF_B)), dim3(KF_B), 0, s,
                       (const uint32_t*)colptr(kcol), (int64_t)0, n, keybits.p);
  unsigned long long bits = 0;
  SG_HIP(hipMemcpyAsync(&bits, keybits.p, 8, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  int b = 1;
  while (b < 8 * kw() && (bits >> b) != 0) b++;
  return b;
}

bool KeyedFollowedByExec::run_packed(hipStream_t s, bool materialise, std::vector<Callback>& out) {
  const int64_t nn = n - lo;
  const int64_t m = n_carry + nn;
  int64_t ts_lo = 0, ts_hi = 0;
  SG_HIP(hipMemcpyAsync(&ts_lo, d_ts() + lo, 8, hipMemcpyDeviceToHost, s));
  SG_HIP(hipMemcpyAsync(&ts_hi, d_ts() + n - 1, 8, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  const int64_t ts_base = within >= 0 ? ts_lo - within - 1 : 0;
  if (within >= 0 && ts_hi - ts_base >= (1ll << 31)) return false;   // 31-bit relative timestamps
  const int end_bit = key_end_bit(s);
  kp_keys_in.reserve(m); kp_keys_out.reserve(m); kp_vals_in.reserve(m); kp_vals_out.reserve(m);
  mj.reserve(m); kp_mx.reserve(m); kp_rank.reserve(m);
  cnt.reserve(nn + 1); off.reserve(nn + 1);
  counters.reserve(4);
  SG_HIP(hipMemsetAsync(counters.p, 0, 16, s));
  SG_HIP(hipMemsetAsync(cnt.p, 0, (nn + 1) * 4, s));
  new_carry.reserve(std::max<int64_t>(m, 1));
  KpArgs a;
  std::memset(&a, 0, sizeof(a));
  a.ts = d_ts(); a.keycol = (const uint32_t*)colptr(kcol); a.xcol = (const uint32_t*)colptr(fp.xcol);
  a.f1kind = fp.f1kind; a.f1op = fp.f1op; a.f1t = fp.f1t; a.f1c = fp.f1c;
  if (fp.f1kind == 1) { a.f1col = colptr(fp.f1col); a.f1w = tsize(app->streams[st].types[fp.f1col]); }
  a.carried = carry.p; a.nc = n_carry; a.lo = lo; a.n = n; a.ts_base = ts_base; a.within = within;
  a.keys = kp_keys_in.p; a.vals = kp_vals_in.p;
  timed(0, s);
  hipLaunchKernelGGL(k_kp_entries, dim3((unsigned)((m + KF_B - 1) / KF_B)), dim3(KF_B), 0, s, a);
  SG_HIP(hipGetLastError());
  timed(1, s);
  size_t tmp = 0;
  SG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, kp_keys_in.p, kp_keys_out.p, kp_vals_in.p, kp_vals_out.p,
                                            (int)m, 32, 32 + end_bit, s));
  sort_tmp.reserve(tmp);
  SG_HIP(hipcub::DeviceRadixSort::SortPairs(sort_tmp.p, tmp, kp_keys_in.p, kp_keys_out.p, kp_vals_in.p, kp_vals_out.p,
                                            (int)m, 32, 32 + end_bit, s));
  timed(2, s);
  a.keys = kp_keys_out.p; a.vals = kp_vals_out.p; a.m = m;
  a.mj = mj.p; a.mx = kp_mx.p; a.rank = kp_rank.p; a.cnt = cnt.p; a.carry = new_carry.p; a.ncarry = counters.p;
  if (fp.t == T_FLOAT) kp_scan_op<float>(a, s);
  else kp_scan_op<int32_t>(a, s);
  SG_HIP(hipGetLastError());
  timed(3, s);
  size_t tmp2 = 0;
  SG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp2, cnt.p, off.p, (int)(nn + 1), s));
  if (tmp2 > sort_tmp.cap) sort_tmp.reserve(tmp2, false);
  SG_HIP(hipcub::DeviceScan::ExclusiveSum(sort_tmp.p, tmp2, cnt.p, off.p, (int)(nn + 1), s));
  int32_t total = 0;
  uint32_t nc = 0;
  SG_HIP(hipMemcpyAsync(&total, off.p + nn, 4, hipMemcpyDeviceToHost, s));
  SG_HIP(hipMemcpyAsync(&nc, counters.p, 4, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  KpPlaceArgs pa;
  std::memset(&pa, 0, sizeof(pa));
  pa.m = m; pa.lo = lo; pa.nn = nn; pa.keys = kp_keys_out.p; pa.vals = kp_vals_out.p; pa.mj = mj.p; pa.mx = kp_mx.p;
  pa.rank = kp_rank.p; pa.off = off.p;
  pa.nproj = (int)fp.pslot.size();
  int stride = 2;
  for (int c = 0; c < pa.nproj; c++) {
    const int col = fp.pcol[c], slot = fp.pslot[c];
    const int w = tsize(app->streams[st].types[col]) / 4;
    pa.w[c] = w;
    if (col == kcol) pa.src[c] = KP_KEY;
    else if (col == fp.xcol) pa.src[c] = slot == 0 ? KP_XI : KP_XJ;
    else { pa.src[c] = slot == 0 ? KP_COL_I : KP_COL_J; pa.col[c] = colptr(col); }
    stride += w;
  }
  pa.stride = stride;
  kp_stride = stride;
  kp_rec.reserve((size_t)std::max(total, 1) * stride);
  pa.rec = kp_rec.p;
  timed(4, s);
  hipLaunchKernelGGL(k_kp_place, dim3((unsigned)((m + KF_B - 1) / KF_B)), dim3(KF_B), 0, s, pa);
  hipLaunchKernelGGL(k_kp_order, dim3((unsigned)((nn + KF_B - 1) / KF_B)), dim3(KF_B), 0, s, off.p, nn, kp_rec.p,
                     stride);
  SG_HIP(hipGetLastError());
  timed(5, s);
  SG_HIP(hipStreamSynchronize(s));
  float ms = 0;
  SG_HIP(hipEventElapsedTime(&ms, ev[0], ev[1])); kernel_ms["k_kf_entries"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[1], ev[2])); kernel_ms["radix_sort"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[2], ev[3])); kernel_ms["k_kf_scan"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[4], ev[5])); kernel_ms["k_kf_place_order"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[0], ev[5])); kernel_ms["total"] = ms;
  std::swap(carry, new_carry);
  n_carry = nc;
  lo = n;
  nrec = total;
  last_matches = total;
  if (materialise && total > 0) materialise_packed(out, s);
  return true;
}

// Partition pass of the tile matcher: projection sources, the bucket histogram
// per super-tile, its bucket-major exclusive scan (stable scatter bases), bucket starts, and the stable
// scatter into 12-B (or 16-B) entries.  Events ev[0] -> ev[1] time the histogram, ev[1] -> the scatter.
bool KeyedFollowedByExec::kt_partition(hipStream_t s, KtArgs& a, int pb, int64_t ts_lo, int64_t ts_hi, int& stride) {
  const int P = 1 << pb;
  const int64_t nst = (n + KT_ST - 1) / KT_ST;
  kt_pb = pb;
  // projection sources
  std::memset(&a, 0, sizeof(a));
  a.nproj = (int)fp.pslot.size();
  stride = 2;
  for (int c = 0; c < a.nproj; c++) {
    const int col = fp.pcol[c], slot = fp.pslot[c];
    const int w = tsize(app->streams[st].types[col]) / 4;
    a.w[c] = w;
    if (col == kcol) a.src[c] = KT_KEY;
    else if (col == fp.xcol) a.src[c] = slot == 0 ? KT_XI : KT_XJ;
    else { a.src[c] = slot == 0 ? KT_COL_I : KT_COL_J; a.col[c] = colptr(col); }
    stride += w;
  }
  kt_hist.reserve(P * nst); kt_bstart.reserve(P + 1); kt_tprefix.reserve(P + 1); kt_bcur.reserve(P);
  kt_ent.reserve(n + 1); kt_flags.reserve(4);   // + the scatter's dummy slot ent[n]
  kp_rec.reserve((size_t)n * stride);
  new_carry.reserve(std::max<int64_t>(n, 1));
  SG_HIP(hipMemsetAsync(kt_flags.p, 0, 16, s));
  a.ts = d_ts(); a.keycol = (const uint32_t*)colptr(kcol); a.xcol = (const uint32_t*)colptr(fp.xcol);
  a.f1kind = fp.f1kind; a.f1op = fp.f1op; a.f1t = fp.f1t; a.f1c = fp.f1c;
  if (fp.f1kind == 1) { a.f1col = colptr(fp.f1col); a.f1w = tsize(app->streams[st].types[fp.f1col]); }
  a.n = n; a.lo = lo; a.ts0 = ts_lo; a.within = within; a.pb = pb; a.tile_t = kt_T; a.nst = (int32_t)nst;
  a.vec_rec = getenv("SG_KT_VEC") ? atoi(getenv("SG_KT_VEC")) : 1;   // tuning hook
  a.exp = getenv("SG_KT_EXP") ? atoi(getenv("SG_KT_EXP")) : 0;      // measurement hook (wrong results)
  // 12-B entries when the relative timestamps fit 21 bits (the 16-B format serves the tuning variants and
  // the SG_KT_E16 test hook)
  a.ent12 = ts_hi - ts_lo < (1ll << 21) && kt_T == 2048 && !getenv("SG_KT_E16");
  a.hist = kt_hist.p; a.ent = kt_ent.p; a.bstart = kt_bstart.p;
  a.tprefix = kt_tprefix.p; a.tdesc = kt_tdesc.p; a.rec = kp_rec.p; a.stride = stride; a.bcur = kt_bcur.p;
  a.tdir = kt_tdir.p; a.carry = new_carry.p; a.ncarry = kt_flags.p; a.overflow = kt_flags.p + 1;
  a.unsorted = kt_flags.p + 2;
  a.ts_last_rel = ts_hi - ts_lo;
  timed(0, s);
  hipLaunchKernelGGL(k_kt_hist, dim3((unsigned)nst), dim3(KT_NT), 0, s, a);
  size_t tmp = 0;
  SG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, kt_hist.p, kt_hist.p, (int)(P * nst), s));
  sort_tmp.reserve(tmp);
  SG_HIP(hipcub::DeviceScan::ExclusiveSum(sort_tmp.p, tmp, kt_hist.p, kt_hist.p, (int)(P * nst), s));
  hipLaunchKernelGGL(k_kt_buckets, dim3(1), dim3(KT_NT), 0, s, a);
  SG_HIP(hipGetLastError());
  if (getenv("SG_KT_DEBUG"))
    fprintf(stderr, "[kt] n=%lld pb=%d T=%d nst=%lld within=%lld\n", (long long)n, pb, kt_T, (long long)nst,
            (long long)within);
  timed(1, s);
  {
    const int chunk = getenv("SG_KT_CHUNK") ? atoi(getenv("SG_KT_CHUNK")) : 2048;   // tuning hook
    // F1W 1: the start filter reads the compared column itself (no second load)
    const int f1w = fp.f1kind != 1 ? 0 : (a.f1w == 4 && fp.f1col == fp.xcol) ? 1 : a.f1w;
    bool lds_ok = true;
    auto launch = [&](auto kern, int nt) {
      // the bucket histogram / cursors grow with P: raise the dynamic-LDS limit (160 KiB on gfx950)
      const size_t lds = kt_scatter_lds(nt, P, a.ent12 ? chunk : 0);
      if (lds > 160 * 1024) { lds_ok = false; return; }
      SG_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL(kern, dim3((unsigned)nst), dim3(nt), lds, s, a);
    };
    if (a.ent12 && chunk == 8192) {          // tuning variants: longer bucket runs per staged store
      if (f1w == 8) launch(k_kt_scatter<8192, 8, KT_NT, true>, KT_NT);
      else if (f1w == 4) launch(k_kt_scatter<8192, 4, KT_NT, true>, KT_NT);
      else if (f1w == 1) launch(k_kt_scatter<8192, 1, KT_NT, true>, KT_NT);
      else launch(k_kt_scatter<8192, 0, KT_NT, true>, KT_NT);
    } else if (a.ent12 && chunk == 4096) {
      if (f1w == 8) launch(k_kt_scatter<4096, 8, KT_NT, true>, KT_NT);
      else if (f1w == 4) launch(k_kt_scatter<4096, 4, KT_NT, true>, KT_NT);
      else if (f1w == 1) launch(k_kt_scatter<4096, 1, KT_NT, true>, KT_NT);
      else launch(k_kt_scatter<4096, 0, KT_NT, true>, KT_NT);
    } else if (a.ent12) {
      if (f1w == 8) launch(k_kt_scatter<2048, 8, KT_NT, true>, KT_NT);
      else if (f1w == 4) launch(k_kt_scatter<2048, 4, KT_NT, true>, KT_NT);
      else if (f1w == 1) launch(k_kt_scatter<2048, 1, KT_NT, true>, KT_NT);
      else launch(k_kt_scatter<2048, 0, KT_NT, true>, KT_NT);
    } else if (chunk == 8192) {
      if (f1w == 8) launch(k_kt_scatter<8192, 8, 1024>, 1024);
      else if (f1w == 4 || f1w == 1) launch(k_kt_scatter<8192, 4, 1024>, 1024);
      else launch(k_kt_scatter<8192, 0, 1024>, 1024);
    } else if (chunk == 4096) {
      if (f1w == 8) launch(k_kt_scatter<4096, 8, 1024>, 1024);
      else if (f1w == 4) launch(k_kt_scatter<4096, 4, 1024>, 1024);
      else if (f1w == 1) launch(k_kt_scatter<4096, 1, 1024>, 1024);
      else launch(k_kt_scatter<4096, 0, 1024>, 1024);
    } else {
      if (f1w == 8) launch(k_kt_scatter<2048, 8>, KT_NT);
      else if (f1w == 4) launch(k_kt_scatter<2048, 4>, KT_NT);
      else if (f1w == 1) launch(k_kt_scatter<2048, 1>, KT_NT);
      else launch(k_kt_scatter<2048, 0>, KT_NT);
    }
    if (!lds_ok) return false;   // the sort pipeline takes this flush
  }
  return true;
}

bool KeyedFollowedByExec::run_tiled(hipStream_t s, bool materialise, std::vector<Callback>& out) {
  const bool dbg = getenv("SG_KT_DEBUG") != nullptr;
  const auto h0 = std::chrono::steady_clock::now();
  auto hms = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count(); };
  int64_t ts_lo = 0, ts_hi = 0;
  SG_HIP(hipMemcpyAsync(&ts_lo, d_ts(), 8, hipMemcpyDeviceToHost, s));
  SG_HIP(hipMemcpyAsync(&ts_hi, d_ts() + n - 1, 8, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  const double h_sync0 = hms();
  if (ts_hi - ts_lo >= (1ll << 31) || n >= (1ll << 31)) return false;   // 31-bit relative timestamps, u32 indices
  const int kb = key_end_bit(s);
  if (kb > KT_LB + KT_MAXPB) return false;
  // buckets: local keys must fit KT_LB bits, and a bucket's share of the events in one `within` window
  // (at the mean rate) should fill about half of the KT_H back-halo.  Denser windows overflow and fall back.
  const double win = (double)n * (double)(within + 1) / (double)(ts_hi - ts_lo + 1);
  int pb = std::max(0, kb - KT_LB);
  while (pb < KT_MAXPB && win / (double)(1 << pb) > KT_H / 2) pb++;
  const int P = 1 << pb;
  const int64_t nst = (n + KT_ST - 1) / KT_ST;
  kt_T = getenv("SG_KT_TILE") && atoi(getenv("SG_KT_TILE")) == 4096 ? 4096 : 2048;   // tuning hook
  KtArgs a;
  int stride = 0;
  if (!kt_partition(s, a, pb, ts_lo, ts_hi, stride)) return false;
  const int64_t ntiles = n / kt_T + P + 1;            // upper bound on the tiles (slots past the total are empty)
  kt_ntiles = ntiles;
  kt_tdesc.reserve(ntiles); kt_tdir.reserve(ntiles);
  a.ntiles_max = ntiles; a.tdesc = kt_tdesc.p; a.tdir = kt_tdir.p;
  // trigger order on the device (k_kt_order): the matcher notes each order group's boundary per bucket
  const int64_t nh = (n + KS_HQ - 1) / KS_HQ;
  const bool dev_order = P <= 2048 && a.stride >= 2 && !getenv("SG_KT_NO_ORDER");
  if (dev_order) {
    kt_toffs.reserve((size_t)(nh + 1) * P);
    SG_HIP(hipMemsetAsync(kt_toffs.p, 0xff, (size_t)(nh + 1) * P * sizeof(uint2), s));   // empty buckets' rows
    a.toffs = kt_toffs.p;
    a.nh = nh;
  }
  // the tile table places each back-halo from the bucketed timestamps: after the scatter
  if (!(a.exp & 2)) hipLaunchKernelGGL(k_kt_tdesc, dim3((unsigned)((ntiles + KT_NT - 1) / KT_NT)), dim3(KT_NT), 0, s, a);
  SG_HIP(hipGetLastError());
  timed(2, s);
  DBuf<int64_t> dbgbuf;
  const int ndbg = dbg ? 4096 : 0;
  if (dbg) {
    dbgbuf.reserve(ndbg * 8);
    SG_HIP(hipMemsetAsync(dbgbuf.p, 0, ndbg * 64, s));
    a.dbg = dbgbuf.p; a.dbg_n = ndbg;
  }
  // tuning hooks: SG_KT_XCD=1 deals the matcher's tiles XCD-contiguously (measured: no gain, 16.41 vs 16.34
  // ms, profiles/r03q_*); SG_KO_XCD=0 deals the order groups in plain order (XCD-contiguous is 2 % faster)
  a.xcd_tiles = getenv("SG_KT_XCD") && atoi(getenv("SG_KT_XCD")) == 1;
  kt_mgrid = a.xcd_tiles ? 8 * ((ntiles + 7) / 8) : ntiles;
  if (a.exp & 2) {
  } else if (fp.t == T_FLOAT) kt_match_op<float>(a, s);
  else kt_match_op<int32_t>(a, s);
  SG_HIP(hipGetLastError());
  timed(3, s);
  uint32_t total_dev = 0;
  if (dev_order) {
    KtOrderArgs o{};
    o.toffs = kt_toffs.p; o.tdir = kt_tdir.p; o.flags = kt_flags.p; o.rec = kp_rec.p; o.stride = stride; o.pb = pb;
    o.nh = nh;
    o.xcd = !(getenv("SG_KO_XCD") && atoi(getenv("SG_KO_XCD")) == 0);
    const unsigned og = (unsigned)(o.xcd ? 8 * ((nh + 7) / 8) : nh);
    ks_tot.reserve((size_t)nh + 1); ks_hbase.reserve((size_t)nh + 1);
    SG_HIP(hipMemsetAsync(ks_tot.p + nh, 0, 4, s));
    hipLaunchKernelGGL(k_kt_order_count, dim3(og), dim3(256), 0, s, o, ks_tot.p);
    size_t tmp2 = 0;
    SG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp2, ks_tot.p, ks_hbase.p, (int)(nh + 1), s));
    sort_tmp.reserve(tmp2);
    SG_HIP(hipcub::DeviceScan::ExclusiveSum(sort_tmp.p, tmp2, ks_tot.p, ks_hbase.p, (int)(nh + 1), s));
    ks_out.reserve((size_t)std::max<int64_t>(n, 1) * stride);
    timed(5, s);
    const size_t lds = kt_order_lds(P);
    SG_HIP(hipFuncSetAttribute((const void*)k_kt_order, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_kt_order, dim3(og), dim3(KS_ORDER_NT), lds, s, o, ks_hbase.p, ks_out.p);
    SG_HIP(hipGetLastError());
    SG_HIP(hipMemcpyAsync(&total_dev, ks_hbase.p + nh, 4, hipMemcpyDeviceToHost, s));
  }
  timed(4, s);
  if (dbg) {   // mean phase durations of the sampled matcher tiles (10 ns wall-clock ticks)
    std::vector<int64_t> h(ndbg * 8);
    SG_HIP(hipMemcpyAsync(h.data(), dbgbuf.p, h.size() * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    double acc[8] = {0}; int cntd = 0;
    for (int w = 0; w < ndbg; w++) {
      const int64_t* x = h.data() + w * 8;
      if (x[7] == 0 || x[0] == 0) continue;
      cntd++;
      for (int k = 1; k < 8; k++) acc[k] += (double)(x[k] - x[k - 1]) * 0.01;
    }
    fprintf(stderr, "[kt match phases us, %d tiles] load+zero %.2f rank %.2f hscan %.2f place %.2f count %.2f scan+emit %.2f write %.2f\n",
            cntd, acc[1] / cntd, acc[2] / cntd, acc[3] / cntd, acc[4] / cntd, acc[5] / cntd, acc[6] / cntd, acc[7] / cntd);
  }
  const double h_launch = hms();
  uint32_t flags[3] = {0, 0, 0};
  SG_HIP(hipMemcpyAsync(flags, kt_flags.p, 12, hipMemcpyDeviceToHost, s));
  std::vector<uint32_t> hb(P), hc(P);
  SG_HIP(hipMemcpyAsync(hb.data(), kt_bstart.p, P * 4, hipMemcpyDeviceToHost, s));
  SG_HIP(hipMemcpyAsync(hc.data(), kt_bcur.p, P * 4, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  const double h_sync1 = hms();
  if (dbg) fprintf(stderr, "[kt host] sync0 %.3f launch %.3f sync1 %.3f ms\n", h_sync0, h_launch, h_sync1);
  if (flags[2]) throw Error(-1, "keyed followed-by: event timestamps go backwards (device-resident input must be "
                                 "non-decreasing, as sg_push enforces for host batches)");
  if (flags[1] && !(a.exp & 2)) return false;   // a back-halo longer than KT_H: the sort pipeline takes this flush
  int64_t total = 0;
  for (int b = 0; b < P; b++) total += (int64_t)hc[b] - hb[b];
  float ms = 0;
  SG_HIP(hipEventElapsedTime(&ms, ev[0], ev[1])); kernel_ms["k_kt_hist"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[1], ev[2])); kernel_ms["k_kt_scatter"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[2], ev[3])); kernel_ms["k_kt_match"] = ms;
  if (dev_order) {
    SG_HIP(hipEventElapsedTime(&ms, ev[3], ev[4])); kernel_ms["k_kt_order"] = ms;
    SG_HIP(hipEventElapsedTime(&ms, ev[3], ev[5])); kernel_ms["k_kt_order_count"] = ms;   // counts + scan
  }
  SG_HIP(hipEventElapsedTime(&ms, ev[0], ev[4])); kernel_ms["total"] = ms;
  if (dev_order && total_dev != total) throw Error(-3, "keyed order pass lost records");
  std::swap(carry, new_carry);
  n_carry = flags[0];
  lo = n;
  kp_stride = stride;
  nrec = total;
  last_matches = total;
  if (materialise && total > 0) {
    if (dev_order) materialise_ordered(ks_out.p, total, out, s);   // already in callback order
    else materialise_tiled(out, s);
  }
  return true;
}

// Chunk-sorted pipeline (keyed_chunks.hpp): k_kc_sort (contiguous bucket-sorted chunks), k_kc_slices (halo chunk of
// every slice), k_kc_match (one tile per (slice, bucket)), then the trigger-order pass (keyed_order.hpp) in slice
// mode.  False: the bucketed tiles take the flush (a chunk spanning KC_TSPAN ms or more, a halo or slice that does
// not fit the tile, buckets beyond the order pass, a trigger with more than KT_MAXREC records).
bool KeyedFollowedByExec::run_chunked(hipStream_t s, bool materialise, std::vector<Callback>& out) {
  int64_t ts_lo = 0, ts_hi = 0;
  SG_HIP(hipMemcpyAsync(&ts_lo, d_ts(), 8, hipMemcpyDeviceToHost, s));
  SG_HIP(hipMemcpyAsync(&ts_hi, d_ts() + n - 1, 8, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  if (ts_hi - ts_lo >= (1ll << 31) || n >= (1ll << 31) || within < 0) return false;
  const int kb = key_end_bit(s);
  if (kb > KT_LB + KT_MAXPB) return false;
  // buckets as in run_tiled: local keys fit KT_LB bits, a bucket's share of one `within` window about half of KT_H
  const double win = (double)n * (double)(within + 1) / (double)(ts_hi - ts_lo + 1);
  // (at least 16 buckets: a slice holds whole order groups of KS_HQ trigger indices, at most 0.85 T per bucket).
  // Small tiles when 9-bit local keys and a back-halo of at most 512 entries per bucket fit 2048 buckets.
  int pb = std::max(4, kb - 9);
  while (pb < 11 && win / (double)(1 << pb) > 512) pb++;
  kc_small = getenv("SG_KC_LARGE") == nullptr && pb <= 11 && kb - pb <= 9 && win / (double)(1 << pb) <= 512;
  if (!kc_small) {
    pb = std::max(4, kb - KT_LB);
    while (pb < KT_MAXPB && win / (double)(1 << pb) > KT_H / 2) pb++;
  }
  const int P = 1 << pb;
  if (P > 2048) return false;                                   // the order pass's LDS
  const int T = kc_small ? 1536 : 2048;          // triggers a slice is sized for (the capacity is 2048)
  // slices: about 0.85 T triggers per bucket (6 sigma of the Poisson spread below T at config 4's density), a whole
  // number of order groups (KS_HQ trigger indices) each
  const int gq = KS_HQ / KC_C;
  int spc = (int)((0.85 * T * P / KC_C) / gq) * gq;
  if (spc < gq) spc = gq;
  const int64_t nchunks = (n + KC_C - 1) / KC_C;
  const int64_t nslices = (nchunks + spc - 1) / spc;
  const int64_t ntile = nslices * P;
  const int64_t nh = (n + KS_HQ - 1) / KS_HQ;
  KcArgs a;
  std::memset(&a, 0, sizeof(a));
  a.nproj = (int)fp.pslot.size();
  int stride = 2;
  for (int c = 0; c < a.nproj; c++) {
    const int col = fp.pcol[c], slot = fp.pslot[c];
    const int w = tsize(app->streams[st].types[col]) / 4;
    a.w[c] = w;
    if (col == kcol) a.src[c] = KT_KEY;
    else if (col == fp.xcol) a.src[c] = slot == 0 ? KT_XI : KT_XJ;
    else { a.src[c] = slot == 0 ? KT_COL_I : KT_COL_J; a.col[c] = colptr(col); }
    stride += w;
  }
  kc_ent.reserve((size_t)nchunks * KC_C); kc_off.reserve((size_t)nchunks * P); kc_cts0.reserve((size_t)nchunks);
  kc_shalo.reserve((size_t)nslices); kc_flags.reserve(8);
  kt_tdir.reserve((size_t)ntile);
  const int gps = (int)(((int64_t)spc * KC_C) >> KS_HQB);
  kc_rows.reserve((size_t)ntile * gps);
  // record slots: a fixed region of LC (the matcher's entry capacity) per tile, about 1.8 n at config 4
  const int64_t rcap = ntile * (int64_t)(kc_small ? 2304 : 4096);
  if (rcap > (int64_t)UINT32_MAX) return false;
  kp_rec.reserve((size_t)rcap * stride);
  new_carry.reserve(std::max<int64_t>(n, 1));
  SG_HIP(hipMemsetAsync(kc_flags.p, 0, 32, s));
  a.ts = d_ts(); a.keycol = (const uint32_t*)colptr(kcol); a.xcol = (const uint32_t*)colptr(fp.xcol);
  a.f1kind = fp.f1kind; a.f1op = fp.f1op; a.f1t = fp.f1t; a.f1c = fp.f1c;
  if (fp.f1kind == 1) { a.f1col = colptr(fp.f1col); a.f1w = tsize(app->streams[st].types[fp.f1col]); }
  a.n = n; a.ts0 = ts_lo; a.within = within; a.ts_last_rel = ts_hi - ts_lo; a.pb = pb; a.nchunks = nchunks;
  a.ent = kc_ent.p; a.off = kc_off.p; a.cts0 = kc_cts0.p; a.flags = kc_flags.p;
  a.spc = spc; a.nslices = nslices; a.shalo = kc_shalo.p;
  a.rec = kp_rec.p; a.stride = stride; a.rcap = (uint32_t)rcap; a.tdir = kt_tdir.p;
  a.carry = new_carry.p;
  a.rows16 = kc_rows.p; a.gps = gps; a.hqb = KS_HQB;
  a.vec_rec = getenv("SG_KT_VEC") ? atoi(getenv("SG_KT_VEC")) : 1;   // tuning hook
  a.exp = getenv("SG_KC_EXP") ? atoi(getenv("SG_KC_EXP")) : 0;       // measurement hook (wrong results)
  a.atomic_rank = getenv("SG_KC_PEER_RANK") == nullptr;              // A/B hook
  const bool dbg = getenv("SG_KT_DEBUG") != nullptr;
  DBuf<int64_t> dbgbuf;
  const int ndbg = dbg ? 8192 : 0;
  if (dbg) {
    dbgbuf.reserve((size_t)ndbg * KC_NPROBE);
    SG_HIP(hipMemsetAsync(dbgbuf.p, 0, (size_t)ndbg * KC_NPROBE * 8, s));
    a.dbg = dbgbuf.p; a.dbg_n = ndbg;
  }
  timed(0, s);
  {
    const int f1w = fp.f1kind != 1 ? 0 : (a.f1w == 4 && fp.f1col == fp.xcol) ? 1 : a.f1w;
    const size_t lds = kc_sort_lds(P, KC_NT);
    auto launch = [&](auto kern) {
      SG_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL(kern, dim3((unsigned)nchunks), dim3(KC_NT), lds, s, a);
    };
    if (f1w == 8) launch(k_kc_sort<8>);
    else if (f1w == 4) launch(k_kc_sort<4>);
    else if (f1w == 1) launch(k_kc_sort<1>);
    else launch(k_kc_sort<0>);
  }
  SG_HIP(hipGetLastError());
  timed(1, s);
  hipLaunchKernelGGL(k_kc_slices, dim3((unsigned)((nslices + 255) / 256)), dim3(256), 0, s, a);
  SG_HIP(hipGetLastError());
  timed(2, s);
  if (fp.t == T_FLOAT) kc_match_op<float>(a, (unsigned)ntile, s);
  else kc_match_op<int32_t>(a, (unsigned)ntile, s);
  SG_HIP(hipGetLastError());
  timed(3, s);
  KtOrderArgs o;
  std::memset(&o, 0, sizeof(o));
  o.rows16 = kc_rows.p; o.gps = gps; o.tdir = kt_tdir.p; o.flags = kc_flags.p; o.rec = kp_rec.p; o.stride = stride;
  o.pb = pb;
  o.nh = (a.exp & 1) ? 0 : nh;                     // (a matcher stopped after its gather wrote no order rows)
  o.slice_tiles = 1;
  o.xcd = !(getenv("SG_KO_XCD") && atoi(getenv("SG_KO_XCD")) == 0);
  const unsigned og = (unsigned)(o.xcd ? 8 * ((nh + 7) / 8) : nh);
  ks_tot.reserve((size_t)nh + 1); ks_hbase.reserve((size_t)nh + 1);
  SG_HIP(hipMemsetAsync(ks_tot.p + nh, 0, 4, s));
  hipLaunchKernelGGL(k_kt_order_count, dim3(og), dim3(256), 0, s, o, ks_tot.p);
  size_t tmp2 = 0;
  SG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp2, ks_tot.p, ks_hbase.p, (int)(nh + 1), s));
  sort_tmp.reserve(tmp2);
  SG_HIP(hipcub::DeviceScan::ExclusiveSum(sort_tmp.p, tmp2, ks_tot.p, ks_hbase.p, (int)(nh + 1), s));
  ks_out.reserve((size_t)std::max<int64_t>(n, 1) * stride);
  timed(5, s);
  {
    const size_t lds = kt_order16_lds(P);
    SG_HIP(hipFuncSetAttribute((const void*)k_kt_order, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_kt_order, dim3(og), dim3(KS_ORDER_NT), lds, s, o, ks_hbase.p, ks_out.p);
  }
  SG_HIP(hipGetLastError());
  uint32_t total_dev = 0;
  SG_HIP(hipMemcpyAsync(&total_dev, ks_hbase.p + nh, 4, hipMemcpyDeviceToHost, s));
  timed(4, s);
  uint32_t flags[6] = {0, 0, 0, 0, 0, 0};
  SG_HIP(hipMemcpyAsync(flags, kc_flags.p, 24, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  if (flags[2]) throw Error(-1, "keyed followed-by: event timestamps go backwards (device-resident input must be "
                                 "non-decreasing, as sg_push enforces for host batches)");
  if (getenv("SG_KT_DEBUG"))
    fprintf(stderr, "[kc] n=%lld pb=%d spc=%d slices=%lld small=%d flags ovf=%u wide=%u slots=%u rec=%u\n", (long long)n,
            pb, spc, (long long)nslices, (int)kc_small, flags[1], flags[3], flags[4], total_dev);
  if (dbg) {   // mean phase durations of the sampled matcher tiles (10 ns wall-clock ticks)
    std::vector<int64_t> h((size_t)ndbg * KC_NPROBE);
    SG_HIP(hipMemcpy(h.data(), dbgbuf.p, h.size() * 8, hipMemcpyDeviceToHost));
    double acc[KC_NPROBE] = {0};
    int cnt = 0;
    for (int w = 0; w < ndbg; w++) {
      const int64_t* x = h.data() + (size_t)w * KC_NPROBE;
      if (!x[0] || !x[11]) continue;
      cnt++;
      int64_t prev = x[0];
      for (int k = 1; k < KC_NPROBE; k++) if (x[k]) { acc[k] += (double)(x[k] - prev) * 0.01; prev = x[k]; }
    }
    fprintf(stderr, "[kc match phases us, %d tiles] offsets %.2f lscan %.2f gather %.2f decode %.2f rank %.2f kscan %.2f "
                    "place %.2f walk %.2f slots+sort %.2f write+rows %.2f\n", cnt, acc[1] / cnt, acc[2] / cnt,
            acc[3] / cnt, acc[4] / cnt, acc[5] / cnt, acc[6] / cnt, acc[7] / cnt, acc[8] / cnt, acc[9] / cnt,
            acc[11] / cnt);
  }
  if (a.exp) return true;                          // measurement runs: no outputs
  if (flags[1] || flags[3]) return false;          // the bucketed tiles take this flush
  // the order pass's count of the tiles' records, cross-checked against the matchers' own (one atomic per tile): a
  // row-writing bug would drop or misplace records silently otherwise
  if (flags[5] != total_dev) throw Error(-3, "keyed order pass lost records (chunk pipeline)");
  const int64_t total = total_dev;
  float ms = 0;
  SG_HIP(hipEventElapsedTime(&ms, ev[0], ev[1])); kernel_ms["k_kc_sort"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[1], ev[2])); kernel_ms["k_kc_slices"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[2], ev[3])); kernel_ms["k_kc_match"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[3], ev[4])); kernel_ms["k_kt_order"] = ms;
  SG_HIP(hipEventElapsedTime(&ms, ev[3], ev[5])); kernel_ms["k_kt_order_count"] = ms;   // counts + scan
  SG_HIP(hipEventElapsedTime(&ms, ev[0], ev[4])); kernel_ms["total"] = ms;
  std::swap(carry, new_carry);
  n_carry = flags[0];
  lo = n;
  kp_stride = stride;
  nrec = total;
  last_matches = total;
  if (materialise && total > 0) materialise_ordered(ks_out.p, total, out, s);
  return true;
}

__global__ void __launch_bounds__(256) k_ks_rec_ts(int64_t total, const int32_t* __restrict__ rec, int32_t stride,
                                                   const int64_t* __restrict__ ts, int64_t* __restrict__ out_ts) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r < total) out_ts[r] = ts[rec[r * stride]];
}

// Records already in callback order (ascending j, then i): copy them out with their triggers' timestamps and
// cut one callback per distinct j.
// Callback-ordered records -> the columnar rows of the reference's QueryCallback.receive calls, on the device: each
// record's row (the trigger's timestamp, its projection words decoded into the ABI's 8-B raw slots: FLOAT bits
// zero-extended, other 4-B values sign-extended, 8-B values whole) and whether it opens a callback (its trigger j
// differs from the previous record's: one callback per trigger, ReturnEventHolder per input event,
// MultiProcessStreamReceiver.java:306-316)
struct KoRowArgs {
  const int32_t* rec;
  int32_t stride, nout;
  int32_t w8[FB_MAXP], fl[FB_MAXP];
  const int64_t* ts;
  int64_t total;
  int64_t* ots;
  int64_t* raw;
  uint8_t* first;
};
__global__ void __launch_bounds__(256) k_ko_rows(KoRowArgs a) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= a.total) return;
  const int32_t* x = a.rec + r * a.stride;
  const int32_t j = x[0];
  a.ots[r] = a.ts[j];
  a.first[r] = (uint8_t)(r == 0 || a.rec[(r - 1) * a.stride] != j);
  int wo = 2;
  for (int k = 0; k < a.nout; k++) {
    int64_t v;
    if (a.w8[k]) { v = (int64_t)(uint32_t)x[wo] | ((int64_t)x[wo + 1] << 32); wo += 2; }
    else { v = a.fl[k] ? (int64_t)(uint32_t)x[wo] : (int64_t)x[wo]; wo += 1; }
    a.raw[r * a.nout + k] = v;
  }
}
// one thread per callback (+1 for the closing row bound): its first row, (ts, seq) of its trigger
__global__ void __launch_bounds__(256) k_ko_cbs(const int32_t* __restrict__ ncb_p, const int32_t* __restrict__ first,
                                                const int32_t* __restrict__ rec, int32_t stride,
                                                const int64_t* __restrict__ ots, int64_t total,
                                                const int64_t* __restrict__ dseq, int64_t* __restrict__ cts,
                                                int64_t* __restrict__ crow, int64_t* __restrict__ cseq) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int32_t ncb = *ncb_p;
  if (c > ncb) return;
  if (c == ncb) { crow[c] = total; return; }
  const int32_t r = first[c];
  const int32_t j = rec[(int64_t)r * stride];
  cts[c] = ots[r];
  crow[c] = r;
  cseq[c] = dseq ? dseq[j] : (int64_t)j;   // the trigger's global arrival seq (device ingest), else its index
}

void KeyedFollowedByExec::materialise_ordered(const int32_t* d_rec, int64_t total, std::vector<Callback>& out,
                                              hipStream_t s) {
  if (!getenv("SG_KEYED_OBJECT_OUT")) {           // columnar callbacks formed on the device (one bulk entry)
    const int nout = (int)fp.pslot.size();
    KoRowArgs a;
    std::memset(&a, 0, sizeof(a));
    a.rec = d_rec; a.stride = kp_stride; a.nout = nout; a.ts = d_ts(); a.total = total;
    for (int k = 0; k < nout; k++) {
      const Ty t = app->streams[st].types[fp.pcol[k]];
      a.w8[k] = tsize(t) == 8; a.fl[k] = t == T_FLOAT;
    }
    ko_ts.reserve(total); ko_raw.reserve((size_t)total * std::max(nout, 1)); ko_first.reserve(total);
    ko_cfirst.reserve(total + 1); ko_cts.reserve(total);
    a.ots = ko_ts.p; a.raw = ko_raw.p; a.first = ko_first.p;
    hipLaunchKernelGGL(k_ko_rows, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a);
    SG_HIP(hipGetLastError());
    hipcub::CountingInputIterator<int32_t> idx(0);
    size_t tb = 0;
    SG_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb, idx, ko_first.p, ko_cfirst.p, ko_cfirst.p + total, (int)total, s));
    sort_tmp.reserve(tb);
    SG_HIP(hipcub::DeviceSelect::Flagged(sort_tmp.p, tb, idx, ko_first.p, ko_cfirst.p, ko_cfirst.p + total, (int)total, s));
    ko_crow.reserve(total + 1); ko_cseq.reserve(total);
    hipLaunchKernelGGL(k_ko_cbs, dim3((unsigned)((total + 256) / 256)), dim3(256), 0, s, ko_cfirst.p + total, ko_cfirst.p,
                       d_rec, (int32_t)kp_stride, ko_ts.p, total, ext_seq, ko_cts.p, ko_crow.p, ko_cseq.p);
    SG_HIP(hipGetLastError());
    int32_t ncb = 0;
    SG_HIP(hipMemcpyAsync(&ncb, ko_cfirst.p + total, 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    // every column lands in pooled pinned memory (OutBlock's HostCol): one DMA each, no host pass over rows
    auto blk = std::make_unique<OutBlock>();
    OutBlock& b = *blk;
    b.width = nout;
    b.ts.resize((size_t)total); b.raw.resize((size_t)total * nout);
    b.cb_ts.resize((size_t)ncb); b.cb_row.resize((size_t)ncb + 1); b.cb_seq.resize((size_t)ncb);
    SG_HIP(hipMemcpyAsync(b.ts.data(), ko_ts.p, (size_t)total * 8, hipMemcpyDeviceToHost, s));
    if (nout) SG_HIP(hipMemcpyAsync(b.raw.data(), ko_raw.p, (size_t)total * nout * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(b.cb_ts.data(), ko_cts.p, (size_t)ncb * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(b.cb_row.data(), ko_crow.p, (size_t)(ncb + 1) * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(b.cb_seq.data(), ko_cseq.p, (size_t)ncb * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    if (!ext_seq && !h_seq.empty())                  // host ingest: trigger index -> the app's arrival seq
      for (int32_t c = 0; c < ncb; c++) b.cb_seq[(size_t)c] = h_seq[(size_t)b.cb_seq[(size_t)c]];
    Callback cb;
    cb.seq = ncb ? b.cb_seq[0] : 0;
    cb.order = qi; cb.kind = 0; cb.target = qi;
    cb.ts = ncb ? b.cb_ts[0] : 0;
    cb.blk = blk.get();
    app->blocks.push_back(std::move(blk));
    out.push_back(std::move(cb));
    return;
  }
  fetch_seq(s);
  ks_ots.reserve(total);
  hipLaunchKernelGGL(k_ks_rec_ts, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, total, d_rec,
                     (int32_t)kp_stride, d_ts(), ks_ots.p);
  SG_HIP(hipGetLastError());
  std::vector<int32_t> rec((size_t)total * kp_stride);
  std::vector<int64_t> hts(total);
  SG_HIP(hipMemcpyAsync(rec.data(), d_rec, rec.size() * 4, hipMemcpyDeviceToHost, s));
  SG_HIP(hipMemcpyAsync(hts.data(), ks_ots.p, (size_t)total * 8, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  build_callbacks(rec.data(), hts.data(), total, out);
}

// Records of one bucket, tile after tile, are in (j, i) order, and all records of one trigger j sit in
// one tile.  The reference's global order (ascending j, then i) is therefore a stable sort of the records
// by j, done on the device: the tiles' record runs are listed compactly (k_kt_rec_keys), radix-sorted by
// j (stable: a trigger's records keep ascending i), gathered with the trigger's timestamp
// (k_kt_rec_gather) and copied out in callback order; the host only cuts callbacks where j changes.
__global__ void __launch_bounds__(256) k_kt_rec_count(const uint4* __restrict__ tdesc, const uint2* __restrict__ tdir,
                                                      int64_t ntiles, uint32_t* __restrict__ cnt) {
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (w < ntiles) cnt[w] = tdesc[w].x == 0xffffffffu ? 0u : tdir[w].y;
}

__global__ void __launch_bounds__(256) k_kt_rec_keys(const uint4* __restrict__ tdesc, const uint2* __restrict__ tdir,
                                                     const uint32_t* __restrict__ off, const int32_t* __restrict__ rec,
                                                     int32_t stride, uint32_t* __restrict__ keys,
                                                     uint32_t* __restrict__ slots) {
  const int64_t w = blockIdx.x;
  if (tdesc[w].x == 0xffffffffu) return;
  const uint2 d = tdir[w];
  const uint32_t o = off[w];
  for (uint32_t r = threadIdx.x; r < d.y; r += 256) {
    keys[o + r] = (uint32_t)rec[(int64_t)(d.x + r) * stride];
    slots[o + r] = d.x + r;
  }
}

__global__ void __launch_bounds__(256) k_kt_rec_gather(int64_t total, const uint32_t* __restrict__ slots,
                                                       const int32_t* __restrict__ rec, int32_t stride,
                                                       const int64_t* __restrict__ ts, int32_t* __restrict__ out,
                                                       int64_t* __restrict__ out_ts) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= total) return;
  const int32_t* x = rec + (int64_t)slots[r] * stride;
  for (int k = 0; k < stride; k++) out[r * stride + k] = x[k];
  out_ts[r] = ts[x[0]];
}

void KeyedFollowedByExec::materialise_tiled(std::vector<Callback>& out, hipStream_t s) {
  fetch_seq(s);
  const int64_t nt = kt_ntiles;
  DBuf<uint32_t> cnt, off, keys, keys_s, slots, slots_s;
  cnt.reserve(nt); off.reserve(nt + 1);
  hipLaunchKernelGGL(k_kt_rec_count, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, kt_tdesc.p, kt_tdir.p, nt, cnt.p);
  size_t tmp = 0;
  SG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, cnt.p, off.p, (int)nt, s));
  sort_tmp.reserve(tmp);
  SG_HIP(hipcub::DeviceScan::ExclusiveSum(sort_tmp.p, tmp, cnt.p, off.p, (int)nt, s));
  const int64_t total = nrec;
  if (total == 0) return;
  keys.reserve(total); keys_s.reserve(total); slots.reserve(total); slots_s.reserve(total);
  hipLaunchKernelGGL(k_kt_rec_keys, dim3((unsigned)nt), dim3(256), 0, s, kt_tdesc.p, kt_tdir.p, off.p, kp_rec.p,
                     (int32_t)kp_stride, keys.p, slots.p);
  int bits = 1;
  while (bits < 32 && (1ll << bits) < n) bits++;
  tmp = 0;
  SG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, keys.p, keys_s.p, slots.p, slots_s.p, (int)total, 0, bits, s));
  sort_tmp.reserve(tmp);
  SG_HIP(hipcub::DeviceRadixSort::SortPairs(sort_tmp.p, tmp, keys.p, keys_s.p, slots.p, slots_s.p, (int)total, 0, bits, s));
  DBuf<int32_t> orec;
  DBuf<int64_t> ots;
  orec.reserve((size_t)total * kp_stride); ots.reserve(total);
  hipLaunchKernelGGL(k_kt_rec_gather, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, total, slots_s.p, kp_rec.p,
                     (int32_t)kp_stride, d_ts(), orec.p, ots.p);
  SG_HIP(hipGetLastError());
  std::vector<int32_t> rec((size_t)total * kp_stride);
  std::vector<int64_t> hts(total);
  SG_HIP(hipMemcpyAsync(rec.data(), orec.p, rec.size() * 4, hipMemcpyDeviceToHost, s));
  SG_HIP(hipMemcpyAsync(hts.data(), ots.p, (size_t)total * 8, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  build_callbacks(rec.data(), hts.data(), total, out);
}

void KeyedFollowedByExec::build_callbacks(const int32_t* recs, const int64_t* hts, int64_t total, std::vector<Callback>& out) {
  const int nout = (int)fp.pslot.size();
  Ty pt[FB_MAXP];
  for (int k = 0; k < nout; k++) pt[k] = app->streams[st].types[fp.pcol[k]];
  int64_t curj = -1;
  Callback* cb = nullptr;
  for (int64_t r = 0; r < total; r++) {
    const int32_t* x = recs + (size_t)r * kp_stride;
    const int64_t j = x[0];
    if (j != curj) {
      out.emplace_back();
      cb = &out.back();
      cb->seq = h_seq.empty() ? j : h_seq[j];
      cb->order = qi; cb->kind = 0; cb->target = qi;
      cb->ts = hts[r];
      curj = j;
    }
    OutEvent e;
    e.ts = hts[r];
    int wo = 2;
    for (int k = 0; k < nout; k++) {
      int64_t v;
      if (tsize(pt[k]) == 8) { v = (int64_t)(uint32_t)x[wo] | ((int64_t)x[wo + 1] << 32); wo += 2; }
      else { v = (pt[k] == T_FLOAT) ? (int64_t)(uint32_t)x[wo] : (int64_t)x[wo]; wo += 1; }
      e.raw.push_back(v);
      e.nul.push_back(0);
    }
    cb->ev.push_back(std::move(e));
  }
}


void KeyedFollowedByExec::materialise_packed(std::vector<Callback>& out, hipStream_t s) {
  fetch_seq(s);
  const int nout = (int)fp.pslot.size();
  std::vector<int32_t> rec((size_t)nrec * kp_stride);
  SG_HIP(hipMemcpyAsync(rec.data(), kp_rec.p, rec.size() * 4, hipMemcpyDeviceToHost, s));
  std::vector<int64_t> hts(n);
  SG_HIP(hipMemcpyAsync(hts.data(), d_ts(), n * 8, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  Callback* cur = nullptr;
  int64_t curj = -1;
  for (int64_t r = 0; r < nrec; r++) {
    const int32_t* x = rec.data() + r * kp_stride;
    const int64_t j = x[0];
    if (!cur || j != curj) {
      out.emplace_back();
      cur = &out.back();
      cur->seq = h_seq.empty() ? j : h_seq[j];
      cur->order = qi; cur->kind = 0; cur->target = qi;
      curj = j;
    }
    OutEvent e;
    e.ts = hts[j];
    int wo = 2;
    for (int c = 0; c < nout; c++) {
      Ty t = app->streams[st].types[fp.pcol[c]];
      int64_t v;
      if (tsize(t) == 8) { v = (int64_t)(uint32_t)x[wo] | ((int64_t)x[wo + 1] << 32); wo += 2; }
      else { v = (t == T_FLOAT) ? (int64_t)(uint32_t)x[wo] : (int64_t)x[wo]; wo += 1; }
      e.raw.push_back(v);
      e.nul.push_back(0);
    }
    cur->ts = e.ts;
    cur->ev.push_back(std::move(e));
  }
}

void KeyedFollowedByExec::materialise_records(std::vector<Callback>& out, hipStream_t s) {
  fetch_seq(s);
  const int nout = (int)sel.size();
  std::vector<int32_t> hj(nrec);
  SG_HIP(hipMemcpyAsync(hj.data(), rec_j.p, nrec * 4, hipMemcpyDeviceToHost, s));
  std::vector<std::vector<uint8_t>> pc(pout.size());
  std::vector<int64_t> raw;
  std::vector<uint8_t> nul;
  if (fp.plain_proj) {
    for (size_t c = 0; c < pout.size(); c++) {
      pc[c].resize((size_t)nrec * tsize(app->streams[st].types[fp.pcol[c]]));
      SG_HIP(hipMemcpyAsync(pc[c].data(), pout[c].p, pc[c].size(), hipMemcpyDeviceToHost, s));
    }
  } else if (nout) {
    raw.resize((size_t)nrec * nout);
    nul.resize((size_t)nrec * nout);
    SG_HIP(hipMemcpyAsync(raw.data(), out_raw.p, raw.size() * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(nul.data(), out_null.p, nul.size(), hipMemcpyDeviceToHost, s));
  }
  std::vector<int64_t> hts(n);
  SG_HIP(hipMemcpyAsync(hts.data(), d_ts(), n * 8, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  Callback* cur = nullptr;
  int64_t curj = -1;
  for (int64_t r = 0; r < nrec; r++) {
    const int64_t j = hj[r];
    if (!cur || j != curj) {
      out.emplace_back();
      cur = &out.back();
      cur->seq = h_seq.empty() ? j : h_seq[j];
      cur->order = qi; cur->kind = 0; cur->target = qi;
      curj = j;
    }
    OutEvent e;
    e.ts = hts[j];
    for (int c = 0; c < nout; c++) {
      if (fp.plain_proj) {
        Ty t = app->streams[st].types[fp.pcol[c]];
        int64_t v;
        if (tsize(t) == 8) v = ((const int64_t*)pc[c].data())[r];
        else {
          int32_t x = ((const int32_t*)pc[c].data())[r];
          v = (t == T_FLOAT) ? (int64_t)(uint32_t)x : (int64_t)x;
        }
        e.raw.push_back(v);
        e.nul.push_back(0);
      } else {
        e.raw.push_back(raw[r * nout + c]);
        e.nul.push_back(nul[r * nout + c]);
      }
    }
    cur->ts = e.ts;
    cur->ev.push_back(std::move(e));
  }
}

std::unique_ptr<Exec> make_keyed_followed_by(App& app, int qi, const J& q, std::string& why) {
  const J& in = q["input"];
  if (in["kind"].s != "state") { why = "not a state query"; return nullptr; }
  if (in["type"].s != "PATTERN") { why = "sequence"; return nullptr; }
  if (!q.has("partition")) { why = "not partitioned"; return nullptr; }
  const J& el = in["element"];
  if (el["k"].s != "next" || el["a"]["k"].s != "every" || el["a"]["e"]["k"].s != "stream" || el["b"]["k"].s != "stream") {
    why = "not `every e1 -> e2`";
    return nullptr;
  }
  const J& e1 = el["a"]["e"];
  const J& e2 = el["b"];
  if (e1["stream"].s != e2["stream"].s) { why = "two streams"; return nullptr; }
  if (e1["slot"].as_int() != 0 || e2["slot"].as_int() != 1) { why = "slot layout"; return nullptr; }
  const J& part = q["partition"];
  if (part.o.size() != 1 || !part.has(e1["stream"].s)) { why = "partition does not key the pattern stream"; return nullptr; }
  {
    // @purge: with event-time clocks (playback) and idle.period >= within, every partial a purge would
    // clean has expired by the key's next event anyway, so the purge is invisible here
    std::string pw;
    const PurgeClock* pc = purge_of(app, q, pw);
    if (!pw.empty()) { why = pw; return nullptr; }
    if (pc && !(app.playback && !in["within"].null() && pc->idle >= in["within"].as_int())) {
      why = "@purge that can clean live partials (not playback, or idle.period < within)";
      return nullptr;
    }
  }
  const J& s = q["select"];
  if (s["group_by"].size() || !s["having"].null() || s["order_by"].size() || !s["limit"].null() || !s["offset"].null()) {
    why = "selector features";
    return nullptr;
  }
  if (q["output"]["events"].s != "current" && !q["output"]["events"].s.empty()) { why = "expired events output"; return nullptr; }
  std::function<bool(const J&)> has_agg = [&](const J& e) -> bool {
    if (e["op"].s == "agg" || e["op"].s == "multivar") return true;
    for (const char* c : {"a", "b"}) if (e.has(c) && has_agg(e[c])) return true;
    return false;
  };
  for (size_t k = 0; k < s["attrs"].size(); k++)
    if (has_agg(s["attrs"][k]["e"])) { why = "aggregator in select"; return nullptr; }
  auto ex = std::make_unique<KeyedFollowedByExec>();
  ex->app = &app; ex->qi = qi; ex->path = 4;
  ex->st = app.stream_idx.at(e1["stream"].s);
  const auto& types = app.streams[ex->st].types;
  if (types.size() > KF_MAXC) { why = "too many attributes"; return nullptr; }
  ex->kcol = (int)part[e1["stream"].s].as_int();
  ex->kty = types[ex->kcol];
  if (ex->kty != T_STRING && ex->kty != T_INT && ex->kty != T_LONG && ex->kty != T_BOOL) {
    why = "partition key of a floating-point attribute";
    return nullptr;
  }
  ex->within = in["within"].null() ? -1 : in["within"].as_int();
  auto intern = [&](const std::string& str) { return app.intern(str); };
  auto sm = [&](int slot, int chain) -> int {
    if (slot != 0 && slot != 1) return -1;
    if (chain != -1 && chain != 0) return -1;
    return slot;
  };
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
  ex->fp = recognise(app, ex->st, ex->st, e1, e2, s);
  for (Ty t : types) { ex->cols.emplace_back(); ex->cols.back().w = tsize(t); }
  ex->in_streams = {ex->st};
  return ex;
}

}  // namespace sg
