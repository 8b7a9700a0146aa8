// runtime.hpp — host runtime behind the C ABI (include/siddhi_gfx.h).
//
// One sg_app mirrors one SiddhiAppRuntime (CORE/SiddhiAppRuntimeImpl.java) restricted to the
// hot-path queries.  Each query is lowered to one Exec (an execution path with its own HIP
// kernels).  Input arrives as columnar batches (the JNI shim's pinned SoA buffers); outputs are
// materialised as the callback sequence the reference would fire.
#pragma once
#include <hip/hip_runtime.h>

#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/siddhi_gfx.h"
#include "compile.hpp"
#include "json.hpp"

namespace sg {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define SG_HIP(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) throw ::sg::Error(-3, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

inline int tsize(Ty t) { return (t == T_LONG || t == T_DOUBLE) ? 8 : 4; }

// A growable device buffer.
// Host vector whose resize() leaves new elements uninitialised (default-init): per-event bookkeeping arrays
// of 10^7 elements are written right after they grow, and value-initialising them first doubles the cost.
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U> struct rebind { using other = NoInitAlloc<U>; };
  NoInitAlloc() = default;
  template <class U> NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
  template <class U> void construct(U* p) noexcept { ::new ((void*)p) U; }
  template <class U, class... Args> void construct(U* p, Args&&... args) { ::new ((void*)p) U(std::forward<Args>(args)...); }
};
template <class T> using hvec = std::vector<T, NoInitAlloc<T>>;
// ... in pinned host memory (host arrays the queries upload whole every flush: copies at full PCIe rate)
template <class T>
struct PinAlloc : NoInitAlloc<T> {
  template <class U> struct rebind { using other = PinAlloc<U>; };
  PinAlloc() = default;
  template <class U> PinAlloc(const PinAlloc<U>&) noexcept {}
  T* allocate(size_t n) {
    void* p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(n, 1) * sizeof(T), hipHostMallocDefault) != hipSuccess) throw std::bad_alloc();
    return (T*)p;
  }
  void deallocate(T* p, size_t) noexcept { (void)hipHostFree(p); }
};
template <class T> using pvec = std::vector<T, PinAlloc<T>>;

// Pinned host staging buffer (grow-only): device-to-host copies at full PCIe rate
template <class T>
struct PinBuf {
  T* p = nullptr;
  size_t cap = 0;
  void reserve(size_t n) {
    if (n <= cap) return;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    SG_HIP(hipHostMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T), hipHostMallocDefault));
    cap = n;
  }
  PinBuf() = default;
  PinBuf(const PinBuf&) = delete;
  PinBuf& operator=(const PinBuf&) = delete;
  ~PinBuf() { if (p) (void)hipHostFree(p); }
};

// Process-wide pool of page-locked host blocks.  Output columns are copied into these from the device at full
// PCIe rate and without first-touch page faults; a block returns to the pool when its column is freed
// (sg_out_clear), so a streaming runtime pins its output memory once.  At most 4 GiB stay pooled.
struct PinnedPool {
  static std::mutex& mu() { static std::mutex m; return m; }
  static std::multimap<size_t, void*>& free_blocks() { static std::multimap<size_t, void*> f; return f; }
  static size_t& pooled() { static size_t b = 0; return b; }
  static void* get(size_t bytes, size_t& cap) {
    {
      std::lock_guard<std::mutex> g(mu());
      auto& f = free_blocks();
      auto it = f.lower_bound(bytes);
      if (it != f.end() && it->first <= 2 * bytes + (64u << 20)) {   // reuse unless far larger than needed
        cap = it->first;
        void* p = it->second;
        f.erase(it);
        pooled() -= cap;
        return p;
      }
    }
    cap = (std::max<size_t>(bytes, 1) + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
    void* p = nullptr;
    SG_HIP(hipHostMalloc(&p, cap, hipHostMallocDefault));
    return p;
  }
  static void put(void* p, size_t cap) {
    std::lock_guard<std::mutex> g(mu());
    auto& f = free_blocks();
    f.emplace(cap, p);
    pooled() += cap;
    while (pooled() > ((size_t)4 << 30) && !f.empty()) {   // drop the largest blocks first
      auto last = std::prev(f.end());
      pooled() -= last->first;
      (void)hipHostFree(last->second);
      f.erase(last);
    }
  }
};

// A host column in pooled pinned memory (uninitialised on resize; the device fills it).
template <class T>
struct HostCol {
  T* p = nullptr;
  size_t n = 0, cap = 0;   // cap in bytes
  HostCol() = default;
  HostCol(const HostCol&) = delete;
  HostCol& operator=(const HostCol&) = delete;
  ~HostCol() { if (p) PinnedPool::put(p, cap); }
  void resize(size_t m) {
    if (m * sizeof(T) > cap) {
      if (p) PinnedPool::put(p, cap);
      p = nullptr;
      p = (T*)PinnedPool::get(m * sizeof(T), cap);
    }
    n = m;
  }
  size_t size() const { return n; }
  T* data() { return p; }
  const T* data() const { return p; }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
};

// f(x0, x1) over [0, n) in contiguous ranges on up to 8 host threads (one when n is small)
template <class F>
inline void par_rows(int64_t n, F&& f) {
  const int64_t grain = 1 << 18;
  const int nt = (int)std::min<int64_t>(8, std::max<int64_t>(1, n / grain));
  if (nt <= 1) { if (n > 0) f((int64_t)0, n); return; }
  std::vector<std::thread> th;
  for (int t = 1; t < nt; t++) th.emplace_back([&, t] { f(n * t / nt, n * (t + 1) / nt); });
  f((int64_t)0, n / nt);
  for (auto& x : th) x.join();
}

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t cap = 0;
  DBuf() = default;
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  DBuf(DBuf&& o) noexcept : p(o.p), cap(o.cap) { o.p = nullptr; o.cap = 0; }
  DBuf& operator=(DBuf&& o) noexcept {
    if (this != &o) { if (p) (void)hipFree(p); p = o.p; cap = o.cap; o.p = nullptr; o.cap = 0; }
    return *this;
  }
  ~DBuf() { if (p) (void)hipFree(p); }
  void reserve(size_t n, bool keep = true, hipStream_t s = nullptr, size_t used = 0) {
    if (n <= cap) return;
    size_t nc = cap ? cap : 1024;
    while (nc < n) nc *= 2;
    T* q = nullptr;
    SG_HIP(hipMalloc(&q, nc * sizeof(T)));
    if (p) {
      if (keep && used) SG_HIP(hipMemcpyAsync(q, p, used * sizeof(T), hipMemcpyDeviceToDevice, s));
      SG_HIP(hipStreamSynchronize(s));
      SG_HIP(hipFree(p));
    }
    p = q;
    cap = nc;
  }
};

// Untyped device column (4 or 8 bytes per value).
struct DCol {
  DBuf<uint8_t> b;
  int w = 4;
  void* data() const { return b.p; }
};

// Buffer compaction (flushed events no longer referenced): row k of the compacted buffer is row idx[k]
// of the old one (idx ascending).  Gathered into a scratch buffer and copied back, as rows may move
// onto rows other threads still read.
template <class T>
__global__ void __launch_bounds__(256) k_gather_rows(const T* __restrict__ src, const int64_t* __restrict__ idx,
                                                     int64_t m, T* __restrict__ dst) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k < m) dst[k] = src[idx[k]];
}
template <class T>
inline void compact_rows(T* buf, const int64_t* d_idx, int64_t m, DBuf<uint8_t>& tmp, hipStream_t s) {
  if (m <= 0) return;
  tmp.reserve((size_t)m * sizeof(T), false);
  hipLaunchKernelGGL(k_gather_rows<T>, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, buf, d_idx, m, (T*)tmp.p);
  SG_HIP(hipGetLastError());
  SG_HIP(hipMemcpyAsync(buf, tmp.p, (size_t)m * sizeof(T), hipMemcpyDeviceToDevice, s));
}
// a column of w-byte values (w = 1, 4 or 8)
inline void compact_col(uint8_t* buf, int w, const int64_t* d_idx, int64_t m, DBuf<uint8_t>& tmp, hipStream_t s) {
  if (w == 8) compact_rows((uint64_t*)buf, d_idx, m, tmp, s);
  else if (w == 4) compact_rows((uint32_t*)buf, d_idx, m, tmp, s);
  else compact_rows(buf, d_idx, m, tmp, s);
}
// Device-resident input is adopted unchecked: its timestamps must be non-decreasing, as sg_push enforces
// for host batches (relative-timestamp encodings and window halos rely on it).  One pass, for the paths
// whose kernels do not check it while they stage the events.
template <class T>
__global__ void __launch_bounds__(256) k_ts_order(const T* __restrict__ ts, int64_t n, uint32_t* bad) {
  bool b = false;
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x + 1; k < n; k += (int64_t)gridDim.x * 256)
    b |= ts[k] < ts[k - 1];
  if (__any(b) && (threadIdx.x & 63) == 0) atomicOr(bad, 1u);
}
inline void check_ts_order(const int64_t* ts, int64_t n, DBuf<uint32_t>& flag, hipStream_t s, const char* path) {
  if (n < 2) return;
  flag.reserve(1);
  SG_HIP(hipMemsetAsync(flag.p, 0, 4, s));
  hipLaunchKernelGGL(k_ts_order<int64_t>, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0, s, ts, n,
                     flag.p);
  SG_HIP(hipGetLastError());
  uint32_t h = 0;
  SG_HIP(hipMemcpyAsync(&h, flag.p, 4, hipMemcpyDeviceToHost, s));
  SG_HIP(hipStreamSynchronize(s));
  if (h) throw Error(-1, std::string(path) + ": event timestamps go backwards (device-resident input must be "
                                             "non-decreasing, as sg_push enforces for host batches)");
}

template <class T>
inline std::vector<T> gather_host(const std::vector<T>& v, const std::vector<int64_t>& idx) {
  std::vector<T> o(idx.size());
  for (size_t k = 0; k < idx.size(); k++) o[k] = v[(size_t)idx[k]];
  return o;
}

// A short vector with inline storage: the projection of one output row (a few attributes) without a heap
// allocation per row.  The subset of std::vector the output path uses.
template <class T, int N>
class SVec {
 public:
  SVec() = default;
  SVec(const SVec& o) { assign(o.data(), o.data() + o.n_); }
  SVec(SVec&& o) noexcept { take(std::move(o)); }
  SVec& operator=(const SVec& o) { if (this != &o) assign(o.data(), o.data() + o.n_); return *this; }
  SVec& operator=(SVec&& o) noexcept { if (this != &o) take(std::move(o)); return *this; }
  SVec& operator=(const std::vector<T>& v) { assign(v.begin(), v.end()); return *this; }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  T* data() { return heap_.empty() ? inl_ : heap_.data(); }
  const T* data() const { return heap_.empty() ? inl_ : heap_.data(); }
  T& operator[](size_t i) { return data()[i]; }
  const T& operator[](size_t i) const { return data()[i]; }
  T* begin() { return data(); }
  T* end() { return data() + n_; }
  const T* begin() const { return data(); }
  const T* end() const { return data() + n_; }
  void clear() { n_ = 0; heap_.clear(); }
  void push_back(const T& v) {
    if (heap_.empty() && n_ < (size_t)N) { inl_[n_++] = v; return; }
    if (heap_.empty()) heap_.assign(inl_, inl_ + n_);
    heap_.push_back(v);
    n_++;
  }
  template <class It>
  void assign(It b, It e) {
    clear();
    for (; b != e; ++b) push_back(*b);
  }

 private:
  void take(SVec&& o) {
    n_ = o.n_;
    heap_ = std::move(o.heap_);
    if (heap_.empty()) for (size_t i = 0; i < n_; i++) inl_[i] = o.inl_[i];
    o.n_ = 0;
    o.heap_.clear();
  }
  T inl_[N];
  std::vector<T> heap_;   // used once the row outgrows N (then it holds every element)
  size_t n_ = 0;
};

struct OutEvent {
  int64_t ts;
  bool expired = false;
  SVec<int64_t, 4> raw;
  SVec<uint8_t, 8> nul;
};

// Columnar output of many callbacks of one query (a path that forms its callbacks on the device): per callback its
// arrival seq, timestamp and first row; per row its timestamp and `width` raw slots.  Every row is a CURRENT event
// without nulls.  One bulk Callback entry stands for all of them (no per-event objects on the host).
struct OutBlock {
  int32_t width = 0;
  HostCol<int64_t> cb_seq, cb_ts, cb_row;   // cb_row has one entry more: the row count
  HostCol<int64_t> ts, raw;                 // raw: [row][width]; all pinned, filled by D2H copies
  int64_t ncb() const { return (int64_t)cb_seq.size(); }
};

struct Callback {
  int64_t seq;   // arrival sequence of the event that fired it (for cross-query ordering)
  const OutBlock* blk = nullptr;   // a bulk entry: all callbacks of blk (App::blocks owns it); `ev` unused
  // a Scheduler tick fired it (absent states): its scheduler and the deadline it fired under -- the key that
  // orders the same tick's callbacks of different partition keys (multi-GPU merge); -1 for a send's own
  int32_t tsched = -1;
  int64_t tdl = 0;
  int order;     // query index (subscription order)
  int kind;      // 0 query callback, 1 stream callback
  int target;
  int64_t ts;
  std::vector<OutEvent> ev;   // selector output chunk, in chunk order (expired flag per event)
};

// Selector output of a query feeding other device queries, as columns (one row per output event, in
// callback order): what InsertIntoStreamCallback publishes, without per-event Callback objects.
struct ChainOut {
  hvec<int64_t> ts, seq;                   // event ts, arrival seq of the send that fired its chunk
  std::vector<hvec<int64_t>> raw;          // [attr][row] 8-byte slots (as OutEvent::raw)
  std::vector<int64_t> chunk_end;          // exclusive row ends of the selector output chunks
  bool singles = false;                    // every row is its own chunk (chunk_end left empty: 1, 2, ...)
  bool nulls = false;                      // some attribute was null
  size_t nchunks() const { return singles ? ts.size() : chunk_end.size(); }
  int64_t chunk_end_at(size_t c) const { return singles ? (int64_t)c + 1 : chunk_end[c]; }
};

// A chained export left in HBM (a window query's output feeding NFA queries: config 5): device columns in the
// inserted stream's widths, each row's app clock, and on the host only what the consumers' bookkeeping reads -- the
// rows' arrival seqs and the consumers' partition attribute.  Valid until the exporting query's next flush.
struct DevChain {
  bool done = false;                    // the exporter filled it (else the host ChainOut path runs)
  int key_attr = -1;                    // the attribute the consumers partition by (-1: none)
  std::vector<int> widths;              // bytes per attribute of the inserted stream
  int64_t n = 0;
  const int64_t* d_ts = nullptr;
  const int64_t* d_now = nullptr;
  std::vector<const void*> d_cols;
  const int64_t* seq = nullptr;         // host: arrival seq of the send that fired each row
  const uint8_t* key = nullptr;         // host (pinned): the key attribute's column (widths[key_attr] bytes per row)
};

struct StreamDef {
  std::string name;
  std::vector<Ty> types;
};

struct App;
struct SnapWriter;
struct SnapReader;

// Read-only view of a host array: the caller's buffer for the duration of one push, or storage the
// batch owns (converted columns, chained exports).
template <class T>
struct HSpan {
  const T* p = nullptr;
  size_t n = 0;
  HSpan() = default;
  HSpan(const T* q, size_t m) : p(q), n(m) {}
  template <class A>
  explicit HSpan(const std::vector<T, A>& v) : p(v.data()), n(v.size()) {}
  const T* data() const { return p; }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  const T& operator[](size_t k) const { return p[k]; }
  const T* begin() const { return p; }
  const T* end() const { return p + n; }
};

// Host-side staging of one pushed batch (already split per stream, arrival-ordered).  The arrays are
// views: sg_push points them at the caller's buffers (valid for the call) instead of copying them, so
// a large push costs no allocation or first-touch page faults on the host.
// The Scheduler ticks of one push (TimestampGeneratorImpl listeners), gathered before they are handed to the
// queries: the clock each tick moved to, the arrival seq at that point and the position of the event it precedes.
struct TickBuf {
  hvec<int64_t> now, seq, k;
  void clear() { now.clear(); seq.clear(); k.clear(); }
  void add(int64_t t, int64_t sq, int64_t pos) { now.push_back(t); seq.push_back(sq); k.push_back(pos); }
};

struct HostBatch {
  int stream;
  int64_t n;
  int64_t seq0;                       // global arrival sequence of the first event
  HSpan<int64_t> seqs;                // per-event arrival sequence (chained inputs), else seq0 + k
  HSpan<int64_t> ts;
  std::vector<HSpan<uint8_t>> cols;   // raw column bytes
  bool batch;                         // one send(Event[]) chunk
  int64_t now;                        // wall clock at push
  HSpan<int64_t> now_ev;              // app clock each event is processed at (TimestampGenerator.currentTime)
  bool now_uniform = false;           // every now_ev equals `now` (one batch send under one clock)
  HSpan<uint8_t> nulls;               // n * arity null flags, row-major (empty: no null in the batch)
  // the batch already in HBM (sg_push uploads a stream's batch once when several queries take it to the device;
  // they copy device to device, the host views above stay valid): ts, per-event clock (null when now_uniform),
  // columns (empty: not staged)
  const int64_t* d_ts = nullptr;
  const int64_t* d_now = nullptr;
  std::vector<const uint8_t*> d_cols;
  // storage behind views that do not point at the caller's buffers
  hvec<int64_t> own_seqs, own_ts, own_now;   // (no zero fill on resize: every slot is written)
  std::vector<hvec<uint8_t>> own_cols;
};

struct Exec {
  App* app = nullptr;
  int qi = 0;
  std::string name;
  int path = 0;
  std::vector<int> in_streams;
  virtual ~Exec() = default;
  virtual void push(const HostBatch& b) = 0;
  virtual void push_device(int stream, int64_t n, const int64_t* d_ts, const void* const* d_cols, int batch,
                           hipStream_t s) {
    (void)stream; (void)n; (void)d_ts; (void)d_cols; (void)batch; (void)s;
    throw Error(-2, "device-resident ingest is not implemented for this path");
  }
  // device-resident global arrival seq of the events of the last push_device (multi-GPU ranks)
  virtual void set_device_seq(const int64_t* d_seq) {
    (void)d_seq;
    throw Error(-2, "device arrival sequence numbers are only lowered for the keyed followed-by path");
  }
  // run kernels; append callbacks to out (if materialise)
  virtual void flush(std::vector<Callback>& out, bool materialise, hipStream_t s) = 0;
  virtual void advance_time(int64_t now) { (void)now; }
  // multi-GPU halo: the last n_halo events pushed to `stream` are the next range's leading
  // events -- they complete partials of this range but start none
  virtual void set_halo(int stream, int64_t n_halo) {
    (void)stream; (void)n_halo;
    throw Error(-2, "halo events are only lowered for the unkeyed followed-by path");
  }
  // Scheduler ticks (TimestampGeneratorImpl listeners): the app clock moved to `now` before the k-th event
  // of a push to `stream` (-1: a sleep / advance_time) was dispatched; `seq` = arrival seq at that point
  virtual void on_tick(int64_t now, int64_t seq, int stream, int64_t k) { (void)now; (void)seq; (void)stream; (void)k; }
  // every tick of one push at once (clock, seq and event position per tick, in push order): one call per
  // query and push instead of one per tick (a per-event playback push of 10M sends is 10M ticks).  A query that
  // keeps ticks overrides both; the rest ignore them without a call per tick
  virtual void on_ticks(const TickBuf& t, int stream) { (void)t; (void)stream; }
  virtual void start(int64_t now) { (void)now; }
  // null attribute values reach the bytecode loaders (null -> compare false, null projections)
  virtual bool supports_nulls() const { return false; }
  // sg_snapshot / sg_restore of this query's state (after a flush); default: not implemented
  virtual bool can_snapshot() const { return false; }
  virtual void snapshot(SnapWriter& w, hipStream_t s) { (void)w; (void)s; }
  virtual void restore(SnapReader& r, hipStream_t s) { (void)r; (void)s; }
  virtual void reset() = 0;
  // true when selector chunk boundaries of the input matter (window selectors batch per chunk): a
  // chained input is then pushed one upstream output chunk at a time
  virtual bool chunk_sensitive() const { return true; }
  // push() copies the batch's columns to the device (HostBatch::d_* staging pays off when two such queries share it)
  virtual bool takes_device_batch() const { return false; }
  // run the kernels and hand the selector output over as columns (chained queries with no callback
  // of their own); false: the path has no column export, use flush + Callbacks
  virtual bool flush_export(ChainOut& co, hipStream_t s) { (void)co; (void)s; return false; }
  // device-resident chaining (DevChain): the exporter may leave its next export in HBM; a consumer reports the
  // attribute it partitions by (-1 none; -2 cannot take a device chain) and adopts the chain
  virtual void set_chain_request(DevChain* dc) { (void)dc; }
  virtual int chain_key_attr(int stream) const { (void)stream; return -2; }
  virtual void push_device_chain(int stream, const DevChain& dc, int64_t now, hipStream_t s) {
    (void)stream; (void)dc; (void)now; (void)s;
  }
  // events this query still holds in its buffers (-1: not tracked); bounded by its open state once
  // flushed buffers are compacted
  virtual int64_t buffered() const { return -1; }
  // the query's run-time compiled kernel (SG_PATH_NFA, nfa_rtc.hpp): its generated source, and compiling it into
  // the code-object cache (no GPU needed); false for a path without one
  virtual bool kernel_source(std::string& out) { (void)out; return false; }
  virtual bool compile_kernel(double& ms, bool& from_disk, std::string& err) { (void)ms; (void)from_disk; (void)err; return false; }
  // cross-rank Scheduler collisions (sg_query_shard_mode and friends); false: not a partitioned query
  // with absent states
  virtual bool shard_mode(int mode) { (void)mode; return false; }
  virtual int64_t sched_fires(sg_sched_fire* out, int64_t cap) const { (void)out; (void)cap; return -1; }
  // sg_query_state_json: the pattern state in StreamPreState.snapshot's shape (false: not a pattern path)
  virtual bool state_json(std::string& out, hipStream_t s) { (void)out; (void)s; return false; }
  virtual int64_t sched_ops(sg_sched_op* out, int64_t cap) const { (void)out; (void)cap; return -1; }
  virtual bool sched_defer(int64_t key, int32_t tick, int sched) { (void)key; (void)tick; (void)sched; return false; }
  // streaming shard mode (sg_query_shard_resolver): the driver answers the Scheduler-map questions
  virtual bool shard_resolver(sg_shard_resolver_fn fn, void* user) { (void)fn; (void)user; return false; }
  virtual int64_t sched_clock(int64_t* now, int64_t cap, int64_t* min_wait) const {
    (void)now; (void)cap; (void)min_wait;
    return -1;
  }
  int64_t last_matches = 0;
  std::map<std::string, double> kernel_ms;
};

// @purge of one partition block (PartitionRuntimeImpl.java:79-81, 120-147, 346-402).  Every
// initPartition call (one per key chunk sent into the partition) schedules a purge task at its time
// + k*interval (k >= 1); a task at time c cleans every key with lastSeen + idle < c, so the key's next
// chunk re-initialises its query states.  Restated on the app clock (the reference runs the tasks on the
// wall clock).  The execs apply a purge where it is observable -- the key's next chunk, its timers --
// via task_in(lastSeen + idle, T): does a task fire in (lastSeen + idle, T]?  Calls only ever add
// residues whose first task lies after the call, so the answer for a past T does not change later.
struct PurgeClock {
  int64_t interval = 300000, idle = 0;
  std::map<int64_t, int64_t> first;   // task-time residue mod interval -> earliest call with it
  int64_t t0 = INT64_MAX;             // earliest call
  static int64_t mod(int64_t a, int64_t m) { const int64_t r = a % m; return r < 0 ? r + m : r; }
  void note(int64_t t) {
    auto it = first.find(mod(t, interval));
    if (it == first.end()) first[mod(t, interval)] = t;
    else if (t < it->second) it->second = t;
    if (t < t0) t0 = t;
  }
  bool task_in(int64_t A, int64_t T) const {
    if (T <= A || first.empty() || T < t0 + interval) return false;
    if (T - A >= interval) return true;      // the earliest call's tasks fire in every such span
    const int64_t ra = mod(A + 1, interval), rb = mod(T, interval);
    auto hit = [&](const std::pair<const int64_t, int64_t>& f) {
      const int64_t c = A + 1 + mod(f.first - (A + 1), interval);   // the task time == residue in (A, T]
      return c <= T && c >= f.second + interval;
    };
    if (ra <= rb) {
      for (auto it = first.lower_bound(ra); it != first.end() && it->first <= rb; ++it) if (hit(*it)) return true;
    } else {
      for (auto it = first.lower_bound(ra); it != first.end(); ++it) if (hit(*it)) return true;
      for (auto it = first.begin(); it != first.end() && it->first <= rb; ++it) if (hit(*it)) return true;
    }
    return false;
  }
};

using PurgeFirst = std::vector<std::pair<int64_t, int64_t>>;   // PurgeClock::first, serialised

struct App {
  J desc;
  bool playback = false;
  int device = 0;
  std::map<int, PurgeClock> purges;                 // partition block -> its @purge task schedule
  DBuf<int64_t> stage_ts, stage_now;                // a pushed batch staged once in HBM (HostBatch::d_*)
  std::map<int, DBuf<uint8_t>> stage_cols;
  PinBuf<int64_t> push_now;                         // sg_push: app clock per event of the current push (pinned: the
                                                    // queries copy it to the device)
  TickBuf push_ticks;                               // sg_push / sg_push_shard: the push's Scheduler ticks
  // large host vectors of chained exports, recycled from one flush to the next (pages stay mapped)
  std::vector<hvec<int64_t>> vpool;           // (hvec: a resize does not zero-fill 10M-row columns)
  hvec<int64_t> take64() {
    if (vpool.empty()) return {};
    hvec<int64_t> v = std::move(vpool.back());
    vpool.pop_back();
    v.clear();
    return v;
  }
  void give64(hvec<int64_t>&& v) {
    if (v.capacity() >= ((size_t)1 << 20) && vpool.size() < 16) vpool.push_back(std::move(v));
  }
  // the same for byte vectors (converted 4-byte columns of chained pushes)
  std::vector<hvec<uint8_t>> bpool;
  hvec<uint8_t> take8() {
    if (bpool.empty()) return {};
    hvec<uint8_t> v = std::move(bpool.back());
    bpool.pop_back();
    v.clear();
    return v;
  }
  void give8(hvec<uint8_t>&& v) {
    if (v.capacity() >= ((size_t)1 << 20) && bpool.size() < 16) bpool.push_back(std::move(v));
  }
  std::vector<StreamDef> streams;
  std::map<std::string, int> stream_idx;
  std::vector<std::string> strings;
  std::unordered_map<std::string, int> string_ids;
  std::vector<std::unique_ptr<Exec>> execs;        // one per query
  std::vector<std::string> qnames;
  std::vector<std::vector<Ty>> qout_types;
  std::vector<int> qout_stream;                     // insert-into target (or -1)
  std::vector<bool> feeds;                          // query's output stream is consumed by device queries
  std::vector<Callback> early;                      // callbacks of upstream queries run at push time
  std::vector<bool> query_cb, stream_cb;
  std::vector<std::vector<int>> subscribers;       // stream -> queries
  std::vector<Callback> out;
  std::vector<Callback> cb_spare;                   // an emptied callback vector kept for its capacity (flush_impl)
  std::vector<std::unique_ptr<OutBlock>> blocks;    // columnar outputs the bulk entries of `out` / `early` reference
  int64_t seq = 0;
  int64_t now = 0;
  int64_t last_event_ts = INT64_MIN;                // playback: TimestampGeneratorImpl.lastEventTimestamp
  bool started = false;
  hipStream_t stream = nullptr;

  int intern(const std::string& s) {
    auto it = string_ids.find(s);
    if (it != string_ids.end()) return it->second;
    int id = (int)strings.size();
    strings.push_back(s);
    string_ids[s] = id;
    return id;
  }
};

// Inclusive scan of a u32 across the 64 lanes of a wave with DPP (gfx9 row shifts and row broadcasts): six adds
// of register-to-register moves, where __shfl_up's ds_bpermute costs an LDS round trip per step.
__device__ __forceinline__ uint32_t sg_wave_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);   // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);   // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);   // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);   // row_shr:8 (rows of 16 done)
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// run fn(t) for t in [0, nth) on host threads (O(events) bookkeeping of large flushes)
// Persistent host worker threads for host_parallel (a flush makes a few dozen thread-range passes; spawning and
// joining 15 threads for each costs milliseconds).  One caller at a time; a nested or concurrent call spawns its
// own threads.  A forked child gets a fresh pool (the parent's workers do not exist there).
struct HostPool {
  std::mutex m, busy;
  std::condition_variable cv, done;
  std::vector<std::thread> th;
  std::function<void(int)>* job = nullptr;
  int njob = 0, pending = 0;
  uint64_t gen = 0;
  static bool& in_worker() { static thread_local bool w = false; return w; }
  static HostPool& get() {
    static HostPool* p = nullptr;
    static pid_t owner = 0;
    static std::mutex gm;
    std::lock_guard<std::mutex> l(gm);
    if (!p || owner != getpid()) { p = new HostPool; owner = getpid(); }   // (never freed: workers outlive exit)
    return *p;
  }
  void worker(int id) {
    in_worker() = true;
    uint64_t seen = 0;
    for (;;) {
      std::function<void(int)>* f = nullptr;
      {
        std::unique_lock<std::mutex> l(m);
        cv.wait(l, [&] { return gen != seen; });
        seen = gen;
        if (id >= njob) continue;
        f = job;
      }
      (*f)(id);
      std::lock_guard<std::mutex> l(m);
      if (--pending == 0) done.notify_one();
    }
  }
  void run(int nth, std::function<void(int)>& fn) {
    while ((int)th.size() < nth - 1) {
      const int id = (int)th.size() + 1;
      th.emplace_back([this, id] { worker(id); });
      th.back().detach();
    }
    {
      std::lock_guard<std::mutex> l(m);
      job = &fn; njob = nth; pending = nth - 1; gen++;
    }
    cv.notify_all();
    fn(0);
    std::unique_lock<std::mutex> l(m);
    done.wait(l, [&] { return pending == 0; });
    job = nullptr;
  }
};

template <class F>
inline void host_parallel(int nth, F&& fn) {
  if (nth <= 1) { fn(0); return; }
  HostPool& pool = HostPool::get();
  if (HostPool::in_worker() || !pool.busy.try_lock()) {   // nested, or another thread holds the pool: own threads
    std::vector<std::thread> th;
    for (int t = 1; t < nth; t++) th.emplace_back(fn, t);
    fn(0);
    for (auto& x : th) x.join();
    return;
  }
  std::function<void(int)> job(std::ref(fn));
  pool.run(nth, job);
  pool.busy.unlock();
}
// std::sort over thread ranges: each range sorted on its own, then pairwise merges (the pairs of a round in
// parallel).  cmp must be a strict total order (ties broken by the caller) for a deterministic result.
template <class T, class C>
inline void par_sort(std::vector<T>& v, C cmp, int nth) {
  const int64_t n = (int64_t)v.size();
  if (nth <= 1 || n < 4096) { std::sort(v.begin(), v.end(), cmp); return; }
  std::vector<int64_t> b(nth + 1);
  for (int t = 0; t <= nth; t++) b[t] = n * t / nth;
  host_parallel(nth, [&](int t) { std::sort(v.begin() + b[t], v.begin() + b[t + 1], cmp); });
  std::vector<T> tmp(v.size());
  while (b.size() > 2) {
    const int np = (int)(b.size() - 1) / 2;
    std::vector<int64_t> nb(1, 0);
    for (int q = 0; q < np; q++) nb.push_back(b[2 * q + 2]);
    if ((b.size() - 1) % 2) nb.push_back(b.back());
    host_parallel((int)(b.size() - 1 + 1) / 2, [&](int q) {
      if (2 * q + 2 < (int)b.size())
        std::merge(v.begin() + b[2 * q], v.begin() + b[2 * q + 1], v.begin() + b[2 * q + 1], v.begin() + b[2 * q + 2],
                   tmp.begin() + b[2 * q], cmp);
      else
        std::copy(v.begin() + b[2 * q], v.begin() + b[2 * q + 1], tmp.begin() + b[2 * q]);
    });
    v.swap(tmp);
    b.swap(nb);
  }
}

inline int host_threads(int64_t work) {
  // (SG_HOST_PAR_MIN: a smaller threshold, so that small test inputs take the thread-range paths too)
  const char* e = getenv("SG_HOST_PAR_MIN");
  if (work < (e ? std::max<int64_t>(2, atoll(e)) : (int64_t)1 << 20)) return 1;
  return (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
}

// host-side phase timing (SG_HOST_TIMING=1): prints the milliseconds since the previous mark
struct PhaseClock {
  bool on;
  std::chrono::steady_clock::time_point t;
  explicit PhaseClock(bool enabled) : on(enabled), t(std::chrono::steady_clock::now()) {}
  void mark(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    fprintf(stderr, "[sg phase] %s %.1f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};

// HashMap/HashSet position hash of a partition key: String.hashCode of the key value's toString,
// spread (h ^ h >>> 16) as HashMap.hash does (PartitionRuntimeImpl keys instances by that string)
inline int32_t java_key_hash(const App& app, Ty t, int64_t v) {
  std::string ks;
  switch (t) {
    case T_STRING: ks = app.strings.at((size_t)v); break;
    case T_INT: case T_LONG: ks = std::to_string(v); break;
    case T_BOOL: ks = v ? "true" : "false"; break;
    default: throw Error(-2, "float partition keys in an order-dependent partition structure are not lowered");
  }
  uint32_t h = 0;
  for (unsigned char ch : ks) h = 31u * h + ch;
  return (int32_t)(h ^ (h >> 16));
}

// @purge of a partitioned query: its partition's task schedule, or null.  Execs support it only when the
// query reads every stream its partition keys (then its own chunks are all of the key's initPartition
// calls); `why` says otherwise.
inline PurgeClock* purge_of(App& app, const J& q, std::string& why) {
  if (!q.has("purge") || !q.has("partition")) return nullptr;
  const int part = q.has("partition_id") ? (int)q["partition_id"].as_int() : -1;
  PurgeClock& pc = app.purges[part];
  pc.interval = q["purge"]["interval"].as_int();
  pc.idle = q["purge"]["idle"].as_int();
  if (pc.interval <= 0) { why = "@purge interval must be positive"; return nullptr; }
  return &pc;
}

// factories (one per execution path)
std::unique_ptr<Exec> make_followed_by(App& app, int qi, const J& q, std::string& why);
std::unique_ptr<Exec> make_keyed_followed_by(App& app, int qi, const J& q, std::string& why);
std::unique_ptr<Exec> make_nfa(App& app, int qi, const J& q, std::string& why);
std::unique_ptr<Exec> make_window_agg(App& app, int qi, const J& q, std::string& why);
std::unique_ptr<Exec> make_window_gen(App& app, int qi, const J& q, std::string& why);

}  // namespace sg
