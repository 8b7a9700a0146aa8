// nfa_rtc.hpp — per-query compiled NFA kernels (hipRTC), host side.
//
// The interpreter (k_nfa_lanes<FM>, nfa_lane.hpp) reads the processor table, the column table and the filter /
// projection bytecode from LDS at every step: each processor dispatch is a chain of LDS loads and each filter a
// loop over bytecode with its register file in LDS.  For a query that runs a large flush this file generates a
// kernel specialised to the query's lowered table (StateInputStreamParser.parse restated by NBuilder):
//   * the table is an empty struct whose static constexpr members mirror NTable, so every `t.p[p].kind`,
//     `t.p[p].nextPre`, `t.within` ... is a compile-time constant and the lane's processor loops unroll into a
//     straight-line body per processor (the same Lane code, partially evaluated by the compiler);
//   * every filter and projection program becomes a generated typed function: one statement per bytecode
//     instruction with its operand types, promotions and null rules fixed (expr.hpp semantics, JLS §5.6.2,
//     CompareConditionExpressionExecutor.execute :38-41), registers as locals -- no dispatch, no LDS register file;
//   * every Lane method is force-inlined into the kernel (SG_LI), so the lane's frame lives in registers.
// The source is compiled with hipRTC for gfx950 (options kRtcOpts) and cached: per process by the hash of the
// generated text, the embedded headers and the options, and on disk (SG_RTC_CACHE, default rtc_cache/ next to the
// library) so that a new process of the same query loads the code object instead of compiling again.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <memory>
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "nfa_lane.hpp"

namespace sg {

// header texts embedded into the library at build time (siddhi_amd/build.py -> _build/rtc_embed.cpp)
extern const int kRtcNHdr;
extern const char* const kRtcHdrNames[];
extern const char* const kRtcHdrSrcs[];

static const char* const kRtcOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-DSG_RTC=1"};

struct RtcKernel {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  double compile_ms = 0;     // hipRTC time of this process (0: loaded from the process or disk cache)
  bool from_disk = false;
  std::string err;           // non-empty: generation or compilation failed (the interpreter runs)
};

inline uint64_t rtc_fnv(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : s) { h ^= c; h *= 1099511628211ull; }
  return h;
}

// ---- source generation ----
struct RtcGen {
  std::ostringstream o;
  // A table array as an empty struct with a switch-valued operator[]: indexed by a constant (the unrolled processor
  // loops) it folds to the value; a device global (what a static constexpr array member becomes in HIP: an
  // externally-initialised __constant__ variable) would be re-loaded instead of folded.
  template <class T>
  void arr(const char* ty, const char* name, const T* v, int n) {
    o << "  struct A_" << name << " { __host__ __device__ __attribute__((always_inline)) constexpr " << ty
      << " operator[](int i) const { switch (i) {";
    for (int k = 0; k < n; k++) o << " case " << k << ": return " << (int64_t)v[k] << ";";
    o << " default: return 0; } } };\n  static constexpr A_" << name << " " << name << "{};\n";
  }
  template <class T>
  void arr2(const char* ty, const char* name, const T (*v)[NP], int n0) {
    o << "  struct A_" << name << " { struct Row { int r; __host__ __device__ __attribute__((always_inline)) constexpr "
      << ty << " operator[](int k) const { switch (r * " << NP << " + k) {";
    for (int i = 0; i < n0; i++)
      for (int k = 0; k < NP; k++) o << " case " << i * NP + k << ": return " << (int)v[i][k] << ";";
    o << " default: return 0; } } }; __host__ __device__ __attribute__((always_inline)) constexpr Row operator[](int r) "
         "const { return Row{r}; } };\n  static constexpr A_" << name << " " << name << "{};\n";
  }
  static std::string lit(int64_t v) {
    char b[40];
    snprintf(b, sizeof b, "(int64_t)0x%016" PRIx64 "ull", (uint64_t)v);
    return b;
  }
  // one bytecode program as a straight-line function (expr.hpp `run`, instruction for instruction)
  void prog(int id, const Prog& p) {
    o << "template <class LD> __device__ __attribute__((always_inline)) bool sg_prog" << id
      << "(const LD& ld, int64_t& res, bool& isnull) {\n";
    o << "  int64_t r[" << MAX_REG << "] = {};\n  bool nl[" << MAX_REG << "] = {};\n  (void)ld; (void)res; (void)isnull;\n";
    for (int pc = 0; pc < p.n; pc++) {
      const Ins& in = p.ins[pc];
      const int d = in.dst, a = in.a, b = in.b;
      o << "  { ";
      switch (in.op) {
        case BC_LD:
          o << "int64_t v_ = 0; const bool ok_ = ld.load(" << a << ", " << in.imm << ", v_); r[" << d << "] = v_; nl[" << d
            << "] = !ok_;";
          break;
        case BC_CONST:
          o << "r[" << d << "] = " << lit(p.consts[in.imm]) << "; nl[" << d << "] = " << (in.b ? "true" : "false") << ";";
          break;
        case BC_NULL:
          o << "r[" << d << "] = 0; nl[" << d << "] = true;";
          break;
        case BC_CVT:
          o << "r[" << d << "] = cvt(r[" << a << "], " << ((in.imm >> 4) & 15) << ", " << (in.imm & 15) << "); nl[" << d
            << "] = nl[" << a << "];";
          break;
        case BC_CMP:
          o << "const bool n_ = nl[" << a << "] || nl[" << b << "]; r[" << d << "] = n_ ? 0 : (int64_t)cmp("
            << ((in.imm >> 4) & 15) << ", " << (in.imm & 15) << ", r[" << a << "], r[" << b << "]); nl[" << d << "] = false;";
          break;
        case BC_MATH:
          o << "bool n_ = nl[" << a << "] || nl[" << b << "]; int64_t o_ = 0; if (!n_) n_ = !math(" << ((in.imm >> 4) & 15)
            << ", " << (in.imm & 15) << ", r[" << a << "], r[" << b << "], o_); r[" << d << "] = o_; nl[" << d << "] = n_;";
          break;
        case BC_AND:
        case BC_OR:
          o << "const bool x_ = !nl[" << a << "] && r[" << a << "] != 0, y_ = !nl[" << b << "] && r[" << b << "] != 0; r["
            << d << "] = x_ " << (in.op == BC_AND ? "&&" : "||") << " y_; nl[" << d << "] = false;";
          break;
        case BC_NOT:
          o << "const bool x_ = nl[" << a << "] ? true : (r[" << a << "] == 0); r[" << d << "] = x_; nl[" << d << "] = false;";
          break;
        case BC_ISNULL:
          o << "r[" << d << "] = nl[" << a << "]; nl[" << d << "] = false;";
          break;
        case BC_RET:
          o << "res = r[" << a << "]; isnull = nl[" << a << "]; return true;";
          break;
        default:
          o << "return false;";
      }
      o << " }\n";
    }
    o << "  return false;\n}\n";
  }
};

// The kernel source for one lowered table: the constexpr table, the generated programs, the policy and the
// extern "C" kernel k_nfa_rtc (same arguments as k_nfa_lanes).  Layout checks make the compile fail, never the
// launch, if the run-time compiler ever laid out a shared struct differently from the library.
inline std::string nfa_rtc_source(const NTable& t, const std::vector<Prog>& progs, int fm) {
  RtcGen g;
  auto& o = g.o;
  o << "// generated by nfa_rtc.hpp for one lowered NFA table\n#include \"nfa_lane.hpp\"\nnamespace sg {\n";
  o << "static_assert(sizeof(NArgs) == " << sizeof(NArgs) << " && sizeof(NState) == " << sizeof(NState)
    << " && sizeof(NLds) == " << sizeof(NLds) << " && sizeof(NSpec) == " << sizeof(NSpec) << " && sizeof(NCols) == "
    << sizeof(NCols) << " && sizeof(NTable) == " << sizeof(NTable) << " && sizeof(FireRec) == " << sizeof(FireRec)
    << " && sizeof(OpRec) == " << sizeof(OpRec) << ", \"layout of the shared structs\");\n";
  o << "static_assert(__builtin_offsetof(NArgs, ev_skip) == " << offsetof(NArgs, ev_skip) << " && __builtin_offsetof(NState, tqh) == "
    << offsetof(NState, tqh) << " && __builtin_offsetof(NLds, total) == " << offsetof(NLds, total) << ", \"layout\");\n";
  o << "struct CTab {\n";
  o << "  static constexpr int32_t nproc = " << t.nproc << ", nslots = " << t.nslots << ", seq = " << t.seq
    << ", nstart = " << t.nstart << ";\n";
  o << "  static constexpr int64_t within = " << RtcGen::lit(t.within) << ";\n";
  g.arr("int8_t", "startIds", t.startIds, NS);
  o << "  static constexpr int8_t nall = " << (int)t.nall << ", ninit = " << (int)t.ninit << ", nreset = " << (int)t.nreset
    << ", nupdate = " << (int)t.nupdate << ";\n";
  g.arr("int8_t", "allPre", t.allPre, NP);
  g.arr("int8_t", "initOrder", t.initOrder, NP);
  g.arr("int8_t", "resetOrder", t.resetOrder, NP);
  g.arr("int8_t", "updateOrder", t.updateOrder, NP);
  o << "  static constexpr int32_t nstreams = " << t.nstreams << ";\n";
  g.arr("int8_t", "nnext", t.nnext, NSTR);
  g.arr("int8_t", "nfor", t.nfor, NSTR);
  g.arr("int8_t", "multi", t.multi, NSTR);
  g.arr2("int8_t", "nexts", t.nexts, NSTR);
  g.arr2("int8_t", "forStream", t.forStream, NSTR);
  g.arr("int8_t", "slotStream", t.slotStream, NS);
  o << "  struct A_p { __host__ __device__ __attribute__((always_inline)) constexpr NProc operator[](int i) const { "
       "switch (i) {";
  for (int k = 0; k < NP; k++) {
    const NProc& P = t.p[k];
    o << "\n    case " << k << ": return NProc{" << (int)P.kind << ", " << (int)P.stateId << ", " << (int)P.isStart << ", "
      << (int)P.withinEvery << ", " << (int)P.thisLast << ", " << (int)P.partner << ", " << (int)P.isAnd << ", "
      << (int)P.hasNext << ", " << (int)P.nextPre << ", " << (int)P.nextEveryPre << ", " << (int)P.callbackPre << ", "
      << (int)P.partnerPost << ", " << P.filter << ", " << (int)P.absLog << ", " << (int)P.absIdx << ", " << P.minCount
      << ", " << P.maxCount << "};";
  }
  o << "\n    default: return NProc{}; } } };\n  static constexpr A_p p{};\n";
  o << "  static constexpr int32_t nsel = " << t.nsel << ";\n";
  o << "  struct A_waiting { __host__ __device__ __attribute__((always_inline)) constexpr int64_t operator[](int i) const { "
       "switch (i) {";
  for (int k = 0; k < NP; k++) o << " case " << k << ": return " << RtcGen::lit(t.waiting[k]) << ";";
  o << " default: return -1; } } };\n  static constexpr A_waiting waiting{};\n";
  o << "  static constexpr int8_t nabs = " << (int)t.nabs << ";\n";
  g.arr("int8_t", "absOrder", t.absOrder, NP);
  o << "  static constexpr int8_t partitioned = " << (int)t.partitioned << ";\n};\n";
  for (size_t k = 0; k < progs.size(); k++) g.prog((int)k, progs[k]);
  o << "struct CPol {\n  static constexpr bool compiled = true;\n  using Tab = CTab;\n";
  o << "  template <class LD> __device__ __attribute__((always_inline)) static bool pred(int f, const LD& ld) {\n"
       "    int64_t v = 0; bool n = false;\n    switch (f) {\n";
  for (size_t k = 0; k < progs.size(); k++) {
    if (progs[k].n == 0) o << "      case " << k << ": return true;\n";
    else o << "      case " << k << ": sg_prog" << k << "(ld, v, n); return !n && v != 0;\n";
  }
  o << "      default: return true;\n    }\n  }\n";
  o << "  template <class LD> __device__ __attribute__((always_inline)) static void val(int f, const LD& ld, int64_t& v, "
       "bool& n) {\n    switch (f) {\n";
  for (size_t k = 0; k < progs.size(); k++) o << "      case " << k << ": sg_prog" << k << "(ld, v, n); return;\n";
  o << "      default: return;\n    }\n  }\n};\n}  // namespace sg\n";
  // at least two waves per SIMD (the registers capped at 256): with its pools in global memory a wide speculative launch
  // is latency-bound, and the second wave hides it (config 5's table asked for 269 VGPRs, one wave per SIMD: its
  // 79,000 segments ran 12.7 ms, 8.4 ms with two).  SG_RTC_WPE overrides it (0: no floor); it is part of the source,
  // hence of the cache key.
  const int wpe = getenv("SG_RTC_WPE") ? atoi(getenv("SG_RTC_WPE")) : 2;
  o << "extern \"C\" __global__ void __launch_bounds__(" << NFA_B << ") ";
  if (wpe > 0) o << "__attribute__((amdgpu_waves_per_eu(" << wpe << "))) ";
  o << "k_nfa_rtc(sg::NArgs a, sg::NState g, sg::NLds lay, "
       "const sg::NTable* __restrict__ tab, const sg::NCols* __restrict__ cols, const sg::Prog* __restrict__ progs, "
       "const sg::NSpec* __restrict__ spec) {\n"
       "  (void)tab; (void)progs;\n"
       "  extern __shared__ __align__(16) unsigned char nfa_dyn[];\n"
       "  sg::NCols* lcols = (sg::NCols*)(nfa_dyn + lay.cols_off);\n"
       "  for (int k = threadIdx.x; k < (int)(sizeof(sg::NCols) / 4); k += blockDim.x) ((int32_t*)lcols)[k] = "
       "((const int32_t*)cols)[k];\n"
       "  __syncthreads();\n"
       "  sg::nfa_lanes_run<"
    << fm << ", sg::CPol>(a, g, lay, spec, sg::CTab{}, *(const SG_AS3 sg::NCols*)lcols, nullptr, nfa_dyn);\n}\n";
  return o.str();
}

// ---- compilation and caches ----
inline std::string rtc_cache_dir() {
  if (const char* e = getenv("SG_RTC_CACHE")) return e;
  Dl_info info;
  if (dladdr((const void*)&rtc_cache_dir, &info) && info.dli_fname) {
    std::string p = info.dli_fname;
    const size_t s = p.rfind('/');
    if (s != std::string::npos) return p.substr(0, s) + "/rtc_cache";
  }
  return "/tmp/siddhi_gfx_rtc_cache";
}

// the kernel's private segment (scratch) size from the code object's metadata (msgpack: the key, then an unsigned int)
inline int64_t rtc_scratch_bytes(const std::vector<char>& code) {
  static const std::string key = ".private_segment_fixed_size";
  const std::string blob(code.begin(), code.end());
  const size_t i = blob.find(key);
  if (i == std::string::npos || i + key.size() >= blob.size()) return -1;
  const unsigned char* v = (const unsigned char*)blob.data() + i + key.size();
  const size_t rem = blob.size() - i - key.size();
  if (v[0] <= 0x7f) return v[0];
  if (v[0] == 0xcc && rem >= 2) return v[1];
  if (v[0] == 0xcd && rem >= 3) return (int64_t)v[1] << 8 | v[2];
  if (v[0] == 0xce && rem >= 5) return (int64_t)v[1] << 24 | (int64_t)v[2] << 16 | (int64_t)v[3] << 8 | v[4];
  return -1;
}

inline bool rtc_compile_with(const std::string& src, std::vector<char>& code, std::string& err, bool noreg) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "nfa_rtc.hip", kRtcNHdr, kRtcHdrSrcs, kRtcHdrNames) != HIPRTC_SUCCESS) {
    err = "hiprtcCreateProgram failed";
    return false;
  }
  std::vector<const char*> opts(kRtcOpts, kRtcOpts + sizeof(kRtcOpts) / sizeof(kRtcOpts[0]));
  if (noreg) opts.push_back("-DSG_RTC_NOREG=1");
  const hiprtcResult r = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
  if (r != HIPRTC_SUCCESS) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls + 1, '\0');
    if (ls) hiprtcGetProgramLog(prog, &log[0]);
    err = std::string("hiprtcCompileProgram: ") + hiprtcGetErrorString(r) + "\n" + log.substr(0, 4000);
    hiprtcDestroyProgram(&prog);
    return false;
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  code.resize(cs);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  return true;
}

// The per-processor counters in registers (kRtcRegs) need every processor index to be a constant; when the compiler
// merged paths into a dynamic index the kernel would keep the lane in scratch, so that table is compiled again with
// the counters in the pools (SG_RTC_NOREG), and the variant with less scratch is kept.
inline bool rtc_compile(const std::string& src, std::vector<char>& code, std::string& err) {
  if (!rtc_compile_with(src, code, err, false)) return false;
  if (rtc_scratch_bytes(code) == 0 || getenv("SG_RTC_REGS_ONLY")) return true;
  std::vector<char> alt;
  std::string err2;
  if (rtc_compile_with(src, alt, err2, true) && rtc_scratch_bytes(alt) >= 0 &&
      rtc_scratch_bytes(alt) < rtc_scratch_bytes(code))
    code.swap(alt);
  return true;
}

inline uint64_t rtc_key(const std::string& src) {
  // (the hipRTC version too: code objects an older compiler wrote are not loaded after an upgrade)
  int vmaj = 0, vmin = 0;
  hiprtcVersion(&vmaj, &vmin);
  std::string key_text = "hiprtc " + std::to_string(vmaj) + "." + std::to_string(vmin) + "\n" + src;
  for (int k = 0; k < kRtcNHdr; k++) key_text += kRtcHdrSrcs[k];
  for (const char* o : kRtcOpts) key_text += o;
  return rtc_fnv(key_text);
}
inline std::string rtc_code_path(uint64_t h) {
  char name[64];
  snprintf(name, sizeof name, "/nfa_%016" PRIx64 ".hsaco", h);
  return rtc_cache_dir() + name;
}

// The code object for `src`: from the disk cache, else compiled (and written to the cache).  Needs no GPU, and is
// safe to call from several threads (sg_query_compile warms the cache for many queries in parallel).
inline bool rtc_code(const std::string& src, std::vector<char>& code, RtcKernel& out, bool skip_disk = false) {
  const uint64_t h = rtc_key(src);
  const std::string path = rtc_code_path(h);
  if (!skip_disk) {
    std::ifstream f(path, std::ios::binary);
    if (f) {
      code.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
      out.from_disk = !code.empty();
    }
  }
  if (!code.empty()) return true;
  const auto t0 = std::chrono::steady_clock::now();
  if (!rtc_compile(src, code, out.err)) return false;
  out.compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  mkdir(rtc_cache_dir().c_str(), 0755);
  char sfx[48];
  snprintf(sfx, sizeof sfx, ".tmp%ld.%zx", (long)getpid(), std::hash<std::thread::id>{}(std::this_thread::get_id()));
  const std::string tmp = path + sfx;
  bool written = false;
  {
    std::ofstream f(tmp, std::ios::binary);
    f.write(code.data(), (std::streamsize)code.size());
    f.close();
    written = f.good();
  }
  // a short write (disk full) never reaches the cache's name: every later process would load a truncated object
  if (!written || rename(tmp.c_str(), path.c_str()) != 0) unlink(tmp.c_str());
  return true;
}

// process cache of loaded kernels, per (source hash, device)
struct RtcProcCache {
  std::mutex mu;
  std::map<std::pair<uint64_t, int>, RtcKernel> map;
};
inline RtcProcCache& rtc_proc_cache() { static RtcProcCache* c = new RtcProcCache; return *c; }

inline bool rtc_proc_lookup(uint64_t h, int dev, RtcKernel& out) {
  auto& c = rtc_proc_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.map.find({h, dev});
  if (it == c.map.end()) return false;
  out = it->second;
  out.compile_ms = 0;
  return true;
}
inline RtcKernel rtc_proc_insert(uint64_t h, int dev, const RtcKernel& k) {
  auto& c = rtc_proc_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.map.find({h, dev});
  if (it != c.map.end()) return it->second;          // (another thread loaded it meanwhile)
  c.map[{h, dev}] = k;
  return k;
}
inline bool rtc_load_module(const std::vector<char>& code, RtcKernel& out) {
  out.mod = nullptr;
  out.fn = nullptr;
  if (hipModuleLoadData(&out.mod, code.data()) != hipSuccess ||
      hipModuleGetFunction(&out.fn, out.mod, "k_nfa_rtc") != hipSuccess) {
    (void)hipGetLastError();
    out.err = "hipModuleLoadData / hipModuleGetFunction failed";
    out.fn = nullptr;
    return false;
  }
  return true;
}

// The kernel for `src` if it needs no compile: from the process cache, else loaded from the disk cache (a file read
// and a module load, milliseconds).  False: hipRTC would have to run.
inline bool nfa_rtc_cached(const std::string& src, RtcKernel& out) {
  const uint64_t h = rtc_key(src);
  int dev = 0;
  hipGetDevice(&dev);
  if (rtc_proc_lookup(h, dev, out)) return true;
  std::vector<char> code;
  {
    std::ifstream f(rtc_code_path(h), std::ios::binary);
    if (!f) return false;
    code.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  }
  RtcKernel k;
  k.from_disk = true;
  if (code.empty() || !rtc_load_module(code, k)) {
    unlink(rtc_code_path(h).c_str());                // (corrupt or stale: compiled again by the caller)
    return false;
  }
  out = rtc_proc_insert(h, dev, k);
  return true;
}

// ---- background compiles ----
// A query that starts streaming without a cached code object compiles it on a thread of its own while the
// interpreter serves its flushes (NfaExec::compiled_kernel); the flush thread loads the finished object.  Jobs are
// waited for at process exit (an atexit handler registered with the first job, so it runs before the compiler
// libraries' own static destructors), never when an app is destroyed: the job owns everything it uses.
struct RtcJob {
  std::atomic<bool> done{false};
  bool ok = false;
  std::vector<char> code;
  RtcKernel k;               // compile_ms, from_disk, err
};
struct RtcBgReg {
  std::mutex mu;
  std::condition_variable cv;
  int running = 0;
};
inline RtcBgReg& rtc_bg_reg() { static RtcBgReg* r = new RtcBgReg; return *r; }
inline void rtc_bg_wait_all() {
  auto& r = rtc_bg_reg();
  std::unique_lock<std::mutex> lk(r.mu);
  r.cv.wait(lk, [&] { return r.running == 0; });
}
inline std::shared_ptr<RtcJob> rtc_compile_async(const std::string& src) {
  static std::once_flag once;
  std::call_once(once, [] { std::atexit(rtc_bg_wait_all); });
  auto job = std::make_shared<RtcJob>();
  auto& r = rtc_bg_reg();
  {
    std::lock_guard<std::mutex> lk(r.mu);
    r.running++;
  }
  std::thread([job, src]() {
    job->ok = rtc_code(src, job->code, job->k);
    job->done.store(true, std::memory_order_release);
    auto& reg = rtc_bg_reg();
    std::lock_guard<std::mutex> lk(reg.mu);
    reg.running--;
    reg.cv.notify_all();
  }).detach();
  return job;
}
// the finished job's kernel on the current device (into the process cache)
inline RtcKernel nfa_rtc_from_job(const std::string& src, RtcJob& job) {
  RtcKernel out = job.k;
  if (!job.ok) return out;
  const uint64_t h = rtc_key(src);
  int dev = 0;
  hipGetDevice(&dev);
  if (rtc_proc_lookup(h, dev, out)) return out;
  out = job.k;
  if (!rtc_load_module(job.code, out)) return out;
  return rtc_proc_insert(h, dev, out);
}

// The compiled kernel for `src` on the current device: from the process cache, else the disk cache, else hipRTC.
inline RtcKernel nfa_rtc_get(const std::string& src) {
  const uint64_t h = rtc_key(src);
  int dev = 0;
  hipGetDevice(&dev);
  {
    RtcKernel k;
    if (rtc_proc_lookup(h, dev, k)) return k;
  }
  RtcKernel out;
  auto load = [&](const std::vector<char>& code) { return rtc_load_module(code, out); };
  std::vector<char> code;
  if (rtc_code(src, code, out) && !load(code) && out.from_disk) {
    // a cached object that does not load (corrupt, or from another runtime): dropped from the cache, compiled once more
    unlink(rtc_code_path(h).c_str());
    code.clear();
    out = RtcKernel{};
    if (rtc_code(src, code, out, true)) load(code);
  }
  if (!out.fn) return out;
  return rtc_proc_insert(h, dev, out);
}

}  // namespace sg
