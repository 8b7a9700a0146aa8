// snapshot.hpp — byte-stream writer / reader for sg_snapshot / sg_restore (SiddhiAppRuntime.snapshot()
// / restore(byte[]), CORE/SiddhiAppRuntimeImpl.java; per-processor state maps such as
// StreamPreStateProcessor.StreamPreState.snapshot, CORE/query/input/stream/state/StreamPreStateProcessor.java:450-469).
// Little-endian raw fields; every section is length-checked on read so a truncated or foreign buffer
// fails with SG_E_INVALID instead of restoring garbage.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "runtime.hpp"

namespace sg {

struct SnapWriter {
  std::string b;
  void raw(const void* p, size_t n) { b.append((const char*)p, n); }
  template <class T> void pod(const T& v) { raw(&v, sizeof(T)); }
  template <class T, class A> void vec(const std::vector<T, A>& v) {
    pod<uint64_t>(v.size());
    if (!v.empty()) raw(v.data(), v.size() * sizeof(T));
  }
  template <class T> void deq(const std::deque<T>& v) {
    pod<uint64_t>(v.size());
    for (const T& x : v) pod(x);
  }
  void str(const std::string& s) { pod<uint64_t>(s.size()); raw(s.data(), s.size()); }
  // `count` elements of a device buffer
  template <class T> void dev(const DBuf<T>& d, size_t count, hipStream_t s) { devp(d.p, count, s); }
  template <class T> void devp(const T* d, size_t count, hipStream_t s) {
    pod<uint64_t>(count);
    if (!count) return;
    const size_t at = b.size();
    b.resize(at + count * sizeof(T));
    SG_HIP(hipMemcpyAsync(&b[at], d, count * sizeof(T), hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
  }
};

struct SnapReader {
  const uint8_t* p;
  size_t n, at = 0;
  SnapReader(const uint8_t* d, size_t len) : p(d), n(len) {}
  void need(size_t k) const {
    if (at + k > n) throw Error(-1, "snapshot buffer truncated or from another app");
  }
  void raw(void* dst, size_t k) { need(k); std::memcpy(dst, p + at, k); at += k; }
  template <class T> T pod() { T v; raw(&v, sizeof(T)); return v; }
  template <class T, class A> void vec(std::vector<T, A>& v) {
    const uint64_t k = pod<uint64_t>();
    need(k * sizeof(T));
    v.resize(k);
    if (k) raw(v.data(), k * sizeof(T));
  }
  template <class T> void deq(std::deque<T>& v) {
    const uint64_t k = pod<uint64_t>();
    need(k * sizeof(T));
    v.clear();
    for (uint64_t i = 0; i < k; i++) v.push_back(pod<T>());
  }
  std::string str() {
    const uint64_t k = pod<uint64_t>();
    need(k);
    std::string s((const char*)p + at, k);
    at += k;
    return s;
  }
  // into device memory the caller sized for at most `cap` elements
  template <class T> size_t devp(T* d, size_t cap, hipStream_t s) {
    const uint64_t k = pod<uint64_t>();
    need(k * sizeof(T));
    if (k > cap) throw Error(-1, "snapshot section larger than its buffer");
    if (k) {
      SG_HIP(hipMemcpyAsync(d, p + at, k * sizeof(T), hipMemcpyHostToDevice, s));
      SG_HIP(hipStreamSynchronize(s));
      at += k * sizeof(T);
    }
    return k;
  }
  // the element count of the next device section (without consuming it)
  uint64_t peek_count() const { need(8); uint64_t k; std::memcpy(&k, p + at, 8); return k; }
  // into a device buffer (reserved to the stored count)
  template <class T> size_t dev(DBuf<T>& d, hipStream_t s) {
    const uint64_t k = pod<uint64_t>();
    need(k * sizeof(T));
    if (k) {
      d.reserve(k, false, s, 0);
      SG_HIP(hipMemcpyAsync(d.p, p + at, k * sizeof(T), hipMemcpyHostToDevice, s));
      SG_HIP(hipStreamSynchronize(s));
      at += k * sizeof(T);
    }
    return k;
  }
};

}  // namespace sg
