// PMC calibration (MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are exact or halved depending on the
// access width; other widths "uncalibrated: calibrate on a known byte count in your own access pattern").
// Each kernel moves exactly BYTES of a buffer far larger than the 256 MiB Infinity Cache with one access
// width per lane, coalesced; rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE, a separate pass) over this binary
// gives the factor counter -> bytes per width.
//   hipcc --offload-arch=gfx950 -O3 -o pmc_calib pmc_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr size_t BYTES = size_t(1) << 30;   // 1 GiB per kernel

template <class T>
__global__ void __launch_bounds__(256) k_rd(const T* __restrict__ src, size_t n, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const T v = src[i];
    const uint32_t* w = (const uint32_t*)&v;
    for (int k = 0; k < (int)(sizeof(T) / 4); k++) acc ^= w[k];
  }
  if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;   // never true for the zero-filled buffer: no stores
}

template <class T>
__global__ void __launch_bounds__(256) k_wr(T* __restrict__ dst, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    T v;
    uint32_t* w = (uint32_t*)&v;
    for (int k = 0; k < (int)(sizeof(T) / 4); k++) w[k] = (uint32_t)i + k;
    dst[i] = v;
  }
}

struct U2 { uint32_t a, b; };
struct U3 { uint32_t a, b, c; };

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e)); return 1; } } while (0)

int main() {
  void* buf = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&buf, BYTES));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(buf, 0, BYTES));
  const dim3 g(4096), b(256);
  hipLaunchKernelGGL(k_rd<uint32_t>, g, b, 0, 0, (const uint32_t*)buf, BYTES / 4, out);
  hipLaunchKernelGGL(k_rd<U2>, g, b, 0, 0, (const U2*)buf, BYTES / 8, out);
  hipLaunchKernelGGL(k_rd<U3>, g, b, 0, 0, (const U3*)buf, BYTES / 12, out);
  hipLaunchKernelGGL(k_rd<uint4>, g, b, 0, 0, (const uint4*)buf, BYTES / 16, out);
  hipLaunchKernelGGL(k_wr<uint32_t>, g, b, 0, 0, (uint32_t*)buf, BYTES / 4);
  hipLaunchKernelGGL(k_wr<U2>, g, b, 0, 0, (U2*)buf, BYTES / 8);
  hipLaunchKernelGGL(k_wr<U3>, g, b, 0, 0, (U3*)buf, BYTES / 12);
  hipLaunchKernelGGL(k_wr<uint4>, g, b, 0, 0, (uint4*)buf, BYTES / 16);
  CK(hipDeviceSynchronize());
  printf("pmc_calib: each kernel moves %zu bytes (12-B kernels: %zu)\n", BYTES, (BYTES / 12) * 12);
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
