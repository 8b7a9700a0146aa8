// Dispatch-cost probe: 490k workgroups of 512 threads, with/without 78 KB of static LDS, exiting at once
// or after one global load.  Prints ms per launch for each variant.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int LDS_WORDS, int MODE>
__global__ void __launch_bounds__(512) k(const uint4* __restrict__ in, const int* __restrict__ flag, int* out) {
  __shared__ uint32_t s[LDS_WORDS > 0 ? LDS_WORDS : 1];
  const int f = flag[blockIdx.x & 1023];
  if (MODE == 0) { if (f == 12345) out[0] = 1; return; }
  uint4 v = in[(size_t)blockIdx.x * 512 + threadIdx.x];
  if (MODE == 1) { if (v.x == 0xdeadbeef) out[1] = 1; return; }
  s[threadIdx.x] = v.x;
  __syncthreads();
  if (s[(threadIdx.x + 1) & 511] == 0xdeadbeef) out[2] = 1;
}

template <int W, int M>
float run(const uint4* in, const int* flag, int* out, int nb) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL((k<W, M>), dim3(nb), dim3(512), 0, 0, in, flag, out);
  hipEventRecord(a);
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL((k<W, M>), dim3(nb), dim3(512), 0, 0, in, flag, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 3;
}

int main() {
  const int nb = 490000;
  uint4* in; int* flag; int* out;
  hipMalloc(&in, (size_t)nb * 512 * 16); hipMalloc(&flag, 4096 * 4); hipMalloc(&out, 64);
  hipMemset(in, 0, (size_t)nb * 512 * 16); hipMemset(flag, 0, 4096 * 4);
  printf("lds78K exit:      %.3f ms\n", run<19500, 0>(in, flag, out, nb));
  printf("lds78K load-exit: %.3f ms\n", run<19500, 1>(in, flag, out, nb));
  printf("lds78K load-lds:  %.3f ms\n", run<19500, 2>(in, flag, out, nb));
  printf("lds0 exit:        %.3f ms\n", run<0, 0>(in, flag, out, nb));
  printf("lds0 load-exit:   %.3f ms\n", run<0, 1>(in, flag, out, nb));
  printf("lds2K load-lds:   %.3f ms\n", run<512, 2>(in, flag, out, nb));
  return 0;
}
