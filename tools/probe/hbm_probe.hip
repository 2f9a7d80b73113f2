// HBM bandwidth probe (MI355X calibration for the roofline targets):
// streaming read-reduce and read+write copy with U 16-byte loads in flight per
// lane, grid = CUs x blocks-per-CU (grid-stride), 256-thread blocks.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ void __launch_bounds__(256) rd(const f4* __restrict__ x, long n4, float* out) {
  const long stride = (long)gridDim.x * 256 * U;
  f4 acc = {0, 0, 0, 0};
  for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long j = i + u * 256;
      v[u] = x[j < n4 ? j : n4 - 1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) out[0] = 1.f;
}

template <int U>
__global__ void __launch_bounds__(256) cp(const f4* __restrict__ x, long n4, f4* __restrict__ y) {
  const long stride = (long)gridDim.x * 256 * U;
  for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long j = i + u * 256;
      v[u] = x[j < n4 ? j : n4 - 1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long j = i + u * 256;
      if (j < n4) y[j] = v[u];
    }
  }
}

// write-only (fp32 output stream)
template <int U>
__global__ void __launch_bounds__(256) wr(long n4, f4* __restrict__ y) {
  const long stride = (long)gridDim.x * 256 * U;
  for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long j = i + u * 256;
      if (j < n4) y[j] = f4{(float)j, 0.f, 1.f, 2.f};
    }
  }
}

template <typename L>
static float timeit(L launch, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  launch();
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const long bytes = 6L << 30;  // 6 GiB per stream
  const long n4 = bytes / 16;
  f4 *x, *y;
  float* o;
  if (hipMalloc(&x, bytes) || hipMalloc(&y, bytes) || hipMalloc(&o, 64)) return 1;
  hipMemset(x, 0, bytes);
  hipMemset(y, 0, bytes);
  int ncu;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d, stream %.2f GB\n", ncu, bytes / 1e9);
  for (int bpc : {2, 4, 8}) {
    const int g = ncu * bpc;
#define RUN(U)                                                                                   \
  {                                                                                              \
    float t1 = timeit([&] { hipLaunchKernelGGL(rd<U>, dim3(g), dim3(256), 0, 0, x, n4, o); }, 5); \
    float t2 = timeit([&] { hipLaunchKernelGGL(cp<U>, dim3(g), dim3(256), 0, 0, x, n4, y); }, 5); \
    float t3 = timeit([&] { hipLaunchKernelGGL(wr<U>, dim3(g), dim3(256), 0, 0, n4, y); }, 5);   \
    printf("blocks/CU %d U %d: read %.0f GB/s  copy %.0f GB/s  write %.0f GB/s\n", bpc, U,       \
           bytes / t1 / 1e6, 2 * bytes / t2 / 1e6, bytes / t3 / 1e6);                             \
  }
    RUN(1) RUN(2) RUN(4) RUN(8)
  }
  return 0;
}
