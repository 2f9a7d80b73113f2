// VALU throughput probe: independent fp32 FMA streams as v_fma_f32 vs
// v_pk_fma_f32 (and fp64 v_fma_f64), 8 independent chains per lane, all CUs.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) fma32(float* out, int iters, float a) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], a, 0.5f);
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  if (s == 1.2345f) out[0] = s;
}
__global__ void __launch_bounds__(256) pkfma32(float* out, int iters, float a) {
  f2 x[8];
  for (int i = 0; i < 8; ++i) x[i] = f2{(float)threadIdx.x + i, (float)i};
  const f2 aa = {a, a}, hh = {0.5f, 0.5f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], aa, hh);
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  if (s == 1.2345f) out[0] = s;
}
__global__ void __launch_bounds__(256) fma64(float* out, int iters, double a) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fma(x[i], a, 0.5);
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  if (s == 1.2345) out[0] = (float)s;
}

int main() {
  float* o;
  hipMalloc(&o, 64);
  int ncu;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int bpc : {4, 8}) {
    const int g = ncu * bpc;
    for (int kind = 0; kind < 3; ++kind) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (kind == 0) hipLaunchKernelGGL(fma32, dim3(g), dim3(256), 0, 0, o, iters, 1.0001f);
        if (kind == 1) hipLaunchKernelGGL(pkfma32, dim3(g), dim3(256), 0, 0, o, iters, 1.0001f);
        if (kind == 2) hipLaunchKernelGGL(fma64, dim3(g), dim3(256), 0, 0, o, iters, 1.0001);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double elems = (double)g * 256 * iters * 8 * (kind == 1 ? 2 : 1);
        if (rep == 1)
          printf("blocks/CU %d %s: %.1f TFLOP/s (%.3f ms)\n", bpc,
                 kind == 0 ? "v_fma_f32   " : kind == 1 ? "v_pk_fma_f32" : "v_fma_f64   ",
                 2 * elems / ms / 1e9, ms);
      }
    }
  }
  return 0;
}
