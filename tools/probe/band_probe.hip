// Access-pattern probe for the blur: band-wise row streaming of a 10k x 10k x
// 30 uint16 HWC slide into an fp32 HWC output (no arithmetic), 64-column bands
// x 256 rows, one barrier per row.  Variant W = bytes per lane per load/store
// (4 or 16), prefetch depth in registers = D rows.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int H = 10000, Wd = 10000, C = 30, BW = 64, R = 8, BH = 256;

template <int W, int NT>
__global__ void __launch_bounds__(NT) band(const unsigned short* __restrict__ in, float* __restrict__ out) {
  const int x0 = blockIdx.x * BW, y0 = blockIdx.y * BH;
  const int y1 = min(H, y0 + BH);
  const int bw = min(BW, Wd - x0);
  const int xs = max(0, x0 - R), xe = min(Wd, x0 + BW + R);
  const int in_bytes = (xe - xs) * C * 2;      // input row segment
  const int out_bytes = bw * C * 4;            // output row segment
  float acc = 0.f;
  for (int y = y0 - R; y < y1 + R; ++y) {
    const int yy = min(max(y, 0), H - 1);
    const char* src = (const char*)(in + ((size_t)yy * Wd + xs) * C);
    for (int b = threadIdx.x * W; b < in_bytes; b += NT * W) {
      if (W == 16) {
        u4 v = *(const u4*)(src + b);
        acc += (float)(v.x & 0xffff) + (float)(v.w >> 16);
      } else {
        unsigned v = *(const unsigned*)(src + b);
        acc += (float)(v & 0xffff);
      }
    }
    __syncthreads();
    if (y >= y0 + R && y - 2 * R >= y0 - R) {
      char* dst = (char*)(out + ((size_t)(y - R) * Wd + x0) * C);
      for (int b = threadIdx.x * W; b < out_bytes; b += NT * W) {
        if (W == 16) *(f4*)(dst + b) = f4{acc, acc, acc, acc};
        else *(float*)(dst + b) = acc;
      }
    }
  }
}

template <typename K>
static float run(K k, dim3 g, int nt, const unsigned short* in, float* out) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k, g, dim3(nt), 0, 0, in, out);
  (void)hipEventRecord(a);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, g, dim3(nt), 0, 0, in, out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 3;
}

int main() {
  unsigned short* in;
  float* out;
  (void)hipMalloc(&in, (size_t)H * Wd * C * 2);
  (void)hipMalloc(&out, (size_t)H * Wd * C * 4);
  (void)hipMemset(in, 1, (size_t)H * Wd * C * 2);
  dim3 g((Wd + BW - 1) / BW, (H + BH - 1) / BH);
  const double gb = (double)H * Wd * C * 6 / 1e9;
  float t;
  t = run(band<4, 512>, g, 512, in, out);   printf("W=4  NT=512 : %.3f ms  %.0f GB/s\n", t, gb / t * 1e3);
  t = run(band<16, 512>, g, 512, in, out);  printf("W=16 NT=512 : %.3f ms  %.0f GB/s\n", t, gb / t * 1e3);
  t = run(band<4, 1024>, g, 1024, in, out); printf("W=4  NT=1024: %.3f ms  %.0f GB/s\n", t, gb / t * 1e3);
  t = run(band<16, 256>, g, 256, in, out);  printf("W=16 NT=256 : %.3f ms  %.0f GB/s\n", t, gb / t * 1e3);
  return 0;
}
