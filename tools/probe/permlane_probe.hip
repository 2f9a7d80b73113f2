// v_permlane32_swap semantics probe: each lane prints (lane, r[0], r[1]) for x = lane
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out) {
  const unsigned x = threadIdx.x;
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  out[2 * threadIdx.x] = r[0];
  out[2 * threadIdx.x + 1] = r[1];
}
int main() {
  unsigned* d;
  unsigned h[128];
  (void)hipMalloc(&d, 512);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l += 7) printf("lane %2d: r0=%2u r1=%2u\n", l, h[2 * l], h[2 * l + 1]);
  return 0;
}
