// LDS-DMA layout check: global_load_lds_dwordx4 of a known pattern, LDS dumped back.
#include <hip/hip_runtime.h>
#include <stdio.h>
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__global__ void k(const unsigned* src, unsigned* dump, int shift) {
  __shared__ unsigned lds[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) lds[i] = 0xdeadbeef;
  __syncthreads();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint32_t base = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) unsigned*)lds);
  const char* g = (const char*)src + shift + (w * 64 + lane) * 16;
  glds16(g, base + w * 1024);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) dump[i] = lds[i];
}
int main() {
  unsigned *src, *dump, h[4096], d[1024];
  for (int i = 0; i < 4096; ++i) h[i] = i;
  (void)hipMalloc(&src, 16384); (void)hipMalloc(&dump, 4096);
  (void)hipMemcpy(src, h, 16384, hipMemcpyHostToDevice);
  for (int shift : {0, 4, 8}) {
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, src, dump, shift);
    (void)hipMemcpy(d, dump, 4096, hipMemcpyDeviceToHost);
    int bad = 0, first = -1;
    for (int i = 0; i < 1024; ++i) if (d[i] != (unsigned)(i + shift / 4)) { if (first < 0) first = i; ++bad; }
    printf("shift %d: bad dwords %d (first %d: got %u)\n", shift, bad, first, first >= 0 ? d[first] : 0);
    if (bad) { for (int i = 0; i < 24; ++i) printf("%u ", d[i]); printf("\n"); }
  }
  return 0;
}
