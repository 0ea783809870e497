// Does hipExtLaunchKernel(..., hipExtAnyOrderLaunch) let the next kernel start before the previous one
// ends on gfx950?  Kernel A: one block per CU busy-waits ~40 us; kernel B records its start clock.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

__global__ void spin(unsigned long long* t, int us) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)us * 100) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0 && blockIdx.x == 0) t[0] = __builtin_amdgcn_s_memrealtime();   // A's end (block 0)
}
__global__ void stamp(unsigned long long* t) {
  if (threadIdx.x == 0 && blockIdx.x == 0) t[1] = __builtin_amdgcn_s_memrealtime();  // B's start
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 16);
  hipStream_t s;
  hipStreamCreate(&s);
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipMemsetAsync(d, 0, 16, s);
      int us = 40;
      void* a1[] = {&d, &us};
      void* a2[] = {&d};
      hipExtLaunchKernel((const void*)spin, dim3(256), dim3(64), a1, 0, s, nullptr, nullptr, 0);
      hipExtLaunchKernel((const void*)stamp, dim3(1), dim3(64), a2, 0, s, nullptr, nullptr, mode ? hipExtAnyOrderLaunch : 0);
      hipStreamSynchronize(s);
      unsigned long long h[2];
      hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
      printf("mode %s rep %d: B start - A end = %+.2f us\n", mode ? "anyorder" : "ordered ", rep,
             ((double)h[1] - (double)h[0]) / 100.0);
    }
  }
  return 0;
}
