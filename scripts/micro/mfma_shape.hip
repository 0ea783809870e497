// Bare MFMA loop: 32x32x16 vs 16x16x32 bf16 on random register operands, 4 waves/CU
// (diagnostic for the DVFS effect of the MFMA shape, MI355X_MICROARCH.md DVFS item 7).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k32(float* out, int iters, unsigned seed) {
  bf16x8 a[3], b[2];
  for (int i = 0; i < 3; ++i) for (int e = 0; e < 8; ++e) {
    unsigned h = (threadIdx.x * 131 + i * 17 + e * 7 + seed) * 2654435761u; h ^= h >> 15;
    a[i][e] = (__bf16)((int)(h & 1023) - 512);
  }
  for (int j = 0; j < 2; ++j) for (int e = 0; e < 8; ++e) {
    unsigned h = (threadIdx.x * 37 + j * 29 + e * 11 + seed) * 2246822519u; h ^= h >> 13;
    b[j][e] = (__bf16)((int)(h & 1023) - 512);
  }
  f32x16 acc[3][2] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 3; ++i) for (int j = 0; j < 2; ++j) for (int e = 0; e < 16; ++e) s += acc[i][j][e];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k16(float* out, int iters, unsigned seed) {
  bf16x8 a[6], b[4];
  for (int i = 0; i < 6; ++i) for (int e = 0; e < 8; ++e) {
    unsigned h = (threadIdx.x * 131 + i * 17 + e * 7 + seed) * 2654435761u; h ^= h >> 15;
    a[i][e] = (__bf16)((int)(h & 1023) - 512);
  }
  for (int j = 0; j < 4; ++j) for (int e = 0; e < 8; ++e) {
    unsigned h = (threadIdx.x * 37 + j * 29 + e * 11 + seed) * 2246822519u; h ^= h >> 13;
    b[j][e] = (__bf16)((int)(h & 1023) - 512);
  }
  f32x4 acc[6][4] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 6; ++i) for (int j = 0; j < 4; ++j) for (int e = 0; e < 4; ++e) s += acc[i][j][e];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 256 * 256 * 4 * 4);
  const int iters = 20000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    for (int shape = 0; shape < 2; ++shape) {
      for (int w = 0; w < 3; ++w) {
        if (shape == 0) k32<<<256, 256>>>(out, iters, 1); else k16<<<256, 256>>>(out, iters, 1);
      }
      (void)hipEventRecord(e0);
      if (shape == 0) k32<<<256, 256>>>(out, iters, 2); else k16<<<256, 256>>>(out, iters, 2);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double flop = 256.0 * 4 * iters * 6 * (shape == 0 ? 32.0 * 32 * 16 * 2 : 4 * 16.0 * 16 * 32 * 2 / 4 * 4);
      // both: per wave per iteration 6 x (32x32x16) = 24 x (16x16x32) = 98304 FLOP... computed below
      const double f = 256.0 * 4 * iters * 98304.0;
      printf("%s: %.3f ms, %.1f TF/s\n", shape == 0 ? "32x32x16" : "16x16x32", ms, f / ms * 1e-9);
      (void)flop;
    }
  }
  return 0;
}
