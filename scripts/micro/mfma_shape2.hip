// MFMA shape A/B on the conv kernel's wave tile (96 x 64 per wave, 4 waves per CU, one
// workgroup per CU), operands re-read from LDS by ds_read_b128 every k-step, random bf16 with
// full mantissas (normal-like values), so the DVFS give-back of MI355X_MICROARCH.md item 7 shows.
//   32x32x16: per 32-deep k: 2 x (3 A + 2 B reads, 6 MFMAs)
//   16x16x32: per 32-deep k: 6 A + 4 B reads, 24 MFMAs
// Same FLOP and the same LDS bytes per k for both.  Conflict-free swizzles: 32-row fragments piece ^ (row>>2)&3,
// 16-row fragments piece ^ ((row>>2)&1)*2 (any row shift).  Prints wall TF/s and the in-kernel clock
// (s_memtime / s_memrealtime, stamps into their own buffer).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <algorithm>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef MFMA_ORDER
#define MFMA_ORDER 0
#endif
constexpr int LDS_ROWS = 512;   // 512 rows x 64 B (32 bf16 of k) = 32 KB A/B image

template <int SHAPE>
__global__ __launch_bounds__(256, 1) void kshape(const uint4* src, float* out, unsigned long long* stamps, int iters) {
  __shared__ uint4 lds[LDS_ROWS * 4];
  for (int i = threadIdx.x; i < LDS_ROWS * 4; i += 256) lds[i] = src[(blockIdx.x * 7 + i) % (LDS_ROWS * 4 * 8)];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  if constexpr (SHAPE == 32) {
    f32x16 acc[3][2];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 2; ++j)
        for (int e = 0; e < 16; ++e) acc[i][j][e] = out[i + j + e];
    const int lr = lane & 31, hk = lane >> 5;   // row, k half (8 elements)
    bf16x8 a[2][3], b[2][2];                    // fragments of step s (software-pipelined by one step)
    auto rd = [&](int step, bf16x8 (&aa)[3], bf16x8 (&bb)[2]) {
      const int it = step >> 1, ks = step & 1;
      const int rb = (it * 96 + w * 32) & (LDS_ROWS - 1);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int row = (rb + i * 32 + lr) & (LDS_ROWS - 1);
        aa[i] = *reinterpret_cast<const bf16x8*>(&lds[row * 4 + ((ks * 2 + hk) ^ ((row >> 2) & 3))]);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = (rb + 256 + j * 32 + lr) & (LDS_ROWS - 1);
        bb[j] = *reinterpret_cast<const bf16x8*>(&lds[row * 4 + ((ks * 2 + hk) ^ ((row >> 2) & 3))]);
      }
    };
    rd(0, a[0], b[0]);
    for (int st = 0; st < 2 * iters; st += 2) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        rd(st + u + 1, a[u ^ 1], b[u ^ 1]);
#if MFMA_ORDER == 1   // B-major: each B fragment held for 3 consecutive MFMAs
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < 3; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[u][i], b[u][j], acc[i][j], 0, 0, 0);
#else                 // A-major (the conv kernel's order): each A fragment held for 2
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[u][i], b[u][j], acc[i][j], 0, 0, 0);
#endif
        // M R M R M R M R M R M: one read per MFMA gap
#pragma unroll
        for (int g = 0; g < 5; ++g) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
    }
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 2; ++j) for (int e = 0; e < 16; ++e) s += acc[i][j][e];
  } else {
    f32x4 acc[6][4];
    for (int i = 0; i < 6; ++i)       // opaque initial values: no zero-peeled first iteration
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{out[i], out[j], out[i + j], out[0]};
    const int lr = lane & 15, q = lane >> 4;    // row, k quarter (8 elements of 32)
    bf16x8 a[2][6], b[2][4];
    auto rd = [&](int it, bf16x8 (&aa)[6], bf16x8 (&bb)[4]) {
      const int rb = (it * 96 + w * 32) & (LDS_ROWS - 1);
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int row = (rb + i * 16 + lr) & (LDS_ROWS - 1);
        aa[i] = *reinterpret_cast<const bf16x8*>(&lds[row * 4 + (q ^ (((row >> 2) & 1) << 1))]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = (rb + 256 + j * 16 + lr) & (LDS_ROWS - 1);
        bb[j] = *reinterpret_cast<const bf16x8*>(&lds[row * 4 + (q ^ (((row >> 2) & 1) << 1))]);
      }
    };
    rd(0, a[0], b[0]);
    for (int it = 0; it < iters; it += 2) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        rd(it + u + 1, a[u ^ 1], b[u ^ 1]);
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][i], b[u][j], acc[i][j], 0, 0, 0);
        // (M M R) x 10, M M M M: one read per two 16-cycle MFMAs
#pragma unroll
        for (int g = 0; g < 10; ++g) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      }
    }
    for (int i = 0; i < 6; ++i) for (int j = 0; j < 4; ++j) for (int e = 0; e < 4; ++e) s += acc[i][j][e];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    stamps[blockIdx.x * 2] = t1 - t0;
    stamps[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  const int reps = argc > 2 ? atoi(argv[2]) : 40;
  const size_t n = LDS_ROWS * 4 * 8;
  std::vector<unsigned short> h(n * 8);
  unsigned x = 12345;
  for (auto& v : h) {   // normal-like bf16: random sign, exponent near 0, full random mantissa
    x = x * 1664525u + 1013904223u;
    const unsigned sign = (x >> 31) & 1, mant = (x >> 8) & 0x7f, ex = 124 + ((x >> 16) & 3);
    v = (unsigned short)((sign << 15) | (ex << 7) | mant);
  }
  uint4* src;
  float* out;
  unsigned long long* st;
  (void)hipMalloc(&src, n * 16);
  (void)hipMalloc(&out, 256 * 256 * 4);
  (void)hipMalloc(&st, 256 * 16);
  (void)hipMemcpy(src, h.data(), n * 16, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  std::vector<unsigned long long> hs(512);
  for (int round = 0; round < 2; ++round) {
    for (int shape = 0; shape < 2; ++shape) {
      for (int w = 0; w < 5; ++w) {
        if (shape == 0) kshape<32><<<256, 256>>>(src, out, st, iters); else kshape<16><<<256, 256>>>(src, out, st, iters);
      }
      (void)hipEventRecord(e0);
      for (int r = 0; r < reps; ++r) {
        if (shape == 0) kshape<32><<<256, 256>>>(src, out, st, iters); else kshape<16><<<256, 256>>>(src, out, st, iters);
      }
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      (void)hipMemcpy(hs.data(), st, 256 * 16, hipMemcpyDeviceToHost);
      std::vector<double> clk;
      for (int b = 0; b < 256; ++b) clk.push_back((double)hs[2 * b] / (double)hs[2 * b + 1] * 100.0);  // MHz
      std::sort(clk.begin(), clk.end());
      // per wave per iteration: 32-deep k over a 96 x 64 tile = 96*64*32*2 FLOP
      const double f = 256.0 * 4 * (double)iters * reps * 96 * 64 * 32 * 2;
      printf("{\"shape\": \"%s\", \"round\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"clock_mhz_median\": %.0f}\n",
             shape == 0 ? "32x32x16" : "16x16x32", round, ms, f / ms * 1e-9, clk[128]);
    }
  }
  return 0;
}
