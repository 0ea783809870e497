// Posterior accuracy metrics on the GPU (main_script.py:719-758):
// per-column mean and the sample covariance (ddof = 1, np.cov) of n samples of d
// columns, fp64 accumulation, deterministic two-stage reduction.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "petmetrics.h"

namespace petmetrics {

constexpr int kThreads = 256;
constexpr int kRows = 32;          // samples staged per LDS tile
constexpr int kSub = 6;            // covariance sub-tile per thread: d <= 16 * kSub = 96

template <typename T>
__device__ __forceinline__ double load(const void* x, int64_t row, int col, int ld) {
  return (double)reinterpret_cast<const T*>(x)[row * ld + col];
}

// pass 1: block b sums columns over its row range -> part[b][d]
template <typename T>
__global__ __launch_bounds__(kThreads) void colsum_kernel(const void* x, int64_t n, int d, int ld, int64_t rows_per,
                                                          double* part) {
  const int64_t r0 = (int64_t)blockIdx.x * rows_per, r1 = min(n, r0 + rows_per);
  for (int c = threadIdx.x; c < d; c += kThreads) {
    double s = 0.0;
    for (int64_t r = r0; r < r1; ++r) s += load<T>(x, r, c, ld);
    part[(size_t)blockIdx.x * d + c] = s;
  }
}

// pass 2: block b accumulates the centred cross products of its rows -> part[b][d][d].
// Thread (ta, tb) of a 16 x 16 layout owns entries (ta + 16 i, tb + 16 j), i, j < 6.
template <typename T>
__global__ __launch_bounds__(kThreads) void comoment_kernel(const void* x, int64_t n, int d, int ld, int64_t rows_per,
                                                            const double* mean, double* part) {
  extern __shared__ double tile[];   // [kRows][d]
  const int64_t r0 = (int64_t)blockIdx.x * rows_per, r1 = min(n, r0 + rows_per);
  const int ta = threadIdx.x >> 4, tb = threadIdx.x & 15;
  double acc[kSub][kSub];
#pragma unroll
  for (int i = 0; i < kSub; ++i)
#pragma unroll
    for (int j = 0; j < kSub; ++j) acc[i][j] = 0.0;
  for (int64_t rb = r0; rb < r1; rb += kRows) {
    const int nr = (int)min<int64_t>(kRows, r1 - rb);
    for (int e = threadIdx.x; e < kRows * d; e += kThreads) {
      const int rr = e / d, c = e - rr * d;
      tile[e] = rr < nr ? load<T>(x, rb + rr, c, ld) - mean[c] : 0.0;
    }
    __syncthreads();
    for (int rr = 0; rr < nr; ++rr) {
      double va[kSub], vb[kSub];
#pragma unroll
      for (int i = 0; i < kSub; ++i) {
        const int ca = ta + 16 * i, cb = tb + 16 * i;
        va[i] = ca < d ? tile[rr * d + ca] : 0.0;
        vb[i] = cb < d ? tile[rr * d + cb] : 0.0;
      }
#pragma unroll
      for (int i = 0; i < kSub; ++i)
#pragma unroll
        for (int j = 0; j < kSub; ++j) acc[i][j] = fma(va[i], vb[j], acc[i][j]);
    }
    __syncthreads();
  }
  const int pairs = d * d;
#pragma unroll
  for (int i = 0; i < kSub; ++i)
#pragma unroll
    for (int j = 0; j < kSub; ++j) {
      const int a = ta + 16 * i, b = tb + 16 * j;
      if (a < d && b < d) part[(size_t)blockIdx.x * pairs + a * d + b] = acc[i][j];
    }
}

// ordered sum of the partials: out[j] = scale * sum_b part[b][j]
__global__ void reduce_parts_kernel(const double* part, int nb, int m, double scale, double* out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += part[(size_t)b * m + j];
  out[j] = s * scale;
}

}  // namespace petmetrics

using namespace petmetrics;

static thread_local const char* g_err = "";

extern "C" {

const char* petmetrics_last_error(void) { return g_err; }

int petmetrics_moments(const void* x, int dtype, int64_t n, int d, int ld, double* mean, double* cov, double* work,
                       void* stream) {
  if (!x || !mean || !cov || !work || n < 2 || d <= 0 || ld < d ||
      (dtype != PETMETRICS_F32 && dtype != PETMETRICS_F64)) {
    g_err = "bad arguments (n >= 2, d > 0, ld >= d, dtype PETMETRICS_F32 | PETMETRICS_F64)";
    return 1;
  }
  if (d > 16 * kSub) {
    g_err = "d must be <= 96";
    return 1;
  }
  hipStream_t s = (hipStream_t)stream;
  const int nb = PETMETRICS_BLOCKS;
  const int64_t rows_per = (n + nb - 1) / nb;
  double* part = work;   // [nb][d*d] (>= [nb][d])
  if (dtype == PETMETRICS_F32) hipLaunchKernelGGL(colsum_kernel<float>, dim3(nb), dim3(kThreads), 0, s, x, n, d, ld, rows_per, part);
  else hipLaunchKernelGGL(colsum_kernel<double>, dim3(nb), dim3(kThreads), 0, s, x, n, d, ld, rows_per, part);
  hipLaunchKernelGGL(reduce_parts_kernel, dim3((d + 255) / 256), dim3(256), 0, s, part, nb, d, 1.0 / (double)n, mean);
  const size_t lds = (size_t)kRows * d * sizeof(double);
  if (dtype == PETMETRICS_F32)
    hipLaunchKernelGGL(comoment_kernel<float>, dim3(nb), dim3(kThreads), lds, s, x, n, d, ld, rows_per, mean, part);
  else
    hipLaunchKernelGGL(comoment_kernel<double>, dim3(nb), dim3(kThreads), lds, s, x, n, d, ld, rows_per, mean, part);
  hipLaunchKernelGGL(reduce_parts_kernel, dim3((d * d + 255) / 256), dim3(256), 0, s, part, nb, d * d,
                     1.0 / (double)(n - 1), cov);
  if (hipGetLastError() != hipSuccess) {
    g_err = "kernel launch failed";
    return 2;
  }
  return 0;
}

size_t petmetrics_work_doubles(int d) { return (size_t)PETMETRICS_BLOCKS * (size_t)d * (size_t)d + (size_t)PETMETRICS_BLOCKS * d; }

}  // extern "C"
