// GPU synthetic-TAC generator (include/petsim.h), fp64.
// Restates sample_sim_data.py:139-215 (+ helper_func.py:146-162): truncated
// MvNormal kinetic parameters and reference TAC, SRTM2 activity curves, truncated
// Poisson-like noise.  One 256-thread workgroup per sample.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <set>
#include <string>
#include <vector>
#include "petsim.h"

namespace petsim {

constexpr int NR = 48, NF = 54, NG = 108;    // ROIs, frames, resampling grid (2 x unique frames)
constexpr int kThreads = 256;
constexpr int kMaxAttempts = 1024;           // per rejection loop (the reference loops unbounded)
constexpr int kMaxOuter = 64;                // redraws of (DVR, R1, ref) after a negative TAC

struct Args {
  const double *tv, *dt, *muD, *LD, *muR, *LR, *muC, *LC, *sig;
  double k2p;
  const int* up_i;     // [NG][2] W_up columns (frame indices) of grid point i
  const double* up_w;  // [NG][2]
  const int* dn_i;     // [NF][2] W_down columns (grid indices) of frame f
  const double* dn_w;  // [NF][2]
  const int* y0_j;     // [NG] np.interp segment of grid point i
  const double* xrs;   // [NG]
  double dx;
  uint64_t seed, offset;
  int n;
  double *DVR, *R1, *REF, *TAC, *NOISY;
  float* COND;
  int* ATT;
};

__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

// Normal number `which` (0 cos / 1 sin of the Box-Muller pair) of Philox call `call`
// under tag = purpose << 24 | outer << 12 | inner, for global sample g.
__device__ __forceinline__ double normal(const Args& a, uint64_t g, uint32_t call, uint32_t tag, int which) {
  uint32_t q[4] = {call, tag, (uint32_t)(g & 0xffffffffull), (uint32_t)(g >> 32)};
  philox(q, (uint32_t)(a.seed & 0xffffffffull), (uint32_t)(a.seed >> 32));
  const double u1 = ((double)q[0] + 1.0) * 2.3283064365386963e-10;
  const double u2 = ((double)q[1] + 0.5) * 2.3283064365386963e-10;
  const double r = sqrt(-2.0 * log(u1));
  return which ? r * sinpi(2.0 * u2) : r * cospi(2.0 * u2);
}

// helper_func.truncnormal_samples for one vector: redraw until every component >= 0.
// Thread i < d owns component i; out in LDS.  Returns the draws used (-1: cap hit).
__device__ int draw_truncated_mvn(const Args& a, uint64_t g, int purpose, int outer, const double* mu,
                                  const double* L, int d, double* z, double* out) {
  const int tid = threadIdx.x;
  for (int inner = 0; inner < kMaxAttempts; ++inner) {
    const uint32_t tag = ((uint32_t)purpose << 24) | ((uint32_t)outer << 12) | (uint32_t)inner;
    if (tid < d) z[tid] = normal(a, g, (uint32_t)(tid >> 1), tag, tid & 1);
    __syncthreads();
    double x = 0.0;
    if (tid < d) {
      x = mu[tid];
      for (int k = 0; k <= tid; ++k) x = fma(L[tid * d + k], z[k], x);   // mu + L z, L lower
      out[tid] = x;
    }
    const int neg = __syncthreads_or(tid < d && x < 0.0);
    if (!neg) return inner + 1;
  }
  return -1;
}

__global__ __launch_bounds__(kThreads) void sim_kernel(Args a) {
  const int b = blockIdx.x;
  if (b >= a.n) return;
  const uint64_t g = a.offset + (uint64_t)b;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  __shared__ double z[64], dvr[NR], r1[NR], ref[64], y0[NG];
  __shared__ double e[4][64], y1[4][NG], conv[4][NG];
  __shared__ double tac[NR * NF];
  int used = 0;
  bool capped = false;
  for (int outer = 0; outer < kMaxOuter; ++outer) {
    const int u1 = draw_truncated_mvn(a, g, 0, outer, a.muD, a.LD, NR, z, dvr);
    const int u2 = draw_truncated_mvn(a, g, 1, outer, a.muR, a.LR, NR, z, r1);
    const int u3 = draw_truncated_mvn(a, g, 2, outer, a.muC, a.LC, NF, z, ref);
    capped = capped || u1 < 0 || u2 < 0 || u3 < 0;
    used += (u1 > 0 ? u1 : kMaxAttempts) + (u2 > 0 ? u2 : kMaxAttempts) + (u3 > 0 ? u3 : kMaxAttempts);
    // y0 = np.interp(x_rs, t, ref) (kinetic_model.py:25)
    if (tid < NG) {
      const int j = a.y0_j[tid];
      const double x = a.xrs[tid];
      y0[tid] = j >= NF - 1 ? ref[NF - 1] : (ref[j + 1] - ref[j]) / (a.tv[j + 1] - a.tv[j]) * (x - a.tv[j]) + ref[j];
    }
    __syncthreads();
    bool neg = false;
    for (int r = w; r < NR; r += 4) {              // one wave per ROI (kinetic_model.py:142-158)
      const double R = r1[r], k2 = a.k2p * R, k2a = k2 / dvr[r];
      e[w][lane] = lane < NF ? exp(-k2a * a.tv[lane]) : 0.0;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      for (int i = lane; i < NG; i += 64)          // y1 = interp1d_linear_vec(x_rs, t, exp) (:26)
        y1[w][i] = a.up_w[2 * i] * e[w][a.up_i[2 * i]] + a.up_w[2 * i + 1] * e[w][a.up_i[2 * i + 1]];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      for (int i = lane; i < NG; i += 64) {        // causal convolution * dx (:28-31)
        double s = 0.0;
        for (int j = 0; j <= i; ++j) s = fma(y0[j], y1[w][i - j], s);
        conv[w][i] = s * a.dx;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      if (lane < NF) {                              // back to the frames (:32), SRTM2 (:157-158), * dt
        const double cv = a.dn_w[2 * lane] * conv[w][a.dn_i[2 * lane]] +
                          a.dn_w[2 * lane + 1] * conv[w][a.dn_i[2 * lane + 1]];
        const double v = (R * ref[lane] + (k2 - R * k2a) * cv) * a.dt[lane];
        tac[r * NF + lane] = v;
        neg = neg || v < 0.0;
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (!__syncthreads_or(neg)) break;             // sample_sim_data.py:175-181: redraw all three
    if (outer == kMaxOuter - 1) capped = true;
  }
  // truncated noise: noisy/dt = x/dt + sqrt(x/dt) * TN(0, sigma, low = -sqrt(x/dt))  (:202-209)
  for (int idx = tid; idx < NR * NF; idx += kThreads) {
    const int f = idx % NF;
    const double xc = tac[idx] / a.dt[f];
    const double s = sqrt(xc), sd = a.sig[idx];
    double nz = 0.0;
    int k = 0;
    for (; k < kMaxAttempts; ++k) {
      nz = sd * normal(a, g, (uint32_t)idx, (3u << 24) | (uint32_t)k, 0);
      if (nz >= -s) break;
    }
    if (k == kMaxAttempts) capped = true;
    const double noisy_c = xc + s * nz;
    if (a.NOISY) a.NOISY[(size_t)b * NR * NF + idx] = noisy_c * a.dt[f];
    if (a.TAC) a.TAC[(size_t)b * NR * NF + idx] = tac[idx];
    if (a.COND) a.COND[(size_t)b * (NR + 1) * NF + idx] = (float)noisy_c;    // tac_noisy / dt rows
  }
  if (a.COND && tid < NF) a.COND[(size_t)b * (NR + 1) * NF + NR * NF + tid] = (float)ref[tid];
  if (a.DVR && tid < NR) a.DVR[(size_t)b * NR + tid] = dvr[tid];
  if (a.R1 && tid < NR) a.R1[(size_t)b * NR + tid] = r1[tid];
  if (a.REF && tid < NF) a.REF[(size_t)b * NF + tid] = ref[tid];
  const int any_cap = __syncthreads_or(capped);
  if (a.ATT && tid == 0) a.ATT[b] = any_cap ? -1 : used;
}

}  // namespace petsim

using namespace petsim;

namespace {

thread_local std::string g_err;

int fail(const std::string& m, int code = 1) {
  g_err = m;
  return code;
}

// Lower Cholesky factor L (row-major) of a symmetric positive SEMI-definite A, L L^T = A: a pivot
// s <= 1e-12 max diag(A) is a direction of (numerically) zero variance, so its column of L is zero.
// The reference's Cov_tac_ref (prior_stats_nROI48) has rank 49 of 54 and np.random.multivariate_normal
// (helper_func.py:158) accepts it (SVD factor); this factor draws the same distribution.
// false if A is not positive semi-definite (a pivot below -tol) or not finite.
bool cholesky(const double* A, int n, std::vector<double>& L) {
  L.assign((size_t)n * n, 0.0);
  double dmax = 0.0;
  for (int i = 0; i < n; ++i) dmax = std::max(dmax, A[(size_t)i * n + i]);
  const double tol = 1e-12 * dmax;
  if (!(dmax > 0.0) || !std::isfinite(dmax)) return false;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = A[(size_t)i * n + j];
      for (int k = 0; k < j; ++k) s -= L[(size_t)i * n + k] * L[(size_t)j * n + k];
      if (i == j) {
        if (!std::isfinite(s) || s < -1e-8 * dmax) return false;
        L[(size_t)i * n + i] = s > tol ? std::sqrt(s) : 0.0;
      } else {
        const double d = L[(size_t)j * n + j];
        L[(size_t)i * n + j] = d > 0.0 ? s / d : 0.0;
      }
    }
  return true;
}

// interp1d_linear_vec weights as (column pair, weight pair) per row (kinetic_model.py:42-49,
// including the searchsorted - 1 == -1 wrap of the first point)
void interp_pairs(const std::vector<double>& x, const std::vector<double>& xp, std::vector<int>& ci,
                  std::vector<double>& cw) {
  const int n = (int)x.size(), m = (int)xp.size();
  ci.assign(2 * n, 0);
  cw.assign(2 * n, 0.0);
  for (int i = 0; i < n; ++i) {
    const int idx = (int)(std::lower_bound(xp.begin(), xp.end(), x[i]) - xp.begin());
    const int i0 = idx % m, i1 = (idx - 1 + m) % m;
    const double w0 = std::fabs(xp[i1] - x[i]), w1 = std::fabs(xp[i0] - x[i]);
    const double s = w0 + w1;
    ci[2 * i] = i0;
    ci[2 * i + 1] = i1;
    cw[2 * i] = w0 / s;
    cw[2 * i + 1] = w1 / s;
  }
}

struct DBuf {
  void* p = nullptr;
  ~DBuf() { if (p) (void)hipFree(p); }
};

template <typename T>
hipError_t up(DBuf& b, const T* h, size_t n) {
  hipError_t e = hipMalloc(&b.p, n * sizeof(T));
  if (e != hipSuccess) return e;
  return hipMemcpy(b.p, h, n * sizeof(T), hipMemcpyHostToDevice);
}

}  // namespace

extern "C" {

const char* petsim_last_error(void) { return g_err.c_str(); }

int petsim_generate(const petsim_prior* p, uint64_t seed, uint64_t sample_offset, int n, int device, double* DVR,
                    double* R1, double* REF, double* TAC, double* NOISY, float* COND, int32_t* ATT, void* stream) {
  if (!p || n < 0) return fail("bad arguments");
  if (p->n_roi != NR || p->n_frames != NF) return fail("compiled for 48 ROIs x 54 frames");
  if (!p->time_vector || !p->dt || !p->mu_DVR || !p->cov_DVR || !p->mu_R1 || !p->cov_R1 || !p->mu_ref ||
      !p->cov_ref || !p->sigma_noise)
    return fail("null prior array");
  if (n == 0) return 0;
  std::vector<double> LD, LR, LC;
  if (!cholesky(p->cov_DVR, NR, LD) || !cholesky(p->cov_R1, NR, LR) || !cholesky(p->cov_ref, NF, LC))
    return fail("prior covariance is not positive semi-definite");
  std::vector<double> t(p->time_vector, p->time_vector + NF);
  std::set<double> uniq(t.begin(), t.end());
  if ((int)uniq.size() * 2 != NG) return fail("frame times must be 54 distinct values");
  const double lo = *std::min_element(t.begin(), t.end()), hi = *std::max_element(t.begin(), t.end());
  std::vector<double> xrs(NG);
  for (int i = 0; i < NG; ++i) xrs[i] = lo + i * ((hi - lo) / (NG - 1));
  xrs[NG - 1] = hi;
  std::vector<int> y0j(NG);
  for (int i = 0; i < NG; ++i) {   // np.interp segment: t[j] <= x < t[j+1] (last point -> NF-1)
    int j = (int)(std::upper_bound(t.begin(), t.end(), xrs[i]) - t.begin()) - 1;
    y0j[i] = std::max(0, std::min(j, NF - 1));
  }
  std::vector<int> ui, di;
  std::vector<double> uw, dw;
  interp_pairs(xrs, t, ui, uw);    // W_up   [NG] rows over frames
  interp_pairs(t, xrs, di, dw);    // W_down [NF] rows over grid points
  if (hipSetDevice(device) != hipSuccess) return fail("hipSetDevice failed", 2);
  DBuf bLD, bLR, bLC, bui, buw, bdi, bdw, by0, bx, btv, bdt, bmuD, bmuR, bmuC, bsig;
  hipError_t e = hipSuccess;
  if ((e = up(bLD, LD.data(), LD.size())) || (e = up(bLR, LR.data(), LR.size())) ||
      (e = up(bLC, LC.data(), LC.size())) || (e = up(bui, ui.data(), ui.size())) ||
      (e = up(buw, uw.data(), uw.size())) || (e = up(bdi, di.data(), di.size())) ||
      (e = up(bdw, dw.data(), dw.size())) || (e = up(by0, y0j.data(), y0j.size())) ||
      (e = up(bx, xrs.data(), xrs.size())) || (e = up(btv, p->time_vector, NF)) || (e = up(bdt, p->dt, NF)) ||
      (e = up(bmuD, p->mu_DVR, NR)) || (e = up(bmuR, p->mu_R1, NR)) || (e = up(bmuC, p->mu_ref, NF)) ||
      (e = up(bsig, p->sigma_noise, (size_t)NR * NF)))
    return fail(std::string("upload: ") + hipGetErrorString(e), 2);
  Args a{};
  a.tv = (const double*)btv.p;
  a.dt = (const double*)bdt.p;
  a.muD = (const double*)bmuD.p;
  a.LD = (const double*)bLD.p;
  a.muR = (const double*)bmuR.p;
  a.LR = (const double*)bLR.p;
  a.muC = (const double*)bmuC.p;
  a.LC = (const double*)bLC.p;
  a.sig = (const double*)bsig.p;
  a.k2p = p->k2p;
  a.up_i = (const int*)bui.p;
  a.up_w = (const double*)buw.p;
  a.dn_i = (const int*)bdi.p;
  a.dn_w = (const double*)bdw.p;
  a.y0_j = (const int*)by0.p;
  a.xrs = (const double*)bx.p;
  a.dx = xrs[1] - xrs[0];
  a.seed = seed;
  a.offset = sample_offset;
  a.n = n;
  a.DVR = DVR; a.R1 = R1; a.REF = REF; a.TAC = TAC; a.NOISY = NOISY; a.COND = COND; a.ATT = ATT;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sim_kernel, dim3(n), dim3(kThreads), 0, s, a);
  if ((e = hipGetLastError()) != hipSuccess) return fail(std::string("launch: ") + hipGetErrorString(e), 2);
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return fail(std::string("sync: ") + hipGetErrorString(e), 2);
  return 0;
}

}  // extern "C"
