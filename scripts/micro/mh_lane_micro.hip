// north_star's MH design point, measured on its dominant cost (diagnostic, not the product; DESIGN.md
// section 5, "one lane per chain").
//
// north_star asks for one lane per chain.  The product runs one wavefront per chain
// (mh_kernels.hip mh_chain_batched): 144 ROI log-likelihood evaluations per draw, dealt to the lanes.
// This micro times the same evaluations with one chain per LANE.  Every lane evaluates its own chain's
// (DVR, R1) of ROI i, for the 144 evaluations of a draw, in the product's order:
//   e_g = exp(-k2a t_g) (54 per lane, in registers);
//   conv_f = sum_g M[f][g] e_g, with the operator rows broadcast from LDS (one address for every lane);
//   then the product's per-frame truncated-normal terms: sqrt, one division, log, and the
//   log-Phi polynomial.
// The operator is a lower-triangular stand-in with the real problem's time grid and reference TAC
// (scripts/micro/mh_problem.bin).  Its values only steer branches of equal cost, so this is a timing
// harness, not a parity one.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../pet_posterior_distribution_amd/csrc
//        mh_lane_micro.hip -o mh_lane_micro
// Run:   ./mh_lane_micro mh_problem.bin   -> evaluations/s and the implied chain-steps/s (1 draw = 144
//        evaluations) at 10k chains (configs[2]) and at 64k / 256k chains (a full chip of lanes).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "logphi_coef.h"
#include "fp64_math.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int NF = 54, NR = 48, MLD = 56, NEVAL = 144;
constexpr int LPNI = PETMH_LOGPHI_NI, LPLD = 18;
__constant__ double c_logphi[LPNI][PETMH_LOGPHI_DEG + 1] = PETMH_LOGPHI_COEF;

struct Prob {
  const double *M, *TV, *CR, *Y, *SIG;   // M [f][MLD], Y / SIG [roi][f]
  double k2p;
};

__device__ __forceinline__ double log_phi_poly(const double* tab, double x) {
  int k = (int)x;
  k = k < 0 ? 0 : (k > LPNI - 1 ? LPNI - 1 : k);
  const double u = x - ((double)k + 0.5);
  const double2* row = reinterpret_cast<const double2*>(tab + k * LPLD);
  double p = row[7].x;
#pragma unroll
  for (int j = 6; j >= 0; --j) {
    const double2 cc = row[j];
    p = fma(p, u, cc.y);
    p = fma(p, u, cc.x);
  }
  return p;
}

// one chain per lane: `draws` x 144 evaluations; out[chain] = the sum of its log-likelihoods
__global__ __launch_bounds__(64) void lane_chain_evals(Prob p, const double* dvr0, const double* r10, int n, int draws,
                                                       double* out) {
  __shared__ alignas(16) double M[NF * MLD];
  __shared__ alignas(16) double LPHI[LPNI * LPLD];
  __shared__ double TV[NF], CR[NF];
  for (int k = threadIdx.x; k < NF * MLD; k += 64) M[k] = p.M[k];
  for (int k = threadIdx.x; k < LPNI * LPLD; k += 64) {
    const int r = k / LPLD, j = k - r * LPLD;
    LPHI[k] = j <= PETMH_LOGPHI_DEG ? c_logphi[r][j] : 0.0;
  }
  for (int k = threadIdx.x; k < NF; k += 64) { TV[k] = p.TV[k]; CR[k] = p.CR[k]; }
  __syncthreads();
  const int chain = blockIdx.x * 64 + threadIdx.x;
  const int ch = chain < n ? chain : n - 1;
  double acc = 0.0;
  for (int d = 0; d < draws; ++d) {
    for (int q = 0; q < NEVAL; ++q) {
      const int i = q % NR;                                  // ROI (uniform across the wave)
      const double dvr = dvr0[(size_t)ch * NR + i] * (1.0 + 1e-3 * (q / NR)), r1 = r10[(size_t)ch * NR + i];
      const double k2 = p.k2p * r1, k2a = k2 / dvr;
      double e[MLD];
#pragma unroll
      for (int g = 0; g < NF; ++g) e[g] = exp(-k2a * TV[g]);
      e[54] = e[55] = 0.0;
      double l = 0.0;
      for (int f = 0; f < NF; ++f) {
        const double2* mrow = reinterpret_cast<const double2*>(M + f * MLD);
        double c0 = 0.0, c1 = 0.0;
#pragma unroll
        for (int g = 0; g < MLD / 2; ++g) {
          const double2 m = mrow[g];
          c0 = fma(m.x, e[2 * g], c0);
          c1 = fma(m.y, e[2 * g + 1], c1);
        }
        const double conv = c0 + c1;
        const double tac = r1 * CR[f] + (k2 - r1 * k2a) * conv;
        const double sn = tac < 0.0 ? 1e-6 : tac;
        const double sig = sqrt(sn) * p.SIG[i * NF + f];
        const double inv = 1.0 / sig;
        const double z = (p.Y[i * NF + f] - sn) * inv;
        const double xs = sn * inv;
        const double lnd = xs < 10.0 ? log_phi_poly(LPHI, xs) : 0.0;
        l += -0.5 * z * z - 0.9189385332046727 - log_pos(sig) - lnd;
      }
      acc += l;
    }
  }
  if (chain < n) out[chain] = acc;
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "mh_problem.bin";
  std::vector<double> d(54 + 54 + 1 + 48 * 54 * 2 + 48 * 2 + 48 * 48 * 2);
  FILE* f = fopen(path, "rb");
  if (!f || fread(d.data(), 8, d.size(), f) != d.size()) { printf("bad problem file\n"); return 1; }
  fclose(f);
  const double *tv = d.data(), *cr = tv + 54, k2p = cr[54], *y = cr + 55, *sg = y + NR * NF;
  const double *mud = sg + NR * NF, *mur = mud + NR + NR * NR;
  // lower-triangular stand-in operator: trapezoid weights of the frame grid times the reference TAC
  std::vector<double> M(NF * MLD, 0.0);
  for (int fr = 0; fr < NF; ++fr)
    for (int g = 0; g <= fr; ++g) {
      const double dt = g == 0 ? tv[0] : tv[g] - tv[g - 1];
      M[fr * MLD + g] = cr[fr - g] * dt;
    }
  const int nmax = 262144;
  std::vector<double> dv((size_t)nmax * NR), rv((size_t)nmax * NR);
  for (size_t c = 0; c < (size_t)nmax; ++c)
    for (int i = 0; i < NR; ++i) {
      const double u = ((c * 2654435761u + i * 40503u) % 1000) / 1000.0 - 0.5;
      dv[c * NR + i] = mud[i] * (1.0 + 0.05 * u);
      rv[c * NR + i] = mur[i] * (1.0 - 0.05 * u);
    }
  double *dM, *dTV, *dCR, *dY, *dS, *dD, *dR, *dOut;
  CK(hipMalloc(&dM, M.size() * 8)); CK(hipMemcpy(dM, M.data(), M.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&dTV, NF * 8)); CK(hipMemcpy(dTV, tv, NF * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&dCR, NF * 8)); CK(hipMemcpy(dCR, cr, NF * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&dY, NR * NF * 8)); CK(hipMemcpy(dY, y, NR * NF * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&dS, NR * NF * 8)); CK(hipMemcpy(dS, sg, NR * NF * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&dD, dv.size() * 8)); CK(hipMemcpy(dD, dv.data(), dv.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&dR, rv.size() * 8)); CK(hipMemcpy(dR, rv.data(), rv.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&dOut, (size_t)nmax * 8));
  Prob p{dM, dTV, dCR, dY, dS, k2p};
  auto run = [&](int n, int draws) {
    const int grid = (n + 63) / 64;
    lane_chain_evals<<<grid, 64>>>(p, dD, dR, n, 1, dOut);   // warm-up
    CK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    lane_chain_evals<<<grid, 64>>>(p, dD, dR, n, draws, dOut);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::vector<double> o(n);
    CK(hipMemcpy(o.data(), dOut, n * 8, hipMemcpyDeviceToHost));
    double cs = 0.0;
    int bad = 0;
    for (double v : o) { if (!std::isfinite(v)) ++bad; else cs += v; }
    const double evals = (double)n * draws * NEVAL;
    printf("lane-per-chain  chains %6d  waves %5d  draws %3d  %.3f s  %.3e evals/s  %.3e chain-steps/s  (checksum %.6e, %d non-finite)\n",
           n, grid, draws, s, evals / s, evals / s / NEVAL, cs, bad);
  };
  run(10000, 20);
  run(65536, 4);
  run(262144, 2);
  return 0;
}
