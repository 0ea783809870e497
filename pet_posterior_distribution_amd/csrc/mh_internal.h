// Internal declarations of the Metropolis-Hastings / SRTM2 kernels (mh_kernels.hip)
// shared with their C-ABI host code (mh_api.cpp).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace petmh {

constexpr int kNRoi = 48;      // ROIs (mcmc.py:53)
constexpr int kNFrames = 54;   // frames (sample_sim_data.py:29-85)

struct MHConst {               // device pointers, fp64
  const double* M;             // [54][54] SRTM2 operator, [g][f]
  const double* PD;            // [48][48] inverse Cov_DVR
  const double* PR;            // [48][48] inverse Cov_R1
  const double* Y;             // [48][54]
  const double* SIG;           // [48][54]
  const double* CR;            // [54]
  const double* TV;            // [54]
  const double* MUD;           // [48]
  const double* MUR;           // [48]
  double k2p;
  double prior_const;          // -0.5 (2k log 2pi + logdet Cov_D + logdet Cov_R)
};

struct MHRun {
  const double* x0;            // [n_chains][96] or null
  int n_chains, n_draws, n_tune, tune_interval;
  int vs_sweep_start;          // pymc 5.12: ratios against the sweep-start point
  double scaling;
  unsigned long long seed;
  double* stats;               // [n_chains][96][3]
  double* accept;              // [n_chains][96] or null
  double* last;                // [n_chains][96] or null
  double* draws;               // [n_chains][n_draws][96] or null (kept draws)
  int kernel;                  // petmh_set_kernel: 0 auto, 1 one update at a time, 2 batched
  int wpc;                     // batched: waves per chain (0 auto)
};

hipError_t launch_mh_chains(const MHConst& c, const MHRun& r, hipStream_t s);
hipError_t launch_mh_logp(const MHConst& c, const double* x, int n, double* out, hipStream_t s);
hipError_t launch_srtm2(const double* M, const double* cr, const double* tv, const double* dvr, const double* r1,
                        const double* k2p, int n, int n_roi, double* tac, hipStream_t s);

}  // namespace petmh
