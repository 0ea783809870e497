/*
 * petmh.h -- C ABI of the MI355X Metropolis-Hastings baseline (libpetdiff.so).
 *
 * Replaces the reference's MCMC baseline (yanisdjebra/PET_posterior_distribution):
 *
 *   SRTM2.create_activity_curve   kinetic_model.py:142-158 (+ :12-57)  -> petmh_srtm2_tac
 *   CreateTAC_SRTM2.perform       mcmc.py:27-39                         -> petmh_srtm2_tac
 *   pm.Model log density          mcmc.py:147-155                       -> petmh_logp
 *   pm.sample(Metropolis(NormalProposal), draws, tune)  mcmc.py:156-157 -> petmh_run
 *
 * Model (mcmc.py:147-155): DVR ~ MvNormal(mu_DVR, Cov_DVR), R1 ~ MvNormal(mu_R1,
 * Cov_R1) (48-d each), k2' fixed, sn = SRTM2(DVR, R1, k2').T with sn < 0 -> 1e-6,
 * y_obs ~ TruncatedNormal(mu = sn, sigma = sqrt(sn) * sigma_noise, lower = 0).
 * Sampler: PyMC 5.12 Metropolis with NormalProposal (Metropolis.astep with
 * elemwise_update): per draw one proposal vector delta = N(0,1) * scaling over the
 * 96 coordinates (DVR | R1), the coordinates visited in a freshly shuffled order,
 * each coordinate's log ratio taken against the sweep-start point (pymc's
 * delta_logp(q_temp, q0)) and accepted iff finite and log u < ratio
 * (metrop_select); per-element scaling tuned every 100 tuning draws with PyMC's
 * tune table.  PyMC is not vendored in the reference: this restates its
 * published source (parity with PyMC itself unpinned).  One 64-lane wavefront per chain (lane = frame /
 * ROI), fp64 throughout (mcmc.py:22).  Draws are reduced on the GPU into
 * per-chain Welford accumulators instead of being stored.
 *
 * SRTM2 numerics: the convolution of kinetic_model.py:12-32 is linear in the
 * frame-sampled exponential, so it is applied as the constant 54 x 54 operator
 * M = W_down . Toeplitz(interp(C_r)) . W_up . dx (exact reassociation, fp64).
 */
#ifndef PETMH_H
#define PETMH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct petmh_ctx* petmh_handle;

typedef struct petmh_problem {
  int n_roi;                  /* 48 */
  int n_frames;               /* 54 */
  const double* time_vector;  /* [n_frames] frame end times (min)       mcmc.py:73     */
  const double* tac_ref;      /* [n_frames] reference TAC               mcmc.py:134    */
  double k2p;                 /* fixed k2' (true value)                  mcmc.py:150    */
  const double* y_obs;        /* [n_roi][n_frames] tac_noisy / dt       mcmc.py:79, 109 */
  const double* sigma_noise;  /* [n_roi][n_frames]                       mcmc.py:96     */
  const double* mu_DVR;       /* [n_roi]                                 mcmc.py:87     */
  const double* cov_DVR;      /* [n_roi][n_roi]                          mcmc.py:88     */
  const double* mu_R1;        /* [n_roi]                                 mcmc.py:90     */
  const double* cov_R1;       /* [n_roi][n_roi]                          mcmc.py:91     */
} petmh_problem;

/* Batched SRTM2 forward on the GPU: DVR_dev, R1_dev [n][n_roi] -> tac_dev
 * [n][n_roi][n_frames] (the mcmc.py:39 orientation).  Host time_vector/tac_ref.
 * k2p_dev: [n] per-row k2' values. */
int petmh_srtm2_tac(const double* time_vector, const double* tac_ref, const double* DVR_dev, const double* R1_dev,
                    int n, int n_roi, const double* k2p_dev, double* tac_dev, void* stream);

/* Copies the problem to `device` and precomputes the SRTM2 operator and the prior
 * precision matrices. */
int petmh_create(const petmh_problem* p, int device, petmh_handle* out);
int petmh_destroy(petmh_handle h);

/* Runs n_chains independent chains for n_tune + n_draws Metropolis iterations.
 * x0_dev: [n_chains][2*n_roi] initial (DVR | R1) or NULL (prior means).
 * stats_dev: [n_chains][2*n_roi][3] {count, mean, M2} over the kept draws.
 * accept_dev: [n_chains][2*n_roi] acceptance counts over the kept draws (may be NULL).
 * last_dev: [n_chains][2*n_roi] final state (may be NULL). */
int petmh_run(petmh_handle h, const double* x0_dev, int n_chains, int n_draws, int n_tune, uint64_t seed,
              double* stats_dev, double* accept_dev, double* last_dev, void* stream);

/* petmh_run that also writes the kept draws (the reference's idata trace,
 * mcmc.py:157-165): draws_dev [n_chains][n_draws][2*n_roi] fp64 (DVR | R1). */
int petmh_run_draws(petmh_handle h, const double* x0_dev, int n_chains, int n_draws, int n_tune, uint64_t seed,
                    double* stats_dev, double* accept_dev, double* last_dev, double* draws_dev, void* stream);

/* Sampler options (defaults = pymc Metropolis: tune_interval 100, scaling 1.0,
 * vs_sweep_start 1).  vs_sweep_start 0 compares each element against the running
 * state instead (textbook component-wise MH). */
int petmh_set_sampler(petmh_handle h, int tune_interval, double scaling, int vs_sweep_start);

/* Chain kernel (no reference counterpart: how the GPU runs mcmc.py:156-157's sampler).
 *   kernel 0 = automatic (batched for <= 256 chains, else one update at a time),
 *          1 = one element update at a time (one wave per chain),
 *          2 = batched proposals (the 144 likelihoods a sweep can need, evaluated up front,
 *              then a scan over the shuffled order; latency-optimised).
 *   waves_per_chain (batched kernel only): 0 = automatic, or 1, 2, 4, 12.
 * Both kernels take the same accept/reject path up to the summation order over frames. */
int petmh_set_kernel(petmh_handle h, int kernel, int waves_per_chain);

/* Joint log density of mcmc.py:147-155 at n points x_dev [n][2*n_roi] -> out_dev [n]. */
int petmh_logp(petmh_handle h, const double* x_dev, int n, double* out_dev, void* stream);

const char* petmh_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PETMH_H */
