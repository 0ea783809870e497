/*
 * petsim.h -- C ABI of the GPU synthetic-TAC generator (libpetdiff.so), SURVEY.md
 * 8(f) row 3: the data step before the posterior path, restating
 * sample_sim_data.py:139-215 with helper_func.py:146-162.
 *
 * Per sample g (global index sample_offset + b), fp64:
 *   DVR ~ MvNormal(mu_DVR, Cov_DVR) | all > 0     (helper_func.truncnormal_samples,
 *   R1  ~ MvNormal(mu_R1,  Cov_R1)  | all > 0      rejection, :157-162)
 *   ref ~ MvNormal(mu_ref, Cov_ref) | all > 0      (sample_sim_data.py:139-161)
 *   tac = SRTM2(DVR, R1, k2p, ref) * dt            (:170-183; negative TAC -> redraw all three)
 *   noisy/dt = tac/dt + sqrt(tac/dt) * TN(0, sigma_noise[r][f], low = -sqrt(tac/dt))   (:196-211)
 * sigma_noise [n_roi][n_frames] is the dataset's per-ROI/frame noise std (:190-194),
 * drawn once per dataset by the caller.  Normal draws: Philox4x32-10 keyed by seed,
 * counter (call, purpose/attempt, g_lo, g_hi), Box-Muller pairs; the truncated noise
 * and the positivity constraints by rejection (the reference's scipy truncnorm and
 * resampling loops draw the same distributions from a different stream).  The
 * reference's optional testing-set acceptance test (alpha, :127-135) is not restated.
 */
#ifndef PETSIM_H
#define PETSIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct petsim_prior {
  int n_roi;                 /* 48 */
  int n_frames;              /* 54 */
  const double* time_vector; /* [n_frames] frame end times (min) */
  const double* dt;          /* [n_frames] frame durations (min) */
  const double* mu_DVR;      /* [n_roi] */
  const double* cov_DVR;     /* [n_roi][n_roi] */
  const double* mu_R1;       /* [n_roi] */
  const double* cov_R1;      /* [n_roi][n_roi] */
  const double* mu_ref;      /* [n_frames] reference-TAC mean */
  const double* cov_ref;     /* [n_frames][n_frames] */
  double k2p;                /* fixed k2' (sample_sim_data.py:150-154) */
  const double* sigma_noise; /* [n_roi][n_frames] */
} petsim_prior;

/* Generates n samples on `device`.  Device outputs (any may be NULL):
 *   DVR_dev, R1_dev [n][n_roi]; ref_dev [n][n_frames];
 *   tac_dev, noisy_dev [n][n_roi][n_frames] (activity, i.e. * dt, as the reference saves);
 *   cond_dev [n][n_roi + 1][n_frames] fp32: the network condition [noisy / dt | ref]
 *     (main_script.py:107-113);
 *   attempts_dev [n] int32: redraws used (a sample that hit the attempt cap is
 *     marked with -1 and holds its last draw). */
int petsim_generate(const petsim_prior* prior, uint64_t seed, uint64_t sample_offset, int n, int device,
                    double* DVR_dev, double* R1_dev, double* ref_dev, double* tac_dev, double* noisy_dev,
                    float* cond_dev, int32_t* attempts_dev, void* stream);
const char* petsim_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PETSIM_H */
