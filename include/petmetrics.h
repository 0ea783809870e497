/*
 * petmetrics.h -- C ABI of the GPU posterior-accuracy metrics (libpetdiff.so).
 *
 * the metrics step after the reverse loop, main_script.py:719-758.
 * For each kinetic parameter the reference computes, over the posterior samples of
 * the iDDPM and of the MCMC trace: np.mean, np.cov (ddof = 1), np.corrcoef, the
 * per-ROI std sqrt(diag(cov)) and their relative differences.  This library
 * computes the mean and the full sample covariance of an (n x d) sample matrix on
 * the GPU; the host (pet_posterior_distribution_amd/metrics.py) derives the rest.
 */
#ifndef PETMETRICS_H
#define PETMETRICS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PETMETRICS_F32 0
#define PETMETRICS_F64 1
#define PETMETRICS_BLOCKS 128       /* row blocks of the deterministic reduction */

/* x_dev: n rows of d values (row stride ld elements, fp32 or fp64), device.
 * mean_dev [d], cov_dev [d][d] (ddof = 1), fp64 device outputs; work_dev holds
 * petmetrics_work_doubles(d) doubles.  Requires n >= 2, d <= 96. */
int petmetrics_moments(const void* x_dev, int dtype, int64_t n, int d, int ld, double* mean_dev, double* cov_dev,
                       double* work_dev, void* stream);
size_t petmetrics_work_doubles(int d);
const char* petmetrics_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PETMETRICS_H */
