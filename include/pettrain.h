/*
 * pettrain.h -- C ABI of the MI355X training step of the iDDPM denoiser
 * (libpetdiff.so), SURVEY.md 8(f) row 4: the step before the posterior path,
 * producing weights on MI355X.
 *
 * Replaces (reference file:line, yanisdjebra/PET_posterior_distribution @ 2025-08-29):
 *   ImprovedDDPM.train_step          diffusion_model.py:533-598
 *                                    -> pettrain_step (= pettrain_compute_gradients
 *                                       + pettrain_apply_gradients)
 *   ImprovedDDPM.test_step           diffusion_model.py:600-640 -> pettrain_compute_loss
 *   _vb_terms_bpd / normal_kl /      diffusion_model.py:498-531, networks.py:29-80
 *   discretized_gaussian_log_likelihood
 *   compile(Adam(ExponentialDecay,   main_script.py:169-192, 233-234
 *           clipnorm), 'MeanSquaredError')  -> pettrain_config
 *
 * Objective (what tf.GradientTape differentiates): loss is the [B] vector
 * mse + vlb_b, and the gradient of a vector is the gradient of its SUM, so
 * J = B * mean((target - pred)^2) + sum_b lambda_vlb * vb_terms_bpd_b, with the
 * VLB seeing the prediction through stop_gradient (learned variance only).
 * Optimizer: Keras Adam, each variable's gradient clipped to norm <= clipnorm
 * first, learning rate lr0 * decay_rate^(iterations / decay_steps).
 *
 * Numerics: fp32 everywhere (the reference trains fp32).  Convolutions run as
 * im2col + rocBLAS fp32 GEMMs (forward Y = A W, weight grad A^T dY, data grad
 * dY W^T then col2im); residual 1x1 convs are folded into the centre tap
 * (their gradient is the centre tap's).  Everything else is hand-written HIP.
 *
 * Random draws (t ~ U{0..T-1}, noise ~ N(0,1)) are Philox4x32-10 keyed by
 * `seed`, counter (purpose, iteration, sample_offset + b): bitwise independent
 * of how a global batch is split across ranks.  Tests inject t / noise.
 *
 * Device pointers (*_dev) belong to the handle's device and the caller.
 */
#ifndef PETTRAIN_H
#define PETTRAIN_H

#include <stddef.h>
#include <stdint.h>

#include "petdiff.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pettrain_config {
  float learning_rate;   /* ExponentialDecay initial_learning_rate (main_script.py:170: 2e-4) */
  float decay_steps;     /* lr = learning_rate * decay_rate^(iterations / decay_steps)         */
  float decay_rate;      /* 1 -> constant learning rate                                        */
  float beta_1;          /* Keras Adam defaults 0.9, 0.999, 1e-7                               */
  float beta_2;
  float epsilon;
  float clipnorm;        /* per-variable clip_by_norm (main_script.py:174: 1.5); <= 0 off      */
  float lambda_vlb;      /* diffusion_model lambda_vlb (main_script.py:185: 0.1)               */
} pettrain_config;

typedef struct pettrain_ctx* pettrain_handle;

/* Fills the shipped compile arguments (main_script.py:169-192), constant lr. */
int pettrain_default_config(pettrain_config* opt);

/* net: the network config (petdiff.h, shipped architecture; dtype ignored: fp32).
 * weights: host fp32 blob in the petdiff.h order; tab: host [PETDIFF_NTAB][T]
 * schedule table (as petdiff_set_schedule).  Adam moments start at zero. */
int pettrain_create(const petdiff_config* net, const float* weights, size_t n_weights, const float* tab, int T,
                    const pettrain_config* opt, int device, pettrain_handle* out);
void pettrain_destroy(pettrain_handle h);

/* Forward + loss + backward of one batch.
 *   x0_dev [B][n_roi][n_par] (the training "images"), cond_dev [B][49][54];
 *   t_dev [B] int32 or NULL (drawn), noise_dev [B][n_roi][n_par] or NULL (drawn);
 *   seed / sample_offset select the draws (see above; iteration = pettrain_iterations);
 *   loss_dev [B] or NULL: per-sample loss mse + vlb_b (the reference's `loss`);
 * Leaves the raw (unclipped) gradients in the handle (pettrain_gradients). */
int pettrain_compute_gradients(pettrain_handle h, const float* x0_dev, const float* cond_dev, int B,
                               const int32_t* t_dev, const float* noise_dev, uint64_t seed,
                               uint64_t sample_offset, float* loss_dev, void* stream);
/* Forward + loss only (ImprovedDDPM.test_step, diffusion_model.py:600-640): same draws and
 * outputs as pettrain_compute_gradients, no backward pass; the gradient blob is untouched. */
int pettrain_compute_loss(pettrain_handle h, const float* x0_dev, const float* cond_dev, int B, const int32_t* t_dev,
                          const float* noise_dev, uint64_t seed, uint64_t sample_offset, float* loss_dev,
                          void* stream);
/* Clip (per variable, after scaling by grad_scale) + Adam update; iterations += 1. */
int pettrain_apply_gradients(pettrain_handle h, float grad_scale, void* stream);
/* compute_gradients + apply_gradients(1). */
int pettrain_step(pettrain_handle h, const float* x0_dev, const float* cond_dev, int B, const int32_t* t_dev,
                  const float* noise_dev, uint64_t seed, uint64_t sample_offset, float* loss_dev, void* stream);

/* Device pointer of the gradient blob (petdiff.h order, n_weights floats), e.g. for an
 * RCCL all-reduce between compute_gradients and apply_gradients on data-parallel ranks. */
float* pettrain_gradients(pettrain_handle h);
/* Copy the gradient blob out / in (n_weights floats), the same through a caller buffer. */
int pettrain_get_gradients(pettrain_handle h, float* dst_dev, void* stream);
int pettrain_set_gradients(pettrain_handle h, const float* src_dev, void* stream);
/* Copies the current fp32 weights (n_weights floats) to dst_dev. */
int pettrain_get_weights(pettrain_handle h, float* dst_dev, void* stream);
/* Last compute_gradients: {mean loss, noise_loss (mse), mean vlb} (synchronises `stream`). */
int pettrain_last_stats(pettrain_handle h, double* out3, void* stream);
int64_t pettrain_iterations(pettrain_handle h);
const char* pettrain_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PETTRAIN_H */
