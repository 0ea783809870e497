/*
 * petdiff.h -- C ABI of the MI355X-native iDDPM posterior sampler
 * (libpetdiff.so, built from pet_posterior_distribution_amd/csrc/ for gfx950).
 *
 * Drop-in boundary for the hot path of yanisdjebra/PET_posterior_distribution:
 * the reference's Python entry points (file:line in /root/reference at
 * 2025-08-29) map to these C entry points as follows:
 *
 *   ImprovedDDPM.__init__ schedule buffers  diffusion_model.py:85-105, 337-355
 *                                            -> petdiff_set_schedule (+ petdiff_cosine_schedule)
 *   UnetConditional.build / load_weights     networks.py:781-992, main_script.py:412
 *                                            -> petdiff_create (flat fp32 Keras-layout weights)
 *   condition encoder + label projections   networks.py:915-921, 958-964, 574-586
 *                                            -> petdiff_set_conditions (hoisted once per TAC)
 *   DDPM.call -> UnetConditional.call        diffusion_model.py:141-158, networks.py:994-1093
 *                                            -> petdiff_forward
 *   ImprovedDDPM.ddpm / tfunc_ddpm           diffusion_model.py:651-668  (= p_sample)
 *                                            -> petdiff_p_sample
 *   ImprovedDDPM.ddpm_loop / tfunc_ddpm_loop diffusion_model.py:670-737  (= generate)
 *                                            -> petdiff_generate
 *   per-ROI posterior mean / std             main_script.py:433-436
 *                                            -> petdiff_posterior_stats
 *
 * Conventions: plain C types only.  Every pointer named *_dev is device memory
 * of the handle's device (e.g. a torch-ROCm tensor's data_ptr()); the caller
 * owns it.  `stream` is a hipStream_t (0 = legacy default stream).  Every
 * function returns PETDIFF_OK (0) or an error code; petdiff_last_error()
 * returns a thread-local message for the last failure (the Python wrapper
 * raises the reference's exception types with it).  A handle is bound to one
 * device; calls on one handle must be externally serialised.
 *
 * Weight blob: fp32, the tensors of the shipped UnetConditional concatenated in
 * the order below, each in Keras layout (Dense kernel (in, out); Conv1D kernel
 * (k, Cin, Cout)), kernel before bias:
 *   time_mlp                      Dense(sin_dim -> n_roi)           networks.py:854
 *   cond_enc.hidden{0,1,2}, .z    Encoder_v3_noskip 54-256-128-64-32 networks.py:526-537
 *   down{d}.time_proj, .label_proj, .conv (k=6), .res (k=1)       d = 0..depth-1
 *   up{u}.time_proj, .label_proj, .upconv (k=pool), .conv, .res   u = 0..depth-2
 *   final (k=1, 128 -> n_out)
 * Conv input channel order is [label(49) | time(1) | x] for down/up-conv
 * layers (networks.py:1022, 1043) and [skip | x] for up blocks (:1057).
 */
#ifndef PETDIFF_H
#define PETDIFF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PETDIFF_OK 0
#define PETDIFF_ERR_INVALID 1      /* bad argument (ValueError in the wrapper) */
#define PETDIFF_ERR_HIP 2          /* HIP runtime failure (RuntimeError)      */
#define PETDIFF_ERR_UNSUPPORTED 3  /* config outside the compiled kernels     */

/* Largest batch one call accepts (posterior samples per launch).  Every activation
 * buffer then stays below 2^31 elements and 4 GB, which the kernels' 32-bit row
 * indices and buffer-resource record counts assume.  ImprovedDDPM.ddpm_loop splits
 * larger batches into chunks (the noise stream is keyed by global sample index, so
 * chunked and unchunked runs are identical), as main_script.py:414-427 chunks its
 * own posterior draws. */
#define PETDIFF_MAX_BATCH 65536

#define PETDIFF_DTYPE_F32 0        /* exact-f32 MFMA network (parity mode)    */
#define PETDIFF_DTYPE_BF16 1       /* bf16 MFMA network, fp32 accumulate + fp32 p_sample */
#define PETDIFF_DTYPE_F16 2        /* fp16 MFMA network (BASELINE config 5), fp32 accumulate + p_sample */
#define PETDIFF_DTYPE_BF16X3 3     /* fp32-class network on the bf16 MFMA path: every fp32 operand split
                                      hi + lo into bf16, products hi*hi + hi*lo + lo*hi (3 MFMAs), fp32
                                      accumulate; about 2^-16 relative per product, meets the 1e-4 parity
                                      tolerance of the exact-f32 mode */

#define PETDIFF_LEARN_FIXED 0      /* learn_variance = ''            */
#define PETDIFF_LEARN 1            /* 'learn'                         */
#define PETDIFF_LEARN_RANGED 2     /* 'learn_ranged' (shipped config) */

#define PETDIFF_PARAM_EPS 0        /* parameterization names, diffusion_model.py:323-326 */
#define PETDIFF_PARAM_X0 1
#define PETDIFF_PARAM_V 2
#define PETDIFF_PARAM_XPREV 3

/* Rows of the [PETDIFF_NTAB][T] fp32 schedule table (petdiff_set_schedule). */
#define PETDIFF_TAB_BETA 0            /* beta                                   */
#define PETDIFF_TAB_LOG_BETA 1        /* log(beta)                              */
#define PETDIFF_TAB_PLVC 2            /* posterior_log_variance_clipped         */
#define PETDIFF_TAB_POST_VAR 3        /* posterior_variance ([0] aliased, :349) */
#define PETDIFF_TAB_C1 4              /* posterior_mean_coef1                   */
#define PETDIFF_TAB_C2 5              /* posterior_mean_coef2                   */
#define PETDIFF_TAB_ALPHA_BAR 6       /* cumprod(alpha) (unshifted, :337)       */
#define PETDIFF_TAB_SQRT_AB 7         /* sqrt(alpha_bar)                        */
#define PETDIFF_TAB_SQRT_1M_AB 8      /* sqrt(1 - alpha_bar)                    */
#define PETDIFF_TAB_INV_SQRT_AB 9     /* 1 / sqrt(alpha_bar)          (:374)    */
#define PETDIFF_TAB_SQRT_RECIP_M1 10  /* sqrt(1 / alpha_bar - 1)      (:374)    */
#define PETDIFF_TAB_RECIP_C1 11       /* 1 / coef1                    (:367)    */
#define PETDIFF_TAB_C2_OVER_C1 12     /* coef2 / coef1                (:368)    */
#define PETDIFF_NTAB 13

typedef struct petdiff_config {
  int n_roi;          /* 48   x length (ROIs)                main_script.py:107   */
  int n_par;          /* 2    DVR, R1 channels               main_script.py:116   */
  int n_frames;       /* 54   TAC frames (condition width)   main_script.py:110   */
  int n_cond_rows;    /* 49   48 ROI TACs + reference TAC    main_script.py:110   */
  int num_filt_start; /* 128                                 main_script.py:138   */
  int depth;          /* 4                                   main_script.py:140   */
  int kernel_size;    /* 6                                   main_script.py:146   */
  int pool_size;      /* 2                                   main_script.py:139   */
  int sin_emb_dim;    /* 64                                  main_script.py:164   */
  int enc_size[3];    /* 256,128,64                          main_script.py:152   */
  int latent_dim;     /* 32                                  main_script.py:153   */
  int timesteps;      /* 1000                                main_script.py:131   */
  int learn_variance; /* PETDIFF_LEARN_*                     main_script.py:132   */
  int parameterization; /* PETDIFF_PARAM_*                   diffusion_model.py:319 */
  int dtype;          /* PETDIFF_DTYPE_* network compute type                      */
} petdiff_config;

typedef struct petdiff_ctx* petdiff_handle;

/* Fills the shipped configuration (main_script.py:131-186). */
int petdiff_default_config(petdiff_config* cfg);
/* Number of fp32 values of the weight blob for cfg (11,851,740 for the shipped one). */
size_t petdiff_param_count(const petdiff_config* cfg);

/* Builds a sampler on `device` from the host fp32 weight blob (copied; the
 * library packs it into its MFMA layouts).  Replaces UnetConditional.build +
 * load_weights. */
int petdiff_create(const petdiff_config* cfg, const float* weights_host, size_t n_weights, int device,
                   petdiff_handle* out);
int petdiff_destroy(petdiff_handle h);

/* Per-timestep tables, host fp32 [PETDIFF_NTAB][T] (row order above).  The
 * Python host fills them with NumPy exactly like diffusion_model.py:98-105,
 * 337-355 so they are bit-identical to the reference's buffers. */
int petdiff_set_schedule(petdiff_handle h, const float* tables_host, int T);
/* C restatement of helper_func.cos_beta_schedule (helper_func.py:210-219) for
 * callers without NumPy (cosf may differ from numpy's float32 cos by 1 ulp). */
int petdiff_cosine_schedule(int T, double offset_s, double max_beta, float* beta_out);

/* Conditions (the network's `condition` input): cond_dev fp32 [n_tac][49][54]
 * device.  Runs the encoder + label projections once per condition and folds
 * them into the per-level conv maps.  Sample b then uses condition tac[b]. */
int petdiff_set_conditions(petdiff_handle h, const float* cond_dev, int n_tac, void* stream);

/* Raw network output (DDPM.call): out_dev fp32 [B][n_roi][n_out].
 * t_dev int32 [B]; tac_dev int32 [B] or NULL (all condition 0). */
int petdiff_forward(petdiff_handle h, const float* x_dev, const int32_t* t_dev, const int32_t* tac_dev,
                    float* out_dev, int B, void* stream);

/* One reverse step (ImprovedDDPM.ddpm): returns (mean, var, var_tilde), each
 * fp32 [B][n_roi][n_par]; any output may be NULL.  z_dev = injected N(0,1)
 * noise [B][n_roi][n_par] or NULL -> counter-based Philox keyed by
 * (seed, sample_offset + b, rng_step). */
int petdiff_p_sample(petdiff_handle h, const float* x_dev, const int32_t* t_dev, const int32_t* tac_dev,
                     const float* z_dev, uint64_t seed, uint64_t sample_offset, int rng_step,
                     float* mean_dev, float* var_dev, float* var_tilde_dev, int B, void* stream);

/* Full reverse loop (ImprovedDDPM.ddpm_loop): t_seq_host = the timestep index
 * list (diffusion_model.py:680-691), step i uses t_seq_host[i] and Philox step i.
 * z_all_dev: NULL or injected noise [n_steps][B][n_roi][n_par].
 * all_xt_dev: NULL or [n_steps][B][n_roi][n_par] (keep_all_xt).
 * use_graph != 0 captures the n_steps kernels into one hipGraph (cached per
 * (B, t_seq, flag); requires z_all_dev == all_xt_dev == NULL). */
int petdiff_generate(petdiff_handle h, const float* x_T_dev, const int32_t* tac_dev, const int32_t* t_seq_host,
                     int n_steps, int flag_var_tilde, const float* z_all_dev, uint64_t seed,
                     uint64_t sample_offset, float* x_out_dev, float* all_xt_dev, int B, int use_graph,
                     void* stream);

/* Fills out_dev [B][n_roi][n_par] with N(0,1) from the sampler's counter-based
 * Philox stream (sample g = sample_offset + b, step id rng_step; the reverse loop
 * uses step ids 0..n_steps-1, so x_T conventionally uses 0x7fffffff).  Replaces the
 * caller's tf.random.normal x_T draw (main_script.py:415) when a world-size
 * independent sharded run is wanted. */
int petdiff_philox_normal(petdiff_handle h, uint64_t seed, uint64_t sample_offset, int rng_step, float* out_dev,
                          int B, void* stream);

/* Per (condition, roi, param) {count, mean, M2} in fp64 over the samples of
 * x0_dev [B][n_roi][n_par] (host output [n_tac][n_roi][n_par][3]; synchronises
 * the stream).  mean / sqrt(M2 / count) = main_script.py:433-436. */
int petdiff_posterior_stats(petdiff_handle h, const float* x0_dev, const int32_t* tac_dev, int B, int n_tac,
                            double* stats_host, void* stream);

/* Level outputs of the last petdiff_forward / petdiff_p_sample call, converted to
 * fp32 into out_dev (test and debugging aid: per-level parity of the 16-bit fused
 * path against the exact-f32 path and the oracle).  level (networks.py:1010-1072):
 *   0 skip s0 = down0 ConvBlock output   [B][48][128]
 *   1 skip s1 = down1 ConvBlock output   [B][24][256]
 *   2 skip s2 = down2 ConvBlock output   [B][12][512]
 *   3 down3 ConvBlock output (bottom)    [B][6][1024]
 *   4 up0 ConvBlock output               [B][12][512]
 *   5 up1 ConvBlock output               [B][24][256]
 * (the up2 ConvBlock output stays in LDS: it feeds the fused final conv).  B must
 * not exceed the batch of that call. */
#define PETDIFF_NUM_LEVELS 6
int petdiff_get_activation(petdiff_handle h, int level, float* out_dev, int B, void* stream);

/* Per-layer kernel timing with HIP events on the launch stream (eager mode
 * only).  layer ids: 0 down0, 1..9 = down1, down2, down3, up0.conv2, up0.block,
 * up1.conv2, up1.block, up2.conv2, up2.block(+final+p_sample).
 * enable: 0 off; n >= 1 on, each timed layer launch repeated n times back to back
 * (at most 64; the kernels are idempotent) so the event pair's queue gap is shared
 * by n launches. */
#define PETDIFF_NUM_LAYERS 10
int petdiff_set_timing(petdiff_handle h, int enable);
/* Synchronises; fills total ms and launch count (timed launches, repeats included)
 * per layer, then resets. */
int petdiff_get_timing(petdiff_handle h, float* total_ms, int* count);

const char* petdiff_last_error(void);

/* Diagnostic (no reference counterpart): the XOR key of 16-B piece slots in an LDS row / packed weight
 * row that the kernels and the host weight packer share (petdiff_internal.h piece_key): row index, pieces
 * per row (2, 4 or 8), m16 = 1 for the 16x16x32 layers' 16-row key.  Exported so the CPU tests check the
 * bank-conflict model against the library's own formula. */
int petdiff_piece_key(int row, int cpr, int m16);

#ifdef __cplusplus
}
#endif
#endif /* PETDIFF_H */
