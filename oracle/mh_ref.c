/*
 * mh_ref.c -- CPU restatement of the reference's Metropolis-Hastings baseline
 * (mcmc.py:147-157 model + PyMC 5.12 element-wise Metropolis, NormalProposal,
 * tune_interval 100) in plain C with OpenMP over chains.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/ and bench.py's cpu_baseline leg
 * (through oracle/mh_c.py), never by the product.  It is the checker for the
 * GPU sampler's chain paths at sizes the NumPy oracle cannot reach and the
 * "port" CPU baseline of BASELINE.json config 3.
 *
 * Follows, per element update of ROI i (DVR or R1):
 *   SRTM2 of ROI i      kinetic_model.py:142-158 via the constant operator
 *                       M = W_down . Toeplitz(C_r) . W_up . dx of
 *                       oracle/srtm2_ref.py:srtm2_operator (kinetic_model.py:12-57)
 *   likelihood          mcmc.py:151-155: sn<0 -> 1e-6, sigma = sqrt(sn) sigma_noise,
 *                       TruncatedNormal(lower=0) logpdf summed over frames
 *   prior change        MvNormal (mcmc.py:148-149): d log p = -(d g_i + d^2 P_ii / 2),
 *                       g = P (x - mu), updated on accept
 *   sweep               pymc 5.12 Metropolis.astep (elemwise_update): one proposal
 *                       vector per draw, elements visited in a shuffled order, each
 *                       ratio taken against the sweep-START point (delta_logp(q_temp, q0));
 *                       accept iff the ratio is finite and log(u) < ratio (metrop_select)
 *   tuning              pymc.step_methods.metropolis.tune every tune_interval
 *                       tuning draws from the per-element acceptance rate
 * Noise: Philox4x32-10 keyed by seed, counter (k, it, chain_lo, chain_hi),
 * words 0/1 -> Box-Muller cos, word 2 -> accept uniform, word 3 -> the element's
 * sort key of the sweep order (oracle/srtm2_ref.py:philox_mh_block) -- the
 * stream the GPU sampler uses.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NR 48
#define NF 54

static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

static double log_ndtr(double x) {   /* scipy.special.log_ndtr for the x > -20 range used here */
  if (x > -20.0) return log(0.5 * erfc(-x * 0.7071067811865476));
  return -0.5 * x * x - log(-x) - 0.9189385332046727;   /* leading asymptotic term */
}

typedef struct {
  const double *M, *PD, *PR, *Y, *SIG, *CR, *TV, *MUD, *MUR;
  double k2p;
} prob_t;

/* Truncated-normal log-likelihood of ROI i with parameters (dvr, r1). */
static double roi_loglik(const prob_t* p, int i, double dvr, double r1) {
  double e[NF];
  const double k2 = p->k2p * r1, k2a = k2 / dvr;
  for (int f = 0; f < NF; ++f) e[f] = exp(-k2a * p->TV[f]);
  double l = 0.0;
  for (int f = 0; f < NF; ++f) {
    double conv = 0.0;
    for (int g = 0; g < NF; ++g) conv += p->M[g * NF + f] * e[g];
    const double tac = r1 * p->CR[f] + (k2 - r1 * k2a) * conv;
    const double sn = tac < 0.0 ? 1e-6 : tac;
    const double sig = sqrt(sn) * p->SIG[i * NF + f];
    const double z = (p->Y[i * NF + f] - sn) / sig;
    l += -0.5 * z * z - 0.9189385332046727 - log(sig) - log_ndtr(sn / sig);
  }
  return l;
}

static double tune_scale(double s, double rate) {
  if (rate < 0.001) return s * 0.1;
  if (rate < 0.05) return s * 0.5;
  if (rate < 0.2) return s * 0.9;
  if (rate > 0.95) return s * 10.0;
  if (rate > 0.75) return s * 2.0;
  if (rate > 0.5) return s * 1.1;
  return s;
}

typedef struct { uint64_t key; int k; } keyed_t;

static int cmp_keyed(const void* a, const void* b) {
  const keyed_t *x = (const keyed_t*)a, *y = (const keyed_t*)b;
  if (x->key != y->key) return x->key < y->key ? -1 : 1;
  return x->k - y->k;
}

static void run_chain(const prob_t* p, const double* x0, long chain, int n_draws, int n_tune, int tune_interval,
                      double scaling, uint64_t seed, int vs_sweep_start, double* stats, double* accept,
                      double* last) {
  double x[2 * NR], g[2 * NR], ll[NR], s[2 * NR], mean[2 * NR], m2[2 * NR], acc[2 * NR], z[2 * NR], lu[2 * NR];
  int win[2 * NR];
  keyed_t ord[2 * NR];
  for (int k = 0; k < NR; ++k) {
    x[k] = x0 ? x0[k] : p->MUD[k];
    x[NR + k] = x0 ? x0[NR + k] : p->MUR[k];
  }
  for (int v = 0; v < 2; ++v) {
    const double* P = v ? p->PR : p->PD;
    const double* mu = v ? p->MUR : p->MUD;
    for (int a = 0; a < NR; ++a) {
      double t = 0.0;
      for (int b = 0; b < NR; ++b) t += P[a * NR + b] * (x[v * NR + b] - mu[b]);
      g[v * NR + a] = t;
    }
  }
  for (int i = 0; i < NR; ++i) ll[i] = roi_loglik(p, i, x[i], x[NR + i]);
  for (int k = 0; k < 2 * NR; ++k) { s[k] = scaling; mean[k] = m2[k] = acc[k] = 0.0; win[k] = 0; }
  long nk = 0;
  for (int it = 0; it < n_tune + n_draws; ++it) {
    if (it < n_tune && it > 0 && it % tune_interval == 0)
      for (int k = 0; k < 2 * NR; ++k) { s[k] = tune_scale(s[k], (double)win[k] / tune_interval); win[k] = 0; }
    for (int k = 0; k < 2 * NR; ++k) {     /* the sweep's draws (Metropolis.astep) */
      uint32_t q[4] = {(uint32_t)k, (uint32_t)it, (uint32_t)((uint64_t)chain & 0xffffffffu),
                       (uint32_t)((uint64_t)chain >> 32)};
      philox(q, (uint32_t)(seed & 0xffffffffu), (uint32_t)(seed >> 32));
      const double u1 = ((double)q[0] + 1.0) * 2.3283064365386963e-10;
      const double u2 = ((double)q[1] + 0.5) * 2.3283064365386963e-10;
      z[k] = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
      lu[k] = log(((double)q[2] + 0.5) * 2.3283064365386963e-10);
      ord[k].key = q[3];
      ord[k].k = k;
    }
    qsort(ord, 2 * NR, sizeof(keyed_t), cmp_keyed);
    double run = 0.0;                      /* log p(running state) - log p(sweep start) */
    for (int j = 0; j < 2 * NR; ++j) {
      const int k = ord[j].k, v = k / NR, i = k % NR;
      const double* P = v ? p->PR : p->PD;
      const double delta = z[k] * s[k];
      const double xp = x[k] + delta;
      const double dprior = -0.5 * (2.0 * delta * g[k] + delta * delta * P[i * NR + i]);
      const double lln = roi_loglik(p, i, v ? x[i] : xp, v ? xp : x[NR + i]);
      const double step = dprior + lln - ll[i];
      const double mr = vs_sweep_start ? run + step : step;
      if (isfinite(mr) && lu[k] < mr) {
        x[k] = xp;
        ll[i] = lln;
        run += step;
        win[k] += 1;
        if (it >= n_tune) acc[k] += 1.0;
        for (int a = 0; a < NR; ++a) g[v * NR + a] += delta * P[a * NR + i];
      }
    }
    if (it >= n_tune) {
      ++nk;
      for (int k = 0; k < 2 * NR; ++k) {
        const double d = x[k] - mean[k];
        mean[k] += d / (double)nk;
        m2[k] += d * (x[k] - mean[k]);
      }
    }
  }
  for (int k = 0; k < 2 * NR; ++k) {
    stats[k * 3 + 0] = (double)nk;
    stats[k * 3 + 1] = mean[k];
    stats[k * 3 + 2] = m2[k];
    if (accept) accept[k] = acc[k];
    if (last) last[k] = x[k];
  }
}

/* n_chains independent chains (chain ids chain0 .. chain0 + n_chains - 1);
 * stats [n][96][3] {count, mean, M2}; accept / last [n][96] or NULL. */
int mhref_run(const double* M, const double* PD, const double* PR, const double* Y, const double* SIG,
              const double* CR, const double* TV, const double* MUD, const double* MUR, double k2p,
              const double* x0, long chain0, int n_chains, int n_draws, int n_tune, int tune_interval,
              double scaling, uint64_t seed, int vs_sweep_start, double* stats, double* accept, double* last,
              int n_threads) {
  prob_t p = {M, PD, PR, Y, SIG, CR, TV, MUD, MUR, k2p};
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int c = 0; c < n_chains; ++c)
    run_chain(&p, x0 ? x0 + (size_t)c * 2 * NR : NULL, chain0 + c, n_draws, n_tune, tune_interval, scaling, seed,
              vs_sweep_start, stats + (size_t)c * 2 * NR * 3, accept ? accept + (size_t)c * 2 * NR : NULL,
              last ? last + (size_t)c * 2 * NR : NULL);
  return 0;
}

/* Joint log density without constants of the priors' normalisers:
 * sum_i roi_loglik - (x-mu)^T P (x-mu) / 2 for both blocks, at n points [n][96]. */
int mhref_logp_kernel_part(const double* M, const double* PD, const double* PR, const double* Y, const double* SIG,
                           const double* CR, const double* TV, const double* MUD, const double* MUR, double k2p,
                           const double* x, int n, double* out) {
  prob_t p = {M, PD, PR, Y, SIG, CR, TV, MUD, MUR, k2p};
  for (int t = 0; t < n; ++t) {
    const double* xt = x + (size_t)t * 2 * NR;
    double l = 0.0;
    for (int i = 0; i < NR; ++i) l += roi_loglik(&p, i, xt[i], xt[NR + i]);
    for (int v = 0; v < 2; ++v) {
      const double* P = v ? PR : PD;
      const double* mu = v ? MUR : MUD;
      double q = 0.0;
      for (int a = 0; a < NR; ++a)
        for (int b = 0; b < NR; ++b) q += (xt[v * NR + a] - mu[a]) * P[a * NR + b] * (xt[v * NR + b] - mu[b]);
      l -= 0.5 * q;
    }
    out[t] = l;
  }
  return 0;
}
