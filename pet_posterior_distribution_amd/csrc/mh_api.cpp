// C-ABI implementation of the Metropolis-Hastings / SRTM2 part of libpetdiff.so
// (include/petmh.h): host precomputation of the SRTM2 operator and prior
// precisions (fp64), device buffers and launches.
#include "petmh.h"
#include "mh_internal.h"

#include <algorithm>
#include <cmath>
#include <memory>
#include <set>
#include <string>
#include <vector>

using namespace petmh;

namespace {

thread_local std::string g_err;

int fail(const std::string& m) {
  g_err = m;
  return 1;
}

#define HIPC(expr)                                                                       \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) {                                                              \
      g_err = std::string(#expr) + ": " + hipGetErrorString(e_);                         \
      return 2;                                                                          \
    }                                                                                    \
  } while (0)

// numpy.linspace(a, b, n)
std::vector<double> linspace(double a, double b, int n) {
  std::vector<double> x(n);
  const double step = (b - a) / (n - 1);
  for (int i = 0; i < n; ++i) x[i] = a + i * step;
  x[n - 1] = b;
  return x;
}

// numpy.interp(x, xp, fp) for increasing xp, x inside [xp0, xpN]
double np_interp(double x, const std::vector<double>& xp, const double* fp) {
  const int n = (int)xp.size();
  if (x <= xp[0]) return fp[0];
  if (x >= xp[n - 1]) return fp[n - 1];
  int j = (int)(std::upper_bound(xp.begin(), xp.end(), x) - xp.begin()) - 1;
  const double slope = (fp[j + 1] - fp[j]) / (xp[j + 1] - xp[j]);
  return slope * (x - xp[j]) + fp[j];
}

// kinetic_model.interp1d_linear_vec weights (kinetic_model.py:42-49), incl. the
// searchsorted-1 == -1 wrap of the first point.  W is [x.size][xp.size].
std::vector<double> interp_weights(const std::vector<double>& x, const std::vector<double>& xp) {
  const int n = (int)x.size(), m = (int)xp.size();
  std::vector<double> W((size_t)n * m, 0.0);
  for (int i = 0; i < n; ++i) {
    const int idx = (int)(std::lower_bound(xp.begin(), xp.end(), x[i]) - xp.begin());   // searchsorted left
    const int im1 = (idx - 1 + m) % m;
    const double d_idx = std::fabs(xp[idx % m] - x[i]), d_im1 = std::fabs(xp[im1] - x[i]);
    W[(size_t)i * m + idx % m] = d_im1;
    W[(size_t)i * m + im1] = d_idx;
    double s = 0.0;
    for (int j = 0; j < m; ++j) s += W[(size_t)i * m + j];
    for (int j = 0; j < m; ++j) W[(size_t)i * m + j] /= s;
  }
  return W;
}

// M = W_down . Toeplitz(y0) . W_up . dx  ([f][g] row-major) -- kinetic_model.py:12-32
std::vector<double> srtm2_operator(const double* tv, const double* cr, int nf) {
  std::vector<double> t(tv, tv + nf);
  std::set<double> uniq(t.begin(), t.end());
  const int n = 2 * (int)uniq.size();
  const double lo = *std::min_element(t.begin(), t.end()), hi = *std::max_element(t.begin(), t.end());
  std::vector<double> xrs = linspace(lo, hi, n);
  const double dx = xrs[1] - xrs[0];
  std::vector<double> y0(n);
  for (int i = 0; i < n; ++i) y0[i] = np_interp(xrs[i], t, cr);
  std::vector<double> Wup = interp_weights(xrs, t);     // [n][nf]
  std::vector<double> Wdn = interp_weights(t, xrs);     // [nf][n]
  // TW = Toeplitz(y0) . Wup : [n][nf]
  std::vector<double> TW((size_t)n * nf, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      const double y = y0[i - j];
      for (int g = 0; g < nf; ++g) TW[(size_t)i * nf + g] += y * Wup[(size_t)j * nf + g];
    }
  std::vector<double> M((size_t)nf * nf, 0.0);
  for (int f = 0; f < nf; ++f)
    for (int i = 0; i < n; ++i) {
      const double w = Wdn[(size_t)f * n + i];
      if (w == 0.0) continue;
      for (int g = 0; g < nf; ++g) M[(size_t)f * nf + g] += w * TW[(size_t)i * nf + g] * dx;
    }
  return M;
}

// Cholesky inverse of an SPD matrix; returns log det.
bool spd_inverse(const double* A, int n, std::vector<double>& inv, double& logdet) {
  std::vector<double> L((size_t)n * n, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = A[(size_t)i * n + j];
      for (int k = 0; k < j; ++k) s -= L[(size_t)i * n + k] * L[(size_t)j * n + k];
      if (i == j) {
        if (s <= 0) return false;
        L[(size_t)i * n + i] = std::sqrt(s);
      } else {
        L[(size_t)i * n + j] = s / L[(size_t)j * n + j];
      }
    }
  logdet = 0.0;
  for (int i = 0; i < n; ++i) logdet += 2.0 * std::log(L[(size_t)i * n + i]);
  // inv(L)
  std::vector<double> Li((size_t)n * n, 0.0);
  for (int i = 0; i < n; ++i) {
    Li[(size_t)i * n + i] = 1.0 / L[(size_t)i * n + i];
    for (int j = 0; j < i; ++j) {
      double s = 0.0;
      for (int k = j; k < i; ++k) s += L[(size_t)i * n + k] * Li[(size_t)k * n + j];
      Li[(size_t)i * n + j] = -s / L[(size_t)i * n + i];
    }
  }
  inv.assign((size_t)n * n, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int k = std::max(i, j); k < n; ++k) s += Li[(size_t)k * n + i] * Li[(size_t)k * n + j];
      inv[(size_t)i * n + j] = s;
    }
  return true;
}

struct Buf {
  double* p = nullptr;
  ~Buf() { if (p) (void)hipFree(p); }
};

}  // namespace

struct petmh_ctx {
  int device = 0;
  Buf M, PD, PR, Y, SIG, CR, TV, MUD, MUR;
  MHConst c{};
  int tune_interval = 100;   // pymc Metropolis defaults
  double scaling = 1.0;
  int vs_sweep_start = 1;    // pymc 5.12 elemwise_update compares against the sweep-start point
  int kernel = 0, wpc = 0;   // petmh_set_kernel
};

extern "C" {

const char* petmh_last_error(void) { return g_err.c_str(); }

static int upload(Buf& b, const double* host, size_t n) {
  HIPC(hipMalloc(&b.p, n * sizeof(double)));
  HIPC(hipMemcpy(b.p, host, n * sizeof(double), hipMemcpyHostToDevice));
  return 0;
}

int petmh_create(const petmh_problem* p, int device, petmh_handle* out) {
  if (!p || !out) return fail("null argument");
  if (p->n_roi != kNRoi || p->n_frames != kNFrames)
    return fail("kernels are compiled for 48 ROIs x 54 frames (mcmc.py:53, sample_sim_data.py:29-85)");
  if (!p->time_vector || !p->tac_ref || !p->y_obs || !p->sigma_noise || !p->mu_DVR || !p->cov_DVR || !p->mu_R1 ||
      !p->cov_R1)
    return fail("null problem array");
  std::unique_ptr<petmh_ctx> h(new petmh_ctx());
  h->device = device;
  HIPC(hipSetDevice(device));
  const int nf = kNFrames, nr = kNRoi;
  std::vector<double> Mfg = srtm2_operator(p->time_vector, p->tac_ref, nf);
  std::vector<double> Mgf((size_t)nf * nf);
  for (int f = 0; f < nf; ++f)
    for (int g = 0; g < nf; ++g) Mgf[(size_t)g * nf + f] = Mfg[(size_t)f * nf + g];
  std::vector<double> PD, PR;
  double ldD = 0, ldR = 0;
  if (!spd_inverse(p->cov_DVR, nr, PD, ldD) || !spd_inverse(p->cov_R1, nr, PR, ldR))
    return fail("prior covariance is not positive definite");
  int rc;
  if ((rc = upload(h->M, Mgf.data(), Mgf.size()))) return rc;
  if ((rc = upload(h->PD, PD.data(), PD.size()))) return rc;
  if ((rc = upload(h->PR, PR.data(), PR.size()))) return rc;
  if ((rc = upload(h->Y, p->y_obs, (size_t)nr * nf))) return rc;
  if ((rc = upload(h->SIG, p->sigma_noise, (size_t)nr * nf))) return rc;
  if ((rc = upload(h->CR, p->tac_ref, nf))) return rc;
  if ((rc = upload(h->TV, p->time_vector, nf))) return rc;
  if ((rc = upload(h->MUD, p->mu_DVR, nr))) return rc;
  if ((rc = upload(h->MUR, p->mu_R1, nr))) return rc;
  MHConst& c = h->c;
  c.M = h->M.p;
  c.PD = h->PD.p;
  c.PR = h->PR.p;
  c.Y = h->Y.p;
  c.SIG = h->SIG.p;
  c.CR = h->CR.p;
  c.TV = h->TV.p;
  c.MUD = h->MUD.p;
  c.MUR = h->MUR.p;
  c.k2p = p->k2p;
  c.prior_const = -0.5 * (2.0 * nr * std::log(2.0 * M_PI) + ldD + ldR);
  *out = h.release();
  return 0;
}

int petmh_destroy(petmh_handle h) {
  if (!h) return 0;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  delete h;
  return 0;
}

int petmh_run(petmh_handle h, const double* x0, int n_chains, int n_draws, int n_tune, uint64_t seed, double* stats,
              double* accept, double* last, void* stream) {
  return petmh_run_draws(h, x0, n_chains, n_draws, n_tune, seed, stats, accept, last, nullptr, stream);
}

int petmh_run_draws(petmh_handle h, const double* x0, int n_chains, int n_draws, int n_tune, uint64_t seed,
                    double* stats, double* accept, double* last, double* draws, void* stream) {
  if (!h || !stats || n_chains < 0 || n_draws < 0 || n_tune < 0) return fail("bad arguments");
  HIPC(hipSetDevice(h->device));
  MHRun r{};
  r.x0 = x0;
  r.n_chains = n_chains;
  r.n_draws = n_draws;
  r.n_tune = n_tune;
  r.tune_interval = h->tune_interval;
  r.scaling = h->scaling;
  r.vs_sweep_start = h->vs_sweep_start;
  r.seed = seed;
  r.stats = stats;
  r.accept = accept;
  r.last = last;
  r.draws = draws;
  r.kernel = h->kernel;
  r.wpc = h->wpc;
  HIPC(launch_mh_chains(h->c, r, (hipStream_t)stream));
  return 0;
}

int petmh_set_sampler(petmh_handle h, int tune_interval, double scaling, int vs_sweep_start) {
  if (!h || tune_interval <= 0 || !(scaling > 0.0)) return fail("bad sampler options");
  h->tune_interval = tune_interval;
  h->scaling = scaling;
  h->vs_sweep_start = vs_sweep_start != 0;
  return 0;
}

int petmh_set_kernel(petmh_handle h, int kernel, int waves_per_chain) {
  if (!h || kernel < 0 || kernel > 2) return fail("bad kernel (0 auto, 1 one update at a time, 2 batched)");
  if (!(waves_per_chain == 0 || waves_per_chain == 1 || waves_per_chain == 2 || waves_per_chain == 4 ||
        waves_per_chain == 12))
    return fail("waves_per_chain must be 0 (auto), 1, 2, 4 or 12");
  h->kernel = kernel;
  h->wpc = waves_per_chain;
  return 0;
}

int petmh_logp(petmh_handle h, const double* x, int n, double* out, void* stream) {
  if (!h || n < 0 || (n > 0 && (!x || !out))) return fail("bad arguments");
  HIPC(hipSetDevice(h->device));
  HIPC(launch_mh_logp(h->c, x, n, out, (hipStream_t)stream));
  return 0;
}

int petmh_srtm2_tac(const double* tv, const double* cr, const double* dvr, const double* r1, int n, int n_roi,
                    const double* k2p, double* tac, void* stream) {
  if (!tv || !cr || n < 0 || n_roi <= 0 || (n > 0 && (!dvr || !r1 || !k2p || !tac))) return fail("bad arguments");
  const int nf = kNFrames;
  std::vector<double> Mfg = srtm2_operator(tv, cr, nf);
  std::vector<double> Mgf((size_t)nf * nf);
  for (int f = 0; f < nf; ++f)
    for (int g = 0; g < nf; ++g) Mgf[(size_t)g * nf + f] = Mfg[(size_t)f * nf + g];
  Buf M, C, T;
  int rc;
  if ((rc = upload(M, Mgf.data(), Mgf.size()))) return rc;
  if ((rc = upload(C, cr, nf))) return rc;
  if ((rc = upload(T, tv, nf))) return rc;
  hipStream_t s = (hipStream_t)stream;
  HIPC(launch_srtm2(M.p, C.p, T.p, dvr, r1, k2p, n, n_roi, tac, s));
  HIPC(hipStreamSynchronize(s));   // temporaries are freed on return
  return 0;
}

}  // extern "C"
