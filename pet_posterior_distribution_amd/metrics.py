"""Posterior accuracy metrics: iDDPM samples vs the MCMC trace.

Restates the metrics step after the reverse loop, main_script.py:719-829:

* per kinetic parameter (DVR, R1), over the posterior samples of each method:
  ``np.mean``, ``np.cov`` (ddof = 1), ``np.corrcoef`` - I, the per-ROI std
  ``sqrt(diag(cov))`` and the relative absolute differences ``Norm_diff``
  against MCMC (main_script.py:721-744);
* the effective sample size of ``tfp.mcmc.effective_sample_size`` (TFP 0.24,
  main_script.py:806-812) -- restated in NumPy from TFP's published algorithm;
  TFP is absent here, so ESS parity with TFP is unpinned (its tests pin the
  known AR(1) / iid answers instead).

The moments (mean, full sample covariance) run on the GPU (``petmetrics_moments``,
include/petmetrics.h); the derived quantities are a few 48 x 48 host operations.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib

PARAMS = ('DVR', 'R1')


def sample_moments(x):
    """Mean [d] and sample covariance [d, d] (ddof = 1) of the rows of x (n, d) on the
    GPU, fp64 accumulation.  x: CUDA tensor, fp32 or fp64, n >= 2, d <= 96."""
    if not isinstance(x, torch.Tensor) or not x.is_cuda:
        raise ValueError('sample_moments expects a CUDA tensor')
    x = x.reshape(x.shape[0], -1).contiguous()
    n, d = x.shape
    if x.dtype == torch.float32:
        dt = 0
    elif x.dtype == torch.float64:
        dt = 1
    else:
        raise ValueError('samples must be float32 or float64')
    L = _lib.lib()
    mean = torch.empty(d, dtype=torch.float64, device=x.device)
    cov = torch.empty((d, d), dtype=torch.float64, device=x.device)
    work = torch.empty(int(L.petmetrics_work_doubles(d)), dtype=torch.float64, device=x.device)
    stream = C.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    rc = L.petmetrics_moments(C.c_void_p(x.data_ptr()), dt, n, d, d, C.c_void_p(mean.data_ptr()),
                              C.c_void_p(cov.data_ptr()), C.c_void_p(work.data_ptr()), stream)
    if rc != 0:
        raise ValueError(L.petmetrics_last_error().decode())
    return mean, cov


def _blocks(mean, cov, layout, n_roi=48):
    """Split full moments into per-parameter (mean [48], cov [48, 48]).
    layout 'interleaved': columns roi*2 + p (iDDPM x layout, main_script.py:116);
    'blocked': DVR 0..47 | R1 48..95 (MCMC trace)."""
    out = {}
    for p, name in enumerate(PARAMS):
        idx = np.arange(n_roi) * 2 + p if layout == 'interleaved' else np.arange(n_roi) + p * n_roi
        out[name] = (mean[idx], cov[np.ix_(idx, idx)])
    return out


def method_stats(samples, layout):
    """GPU moments of one method's samples -> {param: dict(mu, cov, corr, std)}."""
    mean, cov = sample_moments(samples)
    mean, cov = mean.cpu().numpy(), cov.cpu().numpy()
    res = {}
    for name, (mu, cv) in _blocks(mean, cov, layout).items():
        sd = np.sqrt(np.diag(cv))
        res[name] = {'mu': mu[:, None], 'cov': cv, 'corr': cv / np.outer(sd, sd) - np.identity(len(sd)),
                     'std': sd[:, None]}
    return res


def posterior_metrics(nn_samples, mcmc_draws):
    """main_script.py:721-744 for both parameters.

    nn_samples: iDDPM posterior samples (n, 48, 2) CUDA tensor ([..., 0] = DVR).
    mcmc_draws: MCMC trace (chains, draws, 96) CUDA tensor (DVR | R1) or (n, 96).
    Returns {param: {'mu'|'std'|'cov'|'corr': {'MCMC', 'NN', 'Norm_diff'}}}."""
    nn = method_stats(nn_samples.reshape(nn_samples.shape[0], -1), 'interleaved')
    mc = method_stats(mcmc_draws.reshape(-1, mcmc_draws.shape[-1]), 'blocked')
    out = {}
    for name in PARAMS:
        a, b = mc[name], nn[name]
        eye = np.identity(a['cov'].shape[0])
        out[name] = {
            'cov': {'MCMC': a['cov'], 'NN': b['cov'], 'Norm_diff': np.abs((a['cov'] - b['cov']) / a['cov'])},
            'corr': {'MCMC': a['corr'], 'NN': b['corr'],
                     'Norm_diff': np.abs((a['corr'] - b['corr']) / (a['corr'] + eye))},
            'mu': {'MCMC': a['mu'], 'NN': b['mu'], 'Norm_diff': np.abs((a['mu'] - b['mu']) / a['mu'])},
            'std': {'MCMC': a['std'], 'NN': b['std'], 'Norm_diff': np.abs((a['std'] - b['std']) / a['std'])},
        }
    return out


def _auto_covariance(x):
    """tfp.stats.auto_correlation(x, axis=0, center=True, normalize=False): the lag-k
    sums of the centred series divided by the number of terms (N - k), via FFT."""
    n = x.shape[0]
    xc = x - x.mean(axis=0, keepdims=True)
    m = 1 << int(np.ceil(np.log2(2 * n - 1)))
    f = np.fft.rfft(xc, n=m, axis=0)
    acov = np.fft.irfft(f * np.conj(f), n=m, axis=0)[:n]
    shape = (n,) + (1,) * (x.ndim - 1)
    return acov / (n - np.arange(n, dtype=np.float64)).reshape(shape)


def effective_sample_size(states, cross_chain_dims=None, filter_threshold=0.0):
    """tfp.mcmc.effective_sample_size (TFP 0.24, default filter_beta = 0).

    states: array (N, ...) with the sample axis first.  cross_chain_dims: axis index
    (or None) of the chain dimension (Vehtari et al. 2019, eq. 10).  The
    autocorrelation sum is truncated at the first lag whose autocorrelation is
    < filter_threshold."""
    x = np.asarray(states, dtype=np.float64)
    n = x.shape[0]
    acov = _auto_covariance(x)
    if cross_chain_dims is not None:
        ax = cross_chain_dims % x.ndim
        num_chains = x.shape[ax]
        if num_chains < 2:
            raise ValueError('cross_chain_dims needs more than one chain')
        between_div_n = np.var(x.mean(axis=0), axis=ax - 1, ddof=1)
        within_biased = acov[0].mean(axis=ax - 1)
        approx_var = within_biased + between_div_n
        auto_corr = 1.0 - (within_biased - acov.mean(axis=ax)) / approx_var
    else:
        num_chains = 1
        auto_corr = acov / acov[:1]
    k = np.arange(auto_corr.shape[0], dtype=np.float64).reshape((-1,) + (1,) * (auto_corr.ndim - 1))
    weighted = auto_corr * (n - k) / n
    if filter_threshold is not None:
        mask = np.cumsum(auto_corr < filter_threshold, axis=0)
        weighted = weighted * np.maximum(1.0 - mask, 0.0)
    return num_chains * n / (-1.0 + 2.0 * weighted.sum(axis=0))


def ess_pair(nn_samples, mcmc_draws):
    """The reference's ESS call pair (main_script.py:806-812): NN samples (n, 48, 2)
    as one sequence; the MCMC trace (chains, draws, 96) across chains.  -> (48, 2) each."""
    nn = np.asarray(nn_samples.cpu().numpy() if isinstance(nn_samples, torch.Tensor) else nn_samples)
    mc = np.asarray(mcmc_draws.cpu().numpy() if isinstance(mcmc_draws, torch.Tensor) else mcmc_draws)
    n_roi = nn.shape[1]
    tmp = np.stack([mc[..., :n_roi], mc[..., n_roi:]], axis=-1)          # (chains, draws, 48, 2)
    ess_mcmc = effective_sample_size(np.moveaxis(tmp, 0, -1), cross_chain_dims=-1)
    ess_nn = effective_sample_size(nn)
    return {'MCMC': ess_mcmc, 'NN': ess_nn}


# ------------------------------------------------------------------ MCMC convergence (mcmc.py:183-194)
RHAT_FLAG = 1.02          # mcmc.py:188: runs with R-hat above this are logged as possibly not converged


def _split_chains(x):
    """(chains, draws, ...) -> (2 chains, draws // 2, ...): each chain's first and last halves (an odd
    middle draw is dropped), as ArviZ's _split_chains."""
    half = x.shape[1] // 2
    return np.concatenate([x[:, :half], x[:, x.shape[1] - half:]], axis=0)


def _z_scale(x):
    """Rank normalisation over all draws of all chains (axes 0, 1; average ranks for ties), then the
    normal quantile of (rank - 3/8) / (S + 1/4) (Vehtari et al. 2021, eq. 14; ArviZ's _z_scale)."""
    from scipy.stats import norm, rankdata
    flat = x.reshape((x.shape[0] * x.shape[1],) + x.shape[2:])
    r = rankdata(flat, method='average', axis=0).reshape(x.shape)
    return norm.ppf((r - 0.375) / (flat.shape[0] + 0.25))


def _rhat_basic(x):
    """Gelman-Rubin R-hat of (chains, draws, ...): sqrt((B / W + n - 1) / n) with B = n var(chain means),
    W = mean within-chain variance (ddof = 1 both).
    W = 0 with B > 0 (chains each stuck at a different value) gives inf, as ArviZ's division does, so the
    reference's 'rhat > 1.02' flag trips; W = B = 0 gives NaN (rhat() masks fully constant draws anyway).
    Neither raises a floating-point warning."""
    n = x.shape[1]
    b = n * np.var(x.mean(axis=1), axis=0, ddof=1)
    w = np.mean(np.var(x, axis=1, ddof=1), axis=0)
    ok = w > 0
    out = np.where(b > 0, np.inf, np.nan) * np.ones(np.shape(w))
    out[ok] = np.sqrt((b[ok] / w[ok] + n - 1) / n)
    return out


def rhat(draws):
    """pm.rhat (PyMC 5.12 -> ArviZ ``rhat(method='rank')``; not vendored here, so this restates the
    published algorithm, Vehtari et al. 2021): per scalar parameter, the maximum of the rank-normalised
    split R-hat of the draws (bulk) and of their folded values |x - median| (tail).  A parameter whose
    draws are constant or not finite gets NaN.

    draws: (chains, draws, n_params) -> (n_params,) float64."""
    x = np.asarray(draws.cpu().numpy() if isinstance(draws, torch.Tensor) else draws, dtype=np.float64)
    if x.ndim == 2:
        x = x[..., None]
    s = _split_chains(x)
    bulk = _rhat_basic(_z_scale(s))
    med = np.median(s.reshape(-1, s.shape[2]), axis=0)
    tail = _rhat_basic(_z_scale(np.abs(s - med)))
    out = np.maximum(bulk, tail)
    bad = ~np.isfinite(s).all(axis=(0, 1)) | (np.ptp(s.reshape(-1, s.shape[2]), axis=0) == 0)
    out[bad] = np.nan
    return out


def convergence_report(draws, n_roi=48, threshold=RHAT_FLAG):
    """mcmc.py:183-194: R-hat of var_DVR and var_R1 from the trace (chains, draws, 2 n_roi) = [DVR | R1];
    ``flag`` is the reference's 'rhat > 1.02' condition (it then logs the file name and rhat_max)."""
    r = rhat(draws)
    rd, rr = r[:n_roi], r[n_roi:2 * n_roi]
    mx = float(np.nanmax(r))
    return {'rhat_DVR': rd, 'rhat_R1': rr, 'rhat_max': mx,
            'flag': bool(np.any(rd > threshold) or np.any(rr > threshold)), 'threshold': threshold}
