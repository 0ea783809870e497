"""Synthetic PET inputs of the reference's shapes (host side, not the hot path).

Restates the data-generation side of the reference so that benchmarks and
tests have realistic conditions without the Git-LFS test set:

* ``acquisition_time_frames`` -- the 54-frame protocol (sample_sim_data.py:29-85);
* ``srtm2_tac`` -- SRTM2 forward model (kinetic_model.py:12-57, 142-158), NumPy
  fp64, used here only to synthesise inputs (the GPU kernel is in petmh);
* ``noisy_tac`` -- the truncated Poisson-like noise model (sample_sim_data.py:193-215);
* ``make_condition`` -- condition rows [tac_noisy/dt (48 ROIs) | tac_ref] as in
  main_script.py:110-113.

The prior is the reference's own (``reference_prior``): the arrays of
``prior_stats_nROI48.pik`` (sample_sim_data.py:106-126, mcmc.py:84-93), shipped as
``data/prior_stats_nROI48.npz``.  They were extracted by tests/golden/make_golden.py,
which parses the pickle's byte stream with a disassembler and rebuilds only literal
data (no unpickling of reference files).  ``synthetic_prior`` (the rounds 1-2
default, seeded synthetic statistics of the same shapes) stays for the G2 fixture.
"""
from __future__ import annotations

import numpy as np

N_ROI, N_FRAMES = 48, 54
MK_HALF_T = 109.8   # sample_sim_data.py:95


def acquisition_time_frames():
    """(54, 2) frame [start, end] in minutes (sample_sim_data.py:29-82)."""
    edges = ([0, 10, 20, 30, 40, 50, 60] + list(range(75, 181, 15)) + list(range(210, 361, 30)) +
             list(range(420, 841, 60)) + list(range(960, 1801, 120)) + list(range(2100, 7201, 300)))
    e = np.asarray(edges, dtype=np.float64) / 60.0
    return np.stack([e[:-1], e[1:]], axis=1)


def time_grid():
    f = acquisition_time_frames()
    return f[:, 1].copy(), (f[:, 1] - f[:, 0]).copy()     # time_vector, dt (:84-85)


def _random_cov_psd(diag, rng, rho=0.5):
    """helper_func.random_cov_psd (helper_func.py:165-204)."""
    std = np.sqrt(diag)
    n = len(diag)
    A = rng.standard_normal((n, n))
    Rm = A @ A.T
    d = np.sqrt(np.diag(Rm))
    Rm = Rm / d[:, None] / d
    eig, Q = np.linalg.eigh(Rm)
    eig = rho * eig + (1 - rho)
    Rm = Q @ np.diag(eig) @ Q.T
    return (std[:, None] * Rm) * std


def reference_tac(time_vector):
    """Smooth cerebellum-like reference TAC (arbitrary units, synthetic)."""
    t = np.asarray(time_vector, dtype=np.float64)
    return 1.2 * (t / 1.5) * np.exp(1 - t / 1.5) + 0.35 * np.exp(-t / 70.0) * (1 - np.exp(-t / 0.8))


_REF_PRIOR = None


def reference_prior():
    """The reference's prior statistics (prior_stats_nROI48.pik): mu_DVR, Cov_DVR, mu_R1, Cov_R1 (48),
    mu_k2p, mu_tac_ref, Cov_tac_ref (54) as float64 arrays, ROI_names; the default prior of every
    generator here (the data the reference's test TACs, training set and MCMC priors come from)."""
    global _REF_PRIOR
    if _REF_PRIOR is None:
        import os
        with np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data', 'prior_stats_nROI48.npz')) as z:
            _REF_PRIOR = {k: (z[k].astype(np.float64) if z[k].dtype.kind == 'f' else z[k]) for k in z.files}
        _REF_PRIOR['mu_k2p'] = np.float64(_REF_PRIOR['mu_k2p'])
    return {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in _REF_PRIOR.items()}


def synthetic_prior(seed=2025):
    """Prior statistics with the shapes of prior_stats_nROI48.pik (synthetic values)."""
    rng = np.random.default_rng(seed)
    tv, _ = time_grid()
    mu_DVR = rng.uniform(0.95, 1.6, N_ROI)
    mu_R1 = rng.uniform(0.6, 1.0, N_ROI)
    mu_tac_ref = reference_tac(tv)
    return dict(mu_DVR=mu_DVR, Cov_DVR=_random_cov_psd((0.08 * mu_DVR) ** 2, rng),
                mu_R1=mu_R1, Cov_R1=_random_cov_psd((0.06 * mu_R1) ** 2, rng),
                mu_k2p=np.float64(0.015), mu_tac_ref=mu_tac_ref,
                Cov_tac_ref=_random_cov_psd((0.03 * mu_tac_ref + 1e-3) ** 2, rng))


def interp_matrix(x, xp):
    """Weights W with  W @ fp == kinetic_model.interp1d_linear_vec(x, xp, fp)  (kinetic_model.py:35-57)."""
    x = np.asarray(x, dtype=np.float64)
    xp = np.asarray(xp, dtype=np.float64)
    dist = np.abs(xp[None, :] - x[:, None])
    idx = np.searchsorted(xp, x)
    W = np.zeros_like(dist)
    r = np.arange(len(idx))
    W[r, idx] = dist[r, idx - 1]
    W[r, idx - 1] = dist[r, idx]
    W /= W.sum(axis=1)[:, None]
    return W


def srtm2_tac(DVR, R1, k2p, tac_ref, time_vector):
    """SRTM2.create_activity_curve (kinetic_model.py:142-158) -> (54, n_roi) fp64."""
    DVR = np.asarray(DVR, dtype=np.float64)
    R1 = np.asarray(R1, dtype=np.float64)
    tv = np.asarray(time_vector, dtype=np.float64)
    c_r = np.asarray(tac_ref, dtype=np.float64)
    k2 = k2p * R1
    k2a = k2 / DVR
    c_exp = np.exp(-k2a[None, :] * tv[:, None])                       # (54, n)
    n = 2 * np.unique(tv).size
    x_rs = np.linspace(tv.min(), tv.max(), n)
    dx = x_rs[1] - x_rs[0]
    y0 = np.interp(x_rs, tv, c_r)
    y1 = interp_matrix(x_rs, tv) @ c_exp                               # (n, n_roi)
    conv = np.stack([np.convolve(y0, y1[:, r])[:n] for r in range(y1.shape[1])], axis=1) * dx
    return R1 * c_r[:, None] + (k2 - R1 * k2a) * (interp_matrix(tv, x_rs) @ conv)


def noisy_tac(tac, dt, time_vector, sigma_roi, rng):
    """Noise model of sample_sim_data.py:193-215; tac (n_roi, 54) concentration."""
    from scipy.stats import truncnorm
    lam = np.log(2) / MK_HALF_T
    sigma_noise = sigma_roi[:, None] / np.sqrt(dt[None, :] * np.exp(-lam * time_vector))
    x = np.maximum(tac, 0.0)
    s = np.sqrt(x)
    low = (-s) / sigma_noise
    e = truncnorm.rvs(low, np.inf, loc=0.0, scale=sigma_noise, random_state=rng)
    return x + s * e, sigma_noise


def make_condition(seed=0, prior=None, mean_sigma_noise=0.1, return_truth=False):
    """One synthetic test TAC -> condition (49, 54) float32 (main_script.py:110-113)."""
    prior = prior or reference_prior()
    rng = np.random.default_rng(seed)
    tv, dt = time_grid()
    while True:
        DVR = rng.multivariate_normal(prior['mu_DVR'], prior['Cov_DVR'])
        R1 = rng.multivariate_normal(prior['mu_R1'], prior['Cov_R1'])
        ref = rng.multivariate_normal(prior['mu_tac_ref'], prior['Cov_tac_ref'])
        if (DVR > 0).all() and (R1 > 0).all() and (ref > 0).all():
            tac = srtm2_tac(DVR, R1, prior['mu_k2p'], ref, tv).T          # (48, 54)
            if (tac >= 0).all():
                break
    from scipy.stats import truncnorm
    sigma_roi = truncnorm.rvs(-1 / 0.3, np.inf, loc=mean_sigma_noise, scale=0.3 * mean_sigma_noise,
                              size=N_ROI, random_state=rng)
    tac_noisy, sigma_noise = noisy_tac(tac, dt, tv, sigma_roi, rng)
    cond = np.concatenate([tac_noisy, ref[None, :]], axis=0).astype(np.float32)
    if return_truth:
        return cond, dict(DVR=DVR, R1=R1, k2p=prior['mu_k2p'], tac_ref=ref, tac=tac,
                          sigma_noise=sigma_noise, time_vector=tv, dt=dt)
    return cond


def mh_problem(seed=0, prior=None, mean_sigma_noise=0.1):
    """The MH inputs of one synthetic test TAC (mcmc.py:73-137): frame times, reference
    TAC, fixed k2', y_obs, per-frame noise sigmas and the MvNormal priors."""
    prior = prior or reference_prior()
    cond, truth = make_condition(seed, prior, mean_sigma_noise, return_truth=True)
    return dict(time_vector=truth['time_vector'], tac_ref=truth['tac_ref'], k2p=float(truth['k2p']),
                y_obs=cond[:N_ROI].astype(np.float64), sigma_noise=truth['sigma_noise'],
                mu_DVR=prior['mu_DVR'], Cov_DVR=prior['Cov_DVR'], mu_R1=prior['mu_R1'], Cov_R1=prior['Cov_R1'])


def dataset_sigma_noise(mean_sigma_noise=0.1, rng=None):
    """sample_sim_data.py:190-194: per-ROI std drawn once per dataset, scaled per frame."""
    from scipy.stats import truncnorm
    rng = np.random.default_rng(0) if rng is None else rng
    tv, dt = time_grid()
    sigma_roi = truncnorm.rvs(-1 / 0.3, np.inf, loc=mean_sigma_noise, scale=0.3 * mean_sigma_noise, size=N_ROI,
                              random_state=rng)
    lam = np.log(2) / MK_HALF_T
    return sigma_roi[:, None] / np.sqrt(dt[None, :] * np.exp(-lam * tv[None, :]))


def simulate_dataset(n, prior=None, mean_sigma_noise=0.1, seed=0, sample_offset=0, sigma_noise=None, device=None):
    """GPU synthetic test set (include/petsim.h; sample_sim_data.py:139-215).

    Returns the reference's saved fields (varDVR, varR1, vark2p, vartacref,
    tac_sampled, tac_noisy_sampled as activity, sigma_noise, time_vector, dt) as
    CUDA tensors / arrays, plus ``condition`` (n, 49, 54) fp32 = [tac_noisy/dt | tac_ref]
    (main_script.py:107-113) and the per-sample redraw counts ``attempts``."""
    import ctypes as C

    import torch

    from . import _lib
    prior = prior or reference_prior()
    tv, dt = time_grid()
    if sigma_noise is None:
        sigma_noise = dataset_sigma_noise(mean_sigma_noise, np.random.default_rng(seed))
    f = lambda a: np.ascontiguousarray(a, dtype=np.float64)   # noqa: E731
    keep = [f(tv), f(dt), f(prior['mu_DVR']), f(prior['Cov_DVR']), f(prior['mu_R1']), f(prior['Cov_R1']),
            f(prior['mu_tac_ref']), f(prior['Cov_tac_ref']), f(sigma_noise)]
    P = _lib.PetsimPrior(N_ROI, N_FRAMES, *(a.ctypes.data for a in keep[:8]), float(prior['mu_k2p']),
                         keep[8].ctypes.data)
    dev = torch.device('cuda', torch.cuda.current_device() if device is None else device)
    o = lambda *shape: torch.empty(shape, dtype=torch.float64, device=dev)   # noqa: E731
    DVR, R1, REF, TAC, NOISY = o(n, N_ROI), o(n, N_ROI), o(n, N_FRAMES), o(n, N_ROI, N_FRAMES), o(n, N_ROI, N_FRAMES)
    cond = torch.empty((n, N_ROI + 1, N_FRAMES), dtype=torch.float32, device=dev)
    att = torch.empty(n, dtype=torch.int32, device=dev)
    ptr = lambda t: C.c_void_p(t.data_ptr())   # noqa: E731
    rc = _lib.lib().petsim_generate(C.byref(P), int(seed), int(sample_offset), int(n), dev.index, ptr(DVR), ptr(R1),
                                    ptr(REF), ptr(TAC), ptr(NOISY), ptr(cond), ptr(att),
                                    C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    if rc != 0:
        raise ValueError(_lib.lib().petsim_last_error().decode())
    return {'varDVR': DVR, 'varR1': R1, 'vark2p': np.full(n, float(prior['mu_k2p'])), 'vartacref': REF,
            'tac_sampled': TAC, 'tac_noisy_sampled': NOISY, 'sigma_noise': sigma_noise, 'time_vector': tv,
            'dt': dt, 'condition': cond, 'attempts': att}
