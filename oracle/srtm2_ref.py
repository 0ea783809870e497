"""CPU oracle for the SRTM2 forward model and the Metropolis-Hastings posterior.

TEST INFRASTRUCTURE ONLY (see oracle/iddpm_ref.py header): imported by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the product.

Restates, in float64 NumPy:
* kinetic_model.interp1d_linear_vec          kinetic_model.py:35-57
* kinetic_model.estimate_continuous_convolution  kinetic_model.py:12-32
* kinetic_model.SRTM2.create_activity_curve  kinetic_model.py:142-158
* the MH model of mcmc.py:147-155 (log posterior) and PyMC's element-wise
  Metropolis with NormalProposal and tune_interval=100 scaling (pymc 5.12,
  requirements.txt:6, ``Metropolis.astep`` with ``elemwise_update``: per draw one
  proposal vector, shuffled element order, each element's ratio taken against
  the sweep-start point).  PyMC is NOT vendored in the reference and is not
  installed here: restated from PyMC's published source, parity with PyMC
  itself is unpinned.

Pinning: SRTM2 and the interpolation are checked bit-for-bit-close (1e-12)
against the imported reference kinetic_model (tests/golden/g2_srtm2.npz,
made by tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np
from scipy.special import log_ndtr


def interp1d_linear_vec(x, xp, fp, dim=0):
    """kinetic_model.py:35-57 (note the index -1 wrap for x == xp[0])."""
    fp_in = fp.reshape([-1, 1]) if fp.ndim == 1 else fp
    distances = np.abs(xp[np.newaxis, :] - x[:, np.newaxis]).astype(np.float64)
    x_indices = np.searchsorted(xp, x)
    weights = np.zeros_like(distances)
    idx = np.arange(len(x_indices))
    weights[idx, x_indices] = distances[idx, x_indices - 1]
    weights[idx, x_indices - 1] = distances[idx, x_indices]
    weights /= np.sum(weights, axis=1)[:, np.newaxis]
    output = np.tensordot(weights, fp_in, axes=[[1], [dim]])
    return output.reshape([x.size] + list(fp.shape[1:]))


def interp_weights(x, xp):
    """The weight matrix W of interp1d_linear_vec: interp1d_linear_vec(x, xp, f) == W @ f."""
    distances = np.abs(xp[np.newaxis, :] - x[:, np.newaxis]).astype(np.float64)
    x_indices = np.searchsorted(xp, x)
    W = np.zeros_like(distances)
    idx = np.arange(len(x_indices))
    W[idx, x_indices] = distances[idx, x_indices - 1]
    W[idx, x_indices - 1] = distances[idx, x_indices]
    return W / W.sum(axis=1)[:, np.newaxis]


def estimate_continuous_convolution(x, y0, y1, num_points_resample=None):
    """kinetic_model.py:12-32.  scipy convolve1d(origin=-n//2) == causal np.convolve[:n]."""
    n = 2 * np.unique(x).size if num_points_resample is None else num_points_resample
    x_rs = np.linspace(np.min(x), np.max(x), n)
    dx = x_rs[1] - x_rs[0]
    y0_rs = np.interp(x_rs, x, y0)
    y1_rs = interp1d_linear_vec(x_rs, x, y1)
    if y1.ndim == 1:
        conv = np.convolve(y0_rs, y1_rs)[:n] * dx
    else:
        conv = np.stack([np.convolve(y0_rs, y1_rs[:, k])[:n] for k in range(y1_rs.shape[1])], axis=1) * dx
    return interp1d_linear_vec(x, x_rs, conv)


def srtm2_tac(time_vector, tac_ref, DVR, R1, k2p):
    """SRTM2.create_activity_curve (kinetic_model.py:142-158): (n_frames, n_roi)."""
    DVR = np.asarray(DVR, dtype=np.float64)
    R1 = np.asarray(R1, dtype=np.float64)
    c_r = np.asarray(tac_ref, dtype=np.float64)
    t = np.asarray(time_vector, dtype=np.float64)
    c_r_v = c_r.reshape([-1] + [1] * DVR.ndim)
    k2 = k2p * R1
    k2a = k2 / DVR
    c_exp = np.exp((-k2a).reshape([1] + list(DVR.shape)) * t.reshape([-1] + [1] * DVR.ndim))
    return R1 * c_r_v + (k2 - R1 * k2a) * estimate_continuous_convolution(t, c_r, c_exp)


def srtm2_operator(time_vector, tac_ref):
    """Constant (n_frames x n_frames) M with  conv_term = M @ exp(-k2a t):
    M = W_down . Toeplitz(y0) . W_up . dx  (exact reassociation of :12-32)."""
    t = np.asarray(time_vector, dtype=np.float64)
    n = 2 * np.unique(t).size
    x_rs = np.linspace(t.min(), t.max(), n)
    dx = x_rs[1] - x_rs[0]
    y0 = np.interp(x_rs, t, np.asarray(tac_ref, dtype=np.float64))
    Tm = np.zeros((n, n))
    for i in range(n):
        Tm[i, :i + 1] = y0[i::-1]
    return interp_weights(t, x_rs) @ Tm @ interp_weights(x_rs, t) * dx


# --------------------------------------------------------------------------
# mcmc.py:147-155 model
# --------------------------------------------------------------------------

def mvn_logpdf(x, mu, cov):
    d = x - mu
    L = np.linalg.cholesky(cov)
    z = np.linalg.solve(L, d)
    return -0.5 * (len(mu) * np.log(2 * np.pi) + 2 * np.log(np.diag(L)).sum() + z @ z)


def trunc_normal_lower0_logpdf(y, mu, sigma):
    """pm.TruncatedNormal(mu, sigma, lower=0) logp: log phi(z) - log sigma - log Phi(mu/sigma)."""
    z = (y - mu) / sigma
    return -0.5 * z * z - 0.5 * np.log(2 * np.pi) - np.log(sigma) - log_ndtr(mu / sigma)


def log_posterior(DVR, R1, k2p, y_obs, sigma_noise, time_vector, tac_ref, mu_DVR, Cov_DVR, mu_R1, Cov_R1):
    """Joint log density of mcmc.py:147-155 (MvN priors + truncated-normal likelihood)."""
    sn = srtm2_tac(time_vector, tac_ref, DVR, R1, k2p).T                  # (48, 54)  :39
    sn = np.where(sn < 0, 1e-6, sn)                                      # :152
    sig = np.sqrt(sn) * sigma_noise                                      # :153
    ll = trunc_normal_lower0_logpdf(y_obs, sn, sig).sum()
    return mvn_logpdf(DVR, mu_DVR, Cov_DVR) + mvn_logpdf(R1, mu_R1, Cov_R1) + ll


def pymc_tune(scale, acc_rate):
    """pymc.step_methods.metropolis.tune (pymc 5.12)."""
    return np.select([acc_rate < 0.001, acc_rate < 0.05, acc_rate < 0.2, acc_rate > 0.95, acc_rate > 0.75,
                      acc_rate > 0.5], [scale * 0.1, scale * 0.5, scale * 0.9, scale * 10.0, scale * 2.0,
                                        scale * 1.1], scale)


def _pymc_sweep(logp, x, lp0, q, order, log_u, tune_acc, kept_acc, keep, vs_sweep_start=True):
    """One Metropolis.astep with element-wise updates (pymc 5.12 metropolis.py):
    q = x + delta was drawn for every element up front; elements are visited in the
    shuffled `order`; element k's proposal is the running state with q[k] swapped in,
    and -- as in pymc's ``delta_logp(q_temp, q0)`` -- it is compared against the
    sweep-START state x (vs_sweep_start=False: against the running state).
    metrop_select accepts iff the ratio is finite and log u < ratio."""
    q_temp = x.copy()
    lp_run = lp0
    for k in order:
        q_temp[k] = q[k]
        lpp = logp(q_temp)
        mr = lpp - (lp0 if vs_sweep_start else lp_run)
        if np.isfinite(mr) and log_u[k] < mr:
            lp_run = lpp
            tune_acc[k] += 1
            if keep:
                kept_acc[k] += 1
        else:
            q_temp[k] = x[k]
    return q_temp, lp_run


def metropolis_elemwise(logp, x0, n_draws, n_tune, rng, tune_interval=100, scaling=1.0, vs_sweep_start=True):
    """PyMC 5.12 Metropolis(NormalProposal) on a vector variable (elemwise_update):
    per draw: tune (every tune_interval tuning draws, per-element pymc_tune on the
    acceptance rate), delta = N(0,1) * scaling for all elements, shuffle the element
    order, then the element-wise accept/reject sweep of _pymc_sweep."""
    x = np.array(x0, dtype=np.float64)
    n = x.size
    s = np.full(n, float(scaling))
    acc = np.zeros(n)
    kept = np.zeros(n)
    out = np.empty((n_draws,) + x.shape)
    for it in range(n_tune + n_draws):
        if it < n_tune and it > 0 and it % tune_interval == 0:
            s = pymc_tune(s, acc / tune_interval)
            acc[:] = 0
        q = x + rng.standard_normal(n) * s
        order = rng.permutation(n)
        log_u = np.log(rng.uniform(size=n))
        x, _ = _pymc_sweep(logp, x, logp(x), q, order, log_u, acc, kept, it >= n_tune, vs_sweep_start)
        if it >= n_tune:
            out[it - n_tune] = x
    return out


def philox_mh_block(seed, chain, it, k):
    """The GPU sampler's counter-based draws for element k of sweep `it` of `chain`:
    Philox4x32-10(counter = (k, it, chain_lo, chain_hi), key = seed) -> N(0,1)
    proposal (Box-Muller cos of words 0, 1), accept uniform (word 2) and the
    element's sort key for the sweep's shuffled order (word 3)."""
    from oracle.iddpm_ref import philox4x32_10
    q = philox4x32_10(k, it, chain & 0xffffffff, chain >> 32, seed & 0xffffffff, (seed >> 32) & 0xffffffff)
    u1 = (float(q[0]) + 1.0) * 2.0 ** -32
    u2 = (float(q[1]) + 0.5) * 2.0 ** -32
    ua = (float(q[2]) + 0.5) * 2.0 ** -32
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2), ua, int(q[3])


def philox_mh_noise(seed, chain, it, k):
    z, ua, _ = philox_mh_block(seed, chain, it, k)
    return z, ua


def philox_sweep(seed, chain, it, n=96):
    """(z[n], ua[n], order): order = elements by ascending (word-3 key, index)."""
    blk = [philox_mh_block(seed, chain, it, k) for k in range(n)]
    z = np.array([b[0] for b in blk])
    ua = np.array([b[1] for b in blk])
    keys = np.array([b[2] for b in blk], dtype=np.uint64)
    return z, ua, np.argsort(keys, kind='stable')


def metropolis_elemwise_philox(logp, x0, n_draws, n_tune, seed, chain, tune_interval=100, scaling=1.0,
                               vs_sweep_start=True):
    """metropolis_elemwise with the GPU sampler's noise stream (identical chain path)."""
    x = np.array(x0, dtype=np.float64)
    n = x.size
    s = np.full(n, float(scaling))
    acc = np.zeros(n)
    kept = np.zeros(n)
    out = np.empty((n_draws,) + x.shape)
    for it in range(n_tune + n_draws):
        if it < n_tune and it > 0 and it % tune_interval == 0:
            s = pymc_tune(s, acc / tune_interval)
            acc[:] = 0
        z, ua, order = philox_sweep(seed, chain, it, n)
        x, _ = _pymc_sweep(logp, x, logp(x), x + z * s, order, np.log(ua), acc, kept, it >= n_tune,
                           vs_sweep_start)
        if it >= n_tune:
            out[it - n_tune] = x
    return out, kept
