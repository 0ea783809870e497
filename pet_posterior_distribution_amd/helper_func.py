"""Host-side helpers mirroring the reference's helper_func.py.

Only what the sampling path needs: the beta schedules (helper_func.py:210-268),
``chunker`` (:12-13) and ``trunc_normal`` (:146-150, used by the synthetic TAC
generator).  Schedules are computed in float32 NumPy exactly like the
reference (NP_DTYPE = float32), so the tables handed to libpetdiff are
bit-identical to the reference's buffers (pinned by tests/golden/G1).
"""
from __future__ import annotations

import numpy as np

NP_DTYPE = np.float32


def chunker(seq, size):
    """helper_func.py:12-13."""
    return (seq[pos:pos + size] for pos in range(0, len(seq), size))


def cos_beta_schedule(timesteps, offset_s=0.008, max_beta=0.999):
    """Cosine schedule (Nichol & Dhariwal 2021), helper_func.py:210-219."""
    def alpha_bar(t):
        return np.cos((t + offset_s) / (1 + offset_s) * np.pi / 2, dtype=NP_DTYPE) ** 2
    beta = [min(1 - alpha_bar((i + 1) / timesteps) / alpha_bar(i / timesteps), max_beta)
            for i in range(timesteps)]
    return np.array(beta, dtype=NP_DTYPE)


def sigmoid_beta_schedule(timesteps, beta_start, beta_end):
    """helper_func.py:222-225."""
    b = np.linspace(-6, 6, timesteps, dtype=NP_DTYPE)
    return 1 / (1 + np.exp(-b, dtype=NP_DTYPE)) * (beta_end - beta_start) + beta_start


def quadratic_beta_schedule(timesteps, beta_start, beta_end):
    """helper_func.py:228-230."""
    return np.linspace(beta_start ** 0.5, beta_end ** 0.5, timesteps, dtype=NP_DTYPE) ** 2


def linear_beta_schedule(timesteps, beta_start, beta_end):
    """helper_func.py:233-234."""
    return np.linspace(beta_start, beta_end, timesteps, dtype=NP_DTYPE)


def get_beta_schedule(schedule_name, timesteps, **kwargs):
    """helper_func.py:237-268 (same names, same NotImplementedError)."""
    beta_start = kwargs.get('beta_start', None)
    beta_end = kwargs.get('beta_end', None)
    offset_s = kwargs.get('offset_s', None)
    max_beta = kwargs.get('max_beta', None)
    name = schedule_name.lower()
    if name in ('lin', 'linear'):
        return linear_beta_schedule(timesteps, beta_start, beta_end)
    if name in ('quad', 'quadratic'):
        return quadratic_beta_schedule(timesteps, beta_start, beta_end)
    if name in ('sig', 'sigmoid'):
        return sigmoid_beta_schedule(timesteps, beta_start, beta_end)
    if name in ('cos', 'cosine'):
        return cos_beta_schedule(timesteps, offset_s=offset_s, max_beta=max_beta)
    raise NotImplementedError('Schedule name ({}) not recognized or not implemented.'.format(schedule_name))


def trunc_normal(mean=0, std=1, low=0, upp=None, **kwargs):
    """helper_func.py:146-150 (scipy truncnorm)."""
    from scipy.stats import truncnorm
    if upp is None:
        upp = np.inf
    return truncnorm.rvs((low - mean) / std, (upp - mean) / std, loc=mean, scale=std, **kwargs)
