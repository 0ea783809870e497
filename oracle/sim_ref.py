"""CPU oracle of the GPU synthetic-TAC generator (include/petsim.h).

TEST INFRASTRUCTURE ONLY (see oracle/iddpm_ref.py header).

Restates sample_sim_data.py:139-215 (+ helper_func.py:146-162) with the generator's
counter-based stream: helper_func.truncnormal_samples as whole-vector rejection of
MvNormal draws (mu + L z, L = cholesky_psd(Cov), a semi-definite Cholesky); SRTM2 activity = create_activity_curve *
dt (kinetic_model.py:142-158 via oracle/srtm2_ref.srtm2_tac, pinned to the
reference's outputs); a negative TAC redraws (DVR, R1, ref) (sample_sim_data.py:175-181);
noise noisy/dt = x/dt + sqrt(x/dt) TN(0, sigma, low = -sqrt(x/dt)) by rejection.
Philox4x32-10(counter = (call, purpose << 24 | outer << 12 | inner, g_lo, g_hi),
key = seed), Box-Muller of words 0/1 (cos for even, sin for odd normal index).
"""
from __future__ import annotations

import numpy as np

from oracle.iddpm_ref import philox4x32_10
from oracle.srtm2_ref import srtm2_tac

MAX_INNER, MAX_OUTER = 1024, 64


def normal(seed, g, call, tag, which):
    q = philox4x32_10(call, tag, g & 0xffffffff, g >> 32, seed & 0xffffffff, (seed >> 32) & 0xffffffff)
    u1 = (float(q[0]) + 1.0) * 2.0 ** -32
    u2 = (float(q[1]) + 0.5) * 2.0 ** -32
    r = np.sqrt(-2.0 * np.log(u1))
    return r * (np.sin(2 * np.pi * u2) if which else np.cos(2 * np.pi * u2))


def draw_truncated_mvn(seed, g, purpose, outer, mu, L):
    d = len(mu)
    for inner in range(MAX_INNER):
        tag = (purpose << 24) | (outer << 12) | inner
        z = np.array([normal(seed, g, i >> 1, tag, i & 1) for i in range(d)])
        x = mu + L @ z
        if not (x < 0).any():
            return x, inner + 1
    return x, -1


def cholesky_psd(A):
    """Lower factor L, L L^T = A, of a positive SEMI-definite A (the GPU generator's, sim_kernels.hip):
    pivots <= 1e-12 max diag(A) give zero columns (the reference's Cov_tac_ref has rank 49 of 54;
    np.random.multivariate_normal at helper_func.py:158 accepts it)."""
    A = np.asarray(A, dtype=np.float64)
    n = A.shape[0]
    tol = 1e-12 * np.diag(A).max()
    L = np.zeros_like(A)
    for i in range(n):
        for j in range(i + 1):
            s = A[i, j] - L[i, :j] @ L[j, :j]
            if i == j:
                if s < -1e-8 * np.diag(A).max():
                    raise np.linalg.LinAlgError('not positive semi-definite')
                L[i, i] = np.sqrt(s) if s > tol else 0.0
            else:
                L[i, j] = s / L[j, j] if L[j, j] > 0 else 0.0
    return L


def simulate_sample(P, seed, g):
    """One sample g: dict(DVR, R1, ref, tac (48, 54) activity, noisy (48, 54) activity)."""
    LD, LR, LC = (cholesky_psd(P[k]) for k in ('Cov_DVR', 'Cov_R1', 'Cov_tac_ref'))
    tv, dt = P['time_vector'], P['dt']
    for outer in range(MAX_OUTER):
        dvr, _ = draw_truncated_mvn(seed, g, 0, outer, P['mu_DVR'], LD)
        r1, _ = draw_truncated_mvn(seed, g, 1, outer, P['mu_R1'], LR)
        ref, _ = draw_truncated_mvn(seed, g, 2, outer, P['mu_tac_ref'], LC)
        tac = (srtm2_tac(tv, ref, dvr, r1, P['k2p']) * dt[:, None]).T        # (48, 54)
        if not (tac < 0).any():
            break
    xc = tac / dt[None, :]
    s = np.sqrt(xc)
    noisy = np.empty_like(tac)
    sig = P['sigma_noise']
    for idx in range(tac.size):
        r, f = divmod(idx, tac.shape[1])
        for k in range(MAX_INNER):
            nz = sig[r, f] * normal(seed, g, idx, (3 << 24) | k, 0)
            if nz >= -s[r, f]:
                break
        noisy[r, f] = (xc[r, f] + s[r, f] * nz) * dt[f]
    return {'DVR': dvr, 'R1': r1, 'ref': ref, 'tac': tac, 'noisy': noisy}
