"""CPU tests of the MH oracles: the C restatement (oracle/mh_ref.c) is pinned to the
NumPy restatement (oracle/srtm2_ref.py), whose SRTM2 is pinned to the reference's own
kinetic_model outputs (tests/golden/g2_srtm2.npz)."""
import os

import numpy as np
import pytest

from oracle import srtm2_ref as K
from tests.helpers import mh_problem

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


@pytest.fixture(scope='module')
def g2():
    return np.load(os.path.join(GOLD, 'g2_srtm2.npz'))


@pytest.fixture(scope='module')
def cmh():
    from oracle import mh_c
    try:
        mh_c.lib()
    except FileNotFoundError:
        import subprocess
        subprocess.check_call(['make', '-C', os.path.join(os.path.dirname(GOLD), '..', 'oracle')])
    return mh_c


def _np_logp(P):
    def logp(x):
        return K.log_posterior(x[:48], x[48:], P['k2p'], P['y_obs'], P['sigma_noise'], P['time_vector'],
                               P['tac_ref'], P['mu_DVR'], P['Cov_DVR'], P['mu_R1'], P['Cov_R1'])
    return logp


def test_c_logp_matches_numpy(g2, cmh):
    P = mh_problem(g2, case=1)
    prob = cmh.MHProblem(**P)
    const = -0.5 * (96 * np.log(2 * np.pi) + np.linalg.slogdet(P['Cov_DVR'])[1] + np.linalg.slogdet(P['Cov_R1'])[1])
    rng = np.random.default_rng(5)
    x = np.concatenate([P['mu_DVR'] * (1 + 0.05 * rng.standard_normal((4, 48))),
                        P['mu_R1'] * (1 + 0.05 * rng.standard_normal((4, 48)))], axis=1)
    got = prob.logp_unnormalised(x) + const
    ref = np.array([_np_logp(P)(xi) for xi in x])
    np.testing.assert_allclose(got, ref, rtol=1e-11)


@pytest.mark.parametrize('tune_interval,vs0', [(100, True), (2, True), (2, False)])
def test_c_chain_path_matches_numpy(g2, cmh, tune_interval, vs0):
    """Incremental C sampler == full-logp NumPy sampler on the same Philox stream
    (tune_interval=2 exercises the PyMC tune table; vs0 = pymc's sweep-start reference)."""
    P = mh_problem(g2, case=2)
    prob = cmh.MHProblem(**P)
    draws, tune, seed = 4, 5, 321
    st, acc, last = prob.run(2, draws, tune, seed, tune_interval=tune_interval, threads=2, vs_sweep_start=vs0)
    x0 = np.concatenate([P['mu_DVR'], P['mu_R1']])
    for ch in range(2):
        dr, kacc = K.metropolis_elemwise_philox(_np_logp(P), x0, draws, tune, seed, ch, tune_interval=tune_interval,
                                                vs_sweep_start=vs0)
        np.testing.assert_allclose(st[ch, :, 1], dr.mean(0), rtol=1e-10, atol=1e-13)
        np.testing.assert_allclose(st[ch, :, 2], ((dr - dr.mean(0)) ** 2).sum(0), rtol=1e-7, atol=1e-13)
        np.testing.assert_allclose(last[ch], dr[-1], rtol=1e-12)
        np.testing.assert_array_equal(acc[ch], kacc)


def test_c_sampler_thread_invariance(g2, cmh):
    P = mh_problem(g2, case=0)
    prob = cmh.MHProblem(**P)
    a = prob.run(6, 20, 30, 99, threads=1)
    b = prob.run(6, 20, 30, 99, threads=4)
    for u, v in zip(a, b):
        np.testing.assert_array_equal(u, v)


def test_logphi_polynomial_vs_scipy():
    """The MH kernels' log Phi (csrc/logphi_coef.h, scripts/gen_logphi.py): piecewise degree-14
    polynomials on [0, 10), evaluated by Horner as the kernel does, against scipy.special.log_ndtr
    (the reference's TruncatedNormal normaliser, mcmc.py:151-155) on a dense grid (<= 1.5e-15: scipy's
    own error) and against the exact function (mpmath, 30 digits) on every 40th point (<= 2.5e-16;
    the values' own fp64 rounding is 1.1e-16 at x = 0)."""
    import re
    from scipy.special import log_ndtr
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            'pet_posterior_distribution_amd', 'csrc', 'logphi_coef.h')).read()
    rows = re.findall(r'\{([^{}]+)\}', hdr[hdr.index('PETMH_LOGPHI_COEF'):])
    tab = np.array([[float(v) for v in r.split(',')] for r in rows])
    assert tab.shape == (10, 15)
    x = np.concatenate([np.linspace(0.0, 10.0, 200001)[:-1], [1e-300, 0.5, 9.999999999]])
    k = np.clip(x.astype(np.int64), 0, 9)
    u = x - (k + 0.5)
    p = np.zeros_like(x)
    for j in range(14, -1, -1):
        p = p * u + tab[k, j]
    err = np.abs(p - log_ndtr(x))          # scipy itself is off by up to ~9e-16 near x = 0
    assert err.max() <= 1.5e-15, (err.max(), x[err.argmax()])
    import mpmath as mp
    mp.mp.dps = 30
    xs = x[::40]
    exact = np.array([float(mp.log(mp.ncdf(mp.mpf(float(v))))) for v in xs])
    e2 = np.abs(p[::40] - exact)
    assert e2.max() <= 2.5e-16, (e2.max(), xs[e2.argmax()])
