"""CPU tests of the metrics host code (pet_posterior_distribution_amd/metrics.py).

ESS restates tfp.mcmc.effective_sample_size (TFP absent here: parity with TFP is
unpinned); it is pinned to the known answers of iid and AR(1) sequences."""
import numpy as np

from pet_posterior_distribution_amd.metrics import _auto_covariance, effective_sample_size


def test_auto_covariance_definition():
    rng = np.random.default_rng(0)
    x = rng.standard_normal(37)
    ac = _auto_covariance(x)
    xc = x - x.mean()
    for k in (0, 1, 5, 36):
        assert abs(ac[k] - np.dot(xc[:37 - k], xc[k:]) / (37 - k)) < 1e-12


def test_ess_iid_close_to_n():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((20000, 3))
    ess = effective_sample_size(x)
    assert np.all(np.abs(ess / 20000 - 1) < 0.1)


def test_ess_ar1_known_answer():
    rng = np.random.default_rng(2)
    rho, n = 0.5, 50000
    e = rng.standard_normal(n)
    x = np.empty(n)
    x[0] = e[0]
    for i in range(1, n):
        x[i] = rho * x[i - 1] + np.sqrt(1 - rho ** 2) * e[i]
    ess = effective_sample_size(x)
    assert abs(ess / (n * (1 - rho) / (1 + rho)) - 1) < 0.1


def test_ess_cross_chain_iid():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((5000, 4, 2))          # (draws, dim, chains)
    ess = effective_sample_size(x, cross_chain_dims=-1)
    assert ess.shape == (4,)
    assert np.all(np.abs(ess / 10000 - 1) < 0.15)
