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


def _rhat_reference_loop(x):
    """Straight restatement of Vehtari et al. (2021) rank-normalised split R-hat, one parameter at a time
    (ranks by argsort with explicit tie averaging), to pin metrics.rhat's vectorised form."""
    from scipy.stats import norm
    out = []
    for p in range(x.shape[2]):
        c = x[..., p]
        h = c.shape[1] // 2
        s = np.concatenate([c[:, :h], c[:, c.shape[1] - h:]], 0)

        def z(a):
            flat = a.reshape(-1)
            order = np.argsort(flat, kind='mergesort')
            ranks = np.empty(flat.size)
            i = 0
            while i < flat.size:
                j = i
                while j + 1 < flat.size and flat[order[j + 1]] == flat[order[i]]:
                    j += 1
                ranks[order[i:j + 1]] = (i + j) / 2 + 1
                i = j + 1
            return norm.ppf((ranks.reshape(a.shape) - 0.375) / (flat.size + 0.25))

        def basic(a):
            n = a.shape[1]
            B = n * a.mean(1).var(ddof=1)
            W = a.var(1, ddof=1).mean()
            return np.sqrt(((n - 1) / n * W + B / n) / W)
        out.append(max(basic(z(s)), basic(z(np.abs(s - np.median(s))))))
    return np.array(out)


def test_rhat_rank_normalised_split():
    """pm.rhat = ArviZ rank-normalised split R-hat (mcmc.py:186-187; ArviZ not vendored: pinned to the
    published formulas, parity with ArviZ itself unpinned).  Mixed chains -> ~1; one shifted chain -> above
    the reference's 1.02 flag; a scale difference is caught by the folded (tail) R-hat; odd draw counts
    and ties handled; the vectorised form equals a per-parameter restatement."""
    from pet_posterior_distribution_amd.metrics import rhat, convergence_report
    rng = np.random.default_rng(3)
    x = rng.standard_normal((4, 1001, 6))
    x[..., 5] = np.round(x[..., 5])                     # heavy ties
    np.testing.assert_allclose(rhat(x), _rhat_reference_loop(x), rtol=1e-12)
    assert np.abs(rhat(x)[:5] - 1).max() < 0.01
    y = x.copy()
    y[0, :, 1] += 1.0                                    # one chain off in location
    y[1, :, 2] *= 3.0                                    # one chain off in scale only
    r = rhat(y)
    assert r[1] > 1.05 and r[2] > 1.02
    np.testing.assert_allclose(r, _rhat_reference_loop(y), rtol=1e-12)
    t = np.concatenate([x[:, :, :4], y[:, :, 1:5]], axis=2)    # 8 "ROI" pairs layout [DVR | R1], n_roi = 4
    rep = convergence_report(t, n_roi=4)
    assert rep['flag'] and rep['rhat_max'] == np.nanmax(rhat(t))
    assert not convergence_report(np.concatenate([x[:, :, :4], x[:, :, :4]], 2), n_roi=4)['flag']


def test_rhat_constant_draws_nan_without_warnings():
    """A parameter whose draws are constant everywhere gets NaN; chains each stuck at a different value
    (an un-tuned MH element that never accepts, W = 0 < B) get inf, as ArviZ's pm.rhat does, so the
    reference's flag (mcmc.py:186-189) trips.  W = 0 raises no floating-point warning (the GPU test log
    carried divide / invalid warnings from it in round 3)."""
    import warnings
    from pet_posterior_distribution_amd.metrics import rhat, convergence_report
    rng = np.random.default_rng(5)
    x = rng.standard_normal((4, 200, 3))
    x[..., 1] = 2.5                                      # constant everywhere
    x[:, :, 2] = np.arange(4)[:, None]                   # constant within each chain, different chains
    with warnings.catch_warnings():
        warnings.simplefilter('error')
        r = rhat(x)
        rep = convergence_report(np.concatenate([x[..., :1], x[..., 2:]], axis=2), n_roi=1)
    assert np.isfinite(r[0]) and np.isnan(r[1])
    assert r[2] > 1e6                                    # W = 0 up to the mean's rounding: inf or huge
    assert rep['flag'] and rep['rhat_max'] > 1e6
    from pet_posterior_distribution_amd.metrics import _rhat_basic
    s = np.repeat(np.array([0.0, 1.0, 2.0, 3.0])[:, None, None], 10, axis=1)   # exact W = 0 < B
    with warnings.catch_warnings():
        warnings.simplefilter('error')
        rb = _rhat_basic(np.concatenate([s, np.zeros_like(s)], axis=2))
    assert rb[0] == np.inf and np.isnan(rb[1])
