"""Shared test fixtures: the shipped config (main_script.py:131-186) and synthetic inputs."""
from pet_posterior_distribution_amd.configs import shipped_net_args, shipped_diff_args  # noqa: F401


def synthetic_condition(seed=0):
    from pet_posterior_distribution_amd.sim_data import make_condition
    return make_condition(seed)


def mh_problem(g2, case=0, noise=0.1, seed=0):
    """One TAC's MH problem (mcmc.py:73-137 inputs) built from the golden SRTM2 case:
    y = SRTM2 truth + sqrt(tac)-scaled Gaussian noise, synthetic MvN priors (the G2 cases are drawn from sim_data.synthetic_prior; the reference's
    prior covariances have condition numbers up to 1e7, which puts the chain-path equality tests'
    accept / reject decisions at the mercy of last-bit differences in the quadratic form)."""
    import numpy as np
    from oracle import srtm2_ref as K
    from pet_posterior_distribution_amd.sim_data import synthetic_prior
    tv = g2['time_vector']
    ref = g2[f'case{case}_tac_ref']
    truth_D, truth_R, k2p = g2[f'case{case}_DVR'], g2[f'case{case}_R1'], float(g2[f'case{case}_k2p'])
    tac = K.srtm2_tac(tv, ref, truth_D, truth_R, k2p).T               # (48, 54)
    rng = np.random.default_rng(seed)
    sig = np.full((48, 54), noise) / np.sqrt(g2['dt'])[None, :]
    y = np.maximum(tac + np.sqrt(np.maximum(tac, 0)) * sig * rng.standard_normal(tac.shape), 1e-3)
    pr = synthetic_prior()
    return dict(time_vector=tv, tac_ref=ref, k2p=k2p, y_obs=y, sigma_noise=sig, mu_DVR=truth_D * 1.02,
                Cov_DVR=pr['Cov_DVR'], mu_R1=truth_R * 0.98, Cov_R1=pr['Cov_R1'])


def assert_same_distribution(x, y, z_mean=5.0, z_cov=5.5, ks_alpha=1e-3):
    """x (n, d) and y (m, d) independent draws of one distribution: every marginal mean within z_mean
    Monte-Carlo standard errors, every covariance entry within z_cov standard errors of the difference
    (se of a sample covariance entry from the fourth moments: var((x_i - m_i)(x_j - m_j)) / n), and every
    marginal passes a two-sample Kolmogorov-Smirnov test at ks_alpha after a Bonferroni split over d.
    Returns the largest statistics (for the test's message)."""
    import numpy as np
    from scipy.stats import ks_2samp
    x, y = np.asarray(x, np.float64), np.asarray(y, np.float64)
    n, m, d = len(x), len(y), x.shape[1]
    se = np.sqrt(x.var(0, ddof=1) / n + y.var(0, ddof=1) / m)
    zm = np.abs(x.mean(0) - y.mean(0)) / se
    cx, cy = x - x.mean(0), y - y.mean(0)
    px, py = cx[:, :, None] * cx[:, None, :], cy[:, :, None] * cy[:, None, :]
    zc = np.abs(px.mean(0) - py.mean(0)) / np.sqrt(px.var(0, ddof=1) / n + py.var(0, ddof=1) / m)
    pks = np.array([ks_2samp(x[:, k], y[:, k]).pvalue for k in range(d)])
    stats = dict(z_mean=float(zm.max()), z_cov=float(zc.max()), ks_p_min=float(pks.min()))
    assert zm.max() < z_mean, stats
    assert zc.max() < z_cov, stats
    assert pks.min() > ks_alpha / d, stats
    return stats


_TRAINED = {}


def quick_trained_weights(steps=800, seed=5, lr=2e-4):
    """Weights of the shipped network after `steps` Adam steps (batch 256, lr 2e-4, clipnorm 1.5,
    main_script.py:169-174) on GPU-simulated training data (sim_data.simulate_dataset, 16,384
    samples): an eps-predictor whose 1000-step reverse chain stays bounded without any identity
    shortcut, so the bf16 / f32 comparisons see the whole network.  About 3 s on one MI355X;
    cached per process.  Returns (weights dict, one condition (49, 54) of the data set)."""
    key = (steps, seed, lr)
    if key in _TRAINED:
        return _TRAINED[key]
    import numpy as np
    import torch
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional, Adam
    from pet_posterior_distribution_amd.networks import glorot_uniform_init
    from pet_posterior_distribution_amd.sim_data import simulate_dataset
    net = UnetConditional(**shipped_net_args())
    net.build((None, 48, 2))
    net.weights = glorot_uniform_init(net.spec(), seed=seed)
    m = ImprovedDDPM(network=net, dtype='float32', **shipped_diff_args())
    m.compile(optimizer=Adam(learning_rate=lr, clipnorm=1.5))
    nb, B = 64, 256
    d = simulate_dataset(nb * B, seed=3)
    x0 = torch.stack([d['varDVR'], d['varR1']], -1).to(torch.float32).contiguous()
    cond = d['condition']
    tr = m._ensure_trainer()
    for i in range(steps):
        k = i % nb
        tr.compute_gradients(x0[k * B:(k + 1) * B], cond[k * B:(k + 1) * B], seed=11)
        tr.apply_gradients(1.0)
    w = tr.weights().cpu().numpy()
    out, o = {}, 0
    for name, sh in net.spec():
        k = int(np.prod(sh))
        out[name] = w[o:o + k].reshape(sh).copy()
        o += k
    tr.close()
    _TRAINED[key] = (out, cond[0].cpu().numpy())
    return _TRAINED[key]
