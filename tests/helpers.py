"""Shared test fixtures: the shipped config (main_script.py:131-186) and synthetic inputs."""
from pet_posterior_distribution_amd.configs import shipped_net_args, shipped_diff_args  # noqa: F401


def synthetic_condition(seed=0):
    from pet_posterior_distribution_amd.sim_data import make_condition
    return make_condition(seed)


def mh_problem(g2, case=0, noise=0.1, seed=0):
    """One TAC's MH problem (mcmc.py:73-137 inputs) built from the golden SRTM2 case:
    y = SRTM2 truth + sqrt(tac)-scaled Gaussian noise, synthetic MvN priors."""
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
