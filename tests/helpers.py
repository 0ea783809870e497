"""Shared test fixtures: the shipped config (main_script.py:131-186) and synthetic inputs."""
from pet_posterior_distribution_amd.configs import shipped_net_args, shipped_diff_args  # noqa: F401


def synthetic_condition(seed=0):
    from pet_posterior_distribution_amd.sim_data import make_condition
    return make_condition(seed)
