"""MH kernel timing for A/B (run once per kernel: PETMH_KERNEL=wave selects the one-update-at-a-time
kernel, default the batched-proposal one): the configs[2] slice (10k chains x 500 steps) and the
reference's 4-chain protocol (4 x (2000 draws + 4000 tune), x 10 = 4 x 60k steps)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    from pet_posterior_distribution_amd.sim_data import mh_problem
    mh = MetropolisSRTM2(**mh_problem(seed=0))
    mh.run(512, 2, 0, seed=1)
    torch.cuda.synchronize()
    out = {'kernel': os.environ.get('PETMH_KERNEL', 'batched'), 'wpc': os.environ.get('PETMH_WPC', 'auto')}
    for n, tune, draws in ((10000, 250, 250), (10000, 1000, 1000)):
        t0 = time.perf_counter()
        res = mh.run(n, draws, tune, seed=7)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out[f'chain_steps_per_s_{tune + draws}'] = round(n * (tune + draws) / el, 1)
        out[f'accept_{tune + draws}'] = round(float(res['accept_rate'].mean()), 5)
        out[f'mean_dvr0_{tune + draws}'] = float(res['mean_DVR'][0])
    t1 = time.perf_counter()
    mh.run(4, 2000, 4000, seed=3)
    torch.cuda.synchronize()
    out['protocol_s_per_tac'] = round((time.perf_counter() - t1) * 10, 3)
    mh.close()
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
