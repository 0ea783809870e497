"""Host-side cost of one posterior job: graph-launch enqueue time of ddpm_loop, bare back-to-back loops vs
sample_posterior_sharded (x_T + loop + stats, host sync per job).  Usage: python scripts/probe/job_overhead.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))


def main():
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    from pet_posterior_distribution_amd.configs import shipped_net_args, shipped_diff_args
    from pet_posterior_distribution_amd.distributed import TacTable, sample_posterior_sharded
    from pet_posterior_distribution_amd.sim_data import make_condition
    net = UnetConditional(**shipped_net_args(), seed=1234)
    net.build((None, 48, 2))
    m = ImprovedDDPM(network=net, dtype=os.environ.get('DT', 'bfloat16'), **shipped_diff_args())
    cond = make_condition(0)
    B = 1024
    x = m.philox_normal(B, seed=1)
    out = {}
    for _ in range(2):
        m.ddpm_loop(x, cond[None], seed=2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.ddpm_loop(x, cond[None], seed=2)
    out['enqueue_ms'] = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    out['one_loop_ms'] = (time.perf_counter() - t0) * 1e3
    K = 5
    t0 = time.perf_counter()
    for _ in range(K):
        m.ddpm_loop(x, cond[None], seed=2)
    torch.cuda.synchronize()
    out['back_to_back_ms'] = (time.perf_counter() - t0) * 1e3 / K
    table = TacTable(1, lambda k: cond)
    sample_posterior_sharded(m, table, B, seed=2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        sample_posterior_sharded(m, table, B, seed=2)
    torch.cuda.synchronize()
    out['sharded_job_ms'] = (time.perf_counter() - t0) * 1e3 / K
    t0 = time.perf_counter()
    for _ in range(K):
        m.ddpm_loop(x, cond[None], seed=2)
        m.posterior_stats(x)
    torch.cuda.synchronize()
    out['loop_plus_stats_ms'] = (time.perf_counter() - t0) * 1e3 / K
    print(json.dumps(out))


if __name__ == '__main__':
    main()
