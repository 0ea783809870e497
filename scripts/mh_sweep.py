"""MH chain-count sweep (diagnostic): chain-steps/s of the selected kernel at n = 4 .. 10000 chains.
Kernel / waves per chain from PETMH_KERNEL / PETMH_WPC (read once per process)."""
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
    mh.run(64, 2, 0, seed=1)
    torch.cuda.synchronize()
    out = {'kernel': os.environ.get('PETMH_KERNEL', 'batched'), 'wpc': os.environ.get('PETMH_WPC', 'auto')}
    for n in (4, 64, 256, 1024, 2048, 4096, 10000):
        steps = 300 if n <= 256 else 100
        t0 = time.perf_counter()
        mh.run(n, steps // 3, steps - steps // 3, seed=7)
        torch.cuda.synchronize()
        out[str(n)] = round(n * steps / (time.perf_counter() - t0))
    mh.close()
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
