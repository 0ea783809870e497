"""Is the step bound by the chip's power budget?  Times the configs[1] loop (1024 samples x 1000 steps,
bf16) with the bench's synthetic weights, with all-zero weights (MFMA operands that toggle nothing) and,
when present, the trained weights of scripts/train_protocol.py.  Usage: python scripts/power_probe.py [out.json]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))


def main(out=None):
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    from pet_posterior_distribution_amd.configs import shipped_diff_args, shipped_net_args
    from pet_posterior_distribution_amd.sim_data import make_condition
    torch.cuda.set_device(0)
    cond = make_condition(seed=0)
    net = UnetConditional(**shipped_net_args(), seed=1234)
    net.build((None, 48, 2))
    variants = {'synthetic': dict(net.weights), 'zeros': {k: np.zeros_like(v) for k, v in net.weights.items()}}
    tw = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'weights', 'trained_r02.npz')
    if os.path.exists(tw):
        with np.load(tw) as z:
            variants['trained'] = {k: z[k] for k in net.weights}
    res = {}
    for rep in range(2):
        for name, w in variants.items():
            net.weights = w
            m = ImprovedDDPM(network=net, dtype='bfloat16', **shipped_diff_args())
            x_T = m.philox_normal(1024, seed=1)
            m.ddpm_loop(x_T, cond[None], num_timesteps=50, seed=2)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                m.ddpm_loop(x_T, cond[None], seed=2)
            torch.cuda.synchronize()
            sps = 3 * 1024 / (time.perf_counter() - t0)
            res.setdefault(name, []).append(round(sps, 1))
            m.close()
            print(name, round(sps, 1), flush=True)
    print(json.dumps(res))
    if out:
        with open(out, 'w') as f:
            json.dump(res, f, indent=1)


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else None)
