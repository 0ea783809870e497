"""Measured accuracy and speed of the bf16x3 network next to exact f32 and bf16 (one JSON line per
dtype): per-level rrms / max errors vs the fp64 oracle (Glorot weights, B = 37, mixed conditions,
as tests/test_gpu_parity16.py), and configs[1] generate throughput (B = 1024, T = 1000, graph).
Usage: python scripts/explore_bf16x3.py [--no-speed]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import iddpm_ref as R                                            # noqa: E402
from tests.helpers import shipped_net_args, shipped_diff_args, synthetic_condition  # noqa: E402


def rrms(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.sqrt(((a - b) ** 2).mean() / ((b ** 2).mean() + 1e-300)))


def relmax(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.sqrt((b ** 2).mean()) + 1e-300))


def main():
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    from pet_posterior_distribution_amd.networks import glorot_uniform_init
    net = UnetConditional(**shipped_net_args())
    net.build((None, 48, 2))
    W = glorot_uniform_init(net.spec(), seed=17, bias_scale=0.05)
    conds = np.stack([synthetic_condition(0), synthetic_condition(1), synthetic_condition(2)])
    rng = np.random.default_rng(3)
    B = 37
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    t = rng.integers(0, 1000, B).astype(np.int32)
    c = conds[rng.integers(0, 3, B)]
    lv = {}
    y = R.unet_forward(W, x, t, c, dt=np.float64, levels=lv)
    speed = '--no-speed' not in sys.argv
    for dt in ('float32', 'bf16x3', 'bfloat16'):
        net = UnetConditional(**shipped_net_args())
        net.build((None, 48, 2))
        net.weights = W
        m = ImprovedDDPM(network=net, dtype=dt, **shipped_diff_args())
        out = m.call({'x': x, 'time': t, 'condition': c}).cpu().numpy()
        rec = {'dtype': dt, 'levels': {k: [rrms(v.cpu().numpy(), lv[k]), relmax(v.cpu().numpy(), lv[k])]
                                       for k, v in m.level_outputs().items()}}
        for k, sl in (('eps', slice(0, 2)), ('v', slice(2, 4))):
            rec['levels'][k] = [rrms(out[..., sl], y[..., sl]), relmax(out[..., sl], y[..., sl])]
        if speed:
            Bs = 1024
            xs = m.philox_normal(Bs, seed=5)
            m.ddpm_loop(xs, conds[:1], seed=2)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m.ddpm_loop(xs, conds[:1], seed=2)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            rec['samples_per_s'] = round(Bs / el, 2)
            rec['ms_per_step'] = round(el, 4)
        m.close()
        print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
