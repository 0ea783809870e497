#!/usr/bin/env python3
"""Exploration run (GPU): how far the 16-bit network paths sit from the fp64 oracle per level
with plain Glorot weights, and which synthetic weights keep a 1000-step reverse chain bounded
(for the configs[1]-size bf16-vs-f32 posterior test).  Prints one JSON line per measurement."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import iddpm_ref as R  # noqa: E402
from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional, Adam  # noqa: E402
from pet_posterior_distribution_amd.networks import glorot_uniform_init, denoiser_init  # noqa: E402
from tests.helpers import shipped_net_args, shipped_diff_args, synthetic_condition  # noqa: E402


def rrms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(((a - b) ** 2).mean() / ((b ** 2).mean() + 1e-300)))


def model(weights, dtype, fuse_up=True):
    os.environ['PETDIFF_FUSE_UP'] = '1' if fuse_up else '0'
    net = UnetConditional(**shipped_net_args())
    net.build((None, 48, 2))
    net.weights = weights
    m = ImprovedDDPM(network=net, dtype=dtype, **shipped_diff_args())
    m._ensure_handle()
    os.environ['PETDIFF_FUSE_UP'] = '1'
    return m


def levels():
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
    for name, dtype, fu in (('f32', 'float32', False), ('bf16_fused', 'bfloat16', True),
                            ('bf16_unfused', 'bfloat16', False), ('f16_fused', 'float16', True)):
        m = model(W, dtype, fu)
        out = m.call({'x': x, 'time': t, 'condition': c}).cpu().numpy()
        got = {k: v.cpu().numpy() for k, v in m.level_outputs().items()}
        rec = {'what': 'levels', 'path': name}
        for k in got:
            rec[k] = rrms(got[k], lv[k])
            rec[k + '_max'] = float(np.abs(got[k] - lv[k]).max() / np.sqrt((lv[k] ** 2).mean()))
        rec['eps'] = rrms(out[..., :2], y[..., :2])
        rec['v'] = rrms(out[..., 2:], y[..., 2:])
        rec['eps_max'] = float(np.abs(out[..., :2] - y[..., :2]).max() / np.sqrt((y[..., :2] ** 2).mean()))
        rec['v_max'] = float(np.abs(out[..., 2:] - y[..., 2:]).max() / np.sqrt((y[..., 2:] ** 2).mean()))
        print(json.dumps(rec), flush=True)
        m.close()


def trained_weights(steps, lr=2e-4, seed=5):
    from pet_posterior_distribution_amd.sim_data import simulate_dataset
    net = UnetConditional(**shipped_net_args())
    net.build((None, 48, 2))
    net.weights = glorot_uniform_init(net.spec(), seed=seed)
    m = ImprovedDDPM(network=net, dtype='float32', **shipped_diff_args())
    m.compile(optimizer=Adam(learning_rate=lr, clipnorm=1.5))
    n = 256 * 64
    d = simulate_dataset(n, seed=3)
    x0 = torch.stack([d['varDVR'], d['varR1']], -1).to(torch.float32).contiguous()
    cond = d['condition']
    tr = m._ensure_trainer()
    loss = torch.empty(256, dtype=torch.float32, device='cuda')
    t0 = time.perf_counter()
    hist = []
    for i in range(steps):
        k = i % 64
        tr.compute_gradients(x0[k * 256:(k + 1) * 256], cond[k * 256:(k + 1) * 256], seed=11, loss=loss)
        tr.apply_gradients(1.0)
        if i % 200 == 0 or i == steps - 1:
            hist.append((i, float(tr.last_stats()[0])))
    torch.cuda.synchronize()
    w = tr.weights().cpu().numpy()
    out, o = {}, 0
    for nme, sh in net.spec():
        k = int(np.prod(sh))
        out[nme] = w[o:o + k].reshape(sh).copy()
        o += k
    print(json.dumps({'what': 'train', 'steps': steps, 'sec': round(time.perf_counter() - t0, 2), 'loss': hist}),
          flush=True)
    return out, d


def loop_pair(W, tag, cond, B=1024):
    m32 = model(W, 'float32', False)
    m16 = model(W, 'bfloat16', True)
    rng = np.random.default_rng(12)
    x = torch.as_tensor(rng.standard_normal((B, 48, 2)).astype(np.float32), device='cuda')
    t0 = time.perf_counter()
    a = m32.ddpm_loop(x, cond[None], seed=77).cpu().numpy().astype(np.float64)
    ta = time.perf_counter() - t0
    b = m16.ddpm_loop(x, cond[None], seed=77).cpu().numpy().astype(np.float64)
    sd = a.std(0)
    rec = {'what': 'loop', 'weights': tag, 'f32_s': round(ta, 2), 'finite32': bool(np.isfinite(a).all()),
           'finite16': bool(np.isfinite(b).all()), 'absmean32': float(np.abs(a).mean()),
           'sd_mean32': float(sd.mean()), 'sd_min32': float(sd.min()),
           'mean_diff_over_mc': float((np.abs(a.mean(0) - b.mean(0)) / (sd * np.sqrt(2.0 / B))).max()),
           'sd_ratio_dev_over_mc': float((np.abs(b.std(0) / sd - 1) / np.sqrt(1.0 / B)).max()),
           'per_sample_rrms': rrms(b, a),
           'corr': float(np.corrcoef(a.ravel(), b.ravel())[0, 1])}
    print(json.dumps(rec), flush=True)
    m32.close()
    m16.close()


def main():
    levels()
    net = UnetConditional(**shipped_net_args())
    net.build((None, 48, 2))
    cond = synthetic_condition(0)
    for vp in (1.0,):
        W = denoiser_init(net.spec(), seed=14, bias_scale=0.05, perturb=0.1, v_perturb=vp)
        loop_pair(W, f'denoiser_v{vp}', cond)
    for steps in (800, 3000):
        W, d = trained_weights(steps)
        loop_pair(W, f'trained{steps}', d['condition'][0].cpu().numpy())


if __name__ == '__main__':
    main()
