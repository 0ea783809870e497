"""Simulation-based calibration of the trained iDDPM posterior (the check DESIGN.md section 9 names next).

N unseen TACs from the training generator (sample_sim_data.py:89-215 on the reference prior; the
likelihood the network learned), n_post posterior samples each through the product path
(distributed.sample_posterior_sharded: one TAC-major batch, 1000 reverse steps, bf16 network), then per
(TAC, ROI, parameter) the rank of the truth among the samples and z = (truth - mean) / SD.
A calibrated posterior gives a flat rank histogram, mean |z| 0.80, z SD 1.00, 50 % / 90 % coverage 0.50 / 0.90.
scripts/mcmc_calibration.py is the same check for the MH baseline.

Usage: python scripts/iddpm_calibration.py WEIGHTS.npz OUT.json [--tacs 128] [--n-post 1000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))


def rank_stats(x, truth, bins=10):
    """x (n_tac, n_post, 48, 2) samples, truth (n_tac, 48, 2): rank histogram, |z|, z SD, coverage."""
    n_post = x.shape[1]
    rank = (x < truth[:, None]).sum(1)                                   # 0 .. n_post
    b = rank.ravel() * bins // (n_post + 1)
    hist = np.bincount(b, minlength=bins)
    exp = np.bincount(np.arange(n_post + 1) * bins // (n_post + 1), minlength=bins) * (rank.size / (n_post + 1))
    chi2 = float(((hist - exp) ** 2 / exp).sum())
    mu, sd = x.mean(1), x.std(1, ddof=1)
    z = (truth - mu) / sd
    lo50, hi50 = np.quantile(x, [0.25, 0.75], axis=1)
    lo90, hi90 = np.quantile(x, [0.05, 0.95], axis=1)
    return {'sbc_rank_hist_10bins': hist.tolist(), 'sbc_chi2_9dof': round(chi2, 2),
            'mean_abs_z': {'DVR': round(float(np.abs(z[..., 0]).mean()), 4), 'R1': round(float(np.abs(z[..., 1]).mean()), 4),
                           'calibrated_gaussian': 0.7979},
            'z_sd': {'DVR': round(float(z[..., 0].std()), 4), 'R1': round(float(z[..., 1].std()), 4), 'calibrated': 1.0},
            'z_mean': {'DVR': round(float(z[..., 0].mean()), 4), 'R1': round(float(z[..., 1].mean()), 4)},
            'coverage50': round(float(((truth >= lo50) & (truth <= hi50)).mean()), 4),
            'coverage90': round(float(((truth >= lo90) & (truth <= hi90)).mean()), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('weights')
    ap.add_argument('out')
    ap.add_argument('--tacs', type=int, default=128)
    ap.add_argument('--n-post', type=int, default=1000)
    ap.add_argument('--dtype', default='bfloat16')
    args = ap.parse_args()

    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    from pet_posterior_distribution_amd.configs import shipped_diff_args, shipped_net_args
    from pet_posterior_distribution_amd.distributed import sample_posterior_sharded
    from pet_posterior_distribution_amd.sim_data import reference_prior, simulate_dataset

    torch.cuda.set_device(0)
    prior = reference_prior()
    net = UnetConditional(**shipped_net_args(), seed=1234)
    net.build((None, 48, 2))
    net.load_weights(args.weights)
    m = ImprovedDDPM(network=net, dtype=args.dtype, **shipped_diff_args())
    t = simulate_dataset(args.tacs, prior, seed=11, sample_offset=(1 << 40) + (1 << 20))   # unseen indices
    cond = t['condition'].cpu().numpy()
    truth = np.stack([t['varDVR'].cpu().numpy(), t['varR1'].cpu().numpy()], -1).astype(np.float64)
    t0 = time.perf_counter()
    _, _, (lo, hi, x0) = sample_posterior_sharded(m, cond, args.n_post, seed=5, x_T_seed=6, return_samples=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    x = x0.double().cpu().numpy().reshape(args.tacs, args.n_post, 48, 2)
    rec = {'protocol': 'SBC of the iDDPM posterior: truths and TACs from the training generator (reference prior), '
                       'unseen sample indices; samples through sample_posterior_sharded',
           'weights': os.path.basename(args.weights), 'dtype': args.dtype, 'tacs': args.tacs, 'n_post': args.n_post,
           'finite': bool(np.isfinite(x).all()), 'seconds': round(el, 2),
           'note_dependence': 'the 96 ranks of one TAC are correlated (one truth vector, one posterior)'}
    rec.update(rank_stats(x, truth))
    with open(args.out, 'w') as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))
    m.close()


if __name__ == '__main__':
    main()
