"""Simulation-based calibration of the MH baseline on the reference's prior.

For K test TACs whose truth is drawn from the prior the MH itself uses (sim_data.make_condition on
sim_data.reference_prior: MvNormal(mu, Cov) of prior_stats_nROI48 -- the MH's pm.MvNormal priors,
mcmc.py:148-149 -- restricted to DVR, R1 > 0, where the SRTM2 likelihood is defined; the MH's
log density is -inf elsewhere), the TAC's noisy observation from the noise model the MH likelihood
states (sample_sim_data.py:193-215 == TruncatedNormal(sn, sqrt(sn) sigma, lower 0), mcmc.py:151-155),
run the reference's protocol (4 chains x (20,000 draws + 40,000 tune), mcmc.py:156-157) and record:

* convergence: rank-normalised split R-hat per ROI (pm.rhat, metrics.rhat) and the reference's
  'R-hat > 1.02' flag (mcmc.py:183-194); cross-chain ESS (tfp's, metrics.effective_sample_size);
* calibration against the truth: SBC rank of the truth among L thinned posterior draws (uniform on
  0..L if the sampler is calibrated), coverage of the central 50 % / 90 % intervals, mean |z| with
  z = (truth - posterior mean) / posterior SD (0.80 for a calibrated Gaussian posterior).

Usage: python scripts/mcmc_calibration.py OUT.json [--tacs 32] [--draws 20000] [--tune 40000] [--textbook]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('out')
    ap.add_argument('--tacs', type=int, default=32)
    ap.add_argument('--draws', type=int, default=20000)
    ap.add_argument('--tune', type=int, default=40000)
    ap.add_argument('--chains', type=int, default=4)
    ap.add_argument('--thin-to', type=int, default=999, help='L: thinned draws per TAC for the SBC rank')
    ap.add_argument('--seed0', type=int, default=7000)
    ap.add_argument('--textbook', action='store_true',
                    help="element ratios against the running state instead of PyMC's sweep-start point")
    args = ap.parse_args()
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    from pet_posterior_distribution_amd.metrics import effective_sample_size
    from pet_posterior_distribution_amd.sim_data import make_condition, reference_prior
    prior = reference_prior()
    torch.cuda.set_device(0)
    per_tac, ranks, z_all, cov50, cov90 = [], [], [], [], []
    t_all = time.perf_counter()
    for k in range(args.tacs):
        seed = args.seed0 + k
        cond, tr = make_condition(seed, prior, return_truth=True)
        P = dict(time_vector=tr['time_vector'], tac_ref=tr['tac_ref'], k2p=float(tr['k2p']),
                 y_obs=cond[:48].astype(np.float64), sigma_noise=tr['sigma_noise'], mu_DVR=prior['mu_DVR'],
                 Cov_DVR=prior['Cov_DVR'], mu_R1=prior['mu_R1'], Cov_R1=prior['Cov_R1'])
        truth = np.concatenate([tr['DVR'], tr['R1']])
        mh = MetropolisSRTM2(**P, vs_sweep_start=not args.textbook)
        t0 = time.perf_counter()
        res = mh.run(args.chains, args.draws, args.tune, seed=seed, return_draws=True)
        torch.cuda.synchronize()
        t_mc = time.perf_counter() - t0
        mh.close()
        dr = res['draws'].cpu().numpy()                                   # (chains, draws, 96)
        conv = res['convergence']
        ess = effective_sample_size(np.moveaxis(dr, 0, -1), cross_chain_dims=-1)   # (96,)
        pooled = dr.reshape(-1, 96)
        mean, sd = pooled.mean(0), pooled.std(0)
        z = (truth - mean) / sd
        step = max(1, dr.shape[1] * dr.shape[0] // args.thin_to)
        thin = dr.transpose(1, 0, 2).reshape(-1, 96)[::step][:args.thin_to]          # interleave chains
        rank = (thin < truth[None, :]).sum(0)
        lo50, hi50 = np.quantile(pooled, [0.25, 0.75], axis=0)
        lo90, hi90 = np.quantile(pooled, [0.05, 0.95], axis=0)
        c50 = (truth >= lo50) & (truth <= hi50)
        c90 = (truth >= lo90) & (truth <= hi90)
        ranks.append(rank)
        z_all.append(z)
        cov50.append(c50)
        cov90.append(c90)
        rec = {'tac': seed, 'mcmc_seconds': round(t_mc, 3), 'accept_rate': round(float(res['accept_rate'].mean()), 4),
               'rhat_max': round(conv['rhat_max'], 5), 'rhat_flag_gt_1.02': conv['flag'],
               'rhat_DVR_max': round(float(np.nanmax(conv['rhat_DVR'])), 5),
               'rhat_R1_max': round(float(np.nanmax(conv['rhat_R1'])), 5),
               'n_rhat_gt_1.02': int(np.sum(np.concatenate([conv['rhat_DVR'], conv['rhat_R1']]) > 1.02)),
               'ess_min': round(float(ess.min()), 1), 'ess_median': round(float(np.median(ess)), 1),
               'mean_abs_z': {'DVR': round(float(np.abs(z[:48]).mean()), 4), 'R1': round(float(np.abs(z[48:]).mean()), 4)},
               'coverage50': round(float(c50.mean()), 4), 'coverage90': round(float(c90.mean()), 4)}
        per_tac.append(rec)
        print(json.dumps(rec), flush=True)
    R = np.stack(ranks)
    Z = np.stack(z_all)
    L = args.thin_to
    nb = 10
    hist = np.histogram(R.reshape(-1), bins=nb, range=(0, L + 1))[0]
    from scipy.stats import chi2
    exp = R.size / nb
    chi = float(((hist - exp) ** 2 / exp).sum())
    summary = {
        'protocol': f'{args.chains} chains x ({args.draws} draws + {args.tune} tune), mcmc.py:156-157',
        'sampler': 'textbook element-wise Metropolis (ratio vs the running state)' if args.textbook else
                   "PyMC 5.12 Metropolis elemwise_update (ratio vs the sweep-start point, delta_logp(q_temp, q0))",
        'prior': 'reference prior_stats_nROI48 (sim_data.reference_prior); truth = MvN restricted to DVR, R1 > 0',
        'tacs': args.tacs, 'seconds': round(time.perf_counter() - t_all, 1),
        'rhat_flagged_tacs': int(sum(r['rhat_flag_gt_1.02'] for r in per_tac)),
        'rhat_max_over_tacs': max(r['rhat_max'] for r in per_tac),
        'sbc_rank_hist_10bins': hist.tolist(), 'sbc_chi2_9dof': round(chi, 2),
        'sbc_chi2_pvalue_if_independent': float(chi2.sf(chi, nb - 1)),
        'note_dependence': 'the 96 ranks of one TAC are correlated (one truth vector, one posterior): the chi2 '
                           'p-value treats them as independent and overstates significance',
        'mean_abs_z': {'DVR': round(float(np.abs(Z[:, :48]).mean()), 4), 'R1': round(float(np.abs(Z[:, 48:]).mean()), 4),
                       'calibrated_gaussian': 0.7979},
        'z_sd': {'DVR': round(float(Z[:, :48].std()), 4), 'R1': round(float(Z[:, 48:].std()), 4), 'calibrated': 1.0},
        'coverage50': round(float(np.mean(cov50)), 4), 'coverage90': round(float(np.mean(cov90)), 4),
        'per_tac': per_tac}
    with open(args.out, 'w') as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != 'per_tac'}))


if __name__ == '__main__':
    main()
