"""Train the shipped network on MI355X with the reference's protocol, then score its posterior against MCMC.

Reference protocol (yanisdjebra/PET_posterior_distribution):
* data: sample_sim_data.py:89-215 -- 100,000 simulated TACs (truncated-MvN prior, SRTM2, truncated noise);
  here the GPU generator (sim_data.simulate_dataset) on the reference prior
  (sim_data.reference_prior: the prior_stats_nROI48 arrays, read by a static pickle parser);
* training: main_script.py:131-271 -- UnetConditional f128/d4, iDDPM T=1000 cosine, lambda_vlb 0.1,
  Adam(ExponentialDecay(2e-4 -> 5e-5 over 500 epochs), clipnorm 1.5), batch 256, 500 epochs,
  validation_split 0.1, WeightsCheckpoint every 50 epochs;
* scoring: main_script.py:363-436 (10,000 posterior samples per test TAC, full 1000-step reverse) and
  :719-829 (per-ROI mean / SD / covariance / correlation relative differences against MCMC, ESS);
  MCMC = mcmc.py:133-157 protocol, 4 chains x (20,000 draws + 40,000 tune), on the same GPU.

The paper's claims (README.md:12): posterior mean within 0.67 % and SD within 7.3 % of MCMC, > 230x faster.

Usage: python scripts/train_protocol.py OUT_DIR [--epochs 500] [--n-samples 100000] [--time-budget S]
       python scripts/train_protocol.py OUT_DIR --weights W.npz --epochs 0      (score saved weights only)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))


class TimeBudget:
    """Stops fit once the next epoch would overrun the budget (keeps a GPU call inside its limit)."""

    def __init__(self, seconds):
        self.seconds = seconds
        self.t0 = time.perf_counter()
        self.last = self.t0
        self.model = None
        self.epochs = 0

    def set_model(self, m):
        self.model = m

    def on_epoch_end(self, epoch, logs=None):
        now = time.perf_counter()
        per = now - self.last
        self.last = now
        self.epochs = epoch + 1
        if now - self.t0 + 1.5 * per > self.seconds:
            self.model.stop_training = True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('out')
    ap.add_argument('--n-samples', type=int, default=100000)
    ap.add_argument('--epochs', type=int, default=500)
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--period', type=int, default=50)
    ap.add_argument('--time-budget', type=float, default=1e9)
    ap.add_argument('--weights', default=None, help='start from / score these weights (.npz)')
    ap.add_argument('--eval-tacs', type=int, default=2)
    ap.add_argument('--n-posterior', type=int, default=10000)
    ap.add_argument('--mh-draws', type=int, default=20000)
    ap.add_argument('--mh-tune', type=int, default=40000)
    ap.add_argument('--f32-eval', action='store_true', help='also sample the posterior with the exact-f32 network')
    ap.add_argument('--mh-textbook', action='store_true',
                    help="also score against the MH with the textbook element ratio (PyMC's is against the sweep start)")
    ap.add_argument('--test-source', default='train-generator', choices=['train-generator', 'independent'],
                    help='train-generator: unseen TACs from the training generator (same per-ROI noise level as the '
                         'training set, the likelihood the network learned); independent: a TAC with its own noise '
                         'draw, like the reference\'s separately simulated test set')
    args = ap.parse_args()

    from pet_posterior_distribution_amd import Adam, ExponentialDecay, ImprovedDDPM, UnetConditional, glorot_uniform_init
    from pet_posterior_distribution_amd.configs import shipped_diff_args, shipped_net_args
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    from pet_posterior_distribution_amd.metrics import ess_pair, posterior_metrics
    from pet_posterior_distribution_amd.sim_data import make_condition, mh_problem, simulate_dataset, reference_prior
    from pet_posterior_distribution_amd.training import WeightsCheckpoint

    os.makedirs(args.out, exist_ok=True)
    torch.cuda.set_device(0)
    prior = reference_prior()
    summary = {'protocol': 'main_script.py:131-271 training, :363-436 + :719-829 scoring',
               'prior': 'sim_data.reference_prior() (the reference prior_stats_nROI48 arrays)'}

    net = UnetConditional(**shipped_net_args(), seed=1234)
    net.build((None, 48, 2))
    if args.weights:
        net.load_weights(args.weights)
    else:   # Keras defaults of the reference's layers: glorot_uniform kernels, zero biases
        net.weights = glorot_uniform_init(net.spec(), seed=1234)
    model = ImprovedDDPM(network=net, dtype='float32', **shipped_diff_args())

    if args.epochs > 0:
        t0 = time.perf_counter()
        d = simulate_dataset(args.n_samples, prior, seed=11)
        x = torch.stack([d['varDVR'], d['varR1']], dim=-1).float().contiguous()   # main_script.py:105
        y = d['condition']                                                        # main_script.py:108-109
        perm = torch.as_tensor(np.random.default_rng(1234).permutation(args.n_samples), device=x.device)
        x, y = x[perm].contiguous(), y[perm].contiguous()                          # main_script.py:123-126
        torch.cuda.synchronize()
        summary['data_seconds'] = round(time.perf_counter() - t0, 2)
        decay_rate = (5e-5 / 2e-4) ** (1 / 500)
        lr = ExponentialDecay(2e-4, args.n_samples // args.batch, decay_rate)      # main_script.py:188-192
        model.compile(optimizer=Adam(learning_rate=lr, clipnorm=1.5), loss='MeanSquaredError')
        budget = TimeBudget(args.time_budget)
        t0 = time.perf_counter()
        hist = model.fit(x, y, batch_size=args.batch, epochs=args.epochs, validation_split=0.1, verbose=1,
                         callbacks=[WeightsCheckpoint(os.path.join(args.out, 'cp'), every_n_epochs=args.period),
                                    budget])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        n_ep = len(hist['loss'])
        summary.update({'epochs_run': n_ep, 'epochs_asked': args.epochs, 'train_seconds': round(el, 1),
                        'train_samples_per_s': round(n_ep * int(args.n_samples * 0.9) / el, 1),
                        'loss_first_last': [hist['loss'][0], hist['loss'][-1]],
                        'val_loss_first_last': [hist['val_loss'][0], hist['val_loss'][-1]],
                        'history': {k: [round(float(v), 6) for v in vals] for k, vals in hist.items()}})
        model._sync_trained_weights()
        net.save_weights(os.path.join(args.out, 'weights.npz'))
        del x, y, d
        torch.cuda.empty_cache()
    model.close()

    evals = []
    if args.test_source == 'train-generator':
        # the training set's per-ROI noise draw (dataset_sigma_noise under the same seed), unseen sample indices
        t = simulate_dataset(args.eval_tacs, prior, seed=11, sample_offset=1 << 40)
        tests = []
        for k in range(args.eval_tacs):
            cond = t['condition'][k].cpu().numpy()
            P = dict(time_vector=t['time_vector'], tac_ref=t['vartacref'][k].cpu().numpy(), k2p=float(prior['mu_k2p']),
                     y_obs=cond[:48].astype(np.float64), sigma_noise=t['sigma_noise'], mu_DVR=prior['mu_DVR'],
                     Cov_DVR=prior['Cov_DVR'], mu_R1=prior['mu_R1'], Cov_R1=prior['Cov_R1'])
            tests.append((k, cond, P, {'DVR': t['varDVR'][k].cpu().numpy(), 'R1': t['varR1'][k].cpu().numpy()}))
    else:
        tests = [(100 + k,) + (lambda ct: (ct[0], mh_problem(100 + k, prior), ct[1]))(
            make_condition(100 + k, prior, return_truth=True)) for k in range(args.eval_tacs)]
    summary['test_source'] = args.test_source
    for k, (seed, cond, P, truth) in enumerate(tests):
        rec = {'tac': seed}
        samplers = [('bf16', 'bfloat16')] + ([('f32', 'float32')] if args.f32_eval and k == 0 else [])
        mh = MetropolisSRTM2(**P)
        mh.run(4, 2, 0, seed=1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = mh.run(4, args.mh_draws, args.mh_tune, seed=3 + k, return_draws=True)
        torch.cuda.synchronize()
        rec['mcmc_seconds'] = round(time.perf_counter() - t0, 3)
        rec['mcmc_accept_rate'] = round(float(res['accept_rate'].mean()), 4)
        conv = res['convergence']                       # mcmc.py:183-194
        rec['mcmc_rhat_max'] = round(conv['rhat_max'], 5)
        rec['mcmc_rhat_flag_gt_1.02'] = conv['flag']
        draws = res['draws']
        tb_draws = None
        if args.mh_textbook:   # the same chains with the textbook element ratio (against the running state)
            mh_tb = MetropolisSRTM2(**P, vs_sweep_start=False)
            rtb = mh_tb.run(4, args.mh_draws, args.mh_tune, seed=3 + k, return_draws=True)
            tb_draws = rtb['draws']
            rec['mcmc_textbook_rhat_max'] = round(rtb['convergence']['rhat_max'], 5)
            mh_tb.close()
        mh.close()
        for tag, dt in samplers:
            m = ImprovedDDPM(network=net, dtype=dt, **shipped_diff_args())
            x_T = m.philox_normal(args.n_posterior, seed=1 + k)
            m.ddpm_loop(x_T[:256], cond[None], num_timesteps=10, seed=2)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            x0 = m.ddpm_loop(x_T, cond[None], seed=2 + k)
            torch.cuda.synchronize()
            t_nn = time.perf_counter() - t0
            met = posterior_metrics(x0, draws)
            ess = ess_pair(x0, draws)
            xs = x0.float().cpu().numpy()
            dr = draws.cpu().numpy()
            r = {'iddpm_seconds': round(t_nn, 3), 'finite': bool(np.isfinite(xs).all()),
                 'speedup_over_mcmc': round(rec['mcmc_seconds'] / t_nn, 2),
                 'norm_diff': {name: {q: {'mean': round(float(np.mean(met[name][q]['Norm_diff'])), 5),
                                          'max': round(float(np.max(met[name][q]['Norm_diff'])), 5)}
                                      for q in ('mu', 'std')} for name in ('DVR', 'R1')},
                 'std_ratio_nn_over_mcmc_mean': {
                     name: round(float(np.mean(met[name]['std']['NN'] / met[name]['std']['MCMC'])), 4)
                     for name in ('DVR', 'R1')},
                 # calibration against the simulation truth: |truth - mean| / SD (0.80 for a calibrated
                 # Gaussian posterior) and the share of ROIs whose truth lies within one SD (0.68)
                 'calibration': {
                     meth: {name: {'mean_abs_z': round(float(np.mean(z)), 4), 'within_1sd': round(float(np.mean(z < 1)), 4)}
                            for name, z in ((nm, np.abs(truth[nm][:, None] - met[nm]['mu'][meth]) / met[nm]['std'][meth])
                                            for nm in ('DVR', 'R1'))}
                     for meth in ('NN', 'MCMC')},
                 'ess_mean': {kk: [round(float(v[:, p].mean()), 1) for p in range(2)] for kk, v in ess.items()},
                 'posterior_mean_abs_err_vs_truth': {
                     'DVR': round(float(np.mean(np.abs(xs[..., 0].mean(0) - truth['DVR']))), 5),
                     'R1': round(float(np.mean(np.abs(xs[..., 1].mean(0) - truth['R1']))), 5)},
                 'mcmc_mean_abs_err_vs_truth': {
                     'DVR': round(float(np.mean(np.abs(dr[..., :48].reshape(-1, 48).mean(0) - truth['DVR']))), 5),
                     'R1': round(float(np.mean(np.abs(dr[..., 48:].reshape(-1, 48).mean(0) - truth['R1']))), 5)}}
            if tb_draws is not None:
                mt = posterior_metrics(x0, tb_draws)
                r['vs_textbook_mh'] = {
                    'norm_diff': {name: {q: round(float(np.mean(mt[name][q]['Norm_diff'])), 5) for q in ('mu', 'std')}
                                  for name in ('DVR', 'R1')},
                    'std_ratio_nn_over_mcmc_mean': {
                        name: round(float(np.mean(mt[name]['std']['NN'] / mt[name]['std']['MCMC'])), 4)
                        for name in ('DVR', 'R1')},
                    'mcmc_calibration': {name: round(float(np.mean(np.abs(truth[name][:, None] - mt[name]['mu']['MCMC'])
                                                                  / mt[name]['std']['MCMC'])), 4)
                                         for name in ('DVR', 'R1')}}
            rec[tag] = r
            m.close()
            print(json.dumps({'tac': seed, tag: r}), flush=True)
        evals.append(rec)
    summary['eval'] = evals
    summary['paper_claim'] = 'mean within 0.67 %, SD within 7.3 % of MCMC, > 230x faster (README.md:12)'
    with open(os.path.join(args.out, 'summary.json'), 'w') as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != 'history'}))


if __name__ == '__main__':
    main()
