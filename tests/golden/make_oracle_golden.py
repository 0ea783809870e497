"""Generate the oracle-side golden fixtures G3-G7 under tests/golden/.

These pin the build's fp64 NumPy restatement of the reference (oracle/) and its inputs, so that a later
change of the oracle, the condition generator or the weight initialiser shows up as a fixture mismatch
on CPU (tests/test_cpu_golden.py), and so that the GPU path is checked against stored vectors as well as
against the live oracle (tests/test_gpu_golden.py).  They are NOT reference outputs: the reference's
U-Net needs TensorFlow, which is absent ("parity unpinned").

* G3 (g3_conditions.npz): 4 synthetic test TACs, sim_data.make_condition(seed, reference prior) for
  seeds 100..103 (main_script.py:110-113 layout (49, 54); sample_sim_data.py:139-215 generator),
  with their truths.
* G4 (g4_unet.npz): the U-Net forward (oracle.iddpm_ref.unet_forward, fp64; networks.py:781-1093) with
  Glorot-uniform weights (seed 1234, biases U(-0.05, 0.05)), B = 4 (one G3 condition per sample),
  t in {0, 1, 500, 998, 999}; plus per-variable checksums of the weights (sum, sum of squares).
* G5 (g5_p_sample.npz): ImprovedDDPM.ddpm with injected z (oracle.ddpm, fp64; diffusion_model.py:651-663)
  on the G4 network at t in {1, 500, 999}: mean, var and var_tilde terms.
* G6 (g6_loop.npz): ddpm_loop (diffusion_model.py:670-715, var_tilde) with denoiser weights (a bounded
  1000-step chain: networks.denoiser_init, seed 1234, biases U(-0.05, 0.05), v rows unscaled), B = 4,
  condition G3[0], x_T seeded, z from the build's counter-based Philox (seed 987654321, samples 0..3):
  the 25-step (linear subsequence) and the full 1000-step outputs, fp64.
* G7 (g7_mh_logp.npz): the MH log density (oracle.srtm2_ref.log_posterior; mcmc.py:147-155) of the
  G3[0] problem (sim_data.mh_problem(100)) at 6 parameter points.

Usage: python tests/golden/make_oracle_golden.py [g3 g4 g5 g6 g7]   (about 3 minutes for all)
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

SEEDS = [100, 101, 102, 103]
T_VALUES = [0, 1, 500, 998, 999]
PS_T = [1, 500, 999]
LOOP_SEED, LOOP_STEPS_SHORT = 987654321, 25


def spec():
    from pet_posterior_distribution_amd import UnetConditional
    from pet_posterior_distribution_amd.configs import shipped_net_args
    net = UnetConditional(**shipped_net_args())
    net.build((None, 48, 2))
    return net.spec()


def g4_weights():
    from pet_posterior_distribution_amd.networks import glorot_uniform_init
    return glorot_uniform_init(spec(), seed=1234, bias_scale=0.05)


def g6_weights():
    from pet_posterior_distribution_amd.networks import denoiser_init
    return denoiser_init(spec(), seed=1234, bias_scale=0.05, v_perturb=1.0)


def checksums(W):
    names = sorted(W)
    return (np.array(names), np.array([float(np.sum(W[n], dtype=np.float64)) for n in names]),
            np.array([float(np.sum(np.asarray(W[n], np.float64) ** 2)) for n in names]))


def g3_inputs():
    from pet_posterior_distribution_amd.sim_data import make_condition
    conds, truth = [], []
    for s in SEEDS:
        c, t = make_condition(s, return_truth=True)
        conds.append(c)
        truth.append(t)
    return np.stack(conds), truth


def g4_x():
    return np.random.default_rng(4).standard_normal((len(T_VALUES), 4, 48, 2))


def g5_inputs():
    rng = np.random.default_rng(5)
    return rng.standard_normal((len(PS_T), 4, 48, 2)), rng.standard_normal((len(PS_T), 4, 48, 2))


def g6_inputs():
    return np.random.default_rng(6).standard_normal((4, 48, 2)).astype(np.float32)


def loop_z(n):
    from oracle import iddpm_ref as R
    return np.stack([R.philox_normal_pairs(LOOP_SEED, np.arange(4), i) for i in range(n)])


def make(which):
    from oracle import iddpm_ref as R
    from oracle import srtm2_ref as K
    S = R.schedule_tables(R.get_beta_schedule('cosine', 1000))
    conds, truth = g3_inputs()
    if 'g3' in which:
        np.savez(os.path.join(HERE, 'g3_conditions.npz'), seeds=np.array(SEEDS), condition=conds,
                 DVR=np.stack([t['DVR'] for t in truth]), R1=np.stack([t['R1'] for t in truth]),
                 tac_ref=np.stack([t['tac_ref'] for t in truth]), sigma_noise=np.stack([t['sigma_noise'] for t in truth]))
        print('g3 written')
    if 'g4' in which or 'g5' in which:
        W = g4_weights()
        names, s1, s2 = checksums(W)
    if 'g4' in which:
        x = g4_x()
        out = np.stack([R.unet_forward(W, x[k], np.full(4, t), conds, dt=np.float64) for k, t in enumerate(T_VALUES)])
        np.savez(os.path.join(HERE, 'g4_unet.npz'), t=np.array(T_VALUES), x=x, out=out, weight_names=names,
                 weight_sum=s1, weight_sumsq=s2)
        print('g4 written', out.shape)
    if 'g5' in which:
        x, z = g5_inputs()
        res = [R.ddpm(W, S, x[k], np.full(4, t), conds, z[k], dt=np.float64) for k, t in enumerate(PS_T)]
        np.savez(os.path.join(HERE, 'g5_p_sample.npz'), t=np.array(PS_T), x=x, z=z,
                 mean=np.stack([r[0] for r in res]), var=np.stack([r[1] for r in res]),
                 var_tilde=np.stack([r[2] for r in res]))
        print('g5 written')
    if 'g6' in which:
        W6 = g6_weights()
        n6, a6, b6 = checksums(W6)
        xT = g6_inputs()
        t0 = time.time()
        idx_s = R.loop_indices(1000, LOOP_STEPS_SHORT)
        short = R.ddpm_loop(W6, S, xT, conds[:1], loop_z(LOOP_STEPS_SHORT), idx_s, dt=np.float64)
        idx = R.loop_indices(1000, None)
        full = R.ddpm_loop(W6, S, xT, conds[:1], loop_z(1000), idx, dt=np.float64)
        np.savez(os.path.join(HERE, 'g6_loop.npz'), seed=np.int64(LOOP_SEED), x_T=xT, out_25=short, out_1000=full,
                 weight_names=n6, weight_sum=a6, weight_sumsq=b6)
        print(f'g6 written ({time.time() - t0:.0f} s)', float(np.abs(full).max()))
    if 'g7' in which:
        from pet_posterior_distribution_amd.sim_data import mh_problem
        P = mh_problem(SEEDS[0])
        t = truth[0]
        rng = np.random.default_rng(7)
        pts = [(t['DVR'], t['R1']), (P['mu_DVR'], P['mu_R1'])]
        for s in (0.01, 0.03, 0.1, 0.3):
            pts.append((t['DVR'] * (1 + s * rng.standard_normal(48)), t['R1'] * (1 + s * rng.standard_normal(48))))
        D = np.stack([p[0] for p in pts])
        R1 = np.stack([p[1] for p in pts])
        lp = np.array([K.log_posterior(d, r, P['k2p'], P['y_obs'], P['sigma_noise'], P['time_vector'], P['tac_ref'],
                                       P['mu_DVR'], P['Cov_DVR'], P['mu_R1'], P['Cov_R1']) for d, r in zip(D, R1)])
        np.savez(os.path.join(HERE, 'g7_mh_logp.npz'), DVR=D, R1=R1, logp=lp)
        print('g7 written', lp)


if __name__ == '__main__':
    make(sys.argv[1:] or ['g3', 'g4', 'g5', 'g6', 'g7'])
