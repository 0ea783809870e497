"""GPU parity tests of the SRTM2 kernel and the Metropolis-Hastings sampler (petmh).

* SRTM2 forward vs the reference's own outputs (tests/golden/g2_srtm2.npz): rtol 1e-10 (fp64).
* joint log density vs the oracle restatement of mcmc.py:147-155: rtol 1e-10.
* MH chains vs the oracle sampler fed the same counter-based noise: identical
  accept/reject path -> per-chain means / M2 equal to 1e-8 relative.
"""
import os

import numpy as np
import pytest
import torch

from oracle import srtm2_ref as K

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


@pytest.fixture(scope='module')
def g2():
    return np.load(os.path.join(GOLD, 'g2_srtm2.npz'))


def make_problem(g2, case=0, noise=0.1, seed=0):
    from tests.helpers import mh_problem
    return mh_problem(g2, case, noise, seed)


def test_srtm2_kernel_vs_reference(g2):
    from pet_posterior_distribution_amd.kinetic_model import SRTM2
    tv, dt = g2['time_vector'], g2['dt']
    for k in range(4):
        m = SRTM2(tv, dt, g2[f'case{k}_tac_ref'])
        tac = m.create_activity_curve(DVR=g2[f'case{k}_DVR'], R1=g2[f'case{k}_R1'], k2p=float(g2[f'case{k}_k2p']))
        np.testing.assert_allclose(tac, g2[f'case{k}_tac'], rtol=1e-10, atol=1e-12)


def test_create_tac_op_vs_reference(g2):
    """mcmc.CreateTAC_SRTM2 (the reference's PyTensor Op, mcmc.py:27-39) through its perform() calling
    convention and as a callable: the (n_roi, 54) TAC of the reference's kinetic_model outputs (G2)."""
    from pet_posterior_distribution_amd.kinetic_model import SRTM2
    from pet_posterior_distribution_amd.mcmc import CreateTAC_SRTM2
    tv, dt = g2['time_vector'], g2['dt']
    for k in range(4):
        op = CreateTAC_SRTM2(SRTM2(tv, dt, g2[f'case{k}_tac_ref']))
        args = (g2[f'case{k}_DVR'], g2[f'case{k}_R1'], float(g2[f'case{k}_k2p']))
        out = [[None]]
        op.perform(None, args, out)
        assert out[0][0].shape == (48, 54)
        np.testing.assert_allclose(out[0][0], g2[f'case{k}_tac'].T, rtol=1e-10, atol=1e-12)
        np.testing.assert_array_equal(op(*args), out[0][0])


def test_srtm2_batched(g2):
    from pet_posterior_distribution_amd.kinetic_model import SRTM2
    tv, dt = g2['time_vector'], g2['dt']
    m = SRTM2(tv, dt, g2['case1_tac_ref'])
    D = np.stack([g2[f'case{k}_DVR'] for k in range(4)])
    R = np.stack([g2[f'case{k}_R1'] for k in range(4)])
    out = m.create_activity_curves(D, R, 0.05).cpu().numpy()
    for k in range(4):
        ref = K.srtm2_tac(tv, g2['case1_tac_ref'], D[k], R[k], 0.05).T
        np.testing.assert_allclose(out[k], ref, rtol=1e-10, atol=1e-12)


def test_logp_vs_oracle(g2):
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    P = make_problem(g2)
    mh = MetropolisSRTM2(**P)
    rng = np.random.default_rng(3)
    pts = np.concatenate([P['mu_DVR'] * (1 + 0.05 * rng.standard_normal((5, 48))),
                          P['mu_R1'] * (1 + 0.05 * rng.standard_normal((5, 48)))], axis=1)
    got = mh.logp(pts).cpu().numpy()
    for k in range(5):
        ref = K.log_posterior(pts[k, :48], pts[k, 48:], P['k2p'], P['y_obs'], P['sigma_noise'], P['time_vector'],
                              P['tac_ref'], P['mu_DVR'], P['Cov_DVR'], P['mu_R1'], P['Cov_R1'])
        assert abs(got[k] - ref) <= 1e-10 * abs(ref)
    mh.close()


def test_mh_chain_path_matches_oracle(g2):
    """Same Philox stream -> the GPU chain takes the oracle's accept/reject path."""
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    P = make_problem(g2, case=2)
    mh = MetropolisSRTM2(**P)
    n_chains, draws, tune, seed = 3, 6, 4, 987
    res = mh.run(n_chains, draws, tune, seed=seed, return_chains=True)

    def logp(x):
        with np.errstate(over='ignore', invalid='ignore'):   # DVR <= 0 proposals: test_mh_chain_rejects_...
            return K.log_posterior(x[:48], x[48:], P['k2p'], P['y_obs'], P['sigma_noise'], P['time_vector'],
                                   P['tac_ref'], P['mu_DVR'], P['Cov_DVR'], P['mu_R1'], P['Cov_R1'])
    x0 = np.concatenate([P['mu_DVR'], P['mu_R1']])
    for ch in range(n_chains):
        dr, acc = K.metropolis_elemwise_philox(logp, x0, draws, tune, seed, ch)
        st = res['chain_stats'][ch]
        np.testing.assert_allclose(st[:, 1], dr.mean(0), rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(st[:, 2], ((dr - dr.mean(0)) ** 2).sum(0), rtol=1e-6, atol=1e-12)
        np.testing.assert_allclose(res['last'][ch], dr[-1], rtol=1e-9)
    mh.close()


def test_mh_tuned_chains_statistics(g2):
    """Many chains with tuning: finite pooled moments, acceptance in a sane band, posterior
    mean close to the truth the data were simulated from."""
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    P = make_problem(g2, case=0, noise=0.05)
    mh = MetropolisSRTM2(**P)
    res = mh.run(256, 300, 400, seed=11)
    for k in ('mean_DVR', 'mean_R1', 'std_DVR', 'std_R1'):
        assert np.isfinite(res[k]).all()
    ar = res['accept_rate'].mean()
    assert 0.05 < ar < 0.95
    assert np.abs(res['mean_DVR'] / g2['case0_DVR'] - 1).mean() < 0.1
    mh.close()


@pytest.mark.parametrize('vs0', [True, False])
def test_mh_chains_match_c_oracle(g2, vs0):
    """64 chains x (130 tune + 30 draws): one tune-table update, GPU vs the C
    restatement on the same Philox stream (vs0: pymc's sweep-start reference)."""
    from oracle import mh_c
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    P = make_problem(g2, case=3, noise=0.08, seed=4)
    mh = MetropolisSRTM2(**P, vs_sweep_start=vs0)
    n, draws, tune, seed = 64, 30, 130, 2024
    res = mh.run(n, draws, tune, seed=seed, return_chains=True)
    st, acc, last = mh_c.MHProblem(**P).run(n, draws, tune, seed, threads=8, vs_sweep_start=vs0)
    # an accept/reject decision within ~1e-12 of the threshold may flip between
    # summation orders; require (almost) every chain to follow the oracle exactly
    same = np.all(np.abs(res['last'] - last) <= 1e-9 * np.abs(last), axis=1)
    assert same.sum() >= n - 1, f'{n - same.sum()} chains diverged from the oracle path'
    np.testing.assert_allclose(res['chain_stats'][same][..., 1], st[same][..., 1], rtol=1e-9)
    np.testing.assert_allclose(res['chain_stats'][same][..., 2], st[same][..., 2], rtol=1e-6, atol=1e-12)
    mh.close()


def test_mh_trace_matches_welford(g2):
    """petmh_run_draws: the stored trace reproduces the on-GPU Welford moments."""
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    P = make_problem(g2, case=1)
    mh = MetropolisSRTM2(**P)
    res = mh.run(16, 40, 30, seed=5, return_chains=True, return_draws=True)
    tr = res['draws'].cpu().numpy()
    assert tr.shape == (16, 40, 96)
    np.testing.assert_allclose(res['chain_stats'][..., 1], tr.mean(1), rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(res['chain_stats'][..., 2], ((tr - tr.mean(1, keepdims=True)) ** 2).sum(1),
                               rtol=1e-9, atol=1e-14)
    np.testing.assert_array_equal(res['last'], tr[:, -1])
    mh.close()


def _same_class(a, b):
    """Both finite and within 1e-10 relative, or the same non-finite value (nan / +inf / -inf)."""
    if np.isfinite(a) and np.isfinite(b):
        return abs(a - b) <= 1e-10 * abs(b)
    return (np.isnan(a) and np.isnan(b)) or a == b


def test_logp_edge_cases_vs_oracle(g2):
    """Deliberate edge cases of the model (mcmc.py:147-155): DVR near 0 (SRTM2 TAC goes negative in
    late frames -> the sn < 0 -> 1e-6 switch of :152), DVR = 0, DVR < 0 (exp(-k2a t) overflows: the
    model TAC is +-inf / nan), R1 < 0.  GPU and oracle agree value for value, non-finite included."""
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    P = make_problem(g2, case=1)
    mh = MetropolisSRTM2(**P)
    base = np.concatenate([P['mu_DVR'], P['mu_R1']])
    pts, hit_clamp = [], False
    for dvr in (0.03, 0.01, 0.0, -0.002, -0.05, -1.0):
        p = base.copy()
        p[[3, 17, 40]] = dvr
        pts.append(p)
        if dvr > 0:
            sn = K.srtm2_tac(P['time_vector'], P['tac_ref'], p[:48], p[48:], P['k2p'])
            hit_clamp |= bool((sn < 0).any())
    p = base.copy()
    p[48 + 5] = -0.3                                    # R1 < 0
    pts.append(p)
    assert hit_clamp, 'no point exercised the sn < 0 switch'
    pts = np.stack(pts)
    got = mh.logp(pts).cpu().numpy()
    with np.errstate(all='ignore'):
        ref = [K.log_posterior(q[:48], q[48:], P['k2p'], P['y_obs'], P['sigma_noise'], P['time_vector'],
                               P['tac_ref'], P['mu_DVR'], P['Cov_DVR'], P['mu_R1'], P['Cov_R1']) for q in pts]
    assert any(not np.isfinite(r) for r in ref), 'no point produced a non-finite density'
    bad = [(k, got[k], ref[k]) for k in range(len(ref)) if not _same_class(got[k], ref[k])]
    assert not bad, bad
    mh.close()


def test_mh_chain_rejects_nonfinite_proposals(g2):
    """Chains started next to DVR = 0 with small proposals (scaling 3e-3): many proposals land in
    DVR <= 0, where exp(-k2a t) overflows and the density is non-finite; metrop_select's isfinite
    rule rejects them.  The GPU chain path equals the oracle's on the same Philox stream, and the
    oracle confirms such proposals occurred."""
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    P = make_problem(g2, case=0)
    scaling = 3e-3
    mh = MetropolisSRTM2(**P, scaling=scaling)
    x0 = np.concatenate([P['mu_DVR'], P['mu_R1']])
    x0[:8] = 5e-4
    n_chains, draws, tune, seed = 2, 5, 3, 4242
    res = mh.run(n_chains, draws, tune, seed=seed, x0=np.repeat(x0[None], n_chains, 0), return_chains=True)
    n_bad = [0]

    def logp(x):
        with np.errstate(all='ignore'):
            v = K.log_posterior(x[:48], x[48:], P['k2p'], P['y_obs'], P['sigma_noise'], P['time_vector'],
                                P['tac_ref'], P['mu_DVR'], P['Cov_DVR'], P['mu_R1'], P['Cov_R1'])
        n_bad[0] += not np.isfinite(v)
        return v
    for ch in range(n_chains):
        dr, acc = K.metropolis_elemwise_philox(logp, x0, draws, tune, seed, ch, scaling=scaling)
        assert np.isfinite(dr).all()
        np.testing.assert_allclose(res['last'][ch], dr[-1], rtol=1e-9)
        np.testing.assert_allclose(res['chain_stats'][ch][:, 1], dr.mean(0), rtol=1e-9, atol=1e-12)
    assert n_bad[0] > 0
    assert np.isfinite(res['last']).all()
    mh.close()


def test_batched_kernel_invariant_to_waves_per_chain(g2):
    """The batched sampler deals a chain's 144 proposal evaluations to 1, 2, 4 or 12 waves.  A chain's
    path depends only on its index: stats, last state, trace and acceptance are bitwise identical
    for every waves-per-chain setting and chain count."""
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    P = make_problem(g2, case=2, noise=0.06, seed=9)
    mh = MetropolisSRTM2(**P)
    ref = None
    for wpc, n in ((12, 40), (4, 700), (2, 1500), (1, 4000), (1, 40)):
        mh.set_kernel('batched', wpc)
        res = mh.run(n, 4, 3, seed=77, return_chains=True, return_draws=True)
        got = (res['chain_stats'][:40], res['last'][:40], res['draws'][:40].cpu().numpy(),
               res['accept_rate'][:40])
        if ref is None:
            ref = got
            continue
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(a, b)
    mh.close()


@pytest.mark.parametrize('vs0', [True, False])
def test_batched_and_update_kernels_same_chain_path(g2, vs0):
    """The batched kernel (likelihoods of every possible proposal state up front, then a scan) and the
    one-update-at-a-time kernel take the same accept/reject path: they differ only in the order of
    the 54-frame sum, so a decision within ~1e-12 of its threshold may flip (allow one chain)."""
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    P = make_problem(g2, case=3, noise=0.08, seed=4)
    mh = MetropolisSRTM2(**P, vs_sweep_start=vs0)
    out = {}
    for k in ('update', 'batched'):
        mh.set_kernel(k)
        out[k] = mh.run(64, 30, 130, seed=2024, return_chains=True)
    a, b = out['update'], out['batched']
    same = np.all(np.abs(a['last'] - b['last']) <= 1e-9 * np.abs(b['last']), axis=1)
    assert same.sum() >= 63, f'{64 - same.sum()} chains diverged between the kernels'
    np.testing.assert_allclose(a['chain_stats'][same][..., 1], b['chain_stats'][same][..., 1], rtol=1e-9)
    np.testing.assert_allclose(a['chain_stats'][same][..., 2], b['chain_stats'][same][..., 2], rtol=1e-6,
                               atol=1e-12)
    with pytest.raises(ValueError):
        mh.set_kernel('batched', 3)
    mh.close()
