"""CPU tests: the oracle against the reference's golden vectors, the host logic of the
product (schedule tables, sub-sequences, weight spec, synthetic data), and the
multi-rank statistics merge over gloo (world_size 2)."""
import os

import numpy as np
import pytest

from oracle import iddpm_ref as R
from oracle import srtm2_ref as K

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


# ---------------------------------------------------------------- G1: schedules
def test_oracle_schedules_bitexact_vs_reference():
    g = np.load(os.path.join(GOLD, 'g1_schedules.npz'))
    np.testing.assert_array_equal(R.get_beta_schedule('cosine', 1000), g['cosine_T1000'])
    np.testing.assert_array_equal(R.get_beta_schedule('cosine', 200), g['cosine_T200'])
    np.testing.assert_array_equal(R.get_beta_schedule('linear', 1000), g['linear_T1000'])
    np.testing.assert_array_equal(R.get_beta_schedule('quadratic', 1000), g['quadratic_T1000'])
    np.testing.assert_array_equal(R.get_beta_schedule('sigmoid', 1000), g['sigmoid_T1000'])


def test_product_schedules_bitexact_vs_reference():
    from pet_posterior_distribution_amd import helper_func as hf
    g = np.load(os.path.join(GOLD, 'g1_schedules.npz'))
    kw = dict(beta_start=1e-4, beta_end=2e-2, offset_s=0.008, max_beta=0.999)
    for name, key in [('cosine', 'cosine_T1000'), ('linear', 'linear_T1000'), ('quadratic', 'quadratic_T1000'),
                      ('sigmoid', 'sigmoid_T1000')]:
        np.testing.assert_array_equal(hf.get_beta_schedule(name, 1000, **kw), g[key])
    with pytest.raises(NotImplementedError):
        hf.get_beta_schedule('exp', 10)


def test_schedule_known_values():
    """Survey a1 known answers (beta_0, beta_999, alpha_bar_999, plvc[0] == plvc[1])."""
    S = R.schedule_tables(R.get_beta_schedule('cosine', 1000))
    assert abs(S['beta'][0] - 4.1246e-5) < 1e-8
    assert S['beta'][-1] == np.float32(0.999)
    assert abs(S['alpha_bar'][-1] - 2.4289e-9) < 1e-12
    assert S['posterior_log_variance_clipped'][0] == S['posterior_log_variance_clipped'][1]
    assert abs(S['posterior_log_variance_clipped'][0] + 10.734668) < 1e-5
    assert S['posterior_variance'][0] == S['posterior_variance'][1]      # the alias quirk (:349-351)


def test_product_tables_match_oracle():
    """ImprovedDDPM's host tables (handed to libpetdiff) == the oracle's restatement."""
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    from pet_posterior_distribution_amd.configs import shipped_net_args, shipped_diff_args
    m = ImprovedDDPM(network=UnetConditional(**shipped_net_args()), **shipped_diff_args())
    S = R.schedule_tables(R.get_beta_schedule('cosine', 1000))
    tab = m.schedule_tables()
    assert tab.shape == (13, 1000) and tab.dtype == np.float32
    np.testing.assert_array_equal(tab[0], S['beta'])
    np.testing.assert_array_equal(tab[2], S['posterior_log_variance_clipped'])
    np.testing.assert_array_equal(tab[4], S['posterior_mean_coef1'])
    np.testing.assert_array_equal(tab[5], S['posterior_mean_coef2'])
    np.testing.assert_array_equal(tab[6], S['alpha_bar'])
    np.testing.assert_array_equal(tab[9], np.float32(1) / S['sqrt_alpha_bar'])


def test_improved_ddpm_errors_match_reference():
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    from pet_posterior_distribution_amd.configs import shipped_net_args, shipped_diff_args
    with pytest.raises(ValueError, match='Input network is required'):
        ImprovedDDPM(network=None, **shipped_diff_args())
    with pytest.raises(ValueError, match='Invalid parameterization'):
        ImprovedDDPM(network=UnetConditional(**shipped_net_args()), parameterization='foo', **shipped_diff_args())
    m = ImprovedDDPM(network=UnetConditional(**shipped_net_args()), **shipped_diff_args())
    with pytest.raises(ValueError, match='Subsequence type not recognized'):
        m.sub_sequence(10, 'cubic')


# ---------------------------------------------------------------- sub-sequences
def test_loop_indices_reference_semantics():
    assert R.loop_indices(1000) == list(range(1000))[::-1]
    lin = R.loop_indices(1000, 100, 'linear')
    assert lin[:5] == [999, 988, 978, 968, 958] and lin[-1] == 0 and len(lin) == 100
    quad = R.loop_indices(1000, 100, 'quadratic')
    assert quad[:3] == [961, 961, 900] and len(set(quad)) == 32          # survey hard-part (a)
    assert R.loop_indices(1000, 10, 'lin') == R.loop_indices(1000, 10, 'linear')   # substring test :683
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    from pet_posterior_distribution_amd.configs import shipped_net_args, shipped_diff_args
    m = ImprovedDDPM(network=UnetConditional(**shipped_net_args()), **shipped_diff_args())
    for n, kind in [(None, 'linear'), (100, 'linear'), (100, 'quadratic'), (1000, 'quadratic'), (7, 'l')]:
        assert m.sub_sequence(n, kind) == R.loop_indices(1000, n, kind)


# ---------------------------------------------------------------- network spec
def test_param_spec_structure():
    from pet_posterior_distribution_amd.networks import param_spec
    spec = param_spec()
    assert spec == R.param_spec()
    assert sum(int(np.prod(s)) for _, s in spec) == 11_851_740
    d = dict(spec)
    assert d['down0.conv.kernel'] == (6, 52, 128) and d['down3.conv.kernel'] == (6, 562, 1024)
    assert d['up0.upconv.kernel'] == (2, 1074, 512) and d['up2.conv.kernel'] == (6, 256, 128)
    assert d['final.kernel'] == (1, 128, 4)


def test_unsupported_configs_raise():
    from pet_posterior_distribution_amd import UnetConditional
    from pet_posterior_distribution_amd.configs import shipped_net_args
    a = shipped_net_args()
    a['depth'] = 5
    with pytest.raises(NotImplementedError):
        UnetConditional(**a)
    a = shipped_net_args()
    a['block_params'] = {'flag_res': True, 'kernel_size': 6, 'norm_list': 'pre'}
    with pytest.raises(NotImplementedError):
        UnetConditional(**a)


def test_denoiser_init_identity_path_and_bounded_chain():
    """The synthetic weights predict eps ~ x (+ small perturbation); a short chain stays finite."""
    from pet_posterior_distribution_amd.networks import denoiser_init, param_spec
    P = denoiser_init(param_spec(), seed=3)
    rng = np.random.default_rng(0)
    x = rng.standard_normal((2, 48, 2))
    cond = np.abs(rng.standard_normal((2, 49, 54)))
    out = R.unet_forward(P, x, np.array([999, 10]), cond)
    assert np.abs(out[..., :2] - x).max() < 1.0
    S = R.schedule_tables(R.get_beta_schedule('cosine', 1000))
    idx = R.loop_indices(1000, 10)
    x0 = R.ddpm_loop(P, S, x, cond[:1], rng.standard_normal((10, 2, 48, 2)), idx, dt=np.float64)
    assert np.isfinite(x0).all()


def test_oracle_keras_semantics():
    """conv1d_same padding (TF SAME: left (k-1)//2), raw reshape, maxpool / upsample."""
    x = np.arange(1, 7, dtype=np.float64).reshape(1, 6, 1)
    W = np.zeros((6, 1, 1))
    W[0] = 1.0                               # tap 0 reads position l - 2
    np.testing.assert_array_equal(R.conv1d_same(x, W, 0.0)[0, :, 0], [0, 0, 1, 2, 3, 4])
    W = np.zeros((2, 1, 1))
    W[1] = 1.0                               # k=2: pad right 1 -> tap 1 reads l + 1
    np.testing.assert_array_equal(R.conv1d_same(x, W, 0.0)[0, :, 0], [2, 3, 4, 5, 6, 0])
    np.testing.assert_array_equal(R.maxpool2(x)[0, :, 0], [2, 4, 6])
    np.testing.assert_array_equal(R.upsample2(x)[0, :4, 0], [1, 1, 2, 2])


def test_oracle_fp32_close_to_fp64():
    from pet_posterior_distribution_amd.networks import denoiser_init, param_spec
    P = denoiser_init(param_spec(), seed=5, bias_scale=0.05)
    rng = np.random.default_rng(1)
    x = rng.standard_normal((2, 48, 2))
    cond = np.abs(rng.standard_normal((2, 49, 54)))
    a = R.unet_forward(P, x, np.array([500, 3]), cond, dt=np.float64)
    b = R.unet_forward(P, x, np.array([500, 3]), cond, dt=np.float32)
    assert np.abs(a - b).max() / np.abs(a).max() < 1e-5


# ---------------------------------------------------------------- Philox
def test_philox_known_answers():
    """Random123 philox4x32-10 known-answer vectors."""
    out = R.philox4x32_10(0, 0, 0, 0, 0, 0)
    assert [int(v) for v in out] == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    f = 0xffffffff
    out = R.philox4x32_10(f, f, f, f, f, f)
    assert [int(v) for v in out] == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    out = R.philox4x32_10(0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0)
    assert [int(v) for v in out] == [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_philox_normals_statistics():
    z = R.philox_normal_pairs(12345, np.arange(4000), 3)
    assert z.shape == (4000, 48, 2)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01


# ---------------------------------------------------------------- G2: SRTM2
def test_srtm2_oracle_vs_reference_golden():
    g = np.load(os.path.join(GOLD, 'g2_srtm2.npz'))
    tv = g['time_vector']
    for k in range(4):
        tac = K.srtm2_tac(tv, g[f'case{k}_tac_ref'], g[f'case{k}_DVR'], g[f'case{k}_R1'], float(g[f'case{k}_k2p']))
        np.testing.assert_allclose(tac, g[f'case{k}_tac'], rtol=1e-12, atol=1e-14)
    up = K.interp1d_linear_vec(g['interp_x'], tv, np.exp(-0.05 * tv)[:, None] * np.arange(1, 4)[None, :])
    np.testing.assert_allclose(up, g['interp_up'], rtol=1e-13, atol=1e-15)


def test_srtm2_operator_reassociation():
    """TAC = R1 C_r + (k2 - R1 k2a) M exp(-k2a t) with the constant 54x54 M (used by the MH kernel)."""
    g = np.load(os.path.join(GOLD, 'g2_srtm2.npz'))
    tv = g['time_vector']
    M = K.srtm2_operator(tv, g['case0_tac_ref'])
    DVR, R1, k2p = g['case0_DVR'], g['case0_R1'], float(g['case0_k2p'])
    k2 = k2p * R1
    k2a = k2 / DVR
    e = np.exp(-k2a[None, :] * tv[:, None])
    tac = R1 * g['case0_tac_ref'][:, None] + (k2 - R1 * k2a) * (M @ e)
    np.testing.assert_allclose(tac, g['case0_tac'], rtol=1e-11, atol=1e-13)


def test_product_srtm2_host_vs_reference_golden():
    from pet_posterior_distribution_amd.sim_data import srtm2_tac, time_grid
    g = np.load(os.path.join(GOLD, 'g2_srtm2.npz'))
    tv, dt = time_grid()
    np.testing.assert_array_equal(tv, g['time_vector'])
    np.testing.assert_array_equal(dt, g['dt'])
    for k in range(4):
        tac = srtm2_tac(g[f'case{k}_DVR'], g[f'case{k}_R1'], float(g[f'case{k}_k2p']), g[f'case{k}_tac_ref'], tv)
        np.testing.assert_allclose(tac, g[f'case{k}_tac'], rtol=1e-12, atol=1e-14)


def test_mh_log_posterior_and_sampler_smoke():
    g = np.load(os.path.join(GOLD, 'g2_srtm2.npz'))
    tv = g['time_vector']
    ref = g['case0_tac_ref']
    mu_D, mu_R = g['case0_DVR'], g['case0_R1']
    cov_D = np.diag((0.1 * mu_D) ** 2)
    cov_R = np.diag((0.1 * mu_R) ** 2)
    sn = g['case0_tac'].T
    sig = np.full_like(sn, 0.1)
    y = sn + np.sqrt(sn) * 0.05
    lp = K.log_posterior(mu_D, mu_R, float(g['case0_k2p']), y, sig, tv, ref, mu_D, cov_D, mu_R, cov_R)
    assert np.isfinite(lp)
    # tune table (pymc 5.12)
    np.testing.assert_allclose(K.pymc_tune(np.ones(7), np.array([0.0005, 0.01, 0.1, 0.3, 0.6, 0.8, 0.99])),
                               [0.1, 0.5, 0.9, 1.0, 1.1, 2.0, 10.0])


# ---------------------------------------------------------------- synthetic data
def test_acquisition_protocol():
    from pet_posterior_distribution_amd.sim_data import acquisition_time_frames
    f = acquisition_time_frames()
    assert f.shape == (54, 2)
    assert abs(f[0, 1] - 10 / 60) < 1e-12 and abs(f[-1, 1] - 120) < 1e-12
    np.testing.assert_allclose(f[1:, 0], f[:-1, 1])


def test_make_condition_shape():
    from pet_posterior_distribution_amd.sim_data import make_condition
    c = make_condition(3)
    assert c.shape == (49, 54) and c.dtype == np.float32 and (c >= 0).all()


# ---------------------------------------------------------------- distributed merge
def test_merge_stats_matches_numpy():
    from pet_posterior_distribution_amd.distributed import merge_stats, local_stats_numpy, summarize
    rng = np.random.default_rng(0)
    x = rng.standard_normal((1000, 48, 2)) * 2 + 3
    parts = [local_stats_numpy(x[a:b]) for a, b in [(0, 100), (100, 601), (601, 1000)]]
    st = merge_stats(parts)
    s = summarize(st)
    np.testing.assert_allclose(s['mean_DVR'][0], x[:, :, 0].mean(0), rtol=1e-12)
    np.testing.assert_allclose(s['std_R1'][0], x[:, :, 1].std(0), rtol=1e-12)


def test_shard_ranges_cover():
    from pet_posterior_distribution_amd.distributed import shard_range
    for n, w in [(10, 3), (8192 * 256, 8), (5, 8)]:
        rs = [shard_range(n, w, r) for r in range(w)]
        assert rs[0][0] == 0 and rs[-1][1] == n
        assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist
    from pet_posterior_distribution_amd.distributed import (allgather_stats, merge_stats, local_stats_numpy,
                                                           shard_range)
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=world)
    rng = np.random.default_rng(42)
    x = rng.standard_normal((777, 48, 2))
    lo, hi = shard_range(777, world, rank)
    parts = allgather_stats(local_stats_numpy(x[lo:hi]))
    st = merge_stats(parts)
    if rank == 0:
        q.put((st[0, :, :, 1] - x.mean(0), np.sqrt(st[0, :, :, 2] / st[0, :, :, 0]) - x.std(0)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_allgather_merge():
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    dm, ds = q.get(timeout=120)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.abs(dm).max() < 1e-12 and np.abs(ds).max() < 1e-12


def test_fused_up_composite_identity():
    """The algebra behind the fused up levels (csrc/unet_kernels.hip compose_kernel):
    UpSampling1D(2) -> Conv1D(k=2, 'same' = pad (0, 1)) -> concat -> Conv1D(k=6, 'same' = pad (2, 3))
    (networks.py:970-975, 1046-1057, 679-691) equals, for output l = 2m + e, the 4-tap conv
    sum_k C[e][k] b[m - 1 + k] on the coarse input, plus (-K1 W1) b[0] at l = 0 and (-K0 W1) b[0]
    at l = 1, plus the k2 bias pushed through the zero-padded k6 conv.  Same term table as the kernel."""
    rng = np.random.default_rng(0)
    for Lh in (3, 6, 12):
        L, cb, cu, co = 2 * Lh, 5, 4, 3
        W = rng.standard_normal((2, cb, cu))
        K = rng.standard_normal((6, cu, co))
        bu = rng.standard_normal(cu)
        b = rng.standard_normal((Lh, cb))
        # direct: upsample, k2 conv (pad right 1), k6 conv over u (pad 2 left, 3 right)
        v = np.repeat(b, 2, axis=0)
        vp = np.concatenate([v, np.zeros((1, cb))])
        u = vp[:L] @ W[0] + vp[1:L + 1] @ W[1] + bu
        up = np.concatenate([np.zeros((2, cu)), u, np.zeros((3, cu))])
        y = sum(up[j:j + L] @ K[j] for j in range(6))
        # composite: term table (j, alpha, beta) of kCompJ / kCompA / kCompB
        terms = [[(0, 1, 1), (1, 1, 0)], [(1, 0, 1), (2, 1, 1), (3, 1, 0)], [(3, 0, 1), (4, 1, 1), (5, 1, 0)],
                 [(5, 0, 1)], [(0, 1, 0)], [(0, 0, 1), (1, 1, 1), (2, 1, 0)], [(2, 0, 1), (3, 1, 1), (4, 1, 0)],
                 [(4, 0, 1), (5, 1, 1)], [(1, 0, -1)], [(0, 0, -1)]]
        C = [sum((al * W[0] + be * W[1]) @ K[j] for j, al, be in tt) for tt in terms]
        bp = np.concatenate([np.zeros((1, cb)), b, np.zeros((2, cb))])   # b[-1], b[Lh], b[Lh+1] = 0
        # bias: u's constant part through the zero-padded k6 conv (map_through_kernel)
        cst = np.concatenate([np.zeros((2, cu)), np.tile(bu, (L, 1)), np.zeros((3, cu))])
        ybias = sum(cst[j:j + L] @ K[j] for j in range(6))
        yc = np.empty_like(y)
        for l in range(L):
            m, e = divmod(l, 2)
            yc[l] = sum(bp[m + k] @ C[4 * e + k] for k in range(4)) + ybias[l]
            if m == 0:
                yc[l] += b[0] @ C[8 + e]
        np.testing.assert_allclose(yc, y, rtol=1e-12, atol=1e-12)


def test_bench_pmc_fields_known_answer():
    """bench.py's PMC-derived roofline extras: HBM GB/s vs 8 TB/s, and MFMA utilisation from
    SQ_VALU_MFMA_BUSY_CYCLES (32 cycles per 32x32x16 MFMA over 1024 SIMDs at 2.4 GHz), which
    must equal executed FLOP/s / dense peak (32768 FLOP per MFMA -> 1024 FLOP per busy cycle)."""
    import bench
    n_mfma = 1_000_000
    pmc = {'traffic': 8e12 * 1e-4, 'mfma_busy': 32 * n_mfma, 'grbm': 8 * 100_000, 'source': 'x'}
    f = bench.pmc_fields(pmc, 1e-4)
    assert f['hbm_gbs'] == 8000.0 and f['hbm_frac'] == 1.0
    exe_tflops = n_mfma * 32768 / 1e-4 / 1e12
    # 2.5 PF / (1024 SIMDs x 2.4 GHz) = 1017 FLOP per SIMD-cycle vs the MFMA's 1024: 0.7% apart
    assert abs(f['mfma_util'] / (exe_tflops / bench.PEAK_BF16_TFLOPS) - 1) < 0.01
    assert f['mfma_busy_vs_active'] == round(32 * n_mfma / (1024 * 100_000), 4)
    none = bench.pmc_fields({'traffic': None, 'mfma_busy': None, 'grbm': None, 'source': None}, 1e-4)
    assert none['hbm_gbs'] is None and none['mfma_util'] is None


def test_default_noise_stream_keys_distinct():
    """diffusion_model.stream_seed: the keys of default-seeded calls differ across call kinds,
    counters and model seeds (the round-1 scheme seed + counter made model seed s at call c+1 reuse
    model seed s+1 at call c, and loops reuse p_sample keys)."""
    from pet_posterior_distribution_amd.diffusion_model import (stream_seed, STREAM_P_SAMPLE, STREAM_LOOP,
                                                                STREAM_EVAL)
    keys = {stream_seed(s, k, c) for s in range(4) for k in (STREAM_P_SAMPLE, STREAM_LOOP, STREAM_EVAL)
            for c in range(50)}
    assert len(keys) == 4 * 3 * 50
    assert all(0 <= k < 2 ** 64 for k in keys)
    assert stream_seed(12345, STREAM_LOOP, 0) not in (12345, 12346)


def test_torch_cpu_baseline_port_matches_oracle():
    """oracle/iddpm_torch_cpu.py (the CPU-baseline timing port) computes the NumPy oracle's
    p_sample: fp32 both, same weights, t, condition and z."""
    import torch
    from oracle import iddpm_torch_cpu as TC
    from pet_posterior_distribution_amd import networks as N
    w = N.glorot_uniform_init(R.param_spec(), seed=3, bias_scale=0.05)
    P = {k: np.asarray(v, np.float32) for k, v in w.items()}
    S = R.schedule_tables(R.get_beta_schedule('cosine', 1000))
    rng = np.random.default_rng(4)
    B = 3
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    t = np.array([0, 500, 999], np.int32)
    cond = rng.standard_normal((B, 49, 54)).astype(np.float32)
    z = rng.standard_normal((B, 48, 2)).astype(np.float32)
    m_ref, v_ref, vt_ref = R.ddpm(P, S, x, t, cond, z, dt=np.float32)
    net = TC.TorchCpuUnet(P)
    m, v, vt = net.ddpm(S, torch.as_tensor(x), t, torch.as_tensor(cond), torch.as_tensor(z))
    for a, b in ((m, m_ref), (vt, vt_ref)):
        a = a.numpy()
        assert np.abs(a - b).max() <= 2e-5 * max(1.0, np.abs(b).max()), np.abs(a - b).max()


def test_down1_pair_position_major_layout():
    """down1's pair-position-major tile (CONV_DOWN1_PP, unet_kernels.hip): fragment F of the 384-row
    tile holds positions 2F (lanes 0-15) and 2F+1 (lanes 16-31) of the tile's 16 samples, the LDS
    input slots are position-major (p * 16 + s), and the C tile is written back as sample-major row
    pairs.  Checks, in the kernel's integer arithmetic: every (sample, position) is one tile row;
    a 16-lane group reads 16 consecutive slots or only the zero row for every tap; the accumulator
    row pairs (rg, rg + 8), rg < 8, land on each sample-major pair (s, 2F | 2F + 1) exactly once."""
    L, S, MT = 24, 16, 384
    seen = set()
    for r in range(MT):
        l, s = 2 * (r >> 5) + ((r >> 4) & 1), r & 15
        seen.add((s, l))
    assert seen == {(s, l) for s in range(S) for l in range(L)}
    ZROW = S * L
    for F in range(MT // 32):
        for j in range(6):
            for g in range(2):
                slots = []
                for lr in range(16 * g, 16 * g + 16):
                    r = 32 * F + lr
                    l, s = 2 * (r >> 5) + ((r >> 4) & 1), r & 15
                    p = l + j - 2
                    slots.append(p * S + s if 0 <= p < L else ZROW)
                assert slots == [ZROW] * 16 or slots == list(range(slots[0], slots[0] + 16))
    pairs = []
    for wm in range(4):
        for i in range(3):
            for h in range(2):
                for rg in range(8):
                    r = wm * 96 + i * 32 + (rg & 3) + 8 * (rg >> 2) + 4 * h
                    assert r & 16 == 0
                    r2 = r + 16        # accumulator element rg + 8 of the same lane
                    assert (r2 & 15, 2 * (r2 >> 5) + ((r2 >> 4) & 1)) == (r & 15, 2 * (r >> 5) + 1)
                    pairs.append(((r & 15) * L + 2 * (r >> 5)) >> 1)
    assert sorted(pairs) == list(range(MT // 2))


def test_bench_pmc_fields_per_dtype_and_build(monkeypatch):
    """bench.py's roofline traffic / MFMA-busy fields come from profiles/pmc_traffic.json, per dtype: the
    bf16 entries are passes over the bf16 network (SQ_VALU_MFMA_BUSY_CYCLES of up0.fused = the analytic
    executed count, 32 busy cycles per 32x32x16 MFMA of 32,768 FLOP), the bf16x3 ones 3x that.  They are
    used only when the code-object hash they were stamped with is the loaded build's
    (_lib.kernel_code_hash); otherwise every field is None (stale counters)."""
    import json
    import bench
    from pet_posterior_distribution_amd import _lib
    d = json.load(open(os.path.join(os.path.dirname(os.path.dirname(__file__)), 'profiles', 'pmc_traffic.json')))
    want = bench.UP0_FUSED_EXEC_FLOP_PER_SAMPLE * 1024 / 32768 * 32
    assert abs(d['up0_fused_mfma_busy_cycles'] / want - 1) < 0.01
    assert d['up0_fused_bytes_per_launch'] < 2.5e8
    if 'up0_fused_bf16x3_mfma_busy_cycles' in d:
        assert abs(d['up0_fused_bf16x3_mfma_busy_cycles'] / (3 * want) - 1) < 0.01
    for dt, pre in (('bfloat16', 'up0_fused'), ('bf16x3', 'up0_fused_bf16x3')):
        stamp = d.get(pre + '_code_hash')
        monkeypatch.setattr(_lib, 'kernel_code_hash', lambda *a, **k: stamp)
        pmc = bench.load_pmc(True, dt)
        if stamp is not None:
            assert not pmc['stale'] and pmc['mfma_busy'] == d[pre + '_mfma_busy_cycles']
        monkeypatch.setattr(_lib, 'kernel_code_hash', lambda *a, **k: 'another build')
        pmc = bench.load_pmc(True, dt)
        assert pmc['stale'] and pmc['mfma_busy'] is None and pmc['traffic'] is None
        assert bench.pmc_fields(pmc, 70e-6)['mfma_util'] is None
        # a build without a recognisable code-object hash never matches, not even a stamp of None
        monkeypatch.setattr(_lib, 'kernel_code_hash', lambda *a, **k: None)
        pmc = bench.load_pmc(True, dt)
        assert pmc['stale'] and pmc['traffic'] is None


def test_bench_step_kernel_table(monkeypatch):
    """bench.py's roofline lists all 6 step kernels of the 16-bit path: launch time,
    algorithmic GFLOP, alg_over_peak, exec_frac (executed MFMA FLOPs / peak) and algorithmic
    bytes; PMC-derived traffic / mfma_util / LDS conflicts only when the committed passes match the build.
    No field named frac exceeds 1 at the kernels' measured speeds, and the App. A MACs add up to the
    SURVEY total."""
    import bench
    from pet_posterior_distribution_amd import _lib
    tot = sum(k[2] for k in bench.STEP_KERNELS) + 48 * 7 * 52 * 128 * 0
    # App. A total (148.18 M MAC) = down0 + the 6 kernels' counts (up2's includes the next step's down0)
    assert tot == bench.FLOP_PER_SAMPLE_STEP // 2
    from pet_posterior_distribution_amd import _lib as L
    us = {'down0': 0, 'down1': 13.4, 'down2': 18.3, 'down3': 25.6, 'up0.block': 59.7, 'up1.block': 37.6,
          'up2.block+final+p_sample': 40.1}
    lm = {k: (0.0, 0) for k in L.LAYER_NAMES}           # the keys ImprovedDDPM.get_kernel_timing returns
    for k, u in us.items():
        lm[k] = (u * 1e-3 * 1000 * bench.TIMING_REPS, 1000 * bench.TIMING_REPS if u else 0)
    monkeypatch.setattr(_lib, 'kernel_code_hash', lambda *a, **k: 'no such build')
    lm3 = {k: (v[0] * 2.6, v[1]) for k, v in lm.items()}     # bf16x3 runs about 2.6 x the bf16 times
    for dt, lmd in (('bfloat16', lm), ('bf16x3', lm3)):
        kt = bench.kernel_table(lmd, 1024, dt)
        assert [r['timing_key'] for r in kt['kernels']] == ['down1', 'down2', 'down3', 'up0.block', 'up1.block',
                                                              'up2.block+final+p_sample']
        assert kt['pmc'] is None and all('mfma_util' not in r for r in kt['kernels'])
        for r in kt['kernels']:
            assert 0 < r['exec_frac'] < 1 and r['alg_bytes'] > 0
    r = {x['timing_key']: x for x in bench.kernel_table(lm, 1024, 'bfloat16')['kernels']}
    assert abs(r['up0.block']['alg_gflop'] - 117.23) < 0.01 and abs(r['up0.block']['alg_over_peak'] - 0.786) < 0.001
    assert abs(r['down3']['alg_gflop'] - 49.50) < 0.01
    assert bench.kernel_table({**lm, 'up0.conv2': (1.0, 1000)}, 1024, 'bfloat16') is None   # unfused path


def test_reference_prior_fixture():
    """G0: the arrays of the reference's prior_stats_nROI48.pik (sample_sim_data.py:106-126), read by
    tests/golden/make_golden.py without unpickling; the package ships an identical copy
    (sim_data.reference_prior), the default prior of the generators, MH problems and the bench TAC.
    Structural pins: SURVEY 2 (48 ROIs, 54 frames, mu_k2p = 0.0126, ROI_names), symmetric positive
    definite covariances."""
    from pet_posterior_distribution_amd.sim_data import reference_prior
    g = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'g0_prior.npz'))
    p = reference_prior()
    assert sorted(g.files) == sorted(p)
    for k in g.files:
        np.testing.assert_array_equal(np.asarray(p[k]), g[k])
    assert p['mu_DVR'].shape == (48,) and p['Cov_R1'].shape == (48, 48) and p['Cov_tac_ref'].shape == (54, 54)
    assert abs(float(p['mu_k2p']) - 0.0126) < 1e-9 and p['ROI_names'][0] == 'Hippocampus' and len(set(p['ROI_names'])) == 48
    from oracle.sim_ref import cholesky_psd
    for c in ('Cov_DVR', 'Cov_R1', 'Cov_tac_ref'):
        np.testing.assert_allclose(p[c], p[c].T, rtol=0, atol=0)
        ev = np.linalg.eigvalsh(p[c])
        assert ev.min() > -1e-12 * ev.max()                   # positive semi-definite
        L = cholesky_psd(p[c])                                 # the generators' factor
        assert np.abs(L @ L.T - p[c]).max() < 1e-13 * np.abs(p[c]).max()
    assert np.linalg.matrix_rank(p['Cov_tac_ref']) < 54       # rank-deficient: a plain Cholesky fails
    assert (p['mu_DVR'] > 0).all() and (p['mu_R1'] > 0).all()


def test_static_pickle_reader_rejects_code():
    """make_golden.read_pickle_data rebuilds literal data only: a pickle that references anything but
    numpy's array / dtype / scalar reconstruction is refused (nothing is imported or called)."""
    import pickle
    import sys
    import tempfile
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), 'golden'))
    from make_golden import read_pickle_data
    with tempfile.TemporaryDirectory() as d:
        ok = os.path.join(d, 'ok.pik')
        with open(ok, 'wb') as f:
            pickle.dump({'a': np.arange(6.0).reshape(2, 3), 'b': [1, 'x'], 's': np.float64(2.5),
                         'f': np.asfortranarray(np.eye(2, 3, dtype=np.float32))}, f)
        got = read_pickle_data(ok)
        np.testing.assert_array_equal(got['a'], np.arange(6.0).reshape(2, 3))
        np.testing.assert_array_equal(got['f'], np.eye(2, 3, dtype=np.float32))
        assert got['b'] == [1, 'x'] and got['s'] == 2.5
        bad = os.path.join(d, 'bad.pik')
        with open(bad, 'wb') as f:
            pickle.dump({'x': os.getcwd}, f)           # a reference to a callable: refused
        with pytest.raises(ValueError):
            read_pickle_data(bad)


# ds_read_b128 lane groups on gfx950 (MI355X_MICROARCH.md, LDS table): one LDS cycle per group when its
# 16 lanes hit 16 distinct 4-bank groups
_B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
                list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
                list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
                list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]


def _piece_key(row, m16):
    """petdiff_internal.h piece_key for 64-B rows (CPR = 4), as the library exports it (petdiff_piece_key)."""
    from pet_posterior_distribution_amd import _lib
    return _lib.lib().petdiff_piece_key(row, 4, int(m16))


def test_piece_key_export_matches_documented_formula():
    """The library's piece_key (the one kernels and host packing use) against the formulas DESIGN.md states:
    64-B rows (row >> 2) & 3, 16x16x32 layers 2 ((row >> 2) & 1), 32-B rows (row >> 3) & 1, 128-B rows
    (row >> 1) & 7 (the test read a Python copy of the formula before)."""
    from pet_posterior_distribution_amd import _lib
    L = _lib.lib()
    for row in range(0, 2048, 3):
        assert L.petdiff_piece_key(row, 4, 0) == (row >> 2) & 3
        assert L.petdiff_piece_key(row, 4, 1) == 2 * ((row >> 2) & 1)
        assert L.petdiff_piece_key(row, 2, 0) == (row >> 3) & 1 == L.petdiff_piece_key(row, 2, 1)
        assert L.petdiff_piece_key(row, 8, 0) == (row >> 1) & 7 == L.petdiff_piece_key(row, 8, 1)


def _b128_conflict_cycles(addr):
    """Extra LDS cycles of one ds_read_b128 wave instruction: per lane group, the largest number of distinct
    16-B slots sharing a 4-bank group ((a / 4) mod 64 banks, 16 B = 4 banks)."""
    extra = 0
    for grp in _B128_GROUPS:
        slots = {}
        for lane in grp:
            a = addr[lane]
            slots.setdefault((a // 16) % 16, set()).add(a)
        extra += max(len(v) for v in slots.values()) - 1
    return extra


@pytest.mark.parametrize('base', [0, 16, 32, 48, 384])
def test_piece_key_conflict_free_for_both_mfma_shapes(base):
    """The XOR swizzle of the 64-B LDS rows is conflict-free for the reads of the MFMA shape each layer uses:
    32x32x16 (lane l: row l & 31, piece 2 g + (l >> 5) of k-group g) with the 32-row key, 16x16x32 (lane l:
    row l & 15, piece l >> 4) with the 16-row key -- and the 32-row key is 2-way on the 16x16x32 pattern, the
    round-4 regression the 16-row key fixed (profiles/r04/r4r_final/pmc vs r4s_swizzle)."""
    def addr32(g, m16):
        return [((base + (l & 31)) * 64 + (((2 * g + (l >> 5)) ^ _piece_key(base + (l & 31), m16)) << 4)) for l in range(64)]

    def addr16(rh, m16):
        return [((base + 16 * rh + (l & 15)) * 64 + (((l >> 4) ^ _piece_key(base + 16 * rh + (l & 15), m16)) << 4))
                for l in range(64)]
    for g in range(2):
        assert _b128_conflict_cycles(addr32(g, False)) == 0
    for rh in range(2):
        assert _b128_conflict_cycles(addr16(rh, True)) == 0
        assert _b128_conflict_cycles(addr16(rh, False)) > 0

    # paired bf16x3 units on 16x16x32 (unet_kernels.hip PX): a cross unit reads B with its halves swapped
    # (piece (l >> 4) ^ 2); the hi-hi unit's lanes 32-63 read piece ((l >> 4) ^ 2) of the same row in the
    # other chunk's stage (a multiple of 256 B away: STAGE is 256-B aligned); both stay conflict-free
    def addr16x(rh, stage_lo, stage_hi):
        out = []
        for l in range(64):
            r = base + 16 * rh + (l & 15)
            hi = l >= 32
            out.append((stage_hi if hi else stage_lo) + r * 64 + ((((l >> 4) ^ (2 if hi or stage_lo == stage_hi
                                                                              else 0)) ^ _piece_key(r, True)) << 4))
        return out
    # the round-5 final level on 16x16x32 (measured and rejected, profiles/r05/rejected_final_level_m16.diff; 32-B
    # rows, two taps per step): lane l reads row l & 15 (+ the tap's row shift for lanes 32-63), piece (l >> 4) & 1
    # -- conflict-free unswizzled; the 32-row key would not be
    def addr32b(shift, key):
        return [((base + (l & 15) + (shift if l >= 32 else 0)) * 32 +
                 ((((l >> 4) & 1) ^ (((base + (l & 15) + (shift if l >= 32 else 0)) >> 3) & 1 if key else 0)) << 4))
                for l in range(64)]
    for shift in (0, 4, 8, 96):
        assert _b128_conflict_cycles(addr32b(shift, False)) == 0
    assert max(_b128_conflict_cycles(addr32b(sh, True)) for sh in (0, 4, 8)) > 0
    for rh in range(2):
        assert _b128_conflict_cycles(addr16x(rh, 0, 0)) == 0                  # cross: every lane swapped
        assert _b128_conflict_cycles(addr16x(rh, 0, 53504)) == 0              # hi-hi: lanes 32-63 in stage Y
        assert _b128_conflict_cycles(addr16x(rh, 107008, 0)) == 0


def test_down1_epilogue_reads_conflict_free():
    """down1's row-pair epilogue (unet_kernels.hip GEN64: 64 output columns, 8 lanes a row pair, L = 24):
    thread t reads row pair rp = t / 8 + 32 i (6 passes) at columns 8 (t % 8) .. + 7, i.e. four 16-B pieces
    of its C-tile line and two 16-B pieces of each of the time / label map rows l, l + 1 (l = 2 rp mod 24).
    With 136-float lines and unswizzled 64-float map rows this costs 1,152 extra LDS cycles per workgroup:
    294,912 per launch over 256 workgroups, the epilogue's share of the PMC count (profiles/r05/r5i:
    442,624 -> 147,712).  The round-5 layout (132-float lines, map piece c of row l in slot c ^ ((l >> 1) & 1))
    is conflict-free."""
    def extra(ct_ld, swz):
        total = 0
        for w in range(4):
            for it in range(6):
                rp = [(64 * w + l) // 8 + 32 * it for l in range(64)]
                c = [(64 * w + l) % 8 for l in range(64)]
                for k in range(4):
                    total += _b128_conflict_cycles([4 * (rp[l] * ct_ld + 16 * c[l] + 4 * k) for l in range(64)])
                for e in range(2):
                    for half in range(2):
                        addr = []
                        for l in range(64):
                            le = (2 * rp[l]) % 24 + e
                            g = (le >> 1) & 1 if swz else 0
                            addr.append(4 * (le * 64 + 4 * ((2 * c[l] + half) ^ g)))
                        total += 2 * _b128_conflict_cycles(addr)        # the time and the label map
        return total
    assert extra(136, False) == 1152
    assert extra(132, True) == 0
