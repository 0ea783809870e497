"""GPU parity tests: libpetdiff (HIP, gfx950) vs the CPU oracle (oracle/iddpm_ref.py).

Tolerances (written per test):
* exact-f32 MFMA network: max|gpu - oracle_fp64| <= 1e-4 * max|oracle| (north_star: 1e-4 rtol);
* 16-bit networks: plain Glorot weights (no identity shortcut) and each output half (eps, v) against
  its own magnitude, with test_gpu_parity16.py's bounds (rrms / max relative to the half's rms):
  bf16 1.2e-2 / 0.1, fp16 1.5e-3 / 1.2e-2; 16-bit loops against f32 within one Monte-Carlo standard
  error (test_gpu_parity16.py); the 16-bit forward / loop tests that bounded the output by a fraction
  of its global max with identity-shortcut weights were retired in round 3;
* p_sample / loop with identical injected noise: posterior mean / SD within 1e-4 rtol.
"""
import numpy as np
import pytest
import torch

from oracle import iddpm_ref as R
from tests.helpers import shipped_net_args, shipped_diff_args, synthetic_condition

pytestmark = pytest.mark.gpu

S = R.schedule_tables(R.get_beta_schedule('cosine', 1000))


def make_model(dtype='float32', seed=11, bias_scale=0.05, learn_variance='learn_ranged', parameterization='eps',
               final_scale=1.0):
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional, denoiser_init
    args = shipped_net_args()
    args['learn_variance'] = learn_variance
    net = UnetConditional(**args)
    net.build((None, 48, 2))
    net.weights = denoiser_init(net.spec(), seed=seed, bias_scale=bias_scale, perturb=0.1 * final_scale)
    return ImprovedDDPM(network=net, dtype=dtype, parameterization=parameterization, **shipped_diff_args())


def rel(a, b):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    return float(np.abs(a.astype(np.float64) - b).max() / (np.abs(b).max() + 1e-30))


# 16-bit bounds of test_gpu_parity16.py: (rrms, max error / rms), each output half on its own magnitude
TOL16 = {'bfloat16': (1.2e-2, 0.1), 'float16': (1.5e-3, 1.2e-2)}


def half_errors(a, b):
    """{'eps': (rrms, max/rms), 'v': ...} of network outputs a vs b (B, 48, n_out); n_out = 2: eps only."""
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    a, b = a.astype(np.float64), np.asarray(b, np.float64)
    out = {}
    for k, sl in (('eps', slice(0, 2)), ('v', slice(2, 4))):
        if b.shape[-1] <= sl.start:
            continue
        d, r = a[..., sl] - b[..., sl], b[..., sl]
        rms = np.sqrt((r ** 2).mean()) + 1e-300
        out[k] = (float(np.sqrt((d ** 2).mean()) / rms), float(np.abs(d).max() / rms))
    return out


def within16(a, b, dtype):
    tr, tm = TOL16[dtype]
    e = half_errors(a, b)
    return all(x <= tr and y <= tm for x, y in e.values()), e


def glorot_model(dtype, seed=17, learn_variance='learn_ranged', parameterization='eps'):
    """Plain Glorot-uniform weights (biases U(-0.05, 0.05)), no identity shortcut."""
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    from pet_posterior_distribution_amd.networks import glorot_uniform_init
    args = shipped_net_args()
    args['learn_variance'] = learn_variance
    net = UnetConditional(**args)
    net.build((None, 48, 2))
    net.weights = glorot_uniform_init(net.spec(), seed=seed, bias_scale=0.05)
    return ImprovedDDPM(network=net, dtype=dtype, parameterization=parameterization, **shipped_diff_args())


@pytest.fixture(scope='module')
def conds():
    return np.stack([synthetic_condition(0), synthetic_condition(1)])


@pytest.fixture(scope='module')
def trained():
    from tests.helpers import quick_trained_weights
    return quick_trained_weights()


@pytest.fixture(scope='module')
def m32():
    return make_model('float32')


@pytest.fixture(scope='module')
def m16():
    return make_model('bfloat16')


def test_unet_forward_f32(m32, conds):
    rng = np.random.default_rng(1)
    B = 8
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    t = np.array([999, 998, 500, 250, 17, 2, 1, 0], dtype=np.int32)
    cond = conds[np.array([0, 1, 1, 0, 0, 1, 0, 1])]
    out = m32.call({'x': x, 'time': t, 'condition': cond})
    ref = R.unet_forward(m32.network.weights, x, t, cond, dt=np.float64)
    assert out.shape == (B, 48, 4)
    assert rel(out, ref) < 1e-4


@pytest.mark.parametrize('B', [1, 5, 37])
def test_ragged_batches_f32(m32, conds, B):
    """Batches that do not fill a 192-row tile (4 samples at L=48, 32 at L=6)."""
    rng = np.random.default_rng(B)
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    t = rng.integers(0, 1000, B).astype(np.int32)
    cond = np.repeat(conds[:1], B, 0)
    out = m32.call({'x': x, 'time': t, 'condition': cond})
    ref = R.unet_forward(m32.network.weights, x, t, cond, dt=np.float64)
    assert rel(out, ref) < 1e-4


def test_p_sample_injected_noise(m32, conds):
    rng = np.random.default_rng(3)
    B = 6
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    t = np.array([999, 600, 100, 2, 1, 0], dtype=np.int32)
    z = rng.standard_normal((B, 48, 2)).astype(np.float32)
    cond = np.repeat(conds[1:], B, 0)
    mean, var, var_t = m32.ddpm(x, t, cond, z=z)
    rm, rv, rvt = R.ddpm(m32.network.weights, S, x, t, cond, z, dt=np.float64)
    assert rel(mean, rm) < 1e-4
    assert rel(var, rv) < 1e-4
    assert rel(var_t, rvt) < 1e-4
    assert float(var[-1].abs().max()) == 0.0          # t == 0: no noise (diffusion_model.py:658)


@pytest.mark.parametrize('lv,param', [('', 'eps'), ('learn', 'eps'), ('learn_ranged', 'v'),
                                      ('learn_ranged', 'x0'), ('learn_ranged', 'x_prev')])
def test_p_sample_variants(conds, lv, param):
    m = make_model('float32', seed=5, learn_variance=lv, parameterization=param, final_scale=0.2)
    rng = np.random.default_rng(4)
    B = 4
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    t = np.array([999, 400, 3, 0], dtype=np.int32)
    z = rng.standard_normal((B, 48, 2)).astype(np.float32)
    cond = np.repeat(conds[:1], B, 0)
    mean, var, var_t = m.ddpm(x, t, cond, z=z)
    rm, rv, rvt = R.ddpm(m.network.weights, S, x, t, cond, z, learn_variance=lv, parameterization=param,
                         dt=np.float64)
    assert rel(mean, rm) < 1e-4
    assert rel(var, rv) < 1e-4
    assert rel(var_t, rvt) < 1e-4
    m.close()


@pytest.mark.parametrize('flag', [True, False])
def test_loop_fixed_variance_flag_var_tilde(conds, flag):
    """Fixed variance (learn_variance=''), where var (log beta) and var_tilde (clipped posterior log var)
    differ: the loop adds var_tilde or var per flag_var_tilde (diffusion_model.py:705-708), graph and
    eager, vs the oracle with the same injected noise."""
    m = make_model('float32', seed=21, learn_variance='', final_scale=0.2)
    rng = np.random.default_rng(22)
    B = 5
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    idx = R.loop_indices(1000, 12, 'quadratic')        # dense near t = 0, where var and var_tilde differ most
    z = rng.standard_normal((len(idx), B, 48, 2)).astype(np.float32)
    out = m.ddpm_loop(x, conds[1:], num_timesteps=12, sub_sequence_type='quadratic', flag_var_tilde=flag, z=z)
    ref = R.ddpm_loop(m.network.weights, S, x, conds[1:], z, idx, flag_var_tilde=flag, learn_variance='',
                      dt=np.float64)
    assert rel(out, ref) < 1e-4
    other = R.ddpm_loop(m.network.weights, S, x, conds[1:], z, idx, flag_var_tilde=not flag, learn_variance='',
                        dt=np.float64)
    assert rel(other, ref) > 5e-4                      # the flag matters in this mode (1.2e-3 here)
    a = m.ddpm_loop(x, conds[1:], num_timesteps=12, flag_var_tilde=flag, seed=4)
    b = m.ddpm_loop(x, conds[1:], num_timesteps=12, flag_var_tilde=flag, seed=4, use_graph=False)
    torch.testing.assert_close(a, b, rtol=0, atol=0)
    m.close()


def test_philox_noise_matches_oracle(m32, conds):
    rng = np.random.default_rng(5)
    B = 4
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    t = np.full(B, 700, dtype=np.int32)
    cond = np.repeat(conds[:1], B, 0)
    seed, off, step = 987654321123, 1000, 17
    mean, var, _ = m32.ddpm(x, t, cond, seed=seed, sample_offset=off, rng_step=step)
    z = R.philox_normal_pairs(seed, off + np.arange(B), step)
    rm, rv, _ = R.ddpm(m32.network.weights, S, x, t, cond, z, dt=np.float64)
    assert rel(var, rv) < 1e-4


@pytest.mark.parametrize('sub', ['linear', 'quadratic'])
def test_loop_injected_noise_f32(m32, conds, sub):
    rng = np.random.default_rng(6)
    B = 8
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    idx = R.loop_indices(1000, 20, sub)
    z = rng.standard_normal((len(idx), B, 48, 2)).astype(np.float32)
    out = m32.ddpm_loop(x, conds[:1], num_timesteps=20, sub_sequence_type=sub, z=z)
    ref = R.ddpm_loop(m32.network.weights, S, x, conds[:1], z, idx, dt=np.float64)
    assert rel(out, ref) < 1e-4
    o = out.cpu().numpy().astype(np.float64)
    for f in (np.mean, np.std):
        assert rel(f(o, axis=0), f(ref, axis=0)) < 1e-4


def test_loop_full_1000_steps_f32(trained):
    """Full T=1000 reverse process (the metric's path) at small B vs the fp64 oracle, 1e-4, with the
    briefly trained eps-predictor (tests.helpers.quick_trained_weights: no identity shortcut, so the
    bound covers the whole U-Net's contribution, as test_loop_full_1000_steps_bf16x3)."""
    from tests.test_gpu_parity16 import make
    W, cond = trained
    m = make(W, 'float32')
    rng = np.random.default_rng(7)
    B = 2
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    idx = R.loop_indices(1000)
    z = rng.standard_normal((len(idx), B, 48, 2)).astype(np.float32)
    out = m.ddpm_loop(x, cond[None], z=z)
    ref = R.ddpm_loop(W, S, x, cond[None], z, idx, dt=np.float64)
    assert rel(out, ref) < 1e-4
    m.close()


def test_config1_posterior_mean_sd_f32(m32, conds):
    """BASELINE configs[0] exactly: one TAC, 48 ROI, n_posterior = 32, 100-step linear sub-sequence
    (main_script.py:419-436).  Same x_T and injected noise as the fp64 oracle; the per-ROI posterior
    mean and population SD (ddof = 0, main_script.py:433-436), computed on the GPU by
    posterior_stats, match the oracle's NumPy moments within the north star's 1e-4 rtol."""
    rng = np.random.default_rng(31)
    B = 32
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    idx = R.loop_indices(1000, 100, 'linear')
    z = rng.standard_normal((len(idx), B, 48, 2)).astype(np.float32)
    out = m32.ddpm_loop(x, conds[:1], num_timesteps=100, sub_sequence_type='linear', z=z)
    ref = R.ddpm_loop(m32.network.weights, S, x, conds[:1], z, idx, dt=np.float64)
    assert rel(out, ref) < 1e-4
    st = m32.posterior_stats(out)[0]                     # (48, 2, [count, mean, M2])
    mean_ref, sd_ref = ref.mean(0), ref.std(0)
    assert rel(st[..., 1], mean_ref) < 1e-4
    assert rel(np.sqrt(st[..., 2] / B), sd_ref) < 1e-4
    np.testing.assert_allclose(np.sqrt(st[..., 2] / B), sd_ref, rtol=1e-4, atol=1e-4 * sd_ref.max())


def test_keep_all_xt(m32, conds):
    rng = np.random.default_rng(8)
    x = rng.standard_normal((3, 48, 2)).astype(np.float32)
    allx = m32.ddpm_loop(x, conds[:1], num_timesteps=5, keep_all_xt=True, seed=3)
    last = m32.ddpm_loop(x, conds[:1], num_timesteps=5, seed=3)
    assert allx.shape == (5, 3, 48, 2)
    np.testing.assert_array_equal(allx[-1], last.cpu().numpy())


def test_graph_equals_eager_and_shard_invariance(m16, conds):
    """hipGraph replay == eager launch, and splitting a batch (sample_offset) is bitwise neutral."""
    rng = np.random.default_rng(9)
    B = 64
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    a = m16.ddpm_loop(x, conds[:1], num_timesteps=50, seed=42, use_graph=True)
    b = m16.ddpm_loop(x, conds[:1], num_timesteps=50, seed=42, use_graph=False)
    c1 = m16.ddpm_loop(x[:24], conds[:1], num_timesteps=50, seed=42, sample_offset=0)
    c2 = m16.ddpm_loop(x[24:], conds[:1], num_timesteps=50, seed=42, sample_offset=24)
    torch.testing.assert_close(a, b, rtol=0, atol=0)
    torch.testing.assert_close(a, torch.cat([c1, c2]), rtol=0, atol=0)


def test_chunked_generate_bitwise(m16, conds, monkeypatch):
    """Batches above PETDIFF_MAX_BATCH run as chunks with advancing sample offsets: bitwise equal to
    one launch (chunk size lowered here so the test stays small), for keep_all_xt and per-sample tac."""
    from pet_posterior_distribution_amd import _lib
    rng = np.random.default_rng(19)
    B = 100
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    tac = (np.arange(B) % 2).astype(np.int32)
    a = m16.ddpm_loop(x, conds, num_timesteps=20, seed=7, tac=tac)
    ka = m16.ddpm_loop(x, conds[:1], num_timesteps=5, seed=8, keep_all_xt=True)
    monkeypatch.setattr(_lib, 'MAX_BATCH', 40)
    b = m16.ddpm_loop(x, conds, num_timesteps=20, seed=7, tac=tac)
    kb = m16.ddpm_loop(x, conds[:1], num_timesteps=5, seed=8, keep_all_xt=True)
    torch.testing.assert_close(a, b, rtol=0, atol=0)
    np.testing.assert_array_equal(ka, kb)


def test_batch_above_max_rejected(m16, conds):
    """The C ABI refuses one launch above PETDIFF_MAX_BATCH (ValueError in the wrapper), before
    allocating or launching anything."""
    from pet_posterior_distribution_amd import _lib
    x = torch.zeros((_lib.MAX_BATCH + 1, 48, 2), device='cuda')
    with pytest.raises(ValueError, match='PETDIFF_MAX_BATCH'):
        m16.ddpm(x, np.zeros(_lib.MAX_BATCH + 1, np.int32), conds[:1])


def test_posterior_stats(m32):
    rng = np.random.default_rng(11)
    B = 1000
    x0 = rng.standard_normal((B, 48, 2)).astype(np.float32) * 3 + 1
    tac = (np.arange(B) % 3).astype(np.int32)
    st = m32.posterior_stats(x0, tac, n_tac=3)
    for k in range(3):
        xs = x0[tac == k].astype(np.float64)
        np.testing.assert_allclose(st[k, :, :, 0], xs.shape[0])
        np.testing.assert_allclose(st[k, :, :, 1], xs.mean(0), rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(np.sqrt(st[k, :, :, 2] / xs.shape[0]), xs.std(0), rtol=1e-10)


def test_full_size_config_properties(m16, conds):
    """BASELINE config 2 at full size (B=1024, 1000 steps, bf16): finite, deterministic, chunk-invariant."""
    rng = np.random.default_rng(12)
    B = 1024
    x = torch.as_tensor(rng.standard_normal((B, 48, 2)).astype(np.float32), device='cuda')
    a = m16.ddpm_loop(x, conds[:1], seed=77)
    b = m16.ddpm_loop(x, conds[:1], seed=77)
    assert torch.isfinite(a).all()
    torch.testing.assert_close(a, b, rtol=0, atol=0)
    half = m16.ddpm_loop(x[512:], conds[:1], seed=77, sample_offset=512)
    torch.testing.assert_close(a[512:], half, rtol=0, atol=0)


def test_loop_mixed_conditions_per_sample_f32(m32, conds):
    """Per-sample conditions interleaved inside a workgroup's samples: the epilogues'
    general path (condition maps read per row) against the oracle, injected noise."""
    rng = np.random.default_rng(21)
    B = 40
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    table = np.stack([conds[0], conds[1], conds[0] * 0.9 + 0.05])
    tac = rng.integers(0, 3, B).astype(np.int32)
    idx = R.loop_indices(1000, 12)
    z = rng.standard_normal((len(idx), B, 48, 2)).astype(np.float32)
    out = m32.ddpm_loop(x, table, num_timesteps=12, z=z, tac=tac)
    ref = R.ddpm_loop(m32.network.weights, S, x, table[tac], z, idx, dt=np.float64)
    assert rel(out, ref) < 1e-4


def test_loop_tac_major_graph_bf16(m16, conds):
    """TAC-major multi-condition batch (config 4 layout) through the captured graph:
    identical to running each TAC's samples separately with the same global indices."""
    rng = np.random.default_rng(22)
    B = 512
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    tac = np.repeat(np.arange(2, dtype=np.int32), B // 2)
    both = m16.ddpm_loop(x, conds, num_timesteps=30, seed=9, tac=tac)
    a = m16.ddpm_loop(x[:B // 2], conds[:1], num_timesteps=30, seed=9, sample_offset=0)
    b = m16.ddpm_loop(x[B // 2:], conds[1:], num_timesteps=30, seed=9, sample_offset=B // 2)
    torch.testing.assert_close(both, torch.cat([a, b]), rtol=0, atol=0)


@pytest.mark.parametrize('dtype', ['bfloat16', 'float32', 'bf16x3'])
def test_fused_next_step_down0_bitwise(conds, dtype, monkeypatch):
    """The loop runs step i+1's first layer (down0) inside step i's final-conv epilogue;
    PETDIFF_FUSE_DOWN0=0 keeps the standalone down0 launch.  Same arithmetic either way:
    bit-identical samples, for a ragged batch with conditions interleaved per sample
    (the epilogue's per-row map path) and for a single condition (the LDS map path)."""
    rng = np.random.default_rng(23)
    B = 37
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    table = np.stack([conds[0], conds[1], conds[0] * 0.9 + 0.05])
    tac = rng.integers(0, 3, B).astype(np.int32)
    monkeypatch.setenv('PETDIFF_FUSE_DOWN0', '0')
    plain = make_model(dtype)
    plain._ensure_handle()                    # the switch is read when the handle is created
    monkeypatch.setenv('PETDIFF_FUSE_DOWN0', '1')
    fused = make_model(dtype)
    fused._ensure_handle()
    for kw in ({'tac': tac}, {}):
        cset = table if kw else conds[:1]
        for g in (True, False):
            a = plain.ddpm_loop(x, cset, num_timesteps=25, seed=4, use_graph=g, **kw)
            b = fused.ddpm_loop(x, cset, num_timesteps=25, seed=4, use_graph=g, **kw)
            torch.testing.assert_close(a, b, rtol=0, atol=0)
    plain.close()
    fused.close()


@pytest.mark.parametrize('fuse_down0', ['1', '0'])
def test_graph_segments_bitwise(conds, fuse_down0, monkeypatch):
    """PETDIFF_GRAPH_SEG=7 captures the 30-step loop as 5 graph segments (the last one ragged: 2 steps)
    launched back to back; the fused next-step down0 crosses every segment boundary (step i's epilogue
    writes step i + 1's s0 / p0).  Bit-identical to the single-graph loop and to eager launches, for one
    condition and for conditions interleaved per sample, with the fused down0 on and off."""
    rng = np.random.default_rng(24)
    B = 200
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    table = np.stack([conds[0], conds[1]])
    tac = rng.integers(0, 2, B).astype(np.int32)
    monkeypatch.setenv('PETDIFF_FUSE_DOWN0', fuse_down0)
    monkeypatch.setenv('PETDIFF_GRAPH_SEG', '0')
    one = make_model('bfloat16')
    one._ensure_handle()                       # the switches are read when the handle is created
    monkeypatch.setenv('PETDIFF_GRAPH_SEG', '7')
    seg = make_model('bfloat16')
    seg._ensure_handle()
    for kw in ({'tac': tac}, {}):
        cset = table if kw else conds[:1]
        a = one.ddpm_loop(x, cset, num_timesteps=30, seed=8, sample_offset=5, **kw)
        b = seg.ddpm_loop(x, cset, num_timesteps=30, seed=8, sample_offset=5, **kw)
        c = seg.ddpm_loop(x, cset, num_timesteps=30, seed=8, sample_offset=5, use_graph=False, **kw)
        torch.testing.assert_close(a, b, rtol=0, atol=0)
        torch.testing.assert_close(a, c, rtol=0, atol=0)
    one.close()
    seg.close()


@pytest.mark.parametrize('dtype', ['bfloat16', 'float16'])
def test_fused_up_levels_forward(conds, dtype, monkeypatch):
    """Fused up levels (k2 conv composed into the block conv, 2-phase 4-tap GEMM on the coarse
    input + left-edge correction, u-path maps through the block) against the fp64 oracle and against
    the separate-launch path (PETDIFF_FUSE_UP=0), Glorot weights, each output half on its own
    magnitude (TOL16): ragged batches, conditions interleaved per sample (the epilogue's per-row map
    path), per-sample t."""
    monkeypatch.setenv('PETDIFF_FUSE_UP', '0')
    plain = glorot_model(dtype, seed=13)
    plain._ensure_handle()
    monkeypatch.setenv('PETDIFF_FUSE_UP', '1')
    fused = glorot_model(dtype, seed=13)
    fused._ensure_handle()
    table = np.stack([conds[0], conds[1], conds[0] * 0.9 + 0.05])
    for B in (1, 5, 37, 96):
        rng = np.random.default_rng(100 + B)
        x = rng.standard_normal((B, 48, 2)).astype(np.float32)
        t = rng.integers(0, 1000, B).astype(np.int32)
        cond = table[rng.integers(0, 3, B)]
        ref = R.unet_forward(fused.network.weights, x, t, cond, dt=np.float64)
        a = fused.call({'x': x, 'time': t, 'condition': cond})
        b = plain.call({'x': x, 'time': t, 'condition': cond})
        for got in (a, b):
            ok, e = within16(got, ref, dtype)
            assert ok, (B, e)
        ok, e = within16(a, b.cpu().numpy(), dtype)
        assert ok, (B, 'fused vs unfused', e)
    plain.close()
    fused.close()


def test_fused_up_loop_vs_unfused(monkeypatch):
    """bf16 loop (graph, fused next-step down0 / down1, one condition -> the LDS map path) with and
    without the fused up levels, on the briefly trained network (tests.helpers.quick_trained_weights:
    an eps-predictor whose chain stays bounded with no identity shortcut): both deterministic; per-ROI
    posterior mean and SD within one Monte-Carlo standard error of each other (the two differ by bf16
    rounding only: u is not rounded in the fused path, the composite weights are rounded once)."""
    from tests.helpers import quick_trained_weights
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    W, cond = quick_trained_weights()

    def mk():
        net = UnetConditional(**shipped_net_args())
        net.build((None, 48, 2))
        net.weights = W
        m = ImprovedDDPM(network=net, dtype='bfloat16', **shipped_diff_args())
        m._ensure_handle()
        return m
    monkeypatch.setenv('PETDIFF_FUSE_UP', '0')
    plain = mk()
    monkeypatch.setenv('PETDIFF_FUSE_UP', '1')
    fused = mk()
    B = 512
    x = fused.philox_normal(B, seed=25)
    a = fused.ddpm_loop(x, cond[None], num_timesteps=100, seed=6).cpu().numpy()
    a2 = fused.ddpm_loop(x, cond[None], num_timesteps=100, seed=6).cpu().numpy()
    b = plain.ddpm_loop(x, cond[None], num_timesteps=100, seed=6).cpu().numpy()
    np.testing.assert_array_equal(a, a2)
    assert np.isfinite(a).all()
    sd = b.std(0)
    assert (sd > 0).all()
    assert (np.abs(a.mean(0) - b.mean(0)) <= sd * np.sqrt(2.0 / B)).all()
    assert (np.abs(a.std(0) / sd - 1) <= np.sqrt(1.0 / B)).all()
    plain.close()
    fused.close()


@pytest.mark.parametrize('lv,param', [('learn_ranged', 'eps'), ('', 'eps'), ('learn_ranged', 'v')])
def test_p_sample_bf16_fused_levels(conds, lv, param):
    """p_sample through the 16-bit network (fused up levels; the final conv + p_sample epilogue
    writing mean / var / var_tilde), Glorot weights.  The bf16 network output is checked against the
    fp64 oracle network (each half on its own magnitude, TOL16), and the fp32 p_sample epilogue against the oracle's p_mean_variance applied
    to that same network output (1e-4); t = 0 exactly noise-free; per-sample conditions and t."""
    m = glorot_model('bfloat16', seed=6, learn_variance=lv, parameterization=param)
    rng = np.random.default_rng(26)
    B = 9
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    t = np.array([999, 800, 600, 400, 100, 10, 2, 1, 0], dtype=np.int32)
    z = rng.standard_normal((B, 48, 2)).astype(np.float32)
    table = np.stack([conds[0], conds[1]])
    cond = table[rng.integers(0, 2, B)]
    net = m.call({'x': x, 'time': t, 'condition': cond}).cpu().numpy().astype(np.float64)
    ok, e = within16(net, R.unet_forward(m.network.weights, x, t, cond, dt=np.float64), 'bfloat16')
    assert ok, e
    mean, var, var_t = m.ddpm(x, t, cond, z=z)
    out = R.p_mean_variance(S, net, x.astype(np.float64), t, lv, param, dt=np.float64)
    mask = np.where(t == 0, 0., 1.).reshape(-1, 1, 1)
    assert rel(mean, out['mean']) < 1e-4
    assert rel(var, mask * np.exp(0.5 * out['log_variance']) * z) < 1e-4
    assert rel(var_t, mask * np.exp(0.5 * out['log_variance_tilde']) * z) < 1e-4
    assert float(var[-1].abs().max()) == 0.0
    m.close()


@pytest.mark.parametrize('dtype', ['bfloat16', 'bf16x3'])
def test_kernel_timing_reps_bitwise(conds, dtype):
    """bench.py's per-layer timing (set_kernel_timing(reps=8): every timed launch repeated back to back
    between its HIP events, petdiff_api.cpp launch) relies on every layer kernel being idempotent: an eager
    loop and a p_sample timed that way are bitwise equal to the untimed ones, and each layer's launch
    count is reps x the untimed count."""
    rng = np.random.default_rng(31)
    B = 150
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    t = rng.integers(0, 1000, B)
    m = make_model(dtype)
    m.set_kernel_timing(True, reps=1)
    a = m.ddpm_loop(x, conds[:1], num_timesteps=12, seed=4, use_graph=False)
    pa = m.ddpm(x, t, conds[:1], seed=6, rng_step=3)
    torch.cuda.synchronize()
    c1 = m.get_kernel_timing()
    m.set_kernel_timing(True, reps=8)
    b = m.ddpm_loop(x, conds[:1], num_timesteps=12, seed=4, use_graph=False)
    pb = m.ddpm(x, t, conds[:1], seed=6, rng_step=3)
    torch.cuda.synchronize()
    c8 = m.get_kernel_timing()
    m.set_kernel_timing(False)
    torch.testing.assert_close(a, b, rtol=0, atol=0)
    for u, v in zip(pa, pb):
        torch.testing.assert_close(u, v, rtol=0, atol=0)
    assert any(n for _, n in c1.values())
    for name in c1:
        assert c8[name][1] == 8 * c1[name][1], (name, c1[name], c8[name])
    m.close()


@pytest.mark.parametrize('dtype', ['bfloat16', 'float16', 'float32', 'bf16x3'])
def test_combined_maps_bitwise(conds, dtype, monkeypatch):
    """One condition: the epilogues read one combined time + label table (tmap[t] + cmap[0], formed once per
    schedule / condition change, petdiff_api.cpp combine_maps) instead of two.  The sum is the one every
    epilogue formed before adding its accumulators, so the outputs are bit-identical to the two-table path
    (PETDIFF_COMBINE_MAPS=0): forward with one t and with per-sample t (the epilogue's general path),
    p_sample, the graph and eager loops, and after the handle moves to two conditions and back."""
    rng = np.random.default_rng(31)
    B = 45
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    t_vec = rng.integers(0, 1000, B).astype(np.int32)
    monkeypatch.setenv('PETDIFF_COMBINE_MAPS', '0')
    two = make_model(dtype)
    two._ensure_handle()                       # the switch is read when the handle is created
    monkeypatch.setenv('PETDIFF_COMBINE_MAPS', '1')
    one = make_model(dtype)
    one._ensure_handle()

    def same(fa, fb):
        ra, rb = fa(two), fb(one)
        for u, v in zip(ra if isinstance(ra, tuple) else (ra,), rb if isinstance(rb, tuple) else (rb,)):
            torch.testing.assert_close(u, v, rtol=0, atol=0)
    c1 = conds[:1]
    for t in (np.full(B, 617, np.int32), t_vec):
        f = lambda m: m.call({'x': x, 'time': t, 'condition': c1})  # noqa: E731
        same(f, f)
    f = lambda m: m.ddpm(x, np.full(B, 311, np.int32), condition=c1, seed=3)  # noqa: E731
    same(f, f)
    for g in (True, False):
        f = lambda m: m.ddpm_loop(x, c1, num_timesteps=20, seed=6, use_graph=g)  # noqa: E731
        same(f, f)
    tac = rng.integers(0, 2, B).astype(np.int32)                # two conditions: both handles use two tables
    f = lambda m: m.ddpm_loop(x, conds[:2], num_timesteps=12, seed=2, tac=tac)  # noqa: E731
    same(f, f)
    f = lambda m: m.ddpm_loop(x, conds[1:2], num_timesteps=12, seed=2)  # noqa: E731  back to one condition
    same(f, f)
    two.close()
    one.close()
