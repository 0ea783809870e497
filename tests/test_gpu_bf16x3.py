"""The bf16x3 network (PETDIFF_DTYPE_BF16X3, dtype='bf16x3'): fp32-class accuracy on the benchmarked
bf16 MFMA kernels.  Every fp32 operand v is split into bf16 hi = bf16(v) and lo = bf16(v - hi);
activations are stored as [hi | lo] rows and each K chunk is walked three times, (a_hi, w_hi),
(a_hi, w_lo), (a_lo, w_hi), accumulating in fp32 (the dropped lo * lo term is about 2^-16 relative).

It is held to the SAME bounds as the exact-f32 mode, i.e. the north star's 1e-4 against the fp64
oracle (oracle/iddpm_ref.py), with the weights of tests/test_gpu_parity16.py (plain Glorot, no
identity shortcut; per level and per output half relative to its own magnitude) and the briefly
trained network for loops (tests.helpers.quick_trained_weights).
"""
import numpy as np
import pytest
import torch

from oracle import iddpm_ref as R
from tests.helpers import synthetic_condition
from tests.test_gpu_parity16 import S, TOL, rrms, relmax, make, glorot, level_case, trained  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('fuse_up', [True, False])
def test_per_level_parity_bf16x3(glorot, level_case, fuse_up, monkeypatch):
    """Every ConvBlock output (read back through petdiff_get_activation's hi + lo) and the eps / v
    halves of the final conv vs the fp64 oracle, within the exact-f32 mode's bounds
    (TOL['float32']: rrms 2e-5, max 2e-4 of the level's rms)."""
    x, t, c, lv, y = level_case
    m = make(glorot, 'bf16x3', fuse_up, monkeypatch)
    out = m.call({'x': x, 'time': t, 'condition': c}).cpu().numpy()
    got = {k: v.cpu().numpy() for k, v in m.level_outputs().items()}
    tr, tm = TOL['float32']
    err = {k: (rrms(g, lv[k]), relmax(g, lv[k])) for k, g in got.items()}
    for k, sl in (('eps', slice(0, 2)), ('v', slice(2, 4))):
        err[k] = (rrms(out[..., sl], y[..., sl]), relmax(out[..., sl], y[..., sl]))
    bad = {k: e for k, e in err.items() if e[0] > tr or e[1] > tm}
    assert not bad, (bad, err)
    m.close()


@pytest.mark.parametrize('B', [1, 5])
def test_ragged_batches_bf16x3(glorot, B):
    """Batches that fill no tile, 1e-4 of max|oracle| like test_ragged_batches_f32."""
    rng = np.random.default_rng(40 + B)
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    t = rng.integers(0, 1000, B).astype(np.int32)
    c = np.repeat(synthetic_condition(1)[None], B, 0)
    m = make(glorot, 'bf16x3')
    out = m.call({'x': x, 'time': t, 'condition': c}).cpu().numpy()
    ref = R.unet_forward(glorot, x, t, c, dt=np.float64)
    assert np.abs(out - ref).max() <= 1e-4 * np.abs(ref).max()
    m.close()


@pytest.fixture(scope='module')
def trained_x3(trained):
    m = make(trained[0], 'bf16x3')
    yield m
    m.close()


def test_p_sample_injected_noise_bf16x3(trained, trained_x3):
    W, cond = trained
    rng = np.random.default_rng(3)
    B = 6
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    t = np.array([999, 600, 100, 2, 1, 0], dtype=np.int32)
    z = rng.standard_normal((B, 48, 2)).astype(np.float32)
    cB = np.repeat(cond[None], B, 0)
    got = trained_x3.ddpm(x, t, cB, z=z)
    ref = R.ddpm(W, S, x, t, cB, z, dt=np.float64)
    for g, r in zip(got, ref):
        g = g.cpu().numpy()
        assert np.abs(g - r).max() <= 1e-4 * np.abs(r).max()


def test_graph_philox_loop_vs_oracle_bf16x3(trained, trained_x3):
    """The captured-graph loop with its own counter-based noise vs the fp64 oracle fed the same
    Philox draws, at the north star's 1e-4 (as test_graph_philox_loop_vs_oracle for exact f32)."""
    W, cond = trained
    B, n, seed, off = 4, 25, 987654321, 4096
    rng = np.random.default_rng(8)
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    out = trained_x3.ddpm_loop(x, cond[None], num_timesteps=n, seed=seed, sample_offset=off).cpu().numpy()
    idx = R.loop_indices(1000, n)
    z = np.stack([R.philox_normal_pairs(seed, off + np.arange(B), i) for i in range(n)])
    ref = R.ddpm_loop(W, S, x, cond[None], z, idx, dt=np.float64)
    assert rrms(out, ref) < 1e-4
    assert np.abs(out - ref).max() <= 1e-4 * np.abs(ref).max()


def test_loop_full_1000_steps_bf16x3(trained, trained_x3):
    """Full T = 1000 reverse process at small B with injected noise vs the fp64 oracle, 1e-4."""
    W, cond = trained
    rng = np.random.default_rng(7)
    B = 2
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    idx = R.loop_indices(1000)
    z = rng.standard_normal((len(idx), B, 48, 2)).astype(np.float32)
    out = trained_x3.ddpm_loop(x, cond[None], z=z).cpu().numpy()
    ref = R.ddpm_loop(W, S, x, cond[None], z, idx, dt=np.float64)
    assert np.abs(out - ref).max() <= 1e-4 * np.abs(ref).max()


def test_config2_full_size_bf16x3_vs_f32(trained, trained_x3):
    """configs[1] size (B = 1024, T = 1000, one TAC, the same x_T and counter-based noise): the
    bf16x3 samples against the exact-f32 path's, per-sample rrms <= 1e-4 (the bf16 path's bound
    in test_config2_full_size_16bit_vs_f32_posterior is 2e-3), and graph == eager bitwise."""
    W, cond = trained
    f32 = make(W, 'float32')
    B = 1024
    x = trained_x3.philox_normal(B, seed=41)
    a = f32.ddpm_loop(x, cond[None], seed=77)
    b = trained_x3.ddpm_loop(x, cond[None], seed=77)
    assert torch.isfinite(b).all()
    assert rrms(b.cpu().numpy(), a.cpu().numpy()) < 1e-4
    e = trained_x3.ddpm_loop(x[:64], cond[None], num_timesteps=40, seed=9, use_graph=False)
    g = trained_x3.ddpm_loop(x[:64], cond[None], num_timesteps=40, seed=9)
    torch.testing.assert_close(e, g, rtol=0, atol=0)
    f32.close()


def test_loop_mixed_conditions_per_sample_bf16x3(trained, trained_x3):
    """Conditions interleaved per sample (the epilogues' per-row map path) through the loop with
    injected noise vs the fp64 oracle, 1e-4 of max|oracle|."""
    W, cond = trained
    rng = np.random.default_rng(21)
    B = 40
    x = rng.standard_normal((B, 48, 2)).astype(np.float32)
    table = np.stack([cond, synthetic_condition(1), cond * 0.9 + 0.05])
    tac = rng.integers(0, 3, B).astype(np.int32)
    idx = R.loop_indices(1000, 12)
    z = rng.standard_normal((len(idx), B, 48, 2)).astype(np.float32)
    out = trained_x3.ddpm_loop(x, table, num_timesteps=12, z=z, tac=tac).cpu().numpy()
    ref = R.ddpm_loop(W, S, x, table[tac], z, idx, dt=np.float64)
    assert np.abs(out - ref).max() <= 1e-4 * np.abs(ref).max()
