"""configs[3]'s product path on the GPU: distributed.sample_posterior_sharded over one rank's full shard
(BASELINE configs[3]: 256 test TACs x 8192 posterior samples over 8 GPUs = 32 TACs x 8192 per GPU,
TAC-major; the reference's caller is main_script.py:414-436, one TAC per ddpm_loop).  The shard is
262,144 samples, run by ddpm_loop as 4 launches of 65,536 with a per-sample condition index.

Pins:
* each TAC's samples equal a separate single-TAC run of the same global sample indices, bitwise (the
  counter-based noise makes the result independent of chunking, sharding and condition batching);
* the per-TAC posterior statistics (GPU fp64 Welford) equal the NumPy moments of the samples (1e-12);
* two TACs at small B, exact-f32 network, against the fp64 oracle loop fed the oracle's Philox draws.
"""
import numpy as np
import pytest
import torch

from oracle import iddpm_ref as R
from pet_posterior_distribution_amd.distributed import TacTable, local_stats_numpy, sample_posterior_sharded
from tests.helpers import shipped_net_args, shipped_diff_args, synthetic_condition, quick_trained_weights

pytestmark = pytest.mark.gpu


def _model(dtype, weights=None):
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    net = UnetConditional(**shipped_net_args(), seed=1234)
    net.build((None, 48, 2))
    if weights is not None:
        net.weights = weights
    return ImprovedDDPM(network=net, dtype=dtype, **shipped_diff_args())


def test_config4_rank_shard_full(capsys):
    """32 TACs x 8192 samples x 1000 steps (bf16, about a minute on one MI355X)."""
    n_tac, n_per, seed, xs = 32, 8192, 2024, 7
    m = _model('bfloat16')
    table = TacTable(n_tac, lambda k: synthetic_condition(1000 + k))
    summ, st, (lo, hi, x0) = sample_posterior_sharded(m, table, n_per, seed=seed, x_T_seed=xs, return_samples=True)
    assert (lo, hi) == (0, n_tac * n_per) and x0.shape == (n_tac * n_per, 48, 2)
    x = x0.cpu().numpy()
    assert np.isfinite(x).all()
    tac = np.repeat(np.arange(n_tac), n_per)
    ref = local_stats_numpy(x, tac, n_tac)
    np.testing.assert_array_equal(st[..., 0], ref[..., 0])
    np.testing.assert_allclose(st[..., 1], ref[..., 1], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(st[..., 2], ref[..., 2], rtol=1e-12)
    np.testing.assert_allclose(summ["std_DVR"], x[..., 0].astype(np.float64).reshape(n_tac, n_per, 48).std(1),
                               rtol=1e-11)
    for k in (0, 5, 11, 16, 21, 26, 31):
        g0 = k * n_per
        xT = m.philox_normal(n_per, seed=xs, sample_offset=g0)
        one = m.ddpm_loop(xT, table.rows([k]), seed=seed, sample_offset=g0).cpu().numpy()
        np.testing.assert_array_equal(one, x[g0:g0 + n_per], err_msg=f'TAC {k}')
    m.close()


def test_two_tacs_small_vs_oracle():
    """2 TACs x 3 samples (ragged), 25 linear sub-sequence steps, exact f32, against the fp64 oracle."""
    W, _ = quick_trained_weights()
    m = _model('float32', W)
    conds = np.stack([synthetic_condition(3), synthetic_condition(4)])
    n_per, n, seed, xs = 3, 25, 555, 9
    summ, st, (lo, hi, x0) = sample_posterior_sharded(m, conds, n_per, seed=seed, x_T_seed=xs, num_timesteps=n,
                                                      return_samples=True)
    got = x0.cpu().numpy()
    S = R.schedule_tables(R.get_beta_schedule('cosine', 1000))
    idx = R.loop_indices(1000, n)
    g = np.arange(2 * n_per)
    xT = R.philox_normal_pairs(xs, g, 0x7fffffff).astype(np.float32)
    z = np.stack([R.philox_normal_pairs(seed, g, i) for i in range(n)]).astype(np.float32)
    ref = R.ddpm_loop(W, S, xT, conds[np.repeat(np.arange(2), n_per)], z, idx, dt=np.float64)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-4 * np.abs(ref).max())
    rs = local_stats_numpy(ref, np.repeat(np.arange(2), n_per), 2)
    np.testing.assert_allclose(st[..., 1], rs[..., 1], rtol=1e-4, atol=1e-4 * np.abs(ref).max())
    m.close()


def test_level_outputs_invalid_after_generate():
    """generate() overwrites the level buffers, so level_outputs() fails until the next
    forward / p_sample instead of returning stale rows."""
    m = _model('bfloat16')
    c = synthetic_condition(0)
    x = np.zeros((8, 48, 2), np.float32)
    m.call({'x': x, 'time': np.full(8, 10, np.int32), 'condition': c[None]})
    assert m.level_outputs()['down1'].shape == (8, 24, 256)
    m.ddpm_loop(x, c[None], num_timesteps=3, seed=1)
    with pytest.raises(Exception, match='B exceeds'):
        m.level_outputs(B=8)
    m.close()


def test_rccl_stats_gather_world1():
    """The configs[3] collective over RCCL on the box's GPU: a one-rank 'nccl' group (the only RCCL group a
    1-GPU box can form; RCCL refuses two ranks on one device), device-side fp64 all-gather of a rank's
    per-TAC Welford partials through gather_merge_own_tacs, then the host merge.  World 1 makes the result
    the rank's own partials, so it must come back bitwise; the N > 1 merge itself is the gloo test's
    (tests/test_cpu_sharded.py)."""
    import os
    import socket
    import torch.distributed as dist
    from pet_posterior_distribution_amd.distributed import gather_merge_own_tacs
    assert not dist.is_initialized()
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    os.environ.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1,
                            device_id=torch.device('cuda', 0))
    try:
        assert dist.get_backend() == 'nccl'
        rng = np.random.default_rng(5)
        n_tac, n_per = 6, 10
        local = np.zeros((n_tac, 48, 2, 3))
        local[..., 0] = n_per
        local[..., 1] = rng.standard_normal((n_tac, 48, 2))
        local[..., 2] = rng.uniform(0.5, 2.0, (n_tac, 48, 2))
        got = gather_merge_own_tacs(local, n_tac, n_per, device=torch.device('cuda', 0))
        np.testing.assert_array_equal(got, local)
        dist.barrier()
    finally:
        dist.destroy_process_group()
