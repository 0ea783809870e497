"""configs[3]'s product path on CPU: distributed.sample_posterior_sharded (the reference's
caller is main_script.py:414-436, one TAC at a time) with a stub sampler that has the sampler's contract --
the samples of global index g depend only on (seed, g, its TAC's condition) -- over world sizes 1 and 2
(gloo).  3 TACs x 5 samples over 2 ranks puts TAC 1 on both ranks, so its statistics are merged from
two partials (one rank's partials of the other TACs have count 0)."""
import multiprocessing as mp
import socket

import numpy as np
import torch

from pet_posterior_distribution_amd.distributed import (TacTable, local_stats_numpy, merge_stats,
                                                       sample_posterior_sharded, tac_major_shards)


class StubSampler:
    """Deterministic stand-in for ImprovedDDPM on the host: x_T(g) = N(0, 1) keyed by (seed, g);
    x_0(g) = x_T(g) * s + the TAC's condition features + a seed/g term."""
    device = torch.device('cpu')

    def philox_normal(self, B, seed=0, sample_offset=0):
        return torch.as_tensor(np.stack([np.random.default_rng([seed, sample_offset + b]).standard_normal((48, 2))
                                         for b in range(B)]))

    def ddpm_loop(self, x_T, cond, num_timesteps=None, seed=0, sample_offset=0, use_graph=True, tac=None):
        x = np.asarray(x_T, np.float64)
        cond = np.asarray(cond, np.float64)
        tac = np.zeros(len(x), np.int64) if tac is None else np.asarray(tac)
        feat = np.stack([cond[:, :48, 0], cond[:, :48, 1]], -1)              # (n_tac, 48, 2)
        g = sample_offset + np.arange(len(x))
        return torch.as_tensor(x * 0.3 + feat[tac] + 1e-3 * np.sin(seed + g)[:, None, None])

    def posterior_stats(self, x0, tac=None, n_tac=1):
        return local_stats_numpy(np.asarray(x0), tac, n_tac)


def _conds(k):
    return np.random.default_rng(100 + k).standard_normal((49, 54)).astype(np.float32) + k


N_TAC, N_PER = 3, 5


def _all_samples():
    s = StubSampler()
    x_T = s.philox_normal(N_TAC * N_PER, seed=1)
    cond = np.stack([_conds(k) for k in range(N_TAC)])
    return s.ddpm_loop(x_T, cond, seed=0, tac=np.repeat(np.arange(N_TAC), N_PER)).numpy()


def _worker(rank, world, port, q):
    import torch.distributed as dist
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=world)
    summ, st, (lo, hi, x0) = sample_posterior_sharded(StubSampler(), TacTable(N_TAC, _conds), N_PER,
                                                      return_samples=True)
    q.put((rank, lo, hi, st, None if x0 is None else np.asarray(x0)))
    dist.barrier()
    dist.destroy_process_group()


def test_tac_major_shards_split_a_tac():
    assert [tac_major_shards(N_TAC, N_PER, 2, r) for r in range(2)] == [(0, 8), (8, 15)]   # TAC 1 = g 5..9


def test_rank_tac_ranges_and_gather_payload():
    """Each rank gathers only its own TAC range: ranges cover every TAC, neighbours share
    at most the TAC their blocks split, and configs[3] (256 TACs x 8192 over 8 ranks) receives 8 x 32 TACs
    x 2,304 B per rank (<= 8 x 80 KB), not 8 x 256."""
    from pet_posterior_distribution_amd.distributed import rank_tac_range
    assert [rank_tac_range(N_TAC, N_PER, 2, r) for r in range(2)] == [(0, 2), (1, 3)]
    for n_tac, n_per, world in ((3, 5, 2), (7, 3, 4), (256, 8192, 8), (2, 1, 5), (1, 1024, 1)):
        rg = [rank_tac_range(n_tac, n_per, world, r) for r in range(world)]
        covered = set()
        for r, (t0, t1) in enumerate(rg):
            lo, hi = tac_major_shards(n_tac, n_per, world, r)
            assert set(range(t0, t1)) == set(g // n_per for g in range(lo, hi))
            covered |= set(range(t0, t1))
        assert covered == set(range(n_tac))
    rg = [rank_tac_range(256, 8192, 8, r) for r in range(8)]
    width = max(t1 - t0 for t0, t1 in rg)
    assert width == 32 and 8 * width * 48 * 2 * 3 * 8 <= 8 * 80 * 1024


def test_world1_matches_numpy():
    summ, st, (lo, hi, x0) = sample_posterior_sharded(StubSampler(), TacTable(N_TAC, _conds), N_PER,
                                                      return_samples=True)
    x = _all_samples()
    assert (lo, hi) == (0, N_TAC * N_PER)
    np.testing.assert_array_equal(np.asarray(x0), x)
    ref = local_stats_numpy(x, np.repeat(np.arange(N_TAC), N_PER), N_TAC)
    np.testing.assert_allclose(st, ref, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(summ['std_R1'], x[..., 1].reshape(N_TAC, N_PER, 48).std(1), rtol=1e-12)


def test_gloo_world2_tac_spanning_ranks_matches_world1():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict((r, rest) for r, *rest in (q.get(timeout=180) for _ in range(2)))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    _, st1 = sample_posterior_sharded(StubSampler(), TacTable(N_TAC, _conds), N_PER)
    x = _all_samples()
    for r in range(2):
        lo, hi, st, x0 = got[r]
        np.testing.assert_array_equal(x0, x[lo:hi])            # the shard's samples = the unsharded ones
        np.testing.assert_allclose(st, st1, rtol=1e-12, atol=1e-12)
    # the merge really combined two partials for TAC 1 (counts 3 + 2)
    p0 = local_stats_numpy(x[0:8], np.repeat(np.arange(N_TAC), N_PER)[0:8], N_TAC)
    p1 = local_stats_numpy(x[8:15], np.repeat(np.arange(N_TAC), N_PER)[8:15], N_TAC)
    assert p0[1, 0, 0, 0] == 3 and p1[1, 0, 0, 0] == 2 and p1[0, 0, 0, 0] == 0
    np.testing.assert_allclose(merge_stats([p0, p1]), st1, rtol=1e-12, atol=1e-12)
