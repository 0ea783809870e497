"""CPU tests of the training-step oracle (oracle/train_ref.py).

The analytic backward is pinned by central finite differences of the forward
objective J = B * mse + sum(vlb) (VLB prediction frozen, as tf.stop_gradient does),
along random directions of individual parameter tensors; the loss terms and the
optimizer against closed forms.
"""
import math
import zlib

import numpy as np
import pytest

from oracle import iddpm_ref as R
from oracle import train_ref as TR

S = R.schedule_tables(R.get_beta_schedule('cosine', 1000))


@pytest.fixture(scope='module')
def setup():
    from pet_posterior_distribution_amd.networks import glorot_uniform_init, param_spec
    P = glorot_uniform_init(param_spec(), seed=7, bias_scale=0.05)
    P = {k: v.astype(np.float64) for k, v in P.items()}
    rng = np.random.default_rng(3)
    B = 3
    x0 = rng.standard_normal((B, 48, 2)) * 1.2
    cond = np.abs(rng.standard_normal((B, 49, 54)))
    t = np.array([0, 1, 640])                  # t == 0 exercises the decoder NLL
    noise = rng.standard_normal((B, 48, 2))
    loss, mse, vlb, G = TR.train_loss_and_grads(P, S, x0, cond, t, noise)
    return P, x0, cond, t, noise, loss, mse, vlb, G


def test_loss_structure(setup):
    P, x0, cond, t, noise, loss, mse, vlb, G = setup
    assert loss.shape == (3,) and np.isfinite(loss).all()
    np.testing.assert_allclose(loss - vlb, mse)
    assert set(G) == set(P)
    for k in P:
        assert G[k].shape == P[k].shape, k


@pytest.mark.parametrize('name', ['time_mlp.kernel', 'cond_enc.hidden0.kernel', 'cond_enc.z.bias',
                                  'down0.conv.kernel', 'down1.res.kernel', 'down2.label_proj.kernel',
                                  'down3.time_proj.bias', 'up0.upconv.kernel', 'up0.conv.kernel',
                                  'up1.res.bias', 'up2.label_proj.bias', 'up2.conv.kernel', 'final.kernel'])
def test_gradient_vs_finite_differences(setup, name):
    P, x0, cond, t, noise, loss, mse, vlb, G = setup
    xt = S['sqrt_alpha_bar'][t].reshape(-1, 1, 1) * x0 + S['sqrt_one_minus_alpha_bar'][t].reshape(-1, 1, 1) * noise
    pred = R.unet_forward(P, xt, t, cond, dt=np.float64)[..., :2]
    # The objective is piecewise smooth (ReLU, max-pool): a direction whose +-eps segment crosses a
    # kink gives a wrong central difference (eps 1e-8 keeps that rare even for the 3M-entry up0 kernel,
    # about 18k ReLU units).  Three fixed directions (str hash() is salted per
    # process, so seeds come from crc32); at least two must agree to 1e-5.
    res = []
    for k in range(3):
        rng = np.random.default_rng(zlib.crc32(name.encode()) + k)
        D = rng.standard_normal(P[name].shape)
        eps = 1e-8 * max(1.0, float(np.abs(P[name]).max())) / max(1.0, float(np.abs(D).max()))

        def J(s):
            Q = dict(P)
            Q[name] = P[name] + s * D
            return TR.objective(Q, S, x0, cond, t, noise, pred)

        fd = (J(eps) - J(-eps)) / (2 * eps)
        an = float((G[name] * D).sum())
        res.append((abs(fd - an) <= 1e-5 * max(abs(an), 1e-3), fd, an))
    assert sum(r[0] for r in res) >= 2, (name, res)


def test_decoder_nll_gradient_finite_differences():
    rng = np.random.default_rng(0)
    x = np.array([-1.5, -0.5, 0.2, 0.999, 1.7, 3.0])
    m = x + rng.standard_normal(6) * 0.05
    lv = np.log(np.full(6, 2e-3))
    bw = 0.1
    _, g = TR.decoder_nll_and_grad(x, m, lv, bw)
    h = 1e-6
    fd = (TR.decoder_nll_and_grad(x, m, lv + h, bw)[0] - TR.decoder_nll_and_grad(x, m, lv - h, bw)[0]) / (2 * h)
    np.testing.assert_allclose(g, fd, rtol=1e-5, atol=1e-8)


def test_adam_clipnorm_closed_form():
    P = {'w': np.array([1.0, -2.0, 3.0])}
    G = {'w': np.array([3.0, 4.0, 0.0])}          # norm 5 -> clipped to 1.5
    m = {'w': np.zeros(3)}
    v = {'w': np.zeros(3)}
    Pn, mn, vn = TR.adam_update(P, G, m, v, step=0, lr=1e-3, clipnorm=1.5)
    g = G['w'] * 1.5 / 5.0
    np.testing.assert_allclose(mn['w'], 0.1 * g)
    np.testing.assert_allclose(vn['w'], 0.001 * g * g)
    alpha = 1e-3 * math.sqrt(1 - 0.999) / (1 - 0.9)
    np.testing.assert_allclose(Pn['w'], P['w'] - 0.1 * g * alpha / (np.sqrt(0.001 * g * g) + 1e-7))
    # ExponentialDecay (main_script.py:189-192)
    assert TR.learning_rate(0, 2e-4, 100, 0.5) == 2e-4
    np.testing.assert_allclose(TR.learning_rate(50, 2e-4, 100, 0.5), 2e-4 * 0.5 ** 0.5)


def _dp_worker(rank, world, port, q):
    """Data-parallel training math on gloo: each rank differentiates its shard's objective; the
    all-reduced SUM equals the full-batch gradient (J_full = sum_r J_r: B*mse splits into the
    shards' B_r*mse_r, the VLB is per sample; t > 0 so the decoder bin width does not enter)."""
    import os
    import torch
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from pet_posterior_distribution_amd.networks import glorot_uniform_init, param_spec
    spec = param_spec()
    P = {k: v.astype(np.float64) for k, v in glorot_uniform_init(spec, seed=5, bias_scale=0.05).items()}
    rng = np.random.default_rng(8)
    B = 4
    x0 = rng.standard_normal((B, 48, 2))
    cond = np.abs(rng.standard_normal((B, 49, 54)))
    t = np.array([3, 250, 640, 999])
    noise = rng.standard_normal((B, 48, 2))
    sl = slice(rank * B // world, (rank + 1) * B // world)
    _, _, _, G = TR.train_loss_and_grads(P, S, x0[sl], cond[sl], t[sl], noise[sl])
    g = torch.as_tensor(np.concatenate([G[n].ravel() for n, _ in spec]))
    dist.all_reduce(g)
    if rank == 0:
        _, _, _, Gf = TR.train_loss_and_grads(P, S, x0, cond, t, noise)
        full = np.concatenate([Gf[n].ravel() for n, _ in spec])
        q.put(float(np.abs(g.numpy() - full).max() / np.abs(full).max()))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_data_parallel_gradient_sum():
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    err = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert err < 1e-12
