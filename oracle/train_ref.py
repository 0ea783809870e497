"""CPU oracle for the iDDPM training step.

TEST INFRASTRUCTURE ONLY (same rules as ``iddpm_ref.py``): nothing in the package
imports it; only ``tests/`` use it, as the checker of the GPU training step.

Restates ``ImprovedDDPM.train_step`` (diffusion_model.py:533-598) with the shipped
compile arguments (main_script.py:169-234):

* t ~ U{0..T-1}, noise ~ N(0, 1) (injected here), x_t = sqrt(ab_t) x0 + sqrt(1-ab_t) noise
  (:546-551); target per parameterization (:553-560);
* the network output splits into prediction | v (:563-565); the VLB term sees the
  prediction through ``tf.stop_gradient`` (:566-569);
* loss = MSE(target, prediction) (Keras ``MeanSquaredError``: the mean over every
  element, compute_loss :177-198) + lambda_vlb * _vb_terms_bpd (:498-527), a [B]
  vector: ``tape.gradient`` of a vector differentiates its SUM, so the objective is
  J = B * mse + sum_b vlb_b;
* _vb_terms_bpd: KL(q(x_{t-1}|x_t,x_0) || p) for t > 0, the discretized-Gaussian
  decoder NLL for t == 0 (bin width 2 * 1.34896 / (B*48)^(1/3), :529-531), each
  averaged over (ROI, parameter) and divided by ln 2 (networks.py:29-80);
* Adam (Keras: beta 0.9 / 0.999, epsilon 1e-7) with per-variable ``clipnorm``
  (g * c / max(||g||, c)) and ExponentialDecay(2e-4, decay_steps, decay_rate)
  evaluated at the pre-increment iteration count (main_script.py:189-192, 233).

The backward pass is the analytic reverse of ``iddpm_ref.unet_forward``; it is pinned
by central finite differences of the forward (tests/test_cpu_train.py), since the
TF reference cannot run here ("parity unpinned" against TF itself).
"""
from __future__ import annotations

import math

import numpy as np
from scipy.special import erf

from oracle import iddpm_ref as R

LN2 = math.log(2.0)


# --------------------------------------------------------------------------
# forward with a tape
# --------------------------------------------------------------------------


def _conv_fwd(x, W, b, tape, key):
    """conv1d_same with the padded input kept for the backward pass."""
    k = W.shape[0]
    B, L, _ = x.shape
    pl = (k - 1) // 2
    xp = np.pad(x, ((0, 0), (pl, k - 1 - pl), (0, 0)))
    out = np.zeros((B, L, W.shape[2]), dtype=x.dtype)
    for j in range(k):
        out += xp[:, j:j + L, :] @ W[j]
    tape[key] = (xp, pl, L)
    return out + b


def _conv_bwd(dout, W, tape, key):
    xp, pl, L = tape[key]
    k = W.shape[0]
    dW = np.empty_like(W)
    dxp = np.zeros_like(xp)
    for j in range(k):
        dW[j] = np.einsum('blc,bld->cd', xp[:, j:j + L, :], dout)
        dxp[:, j:j + L, :] += dout @ W[j].T
    return dxp[:, pl:pl + L, :], dW, dout.sum(axis=(0, 1))


def gelu_grad(a):
    return 0.5 * (1.0 + erf(a / math.sqrt(2.0))) + a * np.exp(-0.5 * a * a) / math.sqrt(2.0 * math.pi)


def unet_forward_tape(P, x, t, cond, depth=4):
    """iddpm_ref.unet_forward (networks.py:994-1093) keeping what the backward needs."""
    tape = {}
    B, n_roi = x.shape[0], x.shape[1]
    down_L, up_L = R.level_lengths(n_roi, depth)
    emb = R.sinusoidal_pos_emb(t, dt=x.dtype.type)
    a_t = R.dense(emb, P['time_mlp.kernel'], P['time_mlp.bias'])
    h_t = R.gelu_exact(a_t)
    tape['time'] = (emb, a_t, h_t)
    enc_in = [cond]
    e = cond
    for i in range(3):
        e = R.relu(R.dense(e, P[f'cond_enc.hidden{i}.kernel'], P[f'cond_enc.hidden{i}.bias']))
        enc_in.append(e)
    z = R.dense(e, P['cond_enc.z.kernel'], P['cond_enc.z.bias'])
    tape['enc'] = enc_in
    tape['z'] = z

    def cond_inputs(prefix, L):
        tim = R.dense(h_t, P[prefix + '.time_proj.kernel'], P[prefix + '.time_proj.bias']).reshape(B, L, 1)
        lab = R.dense(z, P[prefix + '.label_proj.kernel'], P[prefix + '.label_proj.bias']).reshape(B, L, -1)
        return lab, tim

    skips = []
    h = x
    for d in range(depth):
        lab, tim = cond_inputs(f'down{d}', down_L[d])
        hin = np.concatenate([lab, tim, h], axis=-1)
        pre = (_conv_fwd(hin, P[f'down{d}.conv.kernel'], P[f'down{d}.conv.bias'], tape, f'down{d}.conv') +
               _conv_fwd(hin, P[f'down{d}.res.kernel'], P[f'down{d}.res.bias'], tape, f'down{d}.res'))
        h = R.relu(pre)
        tape[f'down{d}.out'] = h
        skips.append(h)
        if d < depth - 1:
            h = R.maxpool2(h)
    for u in range(depth - 1):
        lab, tim = cond_inputs(f'up{u}', up_L[u])
        hin = R.upsample2(np.concatenate([lab, tim, h], axis=-1))
        hu = _conv_fwd(hin, P[f'up{u}.upconv.kernel'], P[f'up{u}.upconv.bias'], tape, f'up{u}.upconv')
        hc = np.concatenate([skips[depth - 2 - u], hu], axis=-1)
        pre = (_conv_fwd(hc, P[f'up{u}.conv.kernel'], P[f'up{u}.conv.bias'], tape, f'up{u}.conv') +
               _conv_fwd(hc, P[f'up{u}.res.kernel'], P[f'up{u}.res.bias'], tape, f'up{u}.res'))
        h = R.relu(pre)
        tape[f'up{u}.out'] = h
    out = _conv_fwd(h, P['final.kernel'], P['final.bias'], tape, 'final')
    return out, tape


def unet_backward(P, tape, dout, depth=4):
    """Gradients of sum(dout * unet_forward(...)) for every parameter."""
    G = {}
    down_L, up_L = R.level_lengths(48, depth)
    dh, G['final.kernel'], G['final.bias'] = _conv_bwd(dout, P['final.kernel'], tape, 'final')
    B = dout.shape[0]
    dz = np.zeros_like(tape['z'])
    emb, a_t, h_t = tape['time']
    dh_t = np.zeros_like(h_t)
    z = tape['z']

    def cond_backward(prefix, dlab, dtim):
        nonlocal dz, dh_t
        dlab = dlab.reshape(B, 49, -1)                      # raw reshape back to (B, 49, L)
        G[prefix + '.label_proj.kernel'] = np.einsum('brk,brl->kl', z, dlab)
        G[prefix + '.label_proj.bias'] = dlab.sum(axis=(0, 1))
        dz = dz + dlab @ P[prefix + '.label_proj.kernel'].T
        dtim = dtim.reshape(B, -1)
        G[prefix + '.time_proj.kernel'] = h_t.T @ dtim
        G[prefix + '.time_proj.bias'] = dtim.sum(axis=0)
        dh_t = dh_t + dtim @ P[prefix + '.time_proj.kernel'].T

    dskip = [None] * depth
    for u in reversed(range(depth - 1)):
        dpre = dh * (tape[f'up{u}.out'] > 0)
        d1, G[f'up{u}.conv.kernel'], G[f'up{u}.conv.bias'] = _conv_bwd(dpre, P[f'up{u}.conv.kernel'], tape,
                                                                       f'up{u}.conv')
        d2, G[f'up{u}.res.kernel'], G[f'up{u}.res.bias'] = _conv_bwd(dpre, P[f'up{u}.res.kernel'], tape,
                                                                     f'up{u}.res')
        dhc = d1 + d2
        cout = dhc.shape[-1] // 2
        dskip[depth - 2 - u] = dhc[..., :cout]
        dhin, G[f'up{u}.upconv.kernel'], G[f'up{u}.upconv.bias'] = _conv_bwd(
            dhc[..., cout:], P[f'up{u}.upconv.kernel'], tape, f'up{u}.upconv')
        dcat = dhin[:, 0::2, :] + dhin[:, 1::2, :]           # UpSampling1D backward
        cond_backward(f'up{u}', dcat[..., :49], dcat[..., 49:50])
        dh = dcat[..., 50:]
    for d in reversed(range(depth)):
        if d < depth - 1:
            out = tape[f'down{d}.out']
            a, b = out[:, 0::2, :], out[:, 1::2, :]
            first = a >= b                                   # MaxPool grad -> first maximum
            dfull = np.zeros_like(out)
            dfull[:, 0::2, :] = np.where(first, dh, 0.0)
            dfull[:, 1::2, :] = np.where(first, 0.0, dh)
            dh = dfull + dskip[d]
        else:
            dh = dh + (dskip[d] if dskip[d] is not None else 0.0)
        dpre = dh * (tape[f'down{d}.out'] > 0)
        d1, G[f'down{d}.conv.kernel'], G[f'down{d}.conv.bias'] = _conv_bwd(dpre, P[f'down{d}.conv.kernel'], tape,
                                                                           f'down{d}.conv')
        d2, G[f'down{d}.res.kernel'], G[f'down{d}.res.bias'] = _conv_bwd(dpre, P[f'down{d}.res.kernel'], tape,
                                                                         f'down{d}.res')
        dhin = d1 + d2
        cond_backward(f'down{d}', dhin[..., :49], dhin[..., 49:50])
        dh = dhin[..., 50:]
    # condition encoder (networks.py:574-586)
    enc = tape['enc']
    G['cond_enc.z.kernel'] = np.einsum('brk,brl->kl', enc[3], dz)
    G['cond_enc.z.bias'] = dz.sum(axis=(0, 1))
    de = dz @ P['cond_enc.z.kernel'].T
    for i in reversed(range(3)):
        de = de * (enc[i + 1] > 0)
        G[f'cond_enc.hidden{i}.kernel'] = np.einsum('brk,brl->kl', enc[i], de)
        G[f'cond_enc.hidden{i}.bias'] = de.sum(axis=(0, 1))
        de = de @ P[f'cond_enc.hidden{i}.kernel'].T
    # time MLP (networks.py:182-198, 235-258, 854)
    da = dh_t * gelu_grad(a_t)
    G['time_mlp.kernel'] = emb.T @ da
    G['time_mlp.bias'] = da.sum(axis=0)
    return G


# --------------------------------------------------------------------------
# loss terms (diffusion_model.py:498-531, networks.py:29-80)
# --------------------------------------------------------------------------


def approx_cdf(x):
    return 0.5 * (1.0 + np.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x ** 3)))


def approx_cdf_grad(x):
    c = math.sqrt(2.0 / math.pi)
    th = np.tanh(c * (x + 0.044715 * x ** 3))
    return 0.5 * (1.0 - th * th) * c * (1.0 + 3 * 0.044715 * x * x)


def decoder_nll_and_grad(x, means, log_var, bin_width):
    """-discretized_gaussian_log_likelihood (networks.py:47-80) with log_scales = lv / 2,
    and its derivative w.r.t. lv (clip_by_value passes gradient only inside the range)."""
    ls = 0.5 * log_var
    cx = x - means
    inv = np.exp(-ls)
    pin, mn = inv * (cx + bin_width), inv * (cx - bin_width)
    cp, cm = approx_cdf(pin), approx_cdf(mn)
    # d(in)/d(ls) = -in
    dcp, dcm = approx_cdf_grad(pin) * (-pin), approx_cdf_grad(mn) * (-mn)
    lo = 1e-12
    v_plus = np.where(cp > lo, np.log(np.maximum(cp, lo)), math.log(lo))
    g_plus = np.where(cp > lo, dcp / np.maximum(cp, lo), 0.0)
    om = 1.0 - cm
    v_om = np.where(om > lo, np.log(np.maximum(om, lo)), math.log(lo))
    g_om = np.where(om > lo, -dcm / np.maximum(om, lo), 0.0)
    dl = cp - cm
    v_dl = np.where(dl > lo, np.log(np.maximum(dl, lo)), math.log(lo))
    g_dl = np.where(dl > lo, (dcp - dcm) / np.maximum(dl, lo), 0.0)
    logp = np.where(x < -0.999, v_plus, np.where(x > 0.999, v_om, v_dl))
    dlogp_dls = np.where(x < -0.999, g_plus, np.where(x > 0.999, g_om, g_dl))
    return -logp, -dlogp_dls * 0.5


def vlb_terms(S, pred, v, x0, x_t, t, lam, learn_variance='learn_ranged', parameterization='eps'):
    """lambda * _vb_terms_bpd per sample, and d/dv of its SUM (prediction frozen)."""
    dt = x0.dtype.type
    out = R.p_mean_variance(S, np.concatenate([pred, v], axis=-1), x_t, t, learn_variance=learn_variance,
                            parameterization=parameterization, dt=dt)
    m2, lv2 = out['mean'], out['log_variance']
    ex = lambda n: np.asarray(S[n], dtype=dt)[np.asarray(t)].reshape(-1, 1, 1)
    m1 = ex('posterior_mean_coef1') * x0 + ex('posterior_mean_coef2') * x_t
    lv1 = ex('posterior_log_variance_clipped')
    kl = 0.5 * (-1.0 + lv2 - lv1 + np.exp(lv1 - lv2) + (m1 - m2) ** 2 * np.exp(-lv2))
    dkl = 0.5 * (1.0 - np.exp(lv1 - lv2) - (m1 - m2) ** 2 * np.exp(-lv2))
    B = x0.shape[0]
    bw = 2 * 1.34896 / float(B * x0.shape[1]) ** (1.0 / 3.0)
    nll, dnll = decoder_nll_and_grad(x0, m2, lv2, bw)
    is0 = (np.asarray(t) == 0).reshape(-1, 1, 1)
    term = np.where(is0, nll, kl)
    dterm = np.where(is0, dnll, dkl)
    n = x0.shape[1] * x0.shape[2]
    vlb = lam * term.mean(axis=(1, 2)) / LN2
    if 'ranged' in learn_variance:
        dlv_dv = 0.5 * (np.log(ex('beta')) - ex('posterior_log_variance_clipped'))
    else:
        dlv_dv = 1.0
    dv = lam * dterm / n / LN2 * dlv_dv
    return vlb, dv


def train_target(S, x0, noise, x_t, t, parameterization='eps'):
    """Regression target per parameterization (diffusion_model.py:553-560)."""
    dt = x0.dtype.type
    ex = lambda n: np.asarray(S[n], dtype=dt)[np.asarray(t)].reshape(-1, 1, 1)
    p = parameterization.lower()
    if p in R.XPREV_NAMES:
        return ex('posterior_mean_coef1') * x0 + ex('posterior_mean_coef2') * x_t
    if p in R.X0_NAMES:
        return x0
    if p in R.V_NAMES:
        return ex('sqrt_alpha_bar') * noise - ex('sqrt_one_minus_alpha_bar') * x0
    return noise


def train_loss_and_grads(P, S, x0, cond, t, noise, lam=0.1, learn_variance='learn_ranged',
                         parameterization='eps', dt=np.float64):
    """One training step's objective and raw gradients (diffusion_model.py:533-578).
    Returns (loss [B], noise_loss, vlb [B], grads dict)."""
    P = {k: np.asarray(v, dtype=dt) for k, v in P.items()}
    x0 = np.asarray(x0, dtype=dt)
    noise = np.asarray(noise, dtype=dt)
    t = np.asarray(t)
    ex = lambda n: np.asarray(S[n], dtype=dt)[t].reshape(-1, 1, 1)
    x_t = ex('sqrt_alpha_bar') * x0 + ex('sqrt_one_minus_alpha_bar') * noise
    out, tape = unet_forward_tape(P, x_t, t, np.asarray(cond, dtype=dt))
    target = train_target(S, x0, noise, x_t, t, parameterization)
    B = x0.shape[0]
    if 'learn' in learn_variance:
        pred, v = out[..., :2], out[..., 2:]
        vlb, dv = vlb_terms(S, pred, v, x0, x_t, t, lam, learn_variance, parameterization)
    else:
        pred, vlb = out, np.zeros(B)
    mse = np.mean((target - pred) ** 2)
    dpred = B * 2.0 * (pred - target) / target.size
    dout = np.concatenate([dpred, dv], axis=-1) if 'learn' in learn_variance else dpred
    G = unet_backward(P, tape, dout)
    return mse + vlb, mse, vlb, G


def objective(P, S, x0, cond, t, noise, pred_frozen, lam=0.1, dt=np.float64):
    """J = B * mse + sum vlb with the VLB's prediction frozen (for finite differences)."""
    P = {k: np.asarray(v, dtype=dt) for k, v in P.items()}
    t = np.asarray(t)
    ex = lambda n: np.asarray(S[n], dtype=dt)[t].reshape(-1, 1, 1)
    x0 = np.asarray(x0, dtype=dt)
    x_t = ex('sqrt_alpha_bar') * x0 + ex('sqrt_one_minus_alpha_bar') * np.asarray(noise, dtype=dt)
    out = R.unet_forward(P, x_t, t, cond, dt=dt)
    vlb, _ = vlb_terms(S, pred_frozen, out[..., 2:], x0, x_t, t, lam)
    return x0.shape[0] * np.mean((np.asarray(noise, dtype=dt) - out[..., :2]) ** 2) + vlb.sum()


# --------------------------------------------------------------------------
# optimizer (Keras Adam with clipnorm; ExponentialDecay)
# --------------------------------------------------------------------------


def learning_rate(step, lr0=2e-4, decay_steps=1, decay_rate=1.0):
    """keras.optimizers.schedules.ExponentialDecay (staircase=False) at iteration `step`."""
    return lr0 * decay_rate ** (step / decay_steps)


def adam_update(P, G, m, v, step, lr, clipnorm=1.5, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
    """Keras Adam.update_step after per-variable clip_by_norm; `step` = iterations before
    this update.  Returns new (P, m, v) dicts (float64)."""
    Pn, mn, vn = {}, {}, {}
    k = step + 1
    alpha = lr * math.sqrt(1 - beta_2 ** k) / (1 - beta_1 ** k)
    for name, g in G.items():
        g = np.asarray(g, dtype=np.float64)
        if clipnorm:
            nrm = math.sqrt(float((g * g).sum()))
            g = g * clipnorm / max(nrm, clipnorm)
        mm = m[name] + (g - m[name]) * (1 - beta_1)
        vv = v[name] + (g * g - v[name]) * (1 - beta_2)
        Pn[name] = np.asarray(P[name], dtype=np.float64) - mm * alpha / (np.sqrt(vv) + epsilon)
        mn[name], vn[name] = mm, vv
    return Pn, mn, vn
