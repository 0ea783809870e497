"""CPU oracle for the iDDPM posterior-sampling hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``pet_posterior_distribution_amd/`` imports
this module; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may use it, and only as the checker / the timed CPU
baseline -- never as the product path.

This is a plain NumPy restatement of the reference algorithm
(yanisdjebra/PET_posterior_distribution @ 2025-08-29).  Every function cites the
reference lines it follows.  The reference is TensorFlow/Keras (not installed
here), so the network part is a restatement of Keras semantics:

* ``Dense`` acts on the last axis, kernel layout ``(in, out)``;
* ``Conv1D(padding='same')`` is a cross-correlation with kernel ``(k, Cin, Cout)``
  and TF SAME padding ``pad_before = (k - 1) // 2``;
* ``Reshape`` is a row-major reinterpretation (NOT a transpose);
* ``MaxPooling1D(2, 'same')`` on even lengths has no padding;
* ``UpSampling1D(2)`` repeats every position twice.

Parity status (see DESIGN.md "Oracle"):
* schedule (a1)      -- PINNED: bit-exact against the imported reference
                        ``helper_func.get_beta_schedule`` (tests/golden/G1).
* U-Net / p_sample / loop (a4-a15) -- the TF reference cannot run here (TF absent,
  trained weights are Git-LFS pointers).  Pinned only STRUCTURALLY: parameter
  count 11,851,740 == the 142,333,243-byte LFS checkpoint (weights + Adam m, v),
  and per-layer shapes.  Numerics are "parity unpinned"
  against TF itself; the GPU path is checked against this restatement.

Parameter naming (shared convention, documented in include/petdiff.h):
``time_mlp``, ``cond_enc.hidden{0,1,2}``, ``cond_enc.z``,
``down{d}.{time_proj,label_proj,conv,res}``,
``up{u}.{time_proj,label_proj,upconv,conv,res}``, ``final``; each with
``.kernel`` / ``.bias`` in Keras layout.
"""
from __future__ import annotations

import math
import numpy as np

F32 = np.float32

# --------------------------------------------------------------------------
# a1: noise schedules (helper_func.py:210-268) -- computed in float32 exactly
# like the reference (NP_DTYPE = float32, diffusion_model.py:7-10).
# --------------------------------------------------------------------------


def cos_beta_schedule(timesteps, offset_s=0.008, max_beta=0.999):
    """helper_func.py:210-219 (cosine schedule, np.cos evaluated in float32)."""
    def alpha_bar(t):
        return np.cos((t + offset_s) / (1 + offset_s) * np.pi / 2, dtype=F32) ** 2
    beta = []
    for i in range(timesteps):
        t1 = i / timesteps
        t2 = (i + 1) / timesteps
        beta.append(min(1 - alpha_bar(t2) / alpha_bar(t1), max_beta))
    return np.array(beta, dtype=F32)


def get_beta_schedule(schedule_name, timesteps, beta_start=1e-4, beta_end=2e-2,
                      offset_s=0.008, max_beta=0.999):
    """helper_func.py:222-268."""
    name = schedule_name.lower()
    if name in ('lin', 'linear'):
        return np.linspace(beta_start, beta_end, timesteps, dtype=F32)
    if name in ('quad', 'quadratic'):
        return np.linspace(beta_start ** 0.5, beta_end ** 0.5, timesteps, dtype=F32) ** 2
    if name in ('sig', 'sigmoid'):
        b = np.linspace(-6, 6, timesteps, dtype=F32)
        return 1 / (1 + np.exp(-b, dtype=F32)) * (beta_end - beta_start) + beta_start
    if name in ('cos', 'cosine'):
        return cos_beta_schedule(timesteps, offset_s=offset_s, max_beta=max_beta)
    raise NotImplementedError(schedule_name)


def schedule_tables(beta):
    """Schedule buffers of ImprovedDDPM (diffusion_model.py:98-105, 337-355).

    ``alpha_bar`` is the UNSHIFTED cumprod (ImprovedDDPM overrides DDPM's
    shifted one at :337); ``posterior_variance[0]`` aliases into the clipped
    log table (:349-351: ``posterior_log_variance_clipped`` IS
    ``posterior_variance`` before the log, so element 0 of BOTH is overwritten).
    """
    beta = np.asarray(beta, dtype=F32)
    alpha = 1 - beta
    alpha_bar = np.cumprod(alpha, 0, dtype=F32)
    alpha_bar_prev = np.concatenate((np.array([1.], dtype=F32), alpha_bar[:-1]), axis=0)
    sqrt_alpha_bar = np.sqrt(alpha_bar, dtype=F32)
    sqrt_one_minus_alpha_bar = np.sqrt(1 - alpha_bar, dtype=F32)
    posterior_variance = beta * (1.0 - alpha_bar_prev) / (1.0 - alpha_bar)
    plvc = posterior_variance           # alias, exactly as the reference
    plvc[0] = plvc[1]
    plvc = np.log(plvc)
    c1 = beta * np.sqrt(alpha_bar_prev) / (1.0 - alpha_bar)
    c2 = (1.0 - alpha_bar_prev) * np.sqrt(alpha) / (1.0 - alpha_bar)
    return dict(beta=beta, alpha=alpha, alpha_bar=alpha_bar, alpha_bar_prev=alpha_bar_prev,
                sqrt_alpha_bar=sqrt_alpha_bar, sqrt_one_minus_alpha_bar=sqrt_one_minus_alpha_bar,
                posterior_variance=posterior_variance, posterior_log_variance_clipped=plvc,
                posterior_mean_coef1=c1, posterior_mean_coef2=c2)


# --------------------------------------------------------------------------
# Architecture of the shipped config (main_script.py:131-167)
# --------------------------------------------------------------------------

N_ROI, N_PAR, N_FRAMES, N_COND_ROWS = 48, 2, 54, 49


def level_lengths(n_roi=N_ROI, depth=4):
    """networks.py:830-973 -- im_size per level (down) and cond length (up)."""
    down = [n_roi]
    for _ in range(depth - 1):
        down.append((down[-1] + 1) // 2)
    up_cond = down[::-1][:-1]           # conditions of the up path use the coarse L
    return down, up_cond


def param_spec(n_roi=N_ROI, n_par=N_PAR, f=128, depth=4, k=6, pool=2, sin_dim=64,
               enc=(256, 128, 64), latent=32, n_frames=N_FRAMES, n_out=4):
    """Ordered (name, shape) list of every trainable tensor (networks.py:781-992)."""
    down_L, up_L = level_lengths(n_roi, depth)
    spec = [('time_mlp.kernel', (sin_dim, n_roi)), ('time_mlp.bias', (n_roi,))]
    prev = n_frames
    for i, e in enumerate(enc):
        spec += [(f'cond_enc.hidden{i}.kernel', (prev, e)), (f'cond_enc.hidden{i}.bias', (e,))]
        prev = e
    spec += [('cond_enc.z.kernel', (prev, latent)), ('cond_enc.z.bias', (latent,))]
    cin = n_par
    for d in range(depth):
        L = down_L[d]
        cout = f * 2 ** d
        c = N_COND_ROWS + 1 + cin
        spec += [(f'down{d}.time_proj.kernel', (n_roi, L)), (f'down{d}.time_proj.bias', (L,)),
                 (f'down{d}.label_proj.kernel', (latent, L)), (f'down{d}.label_proj.bias', (L,)),
                 (f'down{d}.conv.kernel', (k, c, cout)), (f'down{d}.conv.bias', (cout,)),
                 (f'down{d}.res.kernel', (1, c, cout)), (f'down{d}.res.bias', (cout,))]
        cin = cout
    for u in range(depth - 1):
        L = up_L[u]
        cout = f * 2 ** (depth - 2 - u)
        c = N_COND_ROWS + 1 + cin
        spec += [(f'up{u}.time_proj.kernel', (n_roi, L)), (f'up{u}.time_proj.bias', (L,)),
                 (f'up{u}.label_proj.kernel', (latent, L)), (f'up{u}.label_proj.bias', (L,)),
                 (f'up{u}.upconv.kernel', (pool, c, cout)), (f'up{u}.upconv.bias', (cout,)),
                 (f'up{u}.conv.kernel', (k, 2 * cout, cout)), (f'up{u}.conv.bias', (cout,)),
                 (f'up{u}.res.kernel', (1, 2 * cout, cout)), (f'up{u}.res.bias', (cout,))]
        cin = cout
    spec += [('final.kernel', (1, f, n_out)), ('final.bias', (n_out,))]
    return spec


# --------------------------------------------------------------------------
# Keras layer semantics
# --------------------------------------------------------------------------


def dense(x, W, b):
    return x @ W + b


def relu(x):
    return np.maximum(x, 0)


def gelu_exact(x):
    """networks.py:236-241 (approximate=False): 0.5 x (1 + erf(x / sqrt 2))."""
    from scipy.special import erf
    return 0.5 * x * (1.0 + erf(x / x.dtype.type(1.4142135623730951)))


def conv1d_same(x, W, b):
    """tf.keras Conv1D(padding='same'), stride 1: cross-correlation, pad_before=(k-1)//2."""
    k = W.shape[0]
    B, L, _ = x.shape
    pl = (k - 1) // 2
    pr = (k - 1) - pl
    xp = np.pad(x, ((0, 0), (pl, pr), (0, 0)))
    out = np.zeros((B, L, W.shape[2]), dtype=x.dtype)
    for j in range(k):
        out += xp[:, j:j + L, :] @ W[j]
    return out + b


def maxpool2(x):
    B, L, C = x.shape
    assert L % 2 == 0
    return x.reshape(B, L // 2, 2, C).max(axis=2)


def upsample2(x):
    return np.repeat(x, 2, axis=1)


def sinusoidal_pos_emb(t, dim=64, max_positions=10000., dt=F32):
    """networks.py:189-198."""
    x = np.asarray(t).astype(dt)
    half = dim // 2
    emb = dt(np.log(dt(max_positions))) / dt(half - 1)
    emb = np.exp(np.arange(half, dtype=dt) * -emb)
    emb = x[:, None] * emb[None, :]
    return np.concatenate([np.sin(emb), np.cos(emb)], axis=-1)


# --------------------------------------------------------------------------
# a6-a13: UnetConditional.call (networks.py:994-1093) with the shipped config
# --------------------------------------------------------------------------


def unet_forward(P, x, t, cond, dt=np.float64, depth=4, levels=None):
    """UnetConditional.call (networks.py:994-1093), shipped config.

    x (B,48,2), t (B,) int, cond (B,49,54) -> (B,48,n_out).
    Down level d (networks.py:1010-1031): concat [label(49) | time(1) | x] on
    channels (:1022), ConvBlock = relu(conv_k(x) + conv_1(x)) (:679-691), skip
    saved before MaxPool (:1027).  Up level u (:1033-1072): concat
    [label | time | x] at the COARSE length, UpSampling, Conv1D(k=pool) (no
    activation), concat [skip | x] (:1057), ConvBlock.  Final Conv1D 1x1 (:1074).
    ``levels`` (a dict) receives every ConvBlock output: 'down0'..'down3', 'up0'..'up2'.
    """
    P = {k: np.asarray(v, dtype=dt) for k, v in P.items()}
    x = np.asarray(x, dtype=dt)
    cond = np.asarray(cond, dtype=dt)
    B = x.shape[0]
    n_roi = x.shape[1]
    down_L, up_L = level_lengths(n_roi, depth)
    # shared time MLP: SinusoidalPosEmb -> Dense(48) -> GELU (networks.py:854, 912-921)
    h_t = gelu_exact(dense(sinusoidal_pos_emb(t, dt=dt), P['time_mlp.kernel'], P['time_mlp.bias']))
    # shared condition encoder Encoder_v3_noskip (networks.py:526-586)
    e = cond
    for i in range(3):
        e = relu(dense(e, P[f'cond_enc.hidden{i}.kernel'], P[f'cond_enc.hidden{i}.bias']))
    z_lab = dense(e, P['cond_enc.z.kernel'], P['cond_enc.z.bias'])          # (B,49,32)

    def cond_inputs(prefix, L):
        tim = dense(h_t, P[prefix + '.time_proj.kernel'], P[prefix + '.time_proj.bias'])
        tim = tim.reshape(B, L, -1)                                          # Reshape((L,-1))
        lab = dense(z_lab, P[prefix + '.label_proj.kernel'], P[prefix + '.label_proj.bias'])
        lab = lab.reshape(B, L, -1)                                          # raw reshape (B,L,49)
        return lab, tim

    skips = []
    h = x
    for d in range(depth):
        lab, tim = cond_inputs(f'down{d}', down_L[d])
        h = np.concatenate([lab, tim, h], axis=-1)
        h = relu(conv1d_same(h, P[f'down{d}.conv.kernel'], P[f'down{d}.conv.bias']) +
                 conv1d_same(h, P[f'down{d}.res.kernel'], P[f'down{d}.res.bias']))
        skips.append(h)
        if levels is not None:
            levels[f'down{d}'] = h
        if d < depth - 1:
            h = maxpool2(h)
    for u in range(depth - 1):
        lab, tim = cond_inputs(f'up{u}', up_L[u])
        h = np.concatenate([lab, tim, h], axis=-1)
        h = upsample2(h)
        h = conv1d_same(h, P[f'up{u}.upconv.kernel'], P[f'up{u}.upconv.bias'])
        h = np.concatenate([skips[depth - 2 - u], h], axis=-1)
        h = relu(conv1d_same(h, P[f'up{u}.conv.kernel'], P[f'up{u}.conv.bias']) +
                 conv1d_same(h, P[f'up{u}.res.kernel'], P[f'up{u}.res.bias']))
        if levels is not None:
            levels[f'up{u}'] = h
    return conv1d_same(h, P['final.kernel'], P['final.bias'])


# --------------------------------------------------------------------------
# a14/a15: p_mean_variance + ddpm (= p_sample) (diffusion_model.py:366-496, 651-663)
# --------------------------------------------------------------------------

EPS_NAMES = ['eps', 'epsilon']
X0_NAMES = ['x0', 'x_0', 'x_start', 'xstart', 'start_x']
XPREV_NAMES = ['x_{t-1}', 'x_prev', 'xprev', 'prev_x']
V_NAMES = ['v']


def p_mean_variance(S, model_output, x, t, learn_variance='learn_ranged', parameterization='eps',
                    dt=F32):
    """diffusion_model.py:424-496 (+ helpers :366-422)."""
    def ex(name):
        return np.asarray(S[name], dtype=dt)[np.asarray(t)].reshape(-1, 1, 1)
    x = np.asarray(x, dtype=dt)
    mo = np.asarray(model_output, dtype=dt)
    lv = learn_variance.lower()
    if 'learn' in lv:
        mo, var_values = np.split(mo, 2, axis=-1)
        if 'ranged' not in lv:
            logvar = var_values
        else:
            min_log = ex('posterior_log_variance_clipped')
            max_log = np.log(ex('beta'))
            frac = (var_values + 1) / 2
            logvar = frac * max_log + (1 - frac) * min_log
        var = np.exp(logvar)
        var_t, logvar_t = var, logvar
    else:
        var, logvar = ex('beta'), np.log(ex('beta'))
        var_t, logvar_t = ex('posterior_variance'), ex('posterior_log_variance_clipped')
    p = parameterization.lower()
    if p in XPREV_NAMES:
        pred_x0 = (ex('posterior_mean_coef1') ** -1 * mo -
                   (ex('posterior_mean_coef2') / ex('posterior_mean_coef1')) * x)
        mean = mo
    else:
        if p in X0_NAMES:
            pred_x0 = mo
        elif p in V_NAMES:
            pred_x0 = ex('sqrt_alpha_bar') * x - ex('sqrt_one_minus_alpha_bar') * mo
        else:   # eps (:370-374)
            pred_x0 = dt(1.0) / ex('sqrt_alpha_bar') * x - np.sqrt(dt(1.0) / ex('alpha_bar') - 1) * mo
        mean = ex('posterior_mean_coef1') * pred_x0 + ex('posterior_mean_coef2') * x
    return dict(mean=mean, variance=var, log_variance=logvar, variance_tilde=var_t,
                log_variance_tilde=logvar_t, pred_xstart=pred_x0)


def ddpm(P, S, x_t, t, cond, z, learn_variance='learn_ranged', parameterization='eps', dt=F32,
         net_dt=None):
    """ImprovedDDPM.ddpm (diffusion_model.py:651-663) with injected noise ``z``."""
    net_dt = dt if net_dt is None else net_dt
    out_net = unet_forward(P, x_t, t, cond, dt=net_dt).astype(dt)
    out = p_mean_variance(S, out_net, x_t, t, learn_variance, parameterization, dt=dt)
    mask = np.where(np.asarray(t) == 0, 0., 1.).astype(dt).reshape(-1, 1, 1)
    z = np.asarray(z, dtype=dt)
    var = mask * np.exp(dt(0.5) * out['log_variance']) * z
    var_tilde = mask * np.exp(dt(0.5) * out['log_variance_tilde']) * z
    return out['mean'], var, var_tilde


def loop_indices(timesteps, num_timesteps=None, sub_sequence_type='linear'):
    """diffusion_model.py:680-691 (note the substring tests ``in 'linear'``)."""
    if num_timesteps in (None, 0, timesteps):
        return list(range(timesteps))[::-1]
    if sub_sequence_type in 'linear':
        return np.linspace(0, timesteps - 1, num=num_timesteps, dtype=np.int32)[::-1].tolist()
    if sub_sequence_type in 'quadratic':
        return (np.linspace(0, np.sqrt(timesteps - 1), num=num_timesteps,
                            dtype=np.int32)[::-1] ** 2).tolist()
    raise ValueError('Subsequence type not recognized (given {})'.format(sub_sequence_type))


def ddpm_loop(P, S, x_T, cond, z_all, indices, flag_var_tilde=True, keep_all_xt=False,
              learn_variance='learn_ranged', parameterization='eps', dt=F32, net_dt=None):
    """ImprovedDDPM.ddpm_loop (diffusion_model.py:670-715); z_all[i] is the noise of step i."""
    x = np.asarray(x_T, dtype=dt)
    B = x.shape[0]
    cond = np.asarray(cond, dtype=dt)
    if cond.shape[0] != B:
        cond = np.repeat(cond, B, axis=0)                    # :697-699
    out_all = []
    for i, ti in enumerate(indices):
        t = np.full((B,), ti, dtype=np.int32)
        mean, var, var_tilde = ddpm(P, S, x, t, cond, z_all[i], learn_variance, parameterization,
                                    dt=dt, net_dt=net_dt)
        x = mean + (var_tilde if flag_var_tilde else var)
        if keep_all_xt:
            out_all.append(x)
    return np.stack(out_all, 0) if keep_all_xt else x


# --------------------------------------------------------------------------
# Counter-based RNG used by the build for z_t (NOT in the reference, which uses
# TF's stateful Philox): Philox4x32-10 (Salmon et al., SC'11) + Box-Muller.
# Counter = (roi, step, g_lo, g_hi), key = (seed_lo, seed_hi); lanes 0,1 of the
# output feed one Box-Muller pair -> z[..., 0], z[..., 1].
# --------------------------------------------------------------------------

PHILOX_M0, PHILOX_M1 = 0xD2511F53, 0xCD9E8D57
PHILOX_W0, PHILOX_W1 = 0x9E3779B9, 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    c = [np.asarray(v, dtype=np.uint64) & MASK32 for v in (c0, c1, c2, c3)]
    k0 = np.uint64(k0) & MASK32
    k1 = np.uint64(k1) & MASK32
    for _ in range(10):
        p0 = np.uint64(PHILOX_M0) * c[0]
        p1 = np.uint64(PHILOX_M1) * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c = [(hi1 ^ c[1] ^ k0) & MASK32, lo1, (hi0 ^ c[3] ^ k1) & MASK32, lo0]
        k0 = (k0 + np.uint64(PHILOX_W0)) & MASK32
        k1 = (k1 + np.uint64(PHILOX_W1)) & MASK32
    return [v.astype(np.uint32) for v in c]


def philox_normal_pairs(seed, g, step, n_roi=N_ROI):
    """z of shape (len(g), n_roi, 2) for global sample indices g at loop step ``step``."""
    g = np.asarray(g, dtype=np.uint64)
    roi = np.arange(n_roi, dtype=np.uint64)[None, :]
    G = np.broadcast_to(g[:, None], (g.size, n_roi))
    R = np.broadcast_to(roi, (g.size, n_roi))
    x0, x1, _, _ = philox4x32_10(R, np.full(R.shape, step, dtype=np.uint64),
                                 G & MASK32, G >> np.uint64(32),
                                 seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    # uniforms in (0, 1]: (u + 1) * 2^-32 computed exactly in float64
    u1 = (x0.astype(np.float64) + 1.0) * 2.0 ** -32
    u2 = (x1.astype(np.float64) + 0.5) * 2.0 ** -32
    r = np.sqrt(-2.0 * np.log(u1))
    ang = 2.0 * math.pi * u2
    return np.stack([r * np.cos(ang), r * np.sin(ang)], axis=-1)


# --------------------------------------------------------------------------
# a16: caller-side summary (main_script.py:433-436): per-ROI mean and
# population std (ddof = 0) over samples, DVR = channel 0, R1 = channel 1.
# --------------------------------------------------------------------------


def posterior_summary(x0):
    x0 = np.asarray(x0, dtype=np.float64)
    return dict(mean_DVR=x0[:, :, 0].mean(0), mean_R1=x0[:, :, 1].mean(0),
                std_DVR=x0[:, :, 0].std(0), std_R1=x0[:, :, 1].std(0))
