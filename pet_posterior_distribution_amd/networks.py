"""Host-side description of the conditional 1-D U-Net denoiser.

Mirrors ``networks.UnetConditional`` (networks.py:718-1093) as a *plugin object*
the diffusion model consumes: same constructor arguments, ``learn_variance``,
``ndim``, ``build(input_shape)`` and Keras-style weight I/O.  The forward pass
itself runs only inside libpetdiff.so (hand-written gfx950 kernels); this class
holds the configuration and the fp32 weights in Keras layout.

Only the shipped architecture (main_script.py:131-167: f128/d4, pool 2, k=6,
residual ConvBlocks without normalisation, ReLU, Encoder 256-128-64-32 condition
embedding, 64-d sinusoidal time embedding, concat skips) is compiled into the
kernels; other configurations raise ``NotImplementedError`` at construction.
"""
from __future__ import annotations

import json
import os

import numpy as np

from .helper_func import NP_DTYPE

SHIPPED = dict(num_filt_start=128, pool_size=2, depth=4, block_type='conv', kernel_size=6,
               skip_conn_type='concat', sin_emb_dim=64, enc_size=(256, 128, 64), latent_dim=32)


def level_lengths(n_roi, depth):
    down = [n_roi]
    for _ in range(depth - 1):
        down.append((down[-1] + 1) // 2)
    return down, down[::-1][:-1]


def param_spec(n_roi=48, n_par=2, f=128, depth=4, k=6, pool=2, sin_dim=64, enc=(256, 128, 64),
               latent=32, n_frames=54, n_cond_rows=49, n_out=4):
    """Ordered (name, shape) of every weight (networks.py:781-992); order of include/petdiff.h."""
    down_L, up_L = level_lengths(n_roi, depth)
    spec = [('time_mlp.kernel', (sin_dim, n_roi)), ('time_mlp.bias', (n_roi,))]
    prev = n_frames
    for i, e in enumerate(enc):
        spec += [(f'cond_enc.hidden{i}.kernel', (prev, e)), (f'cond_enc.hidden{i}.bias', (e,))]
        prev = e
    spec += [('cond_enc.z.kernel', (prev, latent)), ('cond_enc.z.bias', (latent,))]
    cin = n_par
    for d in range(depth):
        L, cout = down_L[d], f * 2 ** d
        c = n_cond_rows + 1 + cin
        spec += [(f'down{d}.time_proj.kernel', (n_roi, L)), (f'down{d}.time_proj.bias', (L,)),
                 (f'down{d}.label_proj.kernel', (latent, L)), (f'down{d}.label_proj.bias', (L,)),
                 (f'down{d}.conv.kernel', (k, c, cout)), (f'down{d}.conv.bias', (cout,)),
                 (f'down{d}.res.kernel', (1, c, cout)), (f'down{d}.res.bias', (cout,))]
        cin = cout
    for u in range(depth - 1):
        L, cout = up_L[u], f * 2 ** (depth - 2 - u)
        c = n_cond_rows + 1 + cin
        spec += [(f'up{u}.time_proj.kernel', (n_roi, L)), (f'up{u}.time_proj.bias', (L,)),
                 (f'up{u}.label_proj.kernel', (latent, L)), (f'up{u}.label_proj.bias', (L,)),
                 (f'up{u}.upconv.kernel', (pool, c, cout)), (f'up{u}.upconv.bias', (cout,)),
                 (f'up{u}.conv.kernel', (k, 2 * cout, cout)), (f'up{u}.conv.bias', (cout,)),
                 (f'up{u}.res.kernel', (1, 2 * cout, cout)), (f'up{u}.res.bias', (cout,))]
        cin = cout
    spec += [('final.kernel', (1, f, n_out)), ('final.bias', (n_out,))]
    return spec


def glorot_uniform_init(spec, seed=1234, bias_scale=0.0, final_scale=1.0):
    """Keras defaults (glorot_uniform kernels, zero biases), seeded like networks.py:15-17.

    ``bias_scale`` > 0 draws U(-bias_scale, bias_scale) biases (exercises the bias
    paths in parity tests); ``final_scale`` scales the final 1x1 conv.
    """
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in spec:
        if name.endswith('.kernel'):
            if len(shape) == 3:
                fan_in, fan_out = shape[0] * shape[1], shape[0] * shape[2]
            else:
                fan_in, fan_out = shape
            lim = np.sqrt(6.0 / (fan_in + fan_out))
            w = rng.uniform(-lim, lim, shape)
            if name.startswith('final.'):
                w = w * final_scale
        else:
            w = rng.uniform(-bias_scale, bias_scale, shape) if bias_scale > 0 else np.zeros(shape)
        out[name] = w.astype(NP_DTYPE)
    return out


def denoiser_init(spec, seed=1234, perturb=0.1, bias_scale=0.0, v_perturb=None):
    """Synthetic weights that behave like a trained eps-predictor (bounded 1000-step chain).

    An untrained Glorot net predicts eps ~ 0, and at t = 999 the eps
    parameterisation then gives x0 = x / sqrt(alpha_bar) = 2e4 x
    (diffusion_model.py:370-374): the reverse chain diverges.  Here an exact
    identity path is embedded on top of Glorot weights:
    down0 channels 0-3 = relu(+-x) (centre tap), up2 ConvBlock channels 0-3 copy
    them from the skip, and the final 1x1 conv maps them back to eps = x.  All
    other final-conv rows are scaled by ``perturb`` so the rest of the network
    (condition, time, all levels) perturbs eps and v by a small amount.
    ``v_perturb`` (learned variance): scale of the v output rows instead of ``perturb``
    (1.0 = the full Glorot network drives the log-variance interpolation).
    """
    w = glorot_uniform_init(spec, seed=seed, bias_scale=bias_scale)
    names = dict(spec)
    n_out = names['final.kernel'][2]
    n_par = n_out // 2 if n_out == 4 else n_out
    xo = names['down0.conv.kernel'][1] - n_par          # first x channel of the down0 concat
    k = w['down0.conv.kernel']
    k[:, :, :2 * n_par] = 0.0
    w['down0.res.kernel'][:, :, :2 * n_par] = 0.0
    w['down0.conv.bias'][:2 * n_par] = 0.0
    w['down0.res.bias'][:2 * n_par] = 0.0
    ctr = (k.shape[0] - 1) // 2
    for p in range(n_par):
        k[ctr, xo + p, 2 * p] = 1.0
        k[ctr, xo + p, 2 * p + 1] = -1.0
    up = [n for n in names if n.startswith('up') and n.endswith('.conv.kernel')]
    last = sorted(up)[-1].split('.')[0]
    k = w[last + '.conv.kernel']
    k[:, :, :2 * n_par] = 0.0
    w[last + '.res.kernel'][:, :, :2 * n_par] = 0.0
    w[last + '.conv.bias'][:2 * n_par] = 0.0
    w[last + '.res.bias'][:2 * n_par] = 0.0
    for c in range(2 * n_par):
        k[ctr, c, c] = 1.0
    f = w['final.kernel']
    if v_perturb is not None and n_out == 2 * n_par:
        f[..., :n_par] *= perturb
        f[..., n_par:] *= v_perturb
    else:
        f *= perturb
    f[0, :2 * n_par, :] = 0.0
    for p in range(n_par):
        f[0, 2 * p, p] = 1.0
        f[0, 2 * p + 1, p] = -1.0
    return w


class UnetConditional:
    """Conditional U-Net plugin (networks.py:718-1093), weights + config only."""

    def __init__(self, num_filt_start=64, pool_size=2, depth=5, block_type='conv', block_params=None,
                 skip_conn_type='concat', skip_conn_op=None, skip_conn_post_op=None, dropout=None,
                 final_activation=None, cond_params=None, resize_input_len=None, resize_input_type='dense',
                 constrained_func_output=None, sin_emb_dim=None, normalize_feature_dict=None,
                 normalize_label_dict=None, learn_variance=None, pool_type='max', num_channels_out=None,
                 seed=1234, **kwargs):
        self.num_filt_start = num_filt_start
        self.pool_size = pool_size
        self.depth = depth
        self.block_type = block_type
        self.block_params = dict(block_params or {})
        self.skip_conn_type = skip_conn_type
        self.dropout = dropout
        self.final_activation = final_activation
        self.sin_emb_dim = sin_emb_dim
        self.learn_variance = learn_variance or ''
        self.flag_learn_var = 'learn' in self.learn_variance.lower()
        self.cond_params = cond_params if isinstance(cond_params, dict) else {
            'network_name': 'encoder', 'flag_flatten_input': True,
            'network_kwargs': {'enc_size': [256, 128, 64], 'latent_dim': 32}}
        self.seed = seed
        nk = self.cond_params.get('network_kwargs', {})
        unsupported = []
        if (num_filt_start, pool_size, depth, block_type, skip_conn_type, sin_emb_dim) != (
                128, 2, 4, 'conv', 'concat', 64):
            unsupported.append('U-Net geometry')
        if self.block_params.get('kernel_size', 3) != 6 or not self.block_params.get('flag_res', True):
            unsupported.append('block_params')
        if self.block_params.get('norm_list') or self.block_params.get('activation', 'relu') != 'relu' \
                or self.block_params.get('num_convs', 1) != 1:
            unsupported.append('ConvBlock normalisation/activation')
        if self.cond_params.get('network_name', 'encoder').lower() not in 'encoder' or \
                self.cond_params.get('flag_flatten_input', True) or \
                list(nk.get('enc_size', [])) != [256, 128, 64] or nk.get('latent_dim') != 32 or \
                nk.get('final_activation', None) is not None or nk.get('activation', 'relu') != 'relu':
            unsupported.append('cond_params')
        if dropout is not None or final_activation is not None or resize_input_len is not None or \
                constrained_func_output is not None or skip_conn_op is not None or \
                skip_conn_post_op is not None or normalize_feature_dict or normalize_label_dict or \
                'max' not in pool_type.lower():
            unsupported.append('optional branches')
        if unsupported:
            raise NotImplementedError('libpetdiff compiles only the shipped UnetConditional '
                                      '(main_script.py:131-167); unsupported: ' + ', '.join(unsupported))
        self.ndim = None
        self.weights = None
        self.n_out = None

    # Keras Layer.build equivalent (networks.py:781-992)
    def build(self, input_shape):
        if len(input_shape) != 3:
            raise NotImplementedError('only 1-D inputs (B, n_roi, n_par) are supported')
        self.ndim = len(input_shape) - 2
        self.input_shape = tuple(input_shape)
        self.n_roi, self.n_par = int(input_shape[1]), int(input_shape[2])
        if (self.n_roi, self.n_par) != (48, 2):
            raise NotImplementedError('kernels are compiled for x of shape (B, 48, 2)')
        self.n_out = 2 * self.n_par if self.flag_learn_var else self.n_par
        if self.weights is None:
            self.weights = denoiser_init(self.spec(), seed=self.seed)
        return self

    def spec(self):
        return param_spec(n_roi=48, n_par=2, n_out=2 * 2 if self.flag_learn_var else 2)

    def count_params(self):
        return int(sum(np.prod(s) for _, s in self.spec()))

    def get_weights(self):
        return [self.weights[n] for n, _ in self.spec()]

    def set_weights(self, weights):
        if isinstance(weights, dict):
            weights = [weights[n] for n, _ in self.spec()]
        spec = self.spec()
        if len(weights) != len(spec):
            raise ValueError(f'expected {len(spec)} arrays, got {len(weights)}')
        new = {}
        for (n, s), w in zip(spec, weights):
            w = np.asarray(w, dtype=NP_DTYPE)
            if tuple(w.shape) != tuple(s):
                raise ValueError(f'{n}: shape {w.shape} != {s}')
            new[n] = w
        self.weights = new

    def flat_weights(self):
        """Contiguous fp32 blob in the order of include/petdiff.h."""
        return np.concatenate([self.weights[n].ravel() for n, _ in self.spec()]).astype(NP_DTYPE)

    def save_weights(self, path):
        """``.npz`` (+ ``.json`` spec), or Keras-layout HDF5 when the path ends in ``.h5`` (h5.save_unet_h5)."""
        if os.fspath(path).endswith('.h5'):
            from .h5 import save_unet_h5
            save_unet_h5(path, self.weights, network_path='')
            return
        np.savez(path, **self.weights)
        with open(os.path.splitext(path)[0] + '.json', 'w') as f:
            json.dump({'spec': [[n, list(s)] for n, s in self.spec()]}, f)

    def load_weights(self, path, strict=True):
        """Weights from this package's .npz, or from a TensorFlow checkpoint of the reference: a SavedModel
        directory (`cp_<epoch>/`, main_script.py:263) or a TensorBundle prefix (`.../variables/variables`),
        read by checkpoint.py without TensorFlow, or a Keras `.weights.h5` file (main_script.py:412), read by
        h5.py without h5py.  ``strict=False`` (h5 only) keeps the current value of every variable the file lacks
        (Keras 3 does not store layers held in nested Python lists, see h5.unet_h5_paths)."""
        path = os.fspath(path)
        if path.endswith('.index'):
            path = path[:-len('.index')]
        if os.path.isdir(path) or os.path.exists(path + '.index'):
            from .checkpoint import load_unet_weights
            self.set_weights(load_unet_weights(path, self.spec()))
            return
        if path.endswith('.h5'):
            from .h5 import load_unet_h5
            got = load_unet_h5(path, self.spec(), strict=strict)
            if not strict and self.weights is not None:
                got = {**self.weights, **got}
            self.set_weights(got)
            return
        with np.load(path, allow_pickle=False) as z:
            self.set_weights({n: z[n] for n, _ in self.spec()})
