"""Training step of the iDDPM denoiser on MI355X.

Mirrors the reference's training surface (yanisdjebra/PET_posterior_distribution):

================================================  ==========================================
reference (file:line)                             here
================================================  ==========================================
keras.optimizers.Adam(learning_rate, clipnorm)    ``Adam`` (main_script.py:233)
keras.optimizers.schedules.ExponentialDecay       ``ExponentialDecay`` (main_script.py:189-192)
diff_model.compile(optimizer, loss='MeanSq...')   ``ImprovedDDPM.compile``
ImprovedDDPM.train_step   diffusion_model.py:533   ``ImprovedDDPM.train_step`` -> pettrain_step
ImprovedDDPM.test_step    diffusion_model.py:600   ``ImprovedDDPM.test_step``
diff_model.fit(x, y, batch_size, epochs, ...)     ``ImprovedDDPM.fit`` (main_script.py:267-271)
================================================  ==========================================

The step runs in libpetdiff.so (include/pettrain.h): fp32 U-Net forward and
backward (rocBLAS GEMMs + HIP kernels), loss = MSE + lambda_vlb * VLB, per-variable
clip and Adam.  There is no CPU path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib


class ExponentialDecay:
    """keras.optimizers.schedules.ExponentialDecay (staircase=False)."""

    def __init__(self, initial_learning_rate, decay_steps, decay_rate, staircase=False, name=None):
        if staircase:
            raise NotImplementedError('staircase=True is not supported')
        if decay_steps <= 0:
            raise ValueError('decay_steps must be > 0')
        self.initial_learning_rate = float(initial_learning_rate)
        self.decay_steps = float(decay_steps)
        self.decay_rate = float(decay_rate)

    def __call__(self, step):
        return self.initial_learning_rate * self.decay_rate ** (step / self.decay_steps)


class Adam:
    """keras.optimizers.Adam with the arguments the reference uses (clipnorm per variable)."""

    def __init__(self, learning_rate=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7, clipnorm=None, **kwargs):
        if kwargs.get('clipvalue') is not None or kwargs.get('global_clipnorm') is not None or \
                kwargs.get('amsgrad') or kwargs.get('weight_decay'):
            raise NotImplementedError('only learning_rate / betas / epsilon / clipnorm are supported')
        self.learning_rate = learning_rate
        self.beta_1, self.beta_2, self.epsilon = float(beta_1), float(beta_2), float(epsilon)
        self.clipnorm = clipnorm

    def c_config(self, lambda_vlb):
        cfg = _lib.PettrainConfig()
        lr = self.learning_rate
        if isinstance(lr, ExponentialDecay):
            cfg.learning_rate, cfg.decay_steps, cfg.decay_rate = lr.initial_learning_rate, lr.decay_steps, \
                lr.decay_rate
        else:
            cfg.learning_rate, cfg.decay_steps, cfg.decay_rate = float(lr), 1.0, 1.0
        cfg.beta_1, cfg.beta_2, cfg.epsilon = self.beta_1, self.beta_2, self.epsilon
        cfg.clipnorm = float(self.clipnorm) if self.clipnorm else 0.0
        cfg.lambda_vlb = float(lambda_vlb)
        return cfg


class _Mean:
    """keras.metrics.Mean: running mean of every value passed to update_state."""

    def __init__(self, name):
        self.name = name
        self.reset_state()

    def update_state(self, total, count):
        self.total += float(total)
        self.count += float(count)

    def result(self):
        return self.total / self.count if self.count else 0.0

    def reset_state(self):
        self.total = 0.0
        self.count = 0.0


class WeightsCheckpoint:
    """networks.WeightsCheckpoint (networks.py:152-180): every ``every_n_epochs`` epochs save the
    model's weights to ``root_dir/cp_<epoch>/<filename>``, by default the reference's
    ``ckpt.weights.h5`` (Keras HDF5 with the network under ``network/``, the layout
    ``ImprovedDDPM.save_weights`` writes and ``load_weights`` reads, main_script.py:412); another
    extension writes this package's .npz."""

    def __init__(self, root_dir, every_n_epochs=1, filename='ckpt.weights.h5', overwrite=True):
        self.root_dir = root_dir
        self.every_n_epochs = int(every_n_epochs)
        self.filename = filename
        self.overwrite = overwrite
        self.model = None

    def set_model(self, model):
        self.model = model

    def on_epoch_end(self, epoch, logs=None):
        import os
        if (epoch + 1) % self.every_n_epochs != 0:
            return
        sub = os.path.join(self.root_dir, f'cp_{epoch + 1}')
        os.makedirs(sub, exist_ok=True)
        path = os.path.join(sub, self.filename)
        if not self.overwrite and os.path.exists(path):
            return
        self.model.save_weights(path)


def check(rc, what):
    if rc == 0:
        return
    msg = _lib.lib().pettrain_last_error().decode(errors='replace')
    if rc == _lib.PETDIFF_ERR_INVALID:
        raise ValueError(f'{what}: {msg}')
    if rc == _lib.PETDIFF_ERR_UNSUPPORTED:
        raise NotImplementedError(f'{what}: {msg}')
    raise _lib.PetdiffError(f'{what}: {msg}')


class Trainer:
    """Owns one pettrain handle (fp32 weights, gradients, Adam moments on the GPU)."""

    def __init__(self, model, optimizer):
        self.model = model
        self.device = model.device
        net = model.network
        if net.weights is None:
            net.build((None, 48, 2))
        cfg = model._c_config()
        blob = net.flat_weights()
        tabs = model.schedule_tables()
        self.opt_cfg = optimizer.c_config(model.lambda_vlb)
        h = C.c_void_p()
        torch.cuda.set_device(self.device)
        check(_lib.lib().pettrain_create(C.byref(cfg), blob.ctypes.data_as(C.c_void_p), blob.size,
                                         tabs.ctypes.data_as(C.c_void_p), model.timesteps, C.byref(self.opt_cfg),
                                         self.device.index, C.byref(h)), 'pettrain_create')
        self.handle = h
        self.n_weights = blob.size

    def close(self):
        if self.handle is not None:
            _lib.lib().pettrain_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def iterations(self):
        return int(_lib.lib().pettrain_iterations(self.handle))

    def compute_gradients(self, x0, cond, t=None, noise=None, seed=0, sample_offset=0, loss=None):
        B = x0.shape[0]
        st = _stream(self.device)
        check(_lib.lib().pettrain_compute_gradients(self.handle, _p(x0), _p(cond), B, _p(t), _p(noise), int(seed),
                                                    int(sample_offset), _p(loss), st), 'pettrain_compute_gradients')

    def compute_loss(self, x0, cond, t=None, noise=None, seed=0, sample_offset=0, loss=None):
        """Forward + loss only (test_step): the gradient blob is left untouched."""
        B = x0.shape[0]
        st = _stream(self.device)
        check(_lib.lib().pettrain_compute_loss(self.handle, _p(x0), _p(cond), B, _p(t), _p(noise), int(seed),
                                               int(sample_offset), _p(loss), st), 'pettrain_compute_loss')

    def apply_gradients(self, grad_scale=1.0):
        st = _stream(self.device)
        check(_lib.lib().pettrain_apply_gradients(self.handle, float(grad_scale), st), 'pettrain_apply_gradients')

    def gradients(self):
        """Copy of the raw gradient blob (n_weights fp32, petdiff.h order) as a CUDA tensor."""
        g = torch.empty(self.n_weights, dtype=torch.float32, device=self.device)
        check(_lib.lib().pettrain_get_gradients(self.handle, _p(g), _stream(self.device)), 'pettrain_get_gradients')
        return g

    def set_gradients(self, g):
        """Replace the gradient blob (e.g. after an RCCL all-reduce across data-parallel ranks)."""
        g = g.to(device=self.device, dtype=torch.float32).contiguous()
        if g.numel() != self.n_weights:
            raise ValueError('gradient blob size mismatch')
        check(_lib.lib().pettrain_set_gradients(self.handle, _p(g), _stream(self.device)), 'pettrain_set_gradients')

    def last_stats(self):
        out = np.zeros(3, np.float64)
        st = _stream(self.device)
        check(_lib.lib().pettrain_last_stats(self.handle, out.ctypes.data_as(C.c_void_p), st), 'pettrain_last_stats')
        return out

    def weights(self):
        w = torch.empty(self.n_weights, dtype=torch.float32, device=self.device)
        st = _stream(self.device)
        check(_lib.lib().pettrain_get_weights(self.handle, _p(w), st), 'pettrain_get_weights')
        return w


def _p(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream(device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
