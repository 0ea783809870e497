"""Drop-in ``ImprovedDDPM`` sampling API backed by libpetdiff.so (gfx950 HIP).

Mirrors the public sampling surface of the reference's diffusion_model.py
(yanisdjebra/PET_posterior_distribution):

=====================================  ===========================================
reference (file:line)                  here
=====================================  ===========================================
DDPM.__init__ schedule  :85-105        ``ImprovedDDPM.__init__`` (same attributes)
ImprovedDDPM.__init__   :319-357       same (+ ValueError on bad parameterization)
DDPM.call               :141-158       ``call`` / ``__call__`` -> petdiff_forward
ImprovedDDPM.ddpm       :651-663       ``ddpm`` (= ``p_sample``) -> petdiff_p_sample
tfunc_ddpm              :665-668       ``tfunc_ddpm``
ddpm_loop               :670-715       ``ddpm_loop`` (= ``generate``) -> petdiff_generate
tfunc_ddpm_loop         :718-737       ``tfunc_ddpm_loop`` (hipGraph replay)
=====================================  ===========================================

Inputs may be NumPy arrays or torch tensors; outputs are torch tensors on the
sampler's GPU (``keep_all_xt`` returns a NumPy stack, as the reference does at
:712-713).  The network runs in ``dtype``: 'bf16x3' by default -- the reference's fp32
accuracy (1e-4 parity) on the bf16 MFMA kernels, every fp32 operand split hi + lo and
three bf16 products per fp32 product -- or 'bfloat16' / 'float16' (the benchmarked
16-bit networks, about 2.4x faster) or 'float32' (exact-f32 MFMA, 3.7x slower than
'bf16x3'); the p_sample epilogue is always fp32.

Noise: the reference draws ``tf.random.normal`` from TF's stateful Philox.  Here
z is a counter-based Philox4x32-10 normal keyed by (seed, global sample index,
loop step), so results do not depend on batch chunking or on how samples are
sharded over GPUs.  ``z=`` injects explicit noise (used by the parity tests).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from . import _lib
from .helper_func import NP_DTYPE, get_beta_schedule

DTYPE = 'float32'   # dtype of every host-side table and of x (diffusion_model.py:7)


_M64 = (1 << 64) - 1
# noise-stream kinds of the automatically derived seeds (seed=None): p_sample calls, reverse loops
# and test_step draws each get their own Philox key, so no two calls replay each other's noise
STREAM_P_SAMPLE, STREAM_LOOP, STREAM_EVAL = 1, 2, 3


def _mix64(x):
    """splitmix64 finaliser (a bijection of 64-bit words)."""
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def stream_seed(seed, kind, counter=0):
    """Philox key of call ``counter`` of stream ``kind`` under the model seed (distinct model seeds,
    kinds and counters give unrelated keys, unlike seed + counter)."""
    return _mix64(_mix64((int(seed) & _M64) ^ (kind << 56)) ^ (int(counter) & _M64))


def _as_device(x, device, dtype):
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=dtype).contiguous()
    return torch.as_tensor(np.asarray(x), dtype=dtype, device=device).contiguous()


def _stream_ptr(device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


class ImprovedDDPM:
    """iDDPM posterior sampler (diffusion_model.py:317-748, sampling part)."""

    eps_param_name_list = ['eps', 'epsilon']
    x0_param_name_list = ['x0', 'x_0', 'x_start', 'xstart', 'start_x']
    x_prev_param_name_list = ['x_{t-1}', 'x_prev', 'xprev', 'prev_x']
    v_param_name_list = ['v', ]

    def __init__(self, lambda_vlb=0.1, parameterization='eps', timesteps=200, noise_schedule=None,
                 network=None, ndim=None, constrained_func_output_t0=None, dtype='bf16x3', device=None,
                 seed=12345, **kwargs):
        # ---- DDPM.__init__ (diffusion_model.py:79-135) ----
        self.timesteps = timesteps
        self.noise_schedule = noise_schedule
        self.constrained_func_output_t0 = constrained_func_output_t0
        if constrained_func_output_t0 is not None:
            raise NotImplementedError('constrained_func_output_t0 is not supported by the fused kernel')
        ns = noise_schedule or {}
        self.beta_start = ns.get('beta_start', 1e-4)
        self.beta_end = ns.get('beta_end', 2e-2)
        self.offset_s = ns.get('offset_s', 0.008)
        self.max_beta = ns.get('max_beta', 0.999)
        self.schedule_name = ns.get('schedule_name', 'linear') if noise_schedule is not None else 'linear'
        self.beta = get_beta_schedule(self.schedule_name, self.timesteps, beta_start=self.beta_start,
                                      beta_end=self.beta_end, offset_s=self.offset_s, max_beta=self.max_beta)
        self.alpha = 1 - self.beta
        if network is None:
            raise ValueError('Input network is required to create model.')
        self.network = network
        if ndim is not None:
            self.ndim = ndim
        elif getattr(network, 'ndim', None) is not None:
            self.ndim = network.ndim
        elif hasattr(network, 'input_shape'):
            self.ndim = len(network.input_shape) - 2
        else:
            raise AttributeError('``ndim`` was not passed as argument. Could not be retrieved from input '
                                 'network {} (``input_shape`` attribute does not exist).'.format(
                                     type(network).__name__))
        self.reshape_dim = (-1,) + (1,) * (self.ndim + 1)
        self.flag_condition = True
        # ---- ImprovedDDPM.__init__ (diffusion_model.py:319-355) ----
        self.lambda_vlb = lambda_vlb
        self.parameterization = parameterization
        self.all_param_name_list = (self.eps_param_name_list + self.x0_param_name_list +
                                    self.x_prev_param_name_list + self.v_param_name_list)
        if self.parameterization.lower() not in self.all_param_name_list:
            raise ValueError(f'Invalid parameterization (got ``{parameterization}``). '
                             f'Value must be in ``{self.all_param_name_list}``')
        self.learn_variance = network.learn_variance
        self.flag_learn_var = 'learn' in self.learn_variance.lower()
        self.flag_ranged_var = 'ranged' in self.learn_variance.lower()
        self.alpha_bar = np.cumprod(self.alpha, 0, dtype=DTYPE)
        self.alpha_bar_prev = np.concatenate((np.array([1.], dtype=DTYPE), self.alpha_bar[:-1]), axis=0)
        self.sqrt_alpha_bar = np.sqrt(self.alpha_bar, dtype=DTYPE)
        self.sqrt_one_minus_alpha_bar = np.sqrt(1 - self.alpha_bar, dtype=DTYPE)
        self.posterior_variance = self.beta * (1.0 - self.alpha_bar_prev) / (1.0 - self.alpha_bar)
        # the reference's alias (:349-351): element 0 of posterior_variance is overwritten too
        self.posterior_log_variance_clipped = self.posterior_variance
        self.posterior_log_variance_clipped[0] = self.posterior_log_variance_clipped[1]
        self.posterior_log_variance_clipped = np.log(self.posterior_log_variance_clipped)
        self.posterior_mean_coef1 = self.beta * np.sqrt(self.alpha_bar_prev) / (1.0 - self.alpha_bar)
        self.posterior_mean_coef2 = (1.0 - self.alpha_bar_prev) * np.sqrt(self.alpha) / (1.0 - self.alpha_bar)

        self.dtype = {'bfloat16': _lib.DTYPE_BF16, 'bf16': _lib.DTYPE_BF16,
                      'float16': _lib.DTYPE_F16, 'fp16': _lib.DTYPE_F16, 'half': _lib.DTYPE_F16,
                      'float32': _lib.DTYPE_F32, 'fp32': _lib.DTYPE_F32,
                      # fp32-class accuracy on the bf16 MFMA path (hi/lo split, 3 products; petdiff.h)
                      'bf16x3': _lib.DTYPE_BF16X3}[str(dtype)]
        if device is None:
            device = torch.cuda.current_device() if torch.cuda.is_available() else 0
        self.device = torch.device('cuda', device if isinstance(device, int) else torch.device(device).index or 0)
        self.seed = int(seed)
        self._call_counter = 0
        self._last_forward_B = 0
        self._handle = None
        self._cond_cache = None     # (unique-conditions tensor) last sent to the library
        self._cond_cache_host = None  # its host copy when it came from a NumPy condition
        self._inv_cache = None      # (host per-sample index, its device copy)
        self._trainer = None
        self._weights_stale = False
        self.optimizer = None
        self.name = 'improved_ddpm'

    # ------------------------------------------------------------------ setup
    def schedule_tables(self):
        """[NTAB][T] fp32 tables (row order of include/petdiff.h), all NumPy float32 ops."""
        one = NP_DTYPE(1.0)
        c1, c2 = self.posterior_mean_coef1, self.posterior_mean_coef2
        rows = [self.beta, np.log(self.beta), self.posterior_log_variance_clipped, self.posterior_variance,
                c1, c2, self.alpha_bar, self.sqrt_alpha_bar, self.sqrt_one_minus_alpha_bar,
                one / self.sqrt_alpha_bar, np.sqrt(one / self.alpha_bar - one),
                1.0 / c1, c2 / c1]
        return np.ascontiguousarray(np.stack([np.asarray(r, dtype=NP_DTYPE) for r in rows]))

    def _c_config(self):
        """petdiff_config of this model (shipped architecture, schedule length, variance / target)."""
        L = _lib.lib()
        cfg = _lib.PetdiffConfig()
        _lib.check(L.petdiff_default_config(C.byref(cfg)))
        cfg.timesteps = self.timesteps
        lv = self.learn_variance.lower()
        cfg.learn_variance = (_lib.LEARN_RANGED if 'ranged' in lv else _lib.LEARN) if 'learn' in lv \
            else _lib.LEARN_FIXED
        p = self.parameterization.lower()
        cfg.parameterization = (_lib.PARAM_XPREV if p in self.x_prev_param_name_list else
                                _lib.PARAM_X0 if p in self.x0_param_name_list else
                                _lib.PARAM_V if p in self.v_param_name_list else _lib.PARAM_EPS)
        cfg.dtype = self.dtype
        return cfg

    def _ensure_handle(self):
        if self._handle is not None:
            return self._handle
        L = _lib.lib()
        self._sync_trained_weights()
        if self.network.weights is None:
            self.network.build((None, 48, 2))
        cfg = self._c_config()
        blob = self.network.flat_weights()
        h = C.c_void_p()
        torch.cuda.set_device(self.device)
        _lib.check(L.petdiff_create(C.byref(cfg), blob.ctypes.data_as(C.c_void_p), blob.size, self.device.index,
                                    C.byref(h)), 'petdiff_create')
        self._handle = h
        tabs = self.schedule_tables()
        _lib.check(L.petdiff_set_schedule(h, tabs.ctypes.data_as(C.c_void_p), self.timesteps),
                   'petdiff_set_schedule')
        return h

    # ------------------------------------------------------------------ training (8(f) row 4)
    def compile(self, optimizer=None, loss='MeanSquaredError', **kwargs):
        """keras Model.compile as used by the reference (main_script.py:233-234)."""
        from .training import Adam, _Mean
        self._sync_trained_weights()
        name = loss if isinstance(loss, str) else getattr(loss, '__name__', type(loss).__name__)
        if str(name).replace('_', '').lower() not in ('meansquarederror', 'mse'):
            raise NotImplementedError('only the MeanSquaredError loss of the reference is supported')
        self.optimizer = optimizer if optimizer is not None else Adam()
        self.loss_tracker = _Mean('loss')
        self.noise_loss_tracker = _Mean('noise_loss')
        self.lambda_vlb_loss_tracker = _Mean('lambda_vlb_loss')
        self._trainer = None
        self._train_seed = self.seed
        self._eval_calls = 0

    @property
    def metrics(self):
        return [self.loss_tracker, self.noise_loss_tracker, self.lambda_vlb_loss_tracker]

    def _ensure_trainer(self):
        from .training import Trainer
        if getattr(self, 'optimizer', None) is None:
            raise RuntimeError('call compile(optimizer=...) before training')
        if self._trainer is None:
            self._sync_trained_weights()
            self._trainer = Trainer(self, self.optimizer)
        return self._trainer

    def _sync_trained_weights(self):
        """Pull the trainer's weights into network.weights (inference handles re-pack them)."""
        tr = getattr(self, '_trainer', None)
        if tr is None or not getattr(self, '_weights_stale', False):
            return
        blob = tr.weights().cpu().numpy()
        new, o = {}, 0
        for n, sh in self.network.spec():
            k = int(np.prod(sh))
            new[n] = blob[o:o + k].reshape(sh).copy()
            o += k
        self.network.weights = new
        self._weights_stale = False

    def _train_batch(self, data, t, noise, update):
        images, condition = (data[0], data[1]) if isinstance(data, (tuple, list)) else (data, None)
        if condition is None:
            raise NotImplementedError('the shipped UnetConditional requires a condition')
        tr = self._ensure_trainer()
        x0 = _as_device(images, self.device, torch.float32)
        B = x0.shape[0]
        if tuple(x0.shape[1:]) != (48, 2):
            raise ValueError(f'images must be (B, 48, 2), got {tuple(x0.shape)}')
        cond = _as_device(condition, self.device, torch.float32)
        if tuple(cond.shape) != (B, 49, 54):
            raise ValueError(f'condition must be (B, 49, 54), got {tuple(cond.shape)}')
        tt = None if t is None else self._time(t, B)
        nz = None if noise is None else _as_device(noise, self.device, torch.float32)
        if nz is not None and nz.shape != x0.shape:
            raise ValueError('noise must have the shape of images')
        loss = torch.empty(B, dtype=torch.float32, device=self.device)
        if update:
            tr.compute_gradients(x0, cond, tt, nz, seed=self._train_seed, loss=loss)
        else:
            tr.compute_loss(x0, cond, tt, nz, seed=stream_seed(self._train_seed, STREAM_EVAL),
                            sample_offset=self._eval_calls << 32, loss=loss)
            self._eval_calls += 1
        if update:
            tr.apply_gradients(1.0)
            self._weights_stale = True
            self.close()
        mean_loss, noise_loss, mean_vlb = tr.last_stats()
        self.loss_tracker.update_state(mean_loss * B, B)
        self.noise_loss_tracker.update_state(noise_loss, 1)
        self.lambda_vlb_loss_tracker.update_state(mean_vlb * B, B)
        self.last_loss = loss
        return {m.name: m.result() for m in self.metrics}

    def train_step(self, data, t=None, noise=None):
        """ImprovedDDPM.train_step (diffusion_model.py:533-598): one Adam step on (images, condition).
        ``t`` / ``noise`` inject the draws (else counter-based Philox)."""
        return self._train_batch(data, t, noise, update=True)

    def test_step(self, data, t=None, noise=None):
        """ImprovedDDPM.test_step (diffusion_model.py:600-640): loss only (no backward pass), with
        fresh draws per call like the reference's tf.random: its own stream (STREAM_EVAL), and call k
        at sample offset k * 2^32."""
        return self._train_batch(data, t, noise, update=False)

    def fit(self, x=None, y=None, batch_size=32, epochs=1, validation_split=0.0, shuffle=True, verbose=0,
            callbacks=None, **kwargs):
        """keras Model.fit as the reference calls it (main_script.py:267-271): per epoch, shuffled
        batches through train_step, then test_step over the held-out validation tail.  ``callbacks``
        follow the Keras protocol the reference's WeightsCheckpoint uses (networks.py:152-180):
        set_model / on_train_begin / on_epoch_end(epoch, logs) / on_train_end, and a callback may set
        ``model.stop_training``.  ``verbose`` prints one line per epoch."""
        callbacks = list(callbacks or [])
        self.stop_training = False
        for cb in callbacks:
            if hasattr(cb, 'set_model'):
                cb.set_model(self)
            else:
                cb.model = self
            if hasattr(cb, 'on_train_begin'):
                cb.on_train_begin({})
        x = np.asarray(x, dtype=np.float32) if not isinstance(x, torch.Tensor) else x
        y = np.asarray(y, dtype=np.float32) if not isinstance(y, torch.Tensor) else y
        n = x.shape[0]
        n_val = int(n * validation_split)
        n_tr = n - n_val
        xd = _as_device(x, self.device, torch.float32)
        yd = _as_device(y, self.device, torch.float32)
        rng = np.random.default_rng(self.seed)
        history = {m.name: [] for m in self.metrics}
        if n_val:
            history.update({'val_' + m.name: [] for m in self.metrics})
        for epoch in range(epochs):
            if self.stop_training:
                break
            for m in self.metrics:
                m.reset_state()
            order = rng.permutation(n_tr) if shuffle else np.arange(n_tr)
            for s in range(0, n_tr, batch_size):
                idx = torch.as_tensor(order[s:s + batch_size], device=self.device)
                self.train_step((xd[idx], yd[idx]))
            for m in self.metrics:
                history[m.name].append(m.result())
            if n_val:
                for m in self.metrics:
                    m.reset_state()
                for s in range(n_tr, n, batch_size):
                    self.test_step((xd[s:min(s + batch_size, n)], yd[s:min(s + batch_size, n)]))
                for m in self.metrics:
                    history['val_' + m.name].append(m.result())
            logs = {k: v[-1] for k, v in history.items()}
            if verbose:
                print(f'epoch {epoch + 1}/{epochs} ' + ' '.join(f'{k} {v:.5g}' for k, v in logs.items()),
                      flush=True)
            for cb in callbacks:
                if hasattr(cb, 'on_epoch_end'):
                    cb.on_epoch_end(epoch, logs)
        for cb in callbacks:
            if hasattr(cb, 'on_train_end'):
                cb.on_train_end({})
        return history

    def load_weights(self, path, strict=True):
        """diff_model.load_weights (main_script.py:412): the network's weights from an .npz, a SavedModel /
        TensorBundle checkpoint or a Keras ``.weights.h5`` of this model (group ``network``)."""
        self._sync_trained_weights()
        self.network.load_weights(path, strict=strict)
        self._trainer = None
        self.close()

    def save_weights(self, path):
        """model.save_weights as WeightsCheckpoint calls it (networks.py:176): ``.h5`` writes the Keras layout
        with the network under ``network/`` (h5.save_unet_h5), anything else this package's .npz."""
        self._sync_trained_weights()
        if os.fspath(path).endswith('.h5'):
            from .h5 import save_unet_h5
            save_unet_h5(path, self.network.weights, network_path='network')
        else:
            self.network.save_weights(path)

    def close(self):
        if self._handle is not None:
            _lib.lib().petdiff_destroy(self._handle)
            self._handle = None
            self._cond_cache = None
            self._cond_cache_host = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _conditions(self, condition, B, tac=None):
        """Deduplicate conditions -> (per-sample index tensor or None).

        The reference feeds np.repeat(y_obs, B) (main_script.py:419); the kernels
        fold each UNIQUE condition once (encoder + label maps) and index it per sample.
        With ``tac`` given, ``condition`` is the (n_tac, 49, 54) table and tac[b] the
        row of sample b (no deduplication).
        """
        h = self._ensure_handle()
        if condition is None:
            raise NotImplementedError('the shipped UnetConditional requires a condition')
        if not isinstance(condition, torch.Tensor) and not isinstance(tac, torch.Tensor):
            return self._conditions_host(h, condition, B, tac)
        cond = _as_device(condition, self.device, torch.float32)
        if cond.dim() == 2:
            cond = cond[None]
        if cond.shape[1:] != (49, 54):
            raise ValueError(f'condition must be (B, 49, 54), got {tuple(cond.shape)}')
        if tac is not None:
            inv = _as_device(tac, self.device, torch.int32).reshape(-1)
            if inv.numel() != B:
                raise ValueError('tac must have one entry per sample')
            if B and (int(inv.min()) < 0 or int(inv.max()) >= cond.shape[0]):
                raise ValueError('tac index out of range')
            uniq = cond.contiguous()
            if cond.shape[0] == 1:
                inv = None               # one condition: the kernels' single-condition path
        elif cond.shape[0] != B and cond.shape[0] != 1:
            raise ValueError(f'condition batch {cond.shape[0]} != x batch {B}')
        elif cond.shape[0] == 1 or bool((cond == cond[:1]).all()):
            uniq, inv = cond[:1].contiguous(), None
        else:
            uniq, inv = torch.unique(cond.reshape(cond.shape[0], -1), dim=0, return_inverse=True)
            uniq = uniq.reshape(-1, 49, 54).contiguous()
            inv = inv.to(torch.int32).contiguous()
        if self._cond_cache is None or self._cond_cache.shape != uniq.shape or \
                not torch.equal(self._cond_cache, uniq):
            _lib.check(_lib.lib().petdiff_set_conditions(h, _ptr(uniq), uniq.shape[0], _stream_ptr(self.device)),
                       'petdiff_set_conditions')
            # a private copy: the caller may update its condition buffer in place between calls
            self._cond_cache = uniq.clone()
            self._cond_cache_host = None
        return inv, uniq.shape[0]

    def _conditions_host(self, h, condition, B, tac):
        """_conditions for host (NumPy) inputs: validation, deduplication and the comparison with the
        last condition set all run on the host, and the device copies of the unique conditions and of
        the per-sample index are reused while their contents repeat, so a repeated call issues no copy
        that would wait for the GPU work queued before it (a pageable host-to-device copy does)."""
        c = np.ascontiguousarray(np.asarray(condition, dtype=np.float32))
        if c.ndim == 2:
            c = c[None]
        if c.shape[1:] != (49, 54):
            raise ValueError(f'condition must be (B, 49, 54), got {tuple(c.shape)}')
        if tac is not None:
            inv = np.ascontiguousarray(np.asarray(tac).reshape(-1).astype(np.int32))
            if inv.size != B:
                raise ValueError('tac must have one entry per sample')
            if B and (int(inv.min()) < 0 or int(inv.max()) >= c.shape[0]):
                raise ValueError('tac index out of range')
            uniq = c
            if c.shape[0] == 1:
                inv = None               # one condition: the kernels' single-condition path
        elif c.shape[0] != B and c.shape[0] != 1:
            raise ValueError(f'condition batch {c.shape[0]} != x batch {B}')
        elif c.shape[0] == 1 or bool((c == c[:1]).all()):
            uniq, inv = c[:1], None
        else:
            uniq, inv = np.unique(c.reshape(c.shape[0], -1), axis=0, return_inverse=True)
            uniq = np.ascontiguousarray(uniq.reshape(-1, 49, 54))
            inv = np.ascontiguousarray(inv.reshape(-1).astype(np.int32))
        hc = getattr(self, '_cond_cache_host', None)
        if self._cond_cache is None or hc is None or hc.shape != uniq.shape or not np.array_equal(hc, uniq):
            dev = torch.as_tensor(uniq, device=self.device)
            _lib.check(_lib.lib().petdiff_set_conditions(h, _ptr(dev), uniq.shape[0], _stream_ptr(self.device)),
                       'petdiff_set_conditions')
            self._cond_cache = dev
            self._cond_cache_host = uniq.copy()
        if inv is None:
            return None, uniq.shape[0]
        ic = getattr(self, '_inv_cache', None)
        if ic is None or ic[0].shape != inv.shape or not np.array_equal(ic[0], inv):
            self._inv_cache = ic = (inv.copy(), torch.as_tensor(inv, device=self.device))
        return ic[1], uniq.shape[0]

    def _time(self, time, B):
        t = _as_device(time, self.device, torch.int32).reshape(-1)
        if t.numel() == 1 and B != 1:
            t = t.expand(B).contiguous()
        if t.numel() != B:
            raise ValueError('time must have one entry per sample')
        if B and (int(t.min()) < 0 or int(t.max()) >= self.timesteps):
            raise ValueError(f'time must be in [0, {self.timesteps})')
        return t

    # ------------------------------------------------------------------ API
    def call(self, inputs, training=False, **kwargs):
        """DDPM.call (diffusion_model.py:141-158): raw network output (B, 48, n_out)."""
        x = _as_device(inputs['x'], self.device, torch.float32)
        B = x.shape[0]
        t = self._time(inputs.get('time'), B)
        tac, _ = self._conditions(inputs.get('condition'), B)
        out = torch.empty((B, x.shape[1], self.network.n_out), dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().petdiff_forward(self._handle, _ptr(x), _ptr(t), _ptr(tac), _ptr(out), B,
                                              _stream_ptr(self.device)), 'petdiff_forward')
        self._last_forward_B = B
        return out

    __call__ = call

    def ddpm(self, x_t, time, condition=None, z=None, seed=None, sample_offset=0, rng_step=None):
        """ImprovedDDPM.ddpm = p_sample (diffusion_model.py:651-663) -> (mean, var, var_tilde)."""
        x = _as_device(x_t, self.device, torch.float32)
        B = x.shape[0]
        t = self._time(time, B)
        tac, _ = self._conditions(condition, B)
        zt = None if z is None else _as_device(z, self.device, torch.float32)
        if zt is not None and zt.shape != x.shape:
            raise ValueError('z must have the shape of x_t')
        if seed is None:
            seed = stream_seed(self.seed, STREAM_P_SAMPLE)
        if rng_step is None:
            rng_step = self._call_counter & 0x7FFFFFFF
            self._call_counter += 1
        mean = torch.empty_like(x)
        var = torch.empty_like(x)
        var_tilde = torch.empty_like(x)
        _lib.check(_lib.lib().petdiff_p_sample(
            self._handle, _ptr(x), _ptr(t), _ptr(tac), _ptr(zt), int(seed),
            int(sample_offset), int(rng_step), _ptr(mean), _ptr(var), _ptr(var_tilde), B,
            _stream_ptr(self.device)), 'petdiff_p_sample')
        self._last_forward_B = B
        return mean, var, var_tilde

    p_sample = ddpm

    def level_outputs(self, B=None):
        """fp32 copies of the per-level ConvBlock outputs of the last call / ddpm (networks.py:1010-1072):
        {'down0': (B, 48, 128), ..., 'down3': (B, 6, 1024), 'up0': (B, 12, 512), 'up1': (B, 24, 256)}."""
        h = self._ensure_handle()
        out = {}
        for lv, (name, (L, C_)) in enumerate(zip(_lib.LEVEL_NAMES, _lib.LEVEL_SHAPES)):
            n = B if B is not None else self._last_forward_B
            buf = torch.empty((n, L, C_), dtype=torch.float32, device=self.device)
            _lib.check(_lib.lib().petdiff_get_activation(h, lv, _ptr(buf), n, _stream_ptr(self.device)),
                       'petdiff_get_activation')
            out[name] = buf
        return out

    def tfunc_ddpm(self, x_t, time, condition=None, **kwargs):
        """diffusion_model.py:665-668."""
        return self.ddpm(x_t, time, condition, **kwargs)

    def sub_sequence(self, num_timesteps=None, sub_sequence_type='linear'):
        """Index list of ddpm_loop (diffusion_model.py:680-691, same substring semantics)."""
        if num_timesteps in (None, 0, self.timesteps):
            return list(range(self.timesteps))[::-1]
        if sub_sequence_type in 'linear':
            return np.linspace(0, self.timesteps - 1, num=num_timesteps, dtype=np.int32)[::-1].tolist()
        if sub_sequence_type in 'quadratic':
            return (np.linspace(0, np.sqrt(self.timesteps - 1), num=num_timesteps,
                                dtype=np.int32)[::-1] ** 2).tolist()
        raise ValueError('Subsequence type not recognized (given {})'.format(sub_sequence_type))

    def ddpm_loop(self, x_T, condition, num_timesteps=None, sub_sequence_type='linear', flag_var_tilde=True,
                  keep_all_xt=False, z=None, seed=None, sample_offset=0, use_graph=True, tac=None):
        """ImprovedDDPM.ddpm_loop = generate (diffusion_model.py:670-715).

        Extra keywords: ``z`` injected noise (n_steps, B, 48, 2); ``seed`` /
        ``sample_offset`` select the counter-based noise stream (global index of
        sample b is sample_offset + b); ``use_graph`` replays the whole loop as one
        captured hipGraph; ``tac`` indexes a (n_tac, 49, 54) condition table per sample.
        """
        indices = self.sub_sequence(num_timesteps, sub_sequence_type)
        x = _as_device(x_T, self.device, torch.float32)
        B = x.shape[0]
        tac, _ = self._conditions(condition, B, tac)
        n = len(indices)
        zt = None if z is None else _as_device(z, self.device, torch.float32)
        if zt is not None and tuple(zt.shape) != (n,) + tuple(x.shape):
            raise ValueError('z must be (n_steps,) + x_T.shape')
        all_xt = torch.empty((n,) + tuple(x.shape), dtype=torch.float32, device=self.device) \
            if keep_all_xt else None
        out = torch.empty_like(x)
        tseq = np.ascontiguousarray(np.asarray(indices, dtype=np.int32))
        if seed is None:
            seed = stream_seed(self.seed, STREAM_LOOP, self._call_counter)
            self._call_counter += 1
        # batches above PETDIFF_MAX_BATCH run as chunks (main_script.py:414-427 chunks the same way);
        # sample b of chunk c is global sample sample_offset + c0 + b, so the noise is unchanged
        for c0 in range(0, B, _lib.MAX_BATCH):
            c1 = min(B, c0 + _lib.MAX_BATCH)
            whole = c0 == 0 and c1 == B
            xc = x if whole else x[c0:c1].contiguous()
            tc = tac if (whole or tac is None) else tac[c0:c1].contiguous()
            zc = zt if (whole or zt is None) else zt[:, c0:c1].contiguous()
            oc = out if whole else torch.empty_like(xc)
            ac = all_xt if (whole or all_xt is None) else torch.empty((n,) + tuple(xc.shape), dtype=torch.float32,
                                                                      device=self.device)
            _lib.check(_lib.lib().petdiff_generate(
                self._handle, _ptr(xc), _ptr(tc), tseq.ctypes.data_as(C.c_void_p), n, int(bool(flag_var_tilde)),
                _ptr(zc), int(seed), int(sample_offset) + c0, _ptr(oc), _ptr(ac), c1 - c0, int(bool(use_graph)),
                _stream_ptr(self.device)), 'petdiff_generate')
            if not whole:
                out[c0:c1] = oc
                if all_xt is not None:
                    all_xt[:, c0:c1] = ac
        if keep_all_xt:
            return all_xt.cpu().numpy()
        return out

    generate = ddpm_loop

    def tfunc_ddpm_loop(self, x_T, condition, **kwargs):
        """diffusion_model.py:718-737: full-T loop, var_tilde, one captured graph.

        Unlike ddpm_loop (:697-699), the reference passes ``condition`` to the network unchanged
        (no tf.repeat), so its batch must equal x_T's; a mismatch raises ValueError here."""
        B = int(x_T.shape[0])
        cb = 1 if np.ndim(condition) == 2 else int(condition.shape[0])
        if cb != B:
            raise ValueError(f'tfunc_ddpm_loop: condition batch {cb} != x_T batch {B} '
                             '(the reference does not broadcast the condition here)')
        return self.ddpm_loop(x_T, condition, num_timesteps=None, flag_var_tilde=True, use_graph=True, **kwargs)

    def philox_normal(self, B, seed=None, sample_offset=0, rng_step=0x7fffffff):
        """x_T ~ N(0,1) (B, 48, 2) from the counter-based stream: sample b is global sample
        sample_offset + b, so shards of one run reproduce the unsharded draw exactly."""
        h = self._ensure_handle()
        out = torch.empty((B, 48, 2), dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().petdiff_philox_normal(h, self.seed if seed is None else int(seed), int(sample_offset),
                                                    int(rng_step), _ptr(out), B, _stream_ptr(self.device)),
                   'petdiff_philox_normal')
        return out

    # ---------------------------------------------------------- summaries
    def posterior_stats(self, x0, tac=None, n_tac=1):
        """Per (condition, ROI, param) count/mean/M2 (fp64) of samples x0 (main_script.py:433-436)."""
        h = self._ensure_handle()
        x = _as_device(x0, self.device, torch.float32)
        tac_t = None if tac is None else _as_device(tac, self.device, torch.int32)
        stats = np.zeros((n_tac, x.shape[1], x.shape[2], 3), dtype=np.float64)
        _lib.check(_lib.lib().petdiff_posterior_stats(h, _ptr(x), _ptr(tac_t), x.shape[0], n_tac,
                                                      stats.ctypes.data_as(C.c_void_p),
                                                      _stream_ptr(self.device)), 'petdiff_posterior_stats')
        return stats

    # ---------------------------------------------------------- timing
    def set_kernel_timing(self, enable=True, reps=1):
        """Per-layer HIP-event timing of eager launches; reps > 1 repeats every timed launch back to
        back (the kernels are idempotent), so the events' queue gap is amortised over reps launches."""
        _lib.check(_lib.lib().petdiff_set_timing(self._ensure_handle(), int(reps) if enable else 0))

    def get_kernel_timing(self):
        ms = (C.c_float * _lib.NUM_LAYERS)()
        cnt = (C.c_int * _lib.NUM_LAYERS)()
        _lib.check(_lib.lib().petdiff_get_timing(self._handle, ms, cnt))
        return {name: (float(ms[i]), int(cnt[i])) for i, name in enumerate(_lib.LAYER_NAMES)}


def summarize_stats(stats):
    """{count, mean, M2} -> per-ROI mean / population std dicts (main_script.py:433-436)."""
    cnt, mean, m2 = stats[..., 0], stats[..., 1], stats[..., 2]
    std = np.sqrt(m2 / np.maximum(cnt, 1))
    return {'mean_DVR': mean[..., 0], 'mean_R1': mean[..., 1], 'std_DVR': std[..., 0], 'std_R1': std[..., 1]}
