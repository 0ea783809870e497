"""Metropolis-Hastings baseline of the reference (mcmc.py) as a GPU sampler.

``MetropolisSRTM2`` holds one test TAC's problem (mcmc.py:73-137: frame times,
reference TAC, fixed k2', observed y = tac_noisy / dt, noise sigmas, MvNormal
priors) and runs many independent chains of PyMC 5.12's element-wise
Metropolis(NormalProposal) with tune_interval = 100 on the GPU (shuffled
element order per draw, ratios against the sweep-start point as in pymc's
``Metropolis.astep``) (one wavefront per
chain, include/petmh.h).  Draws are reduced on the device to Welford partials;
``run`` returns the pooled posterior mean / population std per ROI (the
quantities the reference compares against iDDPM, main_script.py:719-805).
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np
import torch

from . import _lib
from .distributed import merge_stats


class CreateTAC_SRTM2:
    """The MH model's SRTM2 forward op (mcmc.py:27-39), without PyTensor (absent here): (DVR (n_roi,),
    R1 (n_roi,), k2p scalar) -> the (n_roi, 54) fp64 TAC, computed by ``k_srtm`` (kinetic_model.SRTM2, the
    GPU SRTM2 kernel).  ``perform`` keeps the Op's calling convention (outputs[0][0] = the TAC); the
    samplers below evaluate the same model inside their kernels and do not call it."""
    __props__ = ()
    itypes = ('dvector', 'dvector', 'dscalar')
    otypes = ('dmatrix',)

    def __init__(self, k_srtm):
        self.k_srtm = k_srtm

    def perform(self, node, inputs, outputs, **kwargs):
        outputs[0][0] = self.k_srtm.create_activity_curve(DVR=inputs[0], R1=inputs[1], k2p=inputs[2]).T

    def __call__(self, DVR, R1, k2p):
        out = [[None]]
        self.perform(None, (DVR, R1, k2p), out)
        return out[0][0]


class MetropolisSRTM2:
    def __init__(self, time_vector, tac_ref, k2p, y_obs, sigma_noise, mu_DVR, Cov_DVR, mu_R1, Cov_R1, device=None,
                 tune_interval=100, scaling=1.0, vs_sweep_start=True, kernel='auto', waves_per_chain=0):
        self.device = torch.device('cuda', device if device is not None else torch.cuda.current_device())
        arr = lambda a: np.ascontiguousarray(a, dtype=np.float64)   # noqa: E731
        self._keep = [arr(time_vector), arr(tac_ref), arr(y_obs), arr(sigma_noise), arr(mu_DVR), arr(Cov_DVR),
                      arr(mu_R1), arr(Cov_R1)]
        tv, cr, y, sig, mD, cD, mR, cR = self._keep
        if y.shape != (48, 54) or sig.shape != (48, 54):
            raise NotImplementedError('the MH kernel is compiled for 48 ROIs x 54 frames')
        p = _lib.PetmhProblem(48, 54, *(a.ctypes.data for a in (tv, cr)), float(k2p),
                              *(a.ctypes.data for a in (y, sig, mD, cD, mR, cR)))
        h = C.c_void_p()
        torch.cuda.set_device(self.device)
        _lib.check_mh(_lib.lib().petmh_create(C.byref(p), self.device.index, C.byref(h)), 'petmh_create')
        self._h = h
        _lib.check_mh(_lib.lib().petmh_set_sampler(h, int(tune_interval), float(scaling), int(bool(vs_sweep_start))),
                      'petmh_set_sampler')
        self.set_kernel(kernel, waves_per_chain)

    _KERNELS = {'auto': 0, 'update': 1, 'batched': 2}

    def set_kernel(self, kernel='auto', waves_per_chain=0):
        """GPU chain kernel (petmh_set_kernel): 'update' = one element update at a time, one wave per
        chain; 'batched' = the sweep's 144 possible likelihoods evaluated up front by waves_per_chain
        (1, 2, 4, 12; 0 = auto) waves, then a scan; 'auto' = batched for <= 256 chains."""
        if kernel not in self._KERNELS:
            raise ValueError(f'kernel must be one of {sorted(self._KERNELS)}')
        _lib.check_mh(_lib.lib().petmh_set_kernel(self._h, self._KERNELS[kernel], int(waves_per_chain)),
                      'petmh_set_kernel')

    def close(self):
        if getattr(self, '_h', None) is not None:
            _lib.lib().petmh_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def logp(self, x):
        """Joint log density (mcmc.py:147-155) at x (n, 96) = [DVR | R1]."""
        xt = torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x, dtype=torch.float64,
                             device=self.device).reshape(-1, 96).contiguous()
        out = torch.empty(xt.shape[0], dtype=torch.float64, device=self.device)
        _lib.check_mh(_lib.lib().petmh_logp(self._h, C.c_void_p(xt.data_ptr()), xt.shape[0],
                                            C.c_void_p(out.data_ptr()), self._stream()), 'petmh_logp')
        return out

    def run(self, n_chains, draws, tune, seed=0, x0=None, return_chains=False, return_draws=False):
        """pm.sample(draws, tune, step=Metropolis(NormalProposal)) (mcmc.py:156-157) over n_chains chains.
        return_draws: also keep the trace (the reference's idata, mcmc.py:162-164) as
        res['draws'], a CUDA fp64 tensor (n_chains, draws, 96) = [DVR | R1], and its convergence check
        (mcmc.py:183-194) as res['convergence'] (metrics.convergence_report: R-hat per ROI, rhat_max, and
        the reference's flag R-hat > 1.02)."""
        x0t = None if x0 is None else torch.as_tensor(np.asarray(x0), dtype=torch.float64,
                                                       device=self.device).reshape(n_chains, 96).contiguous()
        stats = torch.empty((n_chains, 96, 3), dtype=torch.float64, device=self.device)
        acc = torch.empty((n_chains, 96), dtype=torch.float64, device=self.device)
        last = torch.empty((n_chains, 96), dtype=torch.float64, device=self.device)
        torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        trace = (torch.empty((n_chains, draws, 96), dtype=torch.float64, device=self.device)
                 if return_draws else None)
        _lib.check_mh(_lib.lib().petmh_run_draws(self._h, None if x0t is None else C.c_void_p(x0t.data_ptr()),
                                                 n_chains, draws, tune, int(seed), C.c_void_p(stats.data_ptr()),
                                                 C.c_void_p(acc.data_ptr()), C.c_void_p(last.data_ptr()),
                                                 None if trace is None else C.c_void_p(trace.data_ptr()),
                                                 self._stream()), 'petmh_run')
        torch.cuda.synchronize(self.device)
        elapsed = time.perf_counter() - t0
        st = stats.cpu().numpy()
        pooled = merge_stats(st)                                     # (96, 3)
        mean, std = pooled[:, 1], np.sqrt(pooled[:, 2] / np.maximum(pooled[:, 0], 1))
        res = {'mean_DVR': mean[:48], 'mean_R1': mean[48:], 'std_DVR': std[:48], 'std_R1': std[48:],
               'accept_rate': acc.cpu().numpy() / max(draws, 1), 'elapsed_s': elapsed,
               'chain_draws_per_s': n_chains * (draws + tune) / elapsed if elapsed > 0 else float('inf')}
        if return_draws:
            res['draws'] = trace
            if draws >= 4 and n_chains >= 1:
                # mcmc.py:183-194: rank-normalised split R-hat per ROI; flag = any R-hat > 1.02
                from .metrics import convergence_report
                res['convergence'] = convergence_report(trace)
        if return_chains:
            res['chain_stats'] = st
            res['last'] = last.cpu().numpy()
        return res
