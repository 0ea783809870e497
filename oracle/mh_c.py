"""ctypes wrapper of oracle/mh_ref.c (the C restatement of the MH baseline).

TEST INFRASTRUCTURE ONLY: used by tests/ and bench.py's cpu_baseline leg, never by
the product.  Built by oracle/Makefile (``make -C oracle``, also run by
__graft_entry__.build()).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from oracle import srtm2_ref as K

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_D = C.POINTER(C.c_double)


def lib():
    global _LIB
    if _LIB is None:
        # MHREF_LIB: an alternative build of the same checker (scripts/asan_check.sh: AddressSanitizer)
        path = os.environ.get('MHREF_LIB') or os.path.join(_HERE, 'lib', 'libmhref.so')
        if not os.path.exists(path):
            raise FileNotFoundError(f'{path} missing: run make -C oracle')
        L = C.CDLL(path)
        L.mhref_run.argtypes = [_D] * 9 + [C.c_double, _D, C.c_long, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                           C.c_uint64, C.c_int, _D, _D, _D, C.c_int]
        L.mhref_run.restype = C.c_int
        L.mhref_logp_kernel_part.argtypes = [_D] * 9 + [C.c_double, _D, C.c_int, _D]
        L.mhref_logp_kernel_part.restype = C.c_int
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(_D)


class MHProblem:
    """Precomputed arrays of one TAC's MH problem (mcmc.py:73-137 inputs)."""

    def __init__(self, time_vector, tac_ref, k2p, y_obs, sigma_noise, mu_DVR, Cov_DVR, mu_R1, Cov_R1):
        f = lambda a: np.ascontiguousarray(a, dtype=np.float64)   # noqa: E731
        self.M = f(K.srtm2_operator(time_vector, tac_ref).T)        # [g][f]
        self.PD, self.PR = f(np.linalg.inv(Cov_DVR)), f(np.linalg.inv(Cov_R1))
        self.Y, self.SIG = f(y_obs), f(sigma_noise)
        self.CR, self.TV = f(tac_ref), f(time_vector)
        self.MUD, self.MUR = f(mu_DVR), f(mu_R1)
        self.k2p = float(k2p)

    def _args(self):
        return [_p(a) for a in (self.M, self.PD, self.PR, self.Y, self.SIG, self.CR, self.TV, self.MUD,
                                self.MUR)] + [self.k2p]

    def run(self, n_chains, n_draws, n_tune, seed, chain0=0, x0=None, tune_interval=100, scaling=1.0, threads=0,
            vs_sweep_start=True):
        stats = np.zeros((n_chains, 96, 3))
        acc = np.zeros((n_chains, 96))
        last = np.zeros((n_chains, 96))
        x0a = None if x0 is None else np.ascontiguousarray(np.broadcast_to(x0, (n_chains, 96)), dtype=np.float64)
        lib().mhref_run(*self._args(), None if x0a is None else _p(x0a), chain0, n_chains, n_draws, n_tune,
                        tune_interval, scaling, seed, int(vs_sweep_start), _p(stats), _p(acc), _p(last), threads)
        return stats, acc, last

    def logp_unnormalised(self, x):
        x = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float64)
        out = np.zeros(x.shape[0])
        lib().mhref_logp_kernel_part(*self._args(), _p(x), x.shape[0], _p(out))
        return out
