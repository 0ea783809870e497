"""SRTM2 kinetic model on the GPU (mirrors the reference's kinetic_model.SRTM2).

``SRTM2.create_activity_curve`` (kinetic_model.py:142-158) and a batched
``create_activity_curves`` run the fp64 HIP kernel behind petmh_srtm2_tac
(include/petmh.h): TAC = R1 C_r + (k2 - R1 k2a) (M exp(-k2a t)) with the constant
54 x 54 operator M of the resampled convolution (kinetic_model.py:12-32).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib


class SRTM2:
    def __init__(self, frame_time_list, frame_duration_list, tac_reference, device=None):
        self._frame_time_list = np.ascontiguousarray(frame_time_list, dtype=np.float64)
        self.frame_duration_list = np.asarray(frame_duration_list, dtype=np.float64)
        self._tac_reference = np.ascontiguousarray(tac_reference, dtype=np.float64)
        if self._frame_time_list.size != 54 or self._tac_reference.size != 54:
            raise NotImplementedError('the SRTM2 kernel is compiled for the 54-frame protocol')
        self.device = torch.device('cuda', device if device is not None else torch.cuda.current_device())

    def create_activity_curves(self, DVR, R1, k2p):
        """Batched: DVR, R1 (n, n_roi); k2p scalar or (n,) -> torch (n, n_roi, 54) fp64 on the GPU."""
        D = torch.as_tensor(np.asarray(DVR) if not isinstance(DVR, torch.Tensor) else DVR, dtype=torch.float64,
                            device=self.device)
        R = torch.as_tensor(np.asarray(R1) if not isinstance(R1, torch.Tensor) else R1, dtype=torch.float64,
                            device=self.device)
        if D.dim() == 1:
            D, R = D[None], R[None]
        D, R = D.contiguous(), R.contiguous()
        n, n_roi = D.shape
        k = torch.as_tensor(k2p, dtype=torch.float64, device=self.device).reshape(-1)
        if k.numel() == 1:
            k = k.expand(n)
        k = k.contiguous()
        out = torch.empty((n, n_roi, 54), dtype=torch.float64, device=self.device)
        _lib.check_mh(_lib.lib().petmh_srtm2_tac(
            self._frame_time_list.ctypes.data_as(C.c_void_p), self._tac_reference.ctypes.data_as(C.c_void_p),
            C.c_void_p(D.data_ptr()), C.c_void_p(R.data_ptr()), n, n_roi, C.c_void_p(k.data_ptr()),
            C.c_void_p(out.data_ptr()), C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
            'petmh_srtm2_tac')
        return out

    def create_activity_curve(self, DVR=None, R1=None, k2p=None):
        """kinetic_model.py:142-158 -> (54, n_roi) NumPy array, like the reference."""
        return self.create_activity_curves(np.atleast_1d(DVR), np.atleast_1d(R1), k2p)[0].T.cpu().numpy()

    __call__ = create_activity_curve
