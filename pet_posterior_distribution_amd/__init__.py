"""MI355X-native iDDPM posterior sampler for PET kinetic parameters.

Drop-in for the sampling hot path of yanisdjebra/PET_posterior_distribution
(``ImprovedDDPM.ddpm`` / ``ddpm_loop``, a.k.a. p_sample / generate) on hand-written
gfx950 HIP kernels behind the C ABI in include/petdiff.h.
"""
from . import _lib
from .helper_func import get_beta_schedule, cos_beta_schedule, chunker
from .networks import UnetConditional, param_spec, glorot_uniform_init, denoiser_init
from .diffusion_model import ImprovedDDPM, summarize_stats
from .training import Adam, ExponentialDecay
from .checkpoint import TensorBundle, load_unet_weights

__all__ = ['ImprovedDDPM', 'UnetConditional', 'get_beta_schedule', 'cos_beta_schedule', 'chunker',
           'param_spec', 'glorot_uniform_init', 'denoiser_init', 'summarize_stats', 'Adam', 'ExponentialDecay',
           'TensorBundle', 'load_unet_weights']
