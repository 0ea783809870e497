"""ctypes binding of libpetdiff.so (the C ABI declared in include/petdiff.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C pet_posterior_distribution_amd/csrc``).  There is no fallback: if the
library is missing every entry point raises ``RuntimeError`` -- the product path
never silently computes on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PETDIFF_LIB: an alternative build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get('PETDIFF_LIB') or os.path.join(_HERE, 'libpetdiff.so')

PETDIFF_OK, PETDIFF_ERR_INVALID, PETDIFF_ERR_HIP, PETDIFF_ERR_UNSUPPORTED = 0, 1, 2, 3
DTYPE_F32, DTYPE_BF16, DTYPE_F16, DTYPE_BF16X3 = 0, 1, 2, 3
LEARN_FIXED, LEARN, LEARN_RANGED = 0, 1, 2
PARAM_EPS, PARAM_X0, PARAM_V, PARAM_XPREV = 0, 1, 2, 3
NTAB = 13
MAX_BATCH = 65536                    # PETDIFF_MAX_BATCH (include/petdiff.h)
NUM_LAYERS = 10
NUM_LEVELS = 6                       # PETDIFF_NUM_LEVELS: petdiff_get_activation levels
LEVEL_SHAPES = [(48, 128), (24, 256), (12, 512), (6, 1024), (12, 512), (24, 256)]
LEVEL_NAMES = ['down0', 'down1', 'down2', 'down3', 'up0', 'up1']
LAYER_NAMES = ['down0', 'down1', 'down2', 'down3', 'up0.conv2', 'up0.block', 'up1.conv2',
               'up1.block', 'up2.conv2', 'up2.block+final+p_sample']


class PetdiffConfig(C.Structure):
    _fields_ = [('n_roi', C.c_int), ('n_par', C.c_int), ('n_frames', C.c_int), ('n_cond_rows', C.c_int),
                ('num_filt_start', C.c_int), ('depth', C.c_int), ('kernel_size', C.c_int),
                ('pool_size', C.c_int), ('sin_emb_dim', C.c_int), ('enc_size', C.c_int * 3),
                ('latent_dim', C.c_int), ('timesteps', C.c_int), ('learn_variance', C.c_int),
                ('parameterization', C.c_int), ('dtype', C.c_int)]


# (name, restype, argtypes) of every exported symbol in include/petdiff.h
SYMBOLS = [
    ('petdiff_default_config', C.c_int, [C.POINTER(PetdiffConfig)]),
    ('petdiff_param_count', C.c_size_t, [C.POINTER(PetdiffConfig)]),
    ('petdiff_create', C.c_int, [C.POINTER(PetdiffConfig), C.c_void_p, C.c_size_t, C.c_int, C.POINTER(C.c_void_p)]),
    ('petdiff_destroy', C.c_int, [C.c_void_p]),
    ('petdiff_set_schedule', C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    ('petdiff_piece_key', C.c_int, [C.c_int, C.c_int, C.c_int]),
    ('petdiff_cosine_schedule', C.c_int, [C.c_int, C.c_double, C.c_double, C.c_void_p]),
    ('petdiff_set_conditions', C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    ('petdiff_forward', C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                  C.c_void_p]),
    ('petdiff_p_sample', C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                   C.c_uint64, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                   C.c_void_p]),
    ('petdiff_generate', C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                   C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                   C.c_void_p]),
    ('petdiff_posterior_stats', C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                          C.c_void_p]),
    ('petdiff_philox_normal', C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.c_void_p, C.c_int,
                                        C.c_void_p]),
    ('petdiff_get_activation', C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p]),
    ('petdiff_set_timing', C.c_int, [C.c_void_p, C.c_int]),
    ('petdiff_get_timing', C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ('petdiff_last_error', C.c_char_p, []),
    # Metropolis-Hastings / SRTM2 (include/petmh.h)
    ('petmh_srtm2_tac', C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                  C.c_void_p, C.c_void_p]),
    ('petmh_create', C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    ('petmh_destroy', C.c_int, [C.c_void_p]),
    ('petmh_run', C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_void_p, C.c_void_p,
                            C.c_void_p, C.c_void_p]),
    ('petmh_set_sampler', C.c_int, [C.c_void_p, C.c_int, C.c_double, C.c_int]),
    ('petmh_set_kernel', C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    ('petmh_run_draws', C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_void_p,
                                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ('petmh_logp', C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    ('petmh_last_error', C.c_char_p, []),
    # synthetic-TAC generator (include/petsim.h)
    ('petsim_generate', C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.c_int] + [C.c_void_p] * 8),
    ('petsim_last_error', C.c_char_p, []),
    # posterior accuracy metrics (include/petmetrics.h)
    ('petmetrics_moments', C.c_int, [C.c_void_p, C.c_int, C.c_int64, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p]),
    ('petmetrics_work_doubles', C.c_size_t, [C.c_int]),
    ('petmetrics_last_error', C.c_char_p, []),
]


class PettrainConfig(C.Structure):
    _fields_ = [('learning_rate', C.c_float), ('decay_steps', C.c_float), ('decay_rate', C.c_float),
                ('beta_1', C.c_float), ('beta_2', C.c_float), ('epsilon', C.c_float), ('clipnorm', C.c_float),
                ('lambda_vlb', C.c_float)]


SYMBOLS += [
    # training step (include/pettrain.h)
    ('pettrain_default_config', C.c_int, [C.POINTER(PettrainConfig)]),
    ('pettrain_create', C.c_int, [C.POINTER(PetdiffConfig), C.c_void_p, C.c_size_t, C.c_void_p, C.c_int,
                                  C.POINTER(PettrainConfig), C.c_int, C.POINTER(C.c_void_p)]),
    ('pettrain_destroy', None, [C.c_void_p]),
    ('pettrain_compute_gradients', C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                             C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p]),
    ('pettrain_compute_loss', C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                        C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p]),
    ('pettrain_apply_gradients', C.c_int, [C.c_void_p, C.c_float, C.c_void_p]),
    ('pettrain_step', C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64,
                                C.c_uint64, C.c_void_p, C.c_void_p]),
    ('pettrain_gradients', C.c_void_p, [C.c_void_p]),
    ('pettrain_get_weights', C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ('pettrain_get_gradients', C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ('pettrain_set_gradients', C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ('pettrain_last_stats', C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ('pettrain_iterations', C.c_int64, [C.c_void_p]),
    ('pettrain_last_error', C.c_char_p, []),
]


class PetsimPrior(C.Structure):
    _fields_ = [('n_roi', C.c_int), ('n_frames', C.c_int), ('time_vector', C.c_void_p), ('dt', C.c_void_p),
                ('mu_DVR', C.c_void_p), ('cov_DVR', C.c_void_p), ('mu_R1', C.c_void_p), ('cov_R1', C.c_void_p),
                ('mu_ref', C.c_void_p), ('cov_ref', C.c_void_p), ('k2p', C.c_double), ('sigma_noise', C.c_void_p)]


class PetmhProblem(C.Structure):
    _fields_ = [('n_roi', C.c_int), ('n_frames', C.c_int), ('time_vector', C.c_void_p), ('tac_ref', C.c_void_p),
                ('k2p', C.c_double), ('y_obs', C.c_void_p), ('sigma_noise', C.c_void_p), ('mu_DVR', C.c_void_p),
                ('cov_DVR', C.c_void_p), ('mu_R1', C.c_void_p), ('cov_R1', C.c_void_p)]


def check_mh(rc, what=''):
    if rc == 0:
        return
    msg = lib().petmh_last_error().decode(errors='replace')
    if rc == 1:
        raise ValueError(f'{what}: {msg}')
    raise PetdiffError(f'{what}: {msg}')

_lib = None


class PetdiffError(RuntimeError):
    pass


def lib():
    """Load libpetdiff.so once; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f'libpetdiff.so not found at {LIB_PATH}: build it with '
                           f'`python -c "import __graft_entry__ as g; g.build()"` (no CPU fallback exists)')
    L = C.CDLL(LIB_PATH)
    for name, res, args in SYMBOLS:
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def last_error():
    return lib().petdiff_last_error().decode(errors='replace')


def check(rc, what=''):
    """Raise the reference's exception type for a C-ABI status code."""
    if rc == PETDIFF_OK:
        return
    msg = f'{what}: {last_error()}' if what else last_error()
    if rc == PETDIFF_ERR_INVALID:
        raise ValueError(msg)
    if rc == PETDIFF_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise PetdiffError(msg)


def exported_symbols():
    """Names of the C entry points this binding expects (for the load test)."""
    return [s[0] for s in SYMBOLS]


def kernel_code_hash(symbol=b'conv_kernel', path=None):
    """sha256 (16 hex digits) of the gfx950 code object in libpetdiff.so's .hip_fatbin that defines
    ``symbol`` (the U-Net kernels' translation unit): it changes exactly when those kernels' machine
    code does, so PMC counters recorded for one build can be recognised as stale for another
    (scripts/pmc_summary.py stamps it, bench.py checks it).  None if the file has no such bundle."""
    import hashlib
    import struct
    with open(path or LIB_PATH, 'rb') as f:
        b = f.read()
    if b[:4] != b'\x7fELF':
        return None
    shoff = struct.unpack_from('<Q', b, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from('<HHH', b, 0x3A)
    secs = [struct.unpack_from('<IIQQQQIIQQ', b, shoff + i * shentsize) for i in range(shnum)]
    stro = secs[shstrndx][4]
    fb = None
    for s in secs:
        if b[stro + s[0]:b.index(b'\0', stro + s[0])] == b'.hip_fatbin':
            fb = b[s[4]:s[4] + s[5]]
    if fb is None:
        return None
    magic = b'__CLANG_OFFLOAD_BUNDLE__'
    i = fb.find(magic)
    while i >= 0:
        n = struct.unpack_from('<Q', fb, i + 24)[0]
        q = i + 32
        for _ in range(n):
            off, sz, idl = struct.unpack_from('<QQQ', fb, q)
            tid = fb[q + 24:q + 24 + idl]
            q += 24 + idl
            co = fb[i + off:i + off + sz]
            if sz and b'gfx950' in tid and symbol in co:
                return hashlib.sha256(co).hexdigest()[:16]
        i = fb.find(magic, i + 1)
    return None
