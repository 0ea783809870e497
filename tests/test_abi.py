"""CPU checks of the C ABI: libpetdiff.so loads and exports every symbol include/*.h declares."""
import ctypes as C
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = []
    for h in sorted(os.listdir(os.path.join(ROOT, 'include'))):
        if h.endswith('.h'):
            txt = open(os.path.join(ROOT, 'include', h)).read()
            names += re.findall(r'^\s*(?:int|size_t|const char\*)\s+(pet\w+)\s*\(', txt, flags=re.M)
    return names


def test_library_loads_and_exports_header_symbols():
    from pet_posterior_distribution_amd import _lib
    L = _lib.lib()
    names = declared_symbols()
    assert 'petdiff_generate' in names and 'petdiff_p_sample' in names
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # every symbol the Python binding declares is exported too
    assert not [n for n in _lib.exported_symbols() if not hasattr(L, n)]


def test_default_config_and_param_count():
    from pet_posterior_distribution_amd import _lib
    L = _lib.lib()
    cfg = _lib.PetdiffConfig()
    assert L.petdiff_default_config(C.byref(cfg)) == 0
    assert (cfg.n_roi, cfg.n_par, cfg.num_filt_start, cfg.depth, cfg.timesteps) == (48, 2, 128, 4, 1000)
    # 11,851,740 params x 12 B (weights + Adam m, v at fp32) ~ the LFS checkpoint blob (142,333,243 B)
    n = L.petdiff_param_count(C.byref(cfg))
    assert n == 11_851_740
    assert abs(n * 12 - 142_333_243) / 142_333_243 < 1e-3


def test_cosine_schedule_c_restatement_close_to_numpy():
    from pet_posterior_distribution_amd import _lib, helper_func
    b = np.zeros(1000, np.float32)
    assert _lib.lib().petdiff_cosine_schedule(1000, 0.008, 0.999, b.ctypes.data_as(C.c_void_p)) == 0
    ref = helper_func.cos_beta_schedule(1000)
    np.testing.assert_allclose(b, ref, rtol=1e-5, atol=1e-6)


def test_errors_map_to_reference_exceptions():
    from pet_posterior_distribution_amd import _lib
    L = _lib.lib()
    cfg = _lib.PetdiffConfig()
    L.petdiff_default_config(C.byref(cfg))
    h = C.c_void_p()
    w = np.zeros(10, np.float32)
    rc = L.petdiff_create(C.byref(cfg), w.ctypes.data_as(C.c_void_p), 10, 0, C.byref(h))
    assert rc == _lib.PETDIFF_ERR_INVALID
    assert 'expected 11851740' in _lib.last_error()
    cfg.depth = 5
    rc = L.petdiff_create(C.byref(cfg), w.ctypes.data_as(C.c_void_p), 10, 0, C.byref(h))
    assert rc == _lib.PETDIFF_ERR_UNSUPPORTED


def test_max_batch_constant_matches_header():
    from pet_posterior_distribution_amd import _lib
    txt = open(os.path.join(ROOT, 'include', 'petdiff.h')).read()
    m = re.search(r'#define\s+PETDIFF_MAX_BATCH\s+(\d+)', txt)
    assert m and int(m.group(1)) == _lib.MAX_BATCH


def test_dtype_constants_match_header():
    """_lib's dtype codes (incl. the bf16x3 network) are the header's PETDIFF_DTYPE_* values, and
    petdiff_create rejects an unknown dtype before touching the device."""
    from pet_posterior_distribution_amd import _lib
    txt = open(os.path.join(ROOT, 'include', 'petdiff.h')).read()
    hdr = {k: int(v) for k, v in re.findall(r'#define\s+PETDIFF_DTYPE_(\w+)\s+(\d+)', txt)}
    assert hdr == {'F32': _lib.DTYPE_F32, 'BF16': _lib.DTYPE_BF16, 'F16': _lib.DTYPE_F16,
                   'BF16X3': _lib.DTYPE_BF16X3}
    L = _lib.lib()
    cfg = _lib.PetdiffConfig()
    assert L.petdiff_default_config(C.byref(cfg)) == 0
    cfg.dtype = 7
    h = C.c_void_p()
    w = np.zeros(_lib.lib().petdiff_param_count(C.byref(cfg)), np.float32)
    rc = L.petdiff_create(C.byref(cfg), w.ctypes.data_as(C.c_void_p), w.size, 0, C.byref(h))
    assert rc == _lib.PETDIFF_ERR_INVALID and 'PETDIFF_DTYPE_BF16X3' in _lib.last_error()
