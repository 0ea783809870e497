"""Bitwise A/B of two builds of libpetdiff.so on the same inputs (layout changes that must not
change a single bit, e.g. CONV_DOWN2_PM: the zero taps a position-major tile skips add +0.0).

  python scripts/lib_bitwise.py dump out.npz        # with PETDIFF_LIB pointing at one build
  python scripts/lib_bitwise.py compare a.npz b.npz

Covers: bf16, fp16 and bf16x3 forward on ragged batches (1, 37, 100, 1024) with interleaved per-sample
conditions and t (the general epilogue), one-condition forward (the LDS-map epilogue) and a
20-step graph loop.
"""
import sys

import numpy as np


def dump(path):
    sys.path.insert(0, '.')
    from tests.test_gpu_parity import make_model
    from tests.helpers import synthetic_condition
    conds = np.stack([synthetic_condition(0), synthetic_condition(1)])
    res = {}
    for dtype in ('bfloat16', 'float16', 'bf16x3'):
        m = make_model(dtype, seed=21)
        rng = np.random.default_rng(3)
        for B in (1, 37, 100, 1024):
            x = rng.standard_normal((B, 48, 2)).astype(np.float32)
            t = rng.integers(0, 1000, B).astype(np.int32)
            cond = conds[np.arange(B) % 2]
            res[f'{dtype}_mixed_{B}'] = m.call({'x': x, 'time': t, 'condition': cond}).cpu().numpy()
            t1 = np.full(B, 500, np.int32)
            res[f'{dtype}_one_{B}'] = m.call({'x': x, 'time': t1, 'condition': np.repeat(conds[:1], B, 0)}).cpu().numpy()
        x = rng.standard_normal((256, 48, 2)).astype(np.float32)
        res[f'{dtype}_loop'] = m.ddpm_loop(x, conds[:1], num_timesteps=20, seed=3).cpu().numpy()
        m.close()
    np.savez(path, **res)
    print('dumped', len(res), 'arrays ->', path)


def compare(pa, pb):
    a, b = np.load(pa), np.load(pb)
    bad = 0
    for k in sorted(a.files):
        same = np.array_equal(a[k], b[k]) and np.isfinite(a[k]).all()
        diff = float(np.abs(a[k].astype(np.float64) - b[k]).max())
        print(f'{k:24s} {"bitwise equal" if same else "DIFFERENT"}  max|a-b| = {diff:.3g}')
        bad += not same
    print('ALL BITWISE EQUAL' if bad == 0 else f'{bad} arrays differ')
    return 0 if bad == 0 else 1


if __name__ == '__main__':
    if sys.argv[1] == 'dump':
        dump(sys.argv[2])
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
