"""Generate the golden fixtures under tests/golden/ from the reference's own code.

Run in the build container only (needs /root/reference, read-only):
    python tests/golden/make_golden.py

* G1 (g1_schedules.npz): helper_func.get_beta_schedule (helper_func.py:237-268) for
  the cosine schedule of the shipped config (T=1000, main_script.py:179-186) and the
  other schedule types with DDPM's defaults (diffusion_model.py:85-90).
  helper_func imports NP_DTYPE from diffusion_model (TensorFlow, absent here), so a
  stub module providing only NP_DTYPE = np.float32 (diffusion_model.py:7-10) is
  inserted into sys.modules before the import.
* G2 (g2_srtm2.npz): kinetic_model.SRTM2.create_activity_curve
  (kinetic_model.py:142-158) and interp1d_linear_vec (:35-57) on synthetic inputs of
  the reference's shapes (54-frame protocol of sample_sim_data.py:29-85, 48 ROIs).

* G0 (g0_prior.npz): the arrays of the reference's prior_stats_nROI48.pik (sample_sim_data.py:106,
  mcmc.py:84-93), the only real data file in the reference.  It is a pickle, and reference pickles are
  never unpickled here: ``read_pickle_data`` parses the byte stream with pickletools.genops (a
  disassembler: nothing in the file is imported, called or constructed) and rebuilds only the literal
  data it holds -- dicts, lists, strings, numbers and numpy arrays / scalars, recognised by the exact
  (module, name) pairs numpy's pickles reference and their argument shapes; anything else raises.
  Run ``python tests/golden/make_golden.py g0`` to (re)write G0 alone.

Only inputs and outputs are stored (data, no reference source).
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'


class _Global:
    """A (module, name) reference in the opcode stream: a label, never resolved or imported."""
    def __init__(self, module, name):
        self.module, self.name = module, name

    def __eq__(self, other):
        return isinstance(other, _Global) and (self.module, self.name) == (other.module, other.name)


class _Call:
    """REDUCE / BUILD record: which label was applied to which literal arguments (and state)."""
    def __init__(self, func, args):
        self.func, self.args, self.state = func, args, None


_NP_MODS = ('numpy.core.multiarray', 'numpy._core.multiarray')


def _np_dtype(rec):
    """numpy.dtype(str, False, True) + BUILD state (3, endian, ...) -> np.dtype of a plain number kind."""
    if not (isinstance(rec, _Call) and rec.func == _Global('numpy', 'dtype') and isinstance(rec.args, tuple)
            and isinstance(rec.args[0], str)):
        raise ValueError('not a numpy dtype record')
    endian = rec.state[1] if isinstance(rec.state, tuple) and len(rec.state) > 1 else '<'
    dt = np.dtype((endian if endian in '<>' else '') + rec.args[0])
    if dt.kind not in 'fiub' or dt.hasobject:
        raise ValueError(f'dtype {dt} not allowed')
    return dt


def _to_data(v):
    """Records -> numpy arrays / scalars; containers recursively; anything unrecognised raises."""
    if isinstance(v, (str, int, float, bool, bytes)) or v is None:
        return v
    if isinstance(v, list):
        return [_to_data(e) for e in v]
    if isinstance(v, tuple):
        return tuple(_to_data(e) for e in v)
    if isinstance(v, dict):
        return {_to_data(k): _to_data(e) for k, e in v.items()}
    if isinstance(v, _Call):
        f = v.func
        if isinstance(f, _Global) and f.module in _NP_MODS and f.name == '_reconstruct':
            if not (v.args[0] == _Global('numpy', 'ndarray') and isinstance(v.state, tuple) and len(v.state) == 5):
                raise ValueError('unexpected ndarray record')
            _, shape, dtrec, fortran, raw = v.state
            dt = _np_dtype(dtrec)
            if not isinstance(raw, bytes) or len(raw) != int(np.prod(shape)) * dt.itemsize:
                raise ValueError('ndarray payload size')
            return np.frombuffer(raw, dtype=dt).reshape(shape, order='F' if fortran else 'C').copy()
        if isinstance(f, _Global) and f.module in _NP_MODS and f.name == 'scalar':
            dt = _np_dtype(v.args[0])
            return np.frombuffer(v.args[1], dtype=dt)[0]
    raise ValueError(f'unsupported pickle content {type(v).__name__}')


def read_pickle_data(path):
    """Literal data of a pickle, read without unpickling (see the module docstring)."""
    import pickletools
    data = open(path, 'rb').read()
    stack, marks, memo = [], [], {}

    def pop_mark():
        k = marks.pop()
        items = stack[k:]
        del stack[k:]
        return items
    for op, arg, _ in pickletools.genops(data):
        n = op.name
        if n in ('PROTO', 'FRAME'):
            continue
        if n == 'STOP':
            break
        if n in ('SHORT_BINUNICODE', 'BINUNICODE', 'BINUNICODE8', 'SHORT_BINBYTES', 'BINBYTES', 'BINBYTES8',
                 'BININT', 'BININT1', 'BININT2', 'BINFLOAT', 'LONG1'):
            stack.append(arg)
        elif n in ('NEWTRUE', 'NEWFALSE', 'NONE'):
            stack.append({'NEWTRUE': True, 'NEWFALSE': False, 'NONE': None}[n])
        elif n == 'EMPTY_DICT':
            stack.append({})
        elif n == 'EMPTY_LIST':
            stack.append([])
        elif n == 'EMPTY_TUPLE':
            stack.append(())
        elif n == 'MARK':
            marks.append(len(stack))
        elif n in ('TUPLE1', 'TUPLE2', 'TUPLE3'):
            k = int(n[-1])
            t = tuple(stack[-k:])
            del stack[-k:]
            stack.append(t)
        elif n == 'TUPLE':
            stack.append(tuple(pop_mark()))
        elif n == 'MEMOIZE':
            memo[len(memo)] = stack[-1]
        elif n in ('BINPUT', 'LONG_BINPUT'):
            memo[arg] = stack[-1]
        elif n in ('BINGET', 'LONG_BINGET'):
            stack.append(memo[arg])
        elif n == 'STACK_GLOBAL':
            name, mod = stack.pop(), stack.pop()
            stack.append(_Global(mod, name))
        elif n == 'GLOBAL':
            mod, name = arg.split(' ', 1)
            stack.append(_Global(mod, name))
        elif n == 'REDUCE':
            args = stack.pop()
            stack.append(_Call(stack.pop(), args))
        elif n == 'BUILD':
            state = stack.pop()
            if not isinstance(stack[-1], _Call):
                raise ValueError('BUILD on a non-record')
            stack[-1].state = state
        elif n == 'APPEND':
            v = stack.pop()
            stack[-1].append(v)
        elif n == 'APPENDS':
            items = pop_mark()
            stack[-1].extend(items)
        elif n == 'SETITEM':
            v, k = stack.pop(), stack.pop()
            stack[-1][k] = v
        elif n == 'SETITEMS':
            items = pop_mark()
            for k, v in zip(items[::2], items[1::2]):
                stack[-1][k] = v
        else:
            raise ValueError(f'opcode {n} not supported')
    if len(stack) != 1:
        raise ValueError('malformed stream')
    return _to_data(stack[0])


def make_g0():
    d = read_pickle_data(os.path.join(REF, 'prior_stats_nROI48.pik'))
    arrays = {k: np.asarray(v, dtype=np.float64) for k, v in d.items() if k != 'ROI_names'}
    arrays['ROI_names'] = np.asarray(d['ROI_names'], dtype='U')
    np.savez(os.path.join(HERE, 'g0_prior.npz'), **arrays)
    # the package's copy (sim_data.reference_prior); tests/test_cpu.py checks the two are identical
    np.savez(os.path.join(os.path.dirname(os.path.dirname(HERE)), 'pet_posterior_distribution_amd', 'data',
                          'prior_stats_nROI48.npz'), **arrays)
    print('g0:', {k: v.shape for k, v in arrays.items()})


def main():
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    stub = types.ModuleType('diffusion_model')
    stub.NP_DTYPE = np.float32
    sys.modules['diffusion_model'] = stub
    sys.path.insert(0, REF)
    import helper_func as hf
    import kinetic_model as km

    g1 = {
        'cosine_T1000': hf.get_beta_schedule('cosine', 1000, beta_start=1e-4, beta_end=2e-2, offset_s=0.008,
                                             max_beta=0.999),
        'cosine_T200': hf.get_beta_schedule('cosine', 200, beta_start=1e-4, beta_end=2e-2, offset_s=0.008,
                                            max_beta=0.999),
        'linear_T1000': hf.get_beta_schedule('linear', 1000, beta_start=1e-4, beta_end=2e-2),
        'quadratic_T1000': hf.get_beta_schedule('quadratic', 1000, beta_start=1e-4, beta_end=2e-2),
        'sigmoid_T1000': hf.get_beta_schedule('sigmoid', 1000, beta_start=1e-4, beta_end=2e-2),
    }
    np.savez(os.path.join(HERE, 'g1_schedules.npz'), **g1)

    from pet_posterior_distribution_amd.sim_data import time_grid, synthetic_prior
    tv, dt = time_grid()
    prior = synthetic_prior()
    rng = np.random.default_rng(20250829)
    cases = {}
    for k in range(4):
        DVR = np.abs(rng.multivariate_normal(prior['mu_DVR'], prior['Cov_DVR'])) + 0.2
        R1 = np.abs(rng.multivariate_normal(prior['mu_R1'], prior['Cov_R1'])) + 0.1
        ref = np.abs(rng.multivariate_normal(prior['mu_tac_ref'], prior['Cov_tac_ref']))
        k2p = 0.0126 if k % 2 == 0 else float(rng.uniform(0.01, 0.2))
        model = km.SRTM2(frame_time_list=tv, frame_duration_list=dt, tac_reference=ref)
        tac = model.create_activity_curve(DVR=DVR, R1=R1, k2p=k2p)
        cases.update({f'case{k}_DVR': DVR, f'case{k}_R1': R1, f'case{k}_tac_ref': ref,
                      f'case{k}_k2p': np.float64(k2p), f'case{k}_tac': tac})
    # scalar-parameter branch (np.isscalar(bp)) of create_activity_curve
    model = km.SRTM2(frame_time_list=tv, frame_duration_list=dt, tac_reference=prior['mu_tac_ref'])
    cases['scalar_tac'] = model.create_activity_curve(DVR=1.3, R1=0.8, k2p=0.05)
    # interpolation kernel on its own (incl. the x == xp[0] wrap of searchsorted - 1)
    x_rs = np.linspace(tv.min(), tv.max(), 108)
    f = np.exp(-0.05 * tv)[:, None] * np.arange(1, 4)[None, :]
    cases['interp_x'] = x_rs
    cases['interp_up'] = km.interp1d_linear_vec(x_rs, tv, f)
    cases['interp_down'] = km.interp1d_linear_vec(tv, x_rs, km.interp1d_linear_vec(x_rs, tv, f))
    cases['time_vector'] = tv
    cases['dt'] = dt
    np.savez(os.path.join(HERE, 'g2_srtm2.npz'), **cases)
    print('wrote', sorted(os.listdir(HERE)))


if __name__ == '__main__':
    if sys.argv[1:] == ['g0']:
        make_g0()
    else:
        main()
        make_g0()
