"""CPU tests of the HDF5 reader / writer and the Keras ``.weights.h5`` importer (h5.py).

Pin: ``tests/golden/testhdf5_7.4_GLNX86.mat`` is an HDF5 file written by the HDF5 library itself (a MATLAB 7.4
v7.3 MAT-file from scipy's test data, BSD): a 512-byte user block, superblock v0, symbol-table root group, one
contiguous float64 dataset ``testdouble`` = pi/4 * (0..8) (scipy's test_mio.py ``theta``; MATLAB stores the
1 x 9 row column-major, so HDF5 sees 9 x 1) with a fixed-length string attribute ``MATLAB_class = 'double'``.
The Keras path layout of the reference's model is parity unpinned (no TF-written file exists offline).
"""
import os

import numpy as np
import pytest

from pet_posterior_distribution_amd import h5
from pet_posterior_distribution_amd.networks import UnetConditional, glorot_uniform_init
from tests.helpers import shipped_net_args

GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'testhdf5_7.4_GLNX86.mat')


def test_reads_library_written_hdf5():
    with h5.File(GOLD) as f:
        assert f._r.base == 512 and f._r.sb_version == 0
        assert f.keys() == ['testdouble']
        d = f['testdouble']
        assert d.shape == (9, 1) and d.dtype == np.float64
        assert d.attrs['MATLAB_class'] == 'double'
        np.testing.assert_array_equal(d.read()[:, 0], np.pi / 4 * np.arange(9, dtype=float))


def test_write_read_roundtrip_nested(tmp_path):
    rng = np.random.default_rng(0)
    tree = {'a': {'vars': {'0': rng.standard_normal((3, 4)).astype(np.float32), '1': np.arange(5.0)}},
            'ints': np.array([[1, -2], [3, 4]], dtype=np.int32), 'empty': {}}
    for i in range(40):          # more members than one symbol-table node holds (2 x leaf K = 8)
        tree['a'][f'g{i}'] = {'vars': {'0': rng.standard_normal((2, i + 1)).astype(np.float32)}}
    p = str(tmp_path / 'x.h5')
    h5.write(p, tree)
    with h5.File(p) as f:
        assert f.keys() == ['a', 'empty', 'ints']
        assert f['empty'].keys() == []
        np.testing.assert_array_equal(f['a/vars/0'].read(), tree['a']['vars']['0'])
        np.testing.assert_array_equal(f['a/vars/1'].read(), tree['a']['vars']['1'])
        np.testing.assert_array_equal(f['ints'].read(), tree['ints'])
        for i in range(40):
            np.testing.assert_array_equal(f[f'a/g{i}/vars/0'].read(), tree['a'][f'g{i}']['vars']['0'])
        seen = []
        f.visit(lambda path, obj: seen.append(path))
        assert 'a/g39/vars/0' in seen and len(seen) == 3 + 1 + 2 + 40 * 3


def _net(seed):
    net = UnetConditional(**shipped_net_args())
    net.build((None, 48, 2))
    net.weights = glorot_uniform_init(net.spec(), seed=seed, bias_scale=0.05)
    return net


def test_unet_weights_h5_roundtrip(tmp_path):
    a, b = _net(1), _net(2)
    p = str(tmp_path / 'ckpt.weights.h5')
    a.save_weights(p)
    b.load_weights(p)
    for n, _ in a.spec():
        np.testing.assert_array_equal(a.weights[n], b.weights[n])


def test_improved_ddpm_layout_and_partial_load(tmp_path):
    """A file of the ImprovedDDPM model keeps the network under ``network/`` (the reference saves diff_model,
    main_script.py:263); a file holding only the variables Keras 3 reaches through attributes and flat
    containers (encoder, final conv) loads with strict=False and leaves the rest unchanged."""
    a, b = _net(3), _net(4)
    full = str(tmp_path / 'full.weights.h5')
    h5.save_unet_h5(full, a.weights, network_path='network')
    with h5.File(full) as f:
        assert f.keys() == ['network']
        assert 'network/final_conv/vars/0' in f and 'network/downs/0/0/conv_l/0/vars/1' in f
    got = h5.load_unet_h5(full, a.spec())
    assert set(got) == {n for n, _ in a.spec()}
    part = str(tmp_path / 'part.weights.h5')
    keep = {n: w for n, w in a.weights.items() if n.startswith(('final', 'cond_enc'))}
    h5.save_unet_h5(part, keep, network_path='network')
    with pytest.raises(KeyError):
        b.load_weights(part)
    before = {n: w.copy() for n, w in b.weights.items()}
    b.load_weights(part, strict=False)
    for n, _ in a.spec():
        np.testing.assert_array_equal(b.weights[n], a.weights[n] if n in keep else before[n])


def test_errors(tmp_path):
    bad = tmp_path / 'bad.h5'
    bad.write_bytes(b'not hdf5' * 100)
    with pytest.raises(h5.H5Error):
        h5.File(str(bad))
    a = _net(5)
    w = dict(a.weights)
    w['final.kernel'] = np.zeros((3, 3), np.float32)
    p = str(tmp_path / 'shape.weights.h5')
    h5.save_unet_h5(p, w, network_path='')
    with pytest.raises(h5.H5Error):
        h5.load_unet_h5(p, a.spec())
