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


def _heap_of_root(f):
    """(data segment size, free-list head, data segment address) of the root group's local heap."""
    r = f._r
    for mtype, _, d in r.messages(r.root):
        if mtype == 0x11:
            heap = int.from_bytes(d[r.so:2 * r.so], 'little')
            p = r.a(heap)
            assert bytes(r.buf[p:p + 4]) == b'HEAP' and r.buf[p + 4] == 0
            q = p + 8
            return r.u(q, r.sl), r.u(q + r.sl, r.sl), r.u(q + 2 * r.sl, r.so)
    raise AssertionError('root is not a symbol-table group')


def _check_free_list(f):
    """HDF5 local-heap free-list rules: the head is 1 (H5HL_FREE_NULL: no free block) or the offset of a
    block {next offset, size} with size >= 2 length fields, inside the data segment; the last block's
    next offset is 1."""
    r = f._r
    size, head, data = _heap_of_root(f)
    seen = 0
    while head != 1:
        assert head % 8 == 0 and head + 2 * r.sl <= size, (head, size)
        nxt, bsz = r.u(r.a(data) + head, r.sl), r.u(r.a(data) + head + r.sl, r.sl)
        assert bsz >= 2 * r.sl and head + bsz <= size, (head, bsz, size)
        head = nxt
        seen += 1
        assert seen < 1000
    return seen


def test_local_heap_free_list_is_valid(tmp_path):
    """the writer's heap must follow the free-list rules libhdf5 enforces (the library-written
    MAT file is the pin for the layout convention)."""
    with h5.File(GOLD) as f:
        _check_free_list(f)
    p = str(tmp_path / 'g.h5')
    h5.write(p, {'a': np.arange(3.0), 'b': {'c': np.ones(2, np.float32)}})
    with h5.File(p) as f:
        assert _check_free_list(f) == 1
        assert f.keys() == ['a', 'b']


def _chunked_dataset(w, arr, chunk):
    """Object header of a chunked, deflate-compressed dataset (layout message v3 class 2, a one-level v1
    chunk B-tree whose keys are {chunk size, filter mask, rank + 1 offsets}), written by hand."""
    import struct
    import zlib
    arr = np.ascontiguousarray(arr, dtype='<f4')
    rank = arr.ndim
    keys, kids = [], []
    for i0 in range(0, arr.shape[0], chunk[0]):
        for i1 in range(0, arr.shape[1], chunk[1]):
            blk = np.zeros(chunk, '<f4')
            part = arr[i0:i0 + chunk[0], i1:i1 + chunk[1]]
            blk[:part.shape[0], :part.shape[1]] = part
            raw = zlib.compress(blk.tobytes())
            kids.append(w.alloc(raw))
            keys.append(struct.pack('<II', len(raw), 0) + struct.pack('<QQQ', i0, i1, 0))
    keys.append(struct.pack('<II', 0, 0) + struct.pack('<QQQ', arr.shape[0], 0, 0))   # final key
    body = b''.join(k + struct.pack('<Q', c) for k, c in zip(keys, kids)) + keys[-1]
    tree = w.alloc(b'TREE' + struct.pack('<BBHQQ', 1, 0, len(kids), h5.UNDEF, h5.UNDEF) + body)
    space = struct.pack('<BBBx4x', 1, rank, 0) + b''.join(struct.pack('<Q', s) for s in arr.shape)
    dtype_msg = bytes([0x11, 0x20, 31, 0]) + struct.pack('<I', 4) + struct.pack('<HHBBBBI', 0, 32, 23, 8, 0, 23, 127)
    layout = struct.pack('<BBB', 3, 2, rank + 1) + struct.pack('<Q', tree) + \
        b''.join(struct.pack('<I', c) for c in chunk) + struct.pack('<I', 4)
    pipeline = struct.pack('<BB6x', 1, 1) + struct.pack('<HHHH', 1, 0, 0, 1) + struct.pack('<II', 6, 0)
    return w.object_header([w._msg(0x01, space), w._msg(0x03, dtype_msg), w._msg(0x08, layout),
                            w._msg(0x0B, pipeline)])


def test_chunked_deflate_dataset(tmp_path):
    """chunk B-tree keys are 8 + 8 (rank + 1) bytes; several chunks (ragged edges) read back."""
    import struct
    arr = np.arange(5 * 7, dtype=np.float32).reshape(5, 7) * 0.5 - 3.0
    w = h5._Writer()
    w.alloc(b'\0' * 96)
    ds = _chunked_dataset(w, arr, (2, 3))
    root, tree_addr, heap_addr = w.group({'c': ds})
    sb = h5.SIGNATURE + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack('<HHI', w.LEAF_K, w.NODE_K, 0)
    sb += struct.pack('<QQQQ', 0, h5.UNDEF, len(w.out), h5.UNDEF)
    sb += struct.pack('<QQII', 0, root, 1, 0) + struct.pack('<QQ', tree_addr, heap_addr)
    w.out[:len(sb)] = sb
    p = tmp_path / 'chunked.h5'
    p.write_bytes(bytes(w.out))
    with h5.File(str(p)) as f:
        np.testing.assert_array_equal(f['c'].read(), arr)


def test_weights_checkpoint_writes_reference_file(tmp_path):
    """WeightsCheckpoint (networks.py:152-180) writes cp_<epoch>/ckpt.weights.h5 in the model-level layout
    (network under ``network/``), which ImprovedDDPM.load_weights reads back (main_script.py:412)."""
    from pet_posterior_distribution_amd import ImprovedDDPM
    from pet_posterior_distribution_amd.training import WeightsCheckpoint
    from tests.helpers import shipped_diff_args
    a, b = _net(6), _net(7)
    ma = ImprovedDDPM(network=a, device=0, **shipped_diff_args())
    mb = ImprovedDDPM(network=b, device=0, **shipped_diff_args())
    cb = WeightsCheckpoint(str(tmp_path), every_n_epochs=2)
    cb.set_model(ma)
    cb.on_epoch_end(0)
    assert not (tmp_path / 'cp_1').exists()
    cb.on_epoch_end(1)
    path = tmp_path / 'cp_2' / 'ckpt.weights.h5'
    assert path.exists()
    with h5.File(str(path)) as f:
        assert f.keys() == ['network']
    mb.load_weights(str(path))
    for n, _ in a.spec():
        np.testing.assert_array_equal(b.weights[n], a.weights[n])
