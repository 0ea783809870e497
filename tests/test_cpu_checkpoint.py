"""CPU tests of the TensorFlow checkpoint reader (pet_posterior_distribution_amd/checkpoint.py).

TensorFlow is not installed and the reference's checkpoints are Git-LFS pointers, so the reader is exercised on
bundles written here by a small writer that follows the published formats: TF table = LevelDB SSTable
(tensorflow/core/lib/io/format.h, block_builder.cc), TensorBundle (tensor_bundle.proto / tensor_bundle.cc string
encoding) and TrackableObjectGraph (trackable_object_graph.proto).  The object graph mirrors the attribute names of the
reference's networks.py (shared time MLP and encoder reachable from several parents).  Parity with a
TensorFlow-written file: unpinned.
"""
import os
import struct

import numpy as np
import pytest

from pet_posterior_distribution_amd import checkpoint as ck
from pet_posterior_distribution_amd.networks import UnetConditional, param_spec
from tests.helpers import shipped_net_args


# ----------------------------------------------------------------- protobuf / table writer (test side)
def varint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def field(num, payload):
    if isinstance(payload, int):
        return varint(num << 3) + varint(payload)
    if isinstance(payload, str):
        payload = payload.encode()
    return varint(num << 3 | 2) + varint(len(payload)) + payload


def fixed32(num, v):
    return varint(num << 3 | 5) + struct.pack('<I', v)


def block(entries, restart_interval=4):
    out, restarts, prev = bytearray(), [], b''
    for i, (k, v) in enumerate(entries):
        if i % restart_interval == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(k), len(prev)) and k[shared] == prev[shared]:
                shared += 1
        out += varint(shared) + varint(len(k) - shared) + varint(len(v)) + k[shared:] + v
        prev = k
    for r in restarts or [0]:
        out += struct.pack('<I', r)
    out += struct.pack('<I', len(restarts or [0]))
    return bytes(out)


def snappy_literal(data):
    """Valid snappy stream made of literal elements only."""
    out = bytearray(varint(len(data)))
    for i in range(0, len(data), 60):
        chunk = data[i:i + 60]
        out.append((len(chunk) - 1) << 2)
        out += chunk
    return bytes(out)


def write_table(path, items, compress=False):
    items = sorted(items, key=lambda kv: kv[0])
    f = bytearray()

    def put(contents, ctype=0):
        off = len(f)
        payload = snappy_literal(contents) if ctype == 1 else contents
        f.extend(payload)
        t = bytes([ctype])
        f.extend(t + struct.pack('<I', ck.mask_crc(ck.crc32c(payload + t))))
        return varint(off) + varint(len(payload))

    half = len(items) // 2                                   # two data blocks
    h1 = put(block(items[:half]), 1 if compress else 0)
    h2 = put(block(items[half:]), 0)
    meta = put(block([]))
    index = put(block([(items[half - 1][0], h1), (items[-1][0], h2)], 1))
    footer = (meta + index).ljust(40, b'\0') + struct.pack('<Q', ck.TABLE_MAGIC)
    f.extend(footer)
    with open(path, 'wb') as fh:
        fh.write(bytes(f))


def string_tensor(values):
    lens = b''.join(varint(len(v)) for v in values)
    return lens + struct.pack('<I', ck.mask_crc(ck.crc32c(lens))) + b''.join(values)


def write_bundle(prefix, tensors, graph, num_shards=2, compress=False):
    """tensors: {key: np.ndarray | [bytes]}; graph: list of (children {name: id}, attributes {name: key})."""
    tensors = dict(tensors)
    nodes = b''
    for children, attrs in graph:
        body = b''.join(field(1, field(1, nid) + field(2, name)) for name, nid in children.items())
        body += b''.join(field(2, field(1, name) + field(2, key) + field(3, key)) for name, key in attrs.items())
        nodes += field(1, body)
    tensors[ck.OBJECT_GRAPH_KEY] = [nodes]
    shards = [bytearray() for _ in range(num_shards)]
    items = [(b'', field(1, num_shards) + field(2, 0))]
    for i, (k, v) in enumerate(sorted(tensors.items())):
        sid = i % num_shards
        if isinstance(v, list):
            raw, dt, shape = string_tensor(v), ck.DT_STRING, ()
        else:
            raw, dt, shape = v.astype('<f4').tobytes(), 1, v.shape
        shp = b''.join(field(2, field(1, d)) for d in shape)
        # CRC32C in pure Python is slow: only small tensors carry one here (the reader checks it on request)
        crc = ck.mask_crc(ck.crc32c(raw)) if len(raw) <= 65536 else 0
        entry = field(1, dt) + field(2, shp) + field(3, sid) + field(4, len(shards[sid])) + field(5, len(raw)) + \
            fixed32(6, crc)
        shards[sid] += raw
        items.append((k.encode(), entry))
    for sid, data in enumerate(shards):
        with open(f'{prefix}.data-{sid:05d}-of-{num_shards:05d}', 'wb') as fh:
            fh.write(bytes(data))
    write_table(prefix + '.index', items, compress)


def reference_object_graph(weights, depth=4):
    """Object graph of an ImprovedDDPM checkpoint with networks.py's attribute names; returns (graph, tensors)."""
    nodes = []

    def node():
        nodes.append(({}, {}))
        return len(nodes) - 1

    tensors = {}

    def var(path, arr):
        nid = node()
        key = path + '/.ATTRIBUTES/VARIABLE_VALUE'
        nodes[nid][1]['VARIABLE_VALUE'] = key
        tensors[key] = arr
        return nid

    def dense(path, name):
        nid = node()
        nodes[nid][0]['kernel'] = var(path + '/kernel', weights[name + '.kernel'])
        nodes[nid][0]['bias'] = var(path + '/bias', weights[name + '.bias'])
        return nid

    def lst(items):
        nid = node()
        for i, c in enumerate(items):
            if c is not None:
                nodes[nid][0][str(i)] = c
        return nid

    root, net = node(), node()
    nodes[root][0]['network'] = net
    nodes[root][0]['optimizer'] = node()
    time_mlp = dense('network/cond_mlp_down/0/0/layer_with_weights-0', 'time_mlp')
    enc = node()
    nodes[enc][0]['encoder'] = node()
    for i in range(3):
        nodes[nodes[enc][0]['encoder']][0][f'layer_{i}'] = dense(f'network/encoder_cond/0/encoder/layer_{i}',
                                                                 f'cond_enc.hidden{i}')
    nodes[enc][0]['dense_z'] = lst([])
    nodes[nodes[enc][0]['dense_z']][0]['layer_0'] = dense('network/encoder_cond/0/dense_z/layer_0', 'cond_enc.z')
    nodes[net][0]['encoder_cond'] = lst([enc])

    def seq(p, first, proj):
        s = node()
        nodes[s][0]['layer_with_weights-0'] = first
        nodes[s][0]['layer_with_weights-1'] = proj
        nodes[s][0]['layer-2'] = first
        return s

    def block_node(p, name):
        b = node()
        nodes[b][0]['conv_l'] = lst([dense(p + '/conv_l/0', name + '.conv')])
        nodes[b][0]['res_conv'] = dense(p + '/res_conv', name + '.res')
        return b

    downs, cdown = [], []
    for d in range(depth):
        p = f'network/cond_mlp_down/{d}'
        cdown.append(lst([seq(p + '/0', time_mlp, dense(p + '/0/layer_with_weights-1', f'down{d}.time_proj')),
                          seq(p + '/1', enc, dense(p + '/1/layer_with_weights-1', f'down{d}.label_proj'))]))
        downs.append(lst([block_node(f'network/downs/{d}/0', f'down{d}'), node(), node()]))
    ups, cup = [], []
    for u in range(depth - 1):
        p = f'network/cond_mlp_up/{u}'
        cup.append(lst([seq(p + '/0', time_mlp, dense(p + '/0/layer_with_weights-1', f'up{u}.time_proj')),
                        seq(p + '/1', enc, dense(p + '/1/layer_with_weights-1', f'up{u}.label_proj'))]))
        ups.append(lst([node(), dense(f'network/ups/{u}/1', f'up{u}.upconv'), node(),
                        block_node(f'network/ups/{u}/3', f'up{u}')]))
    nodes[net][0]['downs'] = lst(downs)
    nodes[net][0]['cond_mlp_down'] = lst(cdown)
    nodes[net][0]['ups'] = lst(ups)
    nodes[net][0]['cond_mlp_up'] = lst(cup)
    nodes[net][0]['final_conv'] = dense('network/final_conv', 'final')
    # an Adam slot variable, as a real training checkpoint holds (ignored by the importer)
    tensors['network/final_conv/kernel/.OPTIMIZER_SLOT/optimizer/m/.ATTRIBUTES/VARIABLE_VALUE'] = \
        np.zeros_like(weights['final.kernel'])
    return nodes, tensors


@pytest.fixture(scope='module')
def weights():
    rng = np.random.default_rng(5)
    return {n: rng.standard_normal(s).astype(np.float32) for n, s in param_spec()}


# ----------------------------------------------------------------- tests
def test_crc32c_known_answer():
    assert ck.crc32c(b'123456789') == 0xE3069283          # CRC-32C check value
    assert ck.crc32c(b'') == 0


def test_snappy_copies():
    # "abcd" literal, then copy(offset 4, length 8): overlapping copy of its own output
    stream = varint(12) + bytes([3 << 2]) + b'abcd' + bytes([((8 - 4) << 2) | 1, 4])
    assert ck.snappy_decompress(stream) == b'abcdabcdabcd'
    data = bytes(range(200)) * 2
    assert ck.snappy_decompress(snappy_literal(data)) == data


@pytest.mark.parametrize('compress', [False, True])
def test_savedmodel_import_roundtrip(tmp_path, weights, compress):
    graph, tensors = reference_object_graph(weights)
    os.makedirs(tmp_path / 'cp_500' / 'variables')
    write_bundle(str(tmp_path / 'cp_500' / 'variables' / 'variables'), tensors, graph, compress=compress)
    b = ck.TensorBundle(str(tmp_path / 'cp_500'))
    assert b.num_shards == 2 and ck.OBJECT_GRAPH_KEY in b.keys()
    k = 'network/final_conv/kernel/.ATTRIBUTES/VARIABLE_VALUE'
    np.testing.assert_array_equal(b.get(k, verify=True), weights['final.kernel'])
    net = UnetConditional(**shipped_net_args())
    net.build((None, 48, 2))
    net.load_weights(str(tmp_path / 'cp_500'))           # SavedModel directory, as main_script.py saves it
    for n, _ in param_spec():
        np.testing.assert_array_equal(net.weights[n], weights[n], err_msg=n)
    net2 = UnetConditional(**shipped_net_args())
    net2.build((None, 48, 2))
    net2.load_weights(str(tmp_path / 'cp_500' / 'variables' / 'variables.index'))
    np.testing.assert_array_equal(net2.weights['final.kernel'], weights['final.kernel'])


def test_import_errors(tmp_path, weights):
    graph, tensors = reference_object_graph(weights)
    bad = dict(tensors)
    key = 'network/final_conv/kernel/.ATTRIBUTES/VARIABLE_VALUE'
    bad[key] = np.zeros((1, 128, 2), np.float32)          # learn_variance mismatch: 2 output channels
    write_bundle(str(tmp_path / 'a'), bad, graph)
    with pytest.raises(ck.CheckpointError, match='final.kernel'):
        ck.load_unet_weights(str(tmp_path / 'a'), param_spec())
    write_bundle(str(tmp_path / 'b'), tensors, graph)
    raw = bytearray(open(str(tmp_path / 'b.index'), 'rb').read())
    raw[10] ^= 0xFF                                       # corrupt the first data block
    open(str(tmp_path / 'b.index'), 'wb').write(bytes(raw))
    with pytest.raises(ck.CheckpointError, match='checksum'):
        ck.TensorBundle(str(tmp_path / 'b'))
    with pytest.raises(ck.CheckpointError, match='magic'):
        open(str(tmp_path / 'c.index'), 'wb').write(b'\0' * 64)
        ck.TensorBundle(str(tmp_path / 'c'))
    net = UnetConditional(**shipped_net_args())
    net.build((None, 48, 2))
    with pytest.raises(FileNotFoundError):                # .weights.h5 is read by h5.py (test_cpu_h5.py)
        net.load_weights(str(tmp_path / 'ckpt.weights.h5'))
