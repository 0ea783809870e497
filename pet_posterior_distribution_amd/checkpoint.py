"""TensorFlow checkpoint (TensorBundle) reader and Keras weight importer.

The reference ships its trained models as SavedModel directories, `cp_<epoch>/variables/variables.index` +
`variables.data-00000-of-00001` (main_script.py:263 WeightsCheckpoint, :299 diff_model.save, `results/nROI48/...`).
That pair is TensorFlow's TensorBundle format, and this module reads it without TensorFlow:

* `variables.index` is a TF table, the LevelDB SSTable layout (tensorflow/core/lib/io/format.h): a 48-byte footer
  (metaindex and index block handles + magic 0xdb4775248b80fb57), prefix-compressed blocks with restart arrays and a
  5-byte trailer (compression type + masked CRC32C).  Type 0 (none) and 1 (snappy) are decoded.
* Entry "" holds a BundleHeaderProto (num_shards, endianness); every other entry a BundleEntryProto (dtype, shape,
  shard_id, offset, size, crc32c) locating the tensor's bytes in `<prefix>.data-<shard>-of-<n>`.
* `_CHECKPOINTABLE_OBJECT_GRAPH` is a string tensor holding the TrackableObjectGraph: nodes with named children and
  the checkpoint key of each variable.  The importer walks it by the attribute names networks.py gives its layers
  (`downs`, `ups`, `cond_mlp_down`, `cond_mlp_up`, `encoder_cond`, `final_conv`; ConvBlock `conv_l` / `res_conv`;
  Encoder `encoder` / `dense_z`; Sequential `layer_with_weights-N`), so shared layers resolve whichever path the
  checkpoint chose as canonical.

Parity: the real checkpoints are Git-LFS pointers in the reference checkout and TensorFlow is not installed, so this
reader is checked against files written by a writer that follows the same published format (tests/test_cpu_checkpoint.py),
not against a TensorFlow-written file: parity unpinned.
"""
import os
import struct

import numpy as np

TABLE_MAGIC = 0xdb4775248b80fb57
FOOTER_LEN = 48
OBJECT_GRAPH_KEY = '_CHECKPOINTABLE_OBJECT_GRAPH'

# tensorflow/core/framework/types.proto
DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
          10: np.bool_, 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
DT_STRING = 7
DT_BFLOAT16 = 14


class CheckpointError(ValueError):
    pass


# ----------------------------------------------------------------- CRC32C (Castagnoli), masked as in TF/LevelDB
def _crc32c_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        t.append(c)
    return t


_CRC_TABLE = _crc32c_table()


def crc32c(data, crc=0):
    c = crc ^ 0xFFFFFFFF
    tab = _CRC_TABLE
    for b in data:
        c = tab[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def mask_crc(c):
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


# ----------------------------------------------------------------- varints and protobuf wire format
def read_varint(buf, pos):
    shift = result = 0
    while True:
        if pos >= len(buf):
            raise CheckpointError('truncated varint')
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift > 63:
            raise CheckpointError('varint too long')


def proto_fields(buf):
    """Yield (field_number, wire_type, value) of a serialized protobuf message."""
    pos = 0
    while pos < len(buf):
        key, pos = read_varint(buf, pos)
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = read_varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from('<Q', buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = read_varint(buf, pos)
            v = bytes(buf[pos:pos + n])
            pos += n
        elif wt == 5:
            v = struct.unpack_from('<I', buf, pos)[0]
            pos += 4
        else:
            raise CheckpointError(f'unsupported wire type {wt}')
        yield field, wt, v


# ----------------------------------------------------------------- snappy (table compression type 1)
def snappy_decompress(buf):
    n, pos = read_varint(buf, 0)
    out = bytearray()
    while pos < len(buf):
        tag = buf[pos]
        pos += 1
        kind = tag & 3
        if kind == 0:                                   # literal
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(buf[pos:pos + nb], 'little')
                pos += nb
            ln += 1
            out += buf[pos:pos + ln]
            pos += ln
            continue
        if kind == 1:
            ln = 4 + ((tag >> 2) & 7)
            off = ((tag >> 5) << 8) | buf[pos]
            pos += 1
        elif kind == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[pos:pos + 2], 'little')
            pos += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[pos:pos + 4], 'little')
            pos += 4
        if off == 0 or off > len(out):
            raise CheckpointError('bad snappy copy offset')
        for _ in range(ln):                              # copies may overlap their own output
            out.append(out[-off])
    if len(out) != n:
        raise CheckpointError('snappy length mismatch')
    return bytes(out)


# ----------------------------------------------------------------- TF table (SSTable) reader
def _block_handle(buf, pos):
    off, pos = read_varint(buf, pos)
    size, pos = read_varint(buf, pos)
    return (off, size), pos


def _read_block(data, handle, verify=True):
    off, size = handle
    if off + size + 5 > len(data):
        raise CheckpointError('block past end of table')
    contents = data[off:off + size]
    ctype = data[off + size]
    if verify:
        want = struct.unpack_from('<I', data, off + size + 1)[0]
        if mask_crc(crc32c(data[off:off + size + 1])) != want:
            raise CheckpointError('table block checksum mismatch')
    if ctype == 1:
        contents = snappy_decompress(contents)
    elif ctype != 0:
        raise CheckpointError(f'unsupported table compression {ctype}')
    return contents


def _block_entries(block):
    if len(block) < 4:
        raise CheckpointError('short block')
    n_restarts = struct.unpack_from('<I', block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * n_restarts
    pos, key = 0, b''
    while pos < end:
        shared, pos = read_varint(block, pos)
        non_shared, pos = read_varint(block, pos)
        vlen, pos = read_varint(block, pos)
        key = key[:shared] + bytes(block[pos:pos + non_shared])
        pos += non_shared
        yield key, bytes(block[pos:pos + vlen])
        pos += vlen


def read_table(path, verify=True):
    """All (key, value) pairs of a TF table file, in key order."""
    with open(path, 'rb') as f:
        data = f.read()
    if len(data) < FOOTER_LEN:
        raise CheckpointError(f'{path}: too short for a table')
    magic = struct.unpack_from('<Q', data, len(data) - 8)[0]
    if magic != TABLE_MAGIC:
        raise CheckpointError(f'{path}: not a TensorFlow table (bad magic)')
    foot = data[len(data) - FOOTER_LEN:]
    _, pos = _block_handle(foot, 0)                     # metaindex (unused)
    index_handle, _ = _block_handle(foot, pos)
    out = {}
    for _, hv in _block_entries(_read_block(data, index_handle, verify)):
        handle, _ = _block_handle(hv, 0)
        for k, v in _block_entries(_read_block(data, handle, verify)):
            out[k] = v
    return out


# ----------------------------------------------------------------- TensorBundle
def _parse_shape(buf):
    dims = []
    for f, _, v in proto_fields(buf):
        if f == 2:
            size = 0
            for g, _, w in proto_fields(v):
                if g == 1:
                    size = w - (1 << 64) if w >= 1 << 63 else w
            dims.append(size)
        elif f == 3 and v:
            raise CheckpointError('unknown-rank tensor')
    return tuple(dims)


def _parse_entry(buf):
    e = {'dtype': 0, 'shape': (), 'shard_id': 0, 'offset': 0, 'size': 0, 'crc32c': None, 'sliced': False}
    for f, _, v in proto_fields(buf):
        if f == 1:
            e['dtype'] = v
        elif f == 2:
            e['shape'] = _parse_shape(v)
        elif f == 3:
            e['shard_id'] = v
        elif f == 4:
            e['offset'] = v
        elif f == 5:
            e['size'] = v
        elif f == 6:
            e['crc32c'] = v
        elif f == 7:
            e['sliced'] = True
    return e


class TensorBundle:
    """Read-only view of a TensorBundle checkpoint `<prefix>.index` / `<prefix>.data-*`."""

    def __init__(self, prefix, verify=True):
        if os.path.isdir(prefix):                         # a SavedModel directory
            prefix = os.path.join(prefix, 'variables', 'variables')
        self.prefix = prefix
        table = read_table(prefix + '.index', verify)
        self.num_shards = 1
        head = table.pop(b'', None)
        if head is not None:
            for f, _, v in proto_fields(head):
                if f == 1:
                    self.num_shards = v
                elif f == 2 and v != 0:
                    raise CheckpointError('big-endian bundles are not supported')
        self.entries = {k.decode(): _parse_entry(v) for k, v in table.items()}
        self._graph = None

    def keys(self):
        return list(self.entries)

    def _raw(self, e):
        fn = f'{self.prefix}.data-{e["shard_id"]:05d}-of-{self.num_shards:05d}'
        with open(fn, 'rb') as f:
            f.seek(e['offset'])
            raw = f.read(e['size'])
        if len(raw) != e['size']:
            raise CheckpointError(f'{fn}: short read')
        return raw

    def get(self, key, verify=False):
        """The tensor `key` as a NumPy array (string tensors: list of bytes).  verify=True also checks the
        entry's CRC32C (pure Python, slow for large tensors)."""
        if key not in self.entries:
            raise KeyError(key)
        e = self.entries[key]
        if e['sliced']:
            raise CheckpointError(f'{key}: partitioned (sliced) variables are not supported')
        raw = self._raw(e)
        if verify and e['crc32c'] is not None and mask_crc(crc32c(raw)) != e['crc32c']:
            raise CheckpointError(f'{key}: checksum mismatch')
        n = int(np.prod(e['shape'])) if e['shape'] else 1
        if e['dtype'] == DT_STRING:
            pos, lens = 0, []
            for _ in range(n):
                ln, pos = read_varint(raw, pos)
                lens.append(ln)
            pos += 4                                      # masked CRC32C of the length varints
            out = []
            for ln in lens:
                out.append(raw[pos:pos + ln])
                pos += ln
            return out
        if e['dtype'] == DT_BFLOAT16:
            u = np.frombuffer(raw, '<u2').astype(np.uint32) << 16
            return u.view(np.float32).reshape(e['shape'])
        if e['dtype'] not in DTYPES:
            raise CheckpointError(f'{key}: unsupported dtype {e["dtype"]}')
        return np.frombuffer(raw, np.dtype(DTYPES[e['dtype']]).newbyteorder('<')).reshape(e['shape']).copy()

    # ------------------------------------------------------------- object graph
    def object_graph(self):
        """TrackableObjectGraph as a list of nodes {'children': {name: id}, 'attributes': {name: checkpoint_key}}."""
        if self._graph is None:
            if OBJECT_GRAPH_KEY not in self.entries:
                raise CheckpointError('checkpoint has no object graph (name-based checkpoint)')
            raw = self.get(OBJECT_GRAPH_KEY)[0]
            nodes = []
            for f, _, v in proto_fields(raw):
                if f != 1:
                    continue
                node = {'children': {}, 'attributes': {}}
                for g, _, w in proto_fields(v):
                    if g == 1:
                        nid, name = 0, ''
                        for h, _, x in proto_fields(w):
                            if h == 1:
                                nid = x
                            elif h == 2:
                                name = x.decode()
                        node['children'][name] = nid
                    elif g == 2:
                        name, key = '', ''
                        for h, _, x in proto_fields(w):
                            if h == 1:
                                name = x.decode()
                            elif h == 3:
                                key = x.decode()
                        node['attributes'][name] = key
                nodes.append(node)
            self._graph = nodes
        return self._graph

    def resolve(self, path, root=0):
        """Node id reached from `root` by a '/'-separated child path; alternatives separated by '|' in one
        component are tried in order."""
        g = self.object_graph()
        nid = root
        for comp in path.split('/'):
            for alt in comp.split('|'):
                if alt in g[nid]['children']:
                    nid = g[nid]['children'][alt]
                    break
            else:
                raise KeyError(f'{path}: no child {comp!r} (has {sorted(g[nid]["children"])[:12]})')
        return nid

    def variable(self, path, root=0):
        node = self.object_graph()[self.resolve(path, root)]
        key = node['attributes'].get('VARIABLE_VALUE')
        if key is None:
            raise KeyError(f'{path}: not a variable')
        return self.get(key)


# ----------------------------------------------------------------- UnetConditional weights
_SEQ_W = 'layer_with_weights-{}'


def unet_object_paths(depth=4):
    """Our parameter name -> object-graph path under the UnetConditional node (networks.py:781-992)."""
    paths = {}

    def dense(name, p):
        paths[name + '.kernel'] = p + '/kernel'
        paths[name + '.bias'] = p + '/bias'

    # shared time MLP Dense(48) (cond_emb_layer[0][0]) and the condition encoder (encoder_cond[0])
    dense('time_mlp', 'cond_mlp_down/0/0/' + _SEQ_W.format(0))
    for i in range(3):
        dense(f'cond_enc.hidden{i}', f'encoder_cond/0/encoder/layer_{i}')
    dense('cond_enc.z', 'encoder_cond/0/dense_z/layer_0')
    for d in range(depth):
        dense(f'down{d}.time_proj', f'cond_mlp_down/{d}/0/' + _SEQ_W.format(1))
        dense(f'down{d}.label_proj', f'cond_mlp_down/{d}/1/' + _SEQ_W.format(1))
        dense(f'down{d}.conv', f'downs/{d}/0/conv_l/0')
        dense(f'down{d}.res', f'downs/{d}/0/res_conv')
    for u in range(depth - 1):
        dense(f'up{u}.time_proj', f'cond_mlp_up/{u}/0/' + _SEQ_W.format(1))
        dense(f'up{u}.label_proj', f'cond_mlp_up/{u}/1/' + _SEQ_W.format(1))
        dense(f'up{u}.upconv', f'ups/{u}/1')
        dense(f'up{u}.conv', f'ups/{u}/3/conv_l/0')
        dense(f'up{u}.res', f'ups/{u}/3/res_conv')
    dense('final', 'final_conv')
    return paths


def load_unet_weights(prefix, spec, network_path=None):
    """{our name: array} for every entry of `spec` ([(name, shape)]) from a TensorBundle checkpoint of the
    ImprovedDDPM model (root child 'network') or of the UnetConditional itself."""
    b = TensorBundle(prefix)
    g = b.object_graph()
    if network_path is None:
        network_path = 'network' if 'network' in g[0]['children'] else ''
    root = b.resolve(network_path) if network_path else 0
    paths = unet_object_paths()
    out = {}
    for name, shape in spec:
        if name not in paths:
            raise KeyError(f'no checkpoint path for {name}')
        arr = np.asarray(b.variable(paths[name], root), dtype=np.float32)
        if tuple(arr.shape) != tuple(shape):
            raise CheckpointError(f'{name} ({paths[name]}): shape {arr.shape} != {tuple(shape)}')
        out[name] = arr
    return out
