"""Minimal HDF5 reader / writer and the Keras ``.weights.h5`` importer.

The reference evaluates from ``cp_<epoch>/ckpt.weights.h5`` (main_script.py:412, written by
``WeightsCheckpoint`` -> ``model.save_weights``, networks.py:152-180).  With TF 2.19, ``tf.keras`` is Keras 3,
whose ``saving_lib`` writes that file through h5py: one group per saveable object along the attribute path,
and each layer's own variables as datasets ``<path>/vars/0, 1, ...`` (kernel, then bias).  h5py is not
installed here, so this module reads the HDF5 file format itself (HDF5 File Format Specification v3):

* superblock versions 0-3 (found at 0, 512, 1024, ... like the library, i.e. behind a user block);
* object headers v1 and v2 ("OHDR"/"OCHK", continuation messages);
* groups: symbol tables (v1 B-tree "TREE" of "SNOD" nodes + local heap "HEAP") and compact link messages;
  dense link storage (fractal heaps) is not supported and raises;
* datasets: dataspace v1/v2, fixed-point / IEEE floating-point / fixed-length string datatypes,
  data layout v1-v3 (compact, contiguous, chunked through a v1 B-tree with deflate / shuffle / fletcher32);
* attributes v1-v3 (numeric and fixed-length strings).

Pinning: the reader's structure parsing is checked against an HDF5 file written by the HDF5 library itself
(MATLAB 7.4 v7.3 MAT-file shipped in scipy's test data, tests/test_cpu_h5.py); the Keras layout is derived from
Keras 3's saving_lib conventions, and no TF-written ``.weights.h5`` of the reference exists offline (the
checkpoints are Git-LFS pointers), so the importer's path mapping is parity unpinned.

The writer (``write``) emits superblock v0 / object header v1 / symbol-table groups / contiguous little-endian
datasets, the layout h5py writes by default, so ``UnetConditional.save_weights('x.weights.h5')`` round-trips.
"""
from __future__ import annotations

import mmap
import struct
import zlib

import numpy as np

SIGNATURE = b'\x89HDF\r\n\x1a\n'
UNDEF = 0xFFFFFFFFFFFFFFFF


class H5Error(ValueError):
    pass


# ============================================================================ reader
class _Reader:
    def __init__(self, buf):
        self.buf = buf
        self.base = None
        for off in [0] + [512 << k for k in range(20)]:
            if off + 8 > len(buf):
                break
            if buf[off:off + 8] == SIGNATURE:
                self.base = off
                break
        if self.base is None:
            raise H5Error('not an HDF5 file (no superblock signature)')
        self._superblock()

    # ---- primitives
    def u(self, pos, n):
        return int.from_bytes(self.buf[pos:pos + n], 'little')

    def addr(self, pos):
        a = self.u(pos, self.so)
        return UNDEF if a == (1 << (8 * self.so)) - 1 else a

    def _superblock(self):
        p = self.base + 8
        ver = self.buf[p]
        self.sb_version = ver
        if ver in (0, 1):
            self.so, self.sl = self.buf[p + 5], self.buf[p + 6]
            self.leaf_k = self.u(p + 8, 2)
            q = p + 16 + (4 if ver == 1 else 0)
            base_addr = self.u(q, self.so)
            q += 4 * self.so                       # base, free-space, EOF, driver info
            # root group symbol table entry: link name offset, object header address, cache type, scratch
            self.root = self.u(q + self.so, self.so)
        elif ver in (2, 3):
            self.so, self.sl = self.buf[p + 1], self.buf[p + 2]
            q = p + 4
            base_addr = self.u(q, self.so)
            self.root = self.u(q + 3 * self.so, self.so)
        else:
            raise H5Error(f'superblock version {ver} not supported')
        # the library constrains the base address to the superblock's own position
        self.off = self.base if base_addr in (0, self.base) else base_addr

    def a(self, rel):
        return self.off + rel

    # ---- object headers: [(type, flags, data)]
    def messages(self, addr):
        pos = self.a(addr)
        if self.buf[pos:pos + 4] == b'OHDR':
            return self._messages_v2(pos)
        if self.buf[pos] != 1:
            raise H5Error(f'object header version {self.buf[pos]} at {addr:#x} not supported')
        n = self.u(pos + 2, 2)
        size = self.u(pos + 8, 4)
        out = []
        blocks = [(pos + 16, size)]
        while blocks and len(out) < n:
            start, length = blocks.pop(0)
            q, end = start, start + length
            while q + 8 <= end and len(out) < n:
                mtype, msize, mflags = self.u(q, 2), self.u(q + 2, 2), self.buf[q + 4]
                data = bytes(self.buf[q + 8:q + 8 + msize])
                if mtype == 0x10:   # continuation
                    blocks.append((self.a(int.from_bytes(data[:self.so], 'little')),
                                   int.from_bytes(data[self.so:self.so + self.sl], 'little')))
                out.append((mtype, mflags, data))
                q += 8 + msize
        return out

    def _messages_v2(self, pos):
        flags = self.buf[pos + 5]
        q = pos + 6
        if flags & 0x20:
            q += 16
        if flags & 0x10:
            q += 4
        nsz = 1 << (flags & 3)
        size = self.u(q, nsz)
        q += nsz
        cre = bool(flags & 0x04)
        out = []
        blocks = [(q, size)]
        while blocks:
            start, length = blocks.pop(0)
            q, end = start, start + length
            hdr = 4 + (2 if cre else 0)
            while q + hdr <= end:
                mtype, msize, mflags = self.buf[q], self.u(q + 1, 2), self.buf[q + 3]
                data = bytes(self.buf[q + hdr:q + hdr + msize])
                if mtype == 0x10:
                    caddr = self.a(int.from_bytes(data[:self.so], 'little'))
                    clen = int.from_bytes(data[self.so:self.so + self.sl], 'little')
                    if self.buf[caddr:caddr + 4] != b'OCHK':
                        raise H5Error('bad continuation block')
                    blocks.append((caddr + 4, clen - 8))
                out.append((mtype, mflags, data))
                q += hdr + msize
        return out

    # ---- groups
    def links(self, addr):
        """{name: object header address} of a group."""
        out = {}
        for mtype, _, data in self.messages(addr):
            if mtype == 0x11:                        # symbol table: B-tree + local heap
                bt = int.from_bytes(data[:self.so], 'little')
                heap = int.from_bytes(data[self.so:2 * self.so], 'little')
                self._walk_group_btree(bt, self._local_heap(heap), out)
            elif mtype == 0x06:                      # link message (compact storage)
                name, target = self._link(data)
                if target is not None:
                    out[name] = target
            elif mtype == 0x02:                      # link info
                fh = int.from_bytes(data[2 + (8 if data[1] & 1 else 0):][:self.so], 'little')
                if fh != (1 << (8 * self.so)) - 1:
                    raise H5Error('dense link storage (fractal heap) is not supported')
        return out

    def _local_heap(self, addr):
        p = self.a(addr)
        if self.buf[p:p + 4] != b'HEAP':
            raise H5Error('bad local heap')
        size = self.u(p + 8, self.sl)
        data = self.a(self.u(p + 8 + 2 * self.sl, self.so))
        return bytes(self.buf[data:data + size])

    @staticmethod
    def _cstr(heap, off):
        e = heap.index(b'\0', off)
        return heap[off:e].decode('utf-8')

    def _walk_group_btree(self, addr, heap, out):
        p = self.a(addr)
        if self.buf[p:p + 4] != b'TREE':
            raise H5Error('bad group B-tree node')
        ntype, level, used = self.buf[p + 4], self.buf[p + 5], self.u(p + 6, 2)
        if ntype != 0:
            raise H5Error('not a group B-tree')
        q = p + 8 + 2 * self.so + self.sl            # past the siblings and key 0
        for _ in range(used):
            child = self.u(q, self.so)
            q += self.so + self.sl
            if level > 0:
                self._walk_group_btree(child, heap, out)
            else:
                self._snod(child, heap, out)

    def _snod(self, addr, heap, out):
        p = self.a(addr)
        if self.buf[p:p + 4] != b'SNOD':
            raise H5Error('bad symbol table node')
        n = self.u(p + 6, 2)
        q = p + 8
        for _ in range(n):
            name = self._cstr(heap, self.u(q, self.so))
            out[name] = self.u(q + self.so, self.so)
            q += 2 * self.so + 24

    def _link(self, d):
        flags = d[1]
        q = 2
        ltype = 0
        if flags & 0x08:
            ltype = d[q]
            q += 1
        if flags & 0x04:
            q += 8
        if flags & 0x10:
            q += 1
        nl = 1 << (flags & 3)
        n = int.from_bytes(d[q:q + nl], 'little')
        q += nl
        name = d[q:q + n].decode('utf-8')
        q += n
        if ltype != 0:                               # soft / external links are not followed
            return name, None
        return name, int.from_bytes(d[q:q + self.so], 'little')

    # ---- datasets and attributes
    def dataspace(self, d):
        ver, rank, flags = d[0], d[1], d[2]
        q = 8 if ver == 1 else 4
        if ver == 2 and d[3] == 2:                   # null dataspace
            return None
        return tuple(int.from_bytes(d[q + i * self.sl:q + (i + 1) * self.sl], 'little') for i in range(rank))

    @staticmethod
    def datatype(d):
        """(numpy dtype or ('S', size), byte length of the message)."""
        cls, bits = d[0] & 0x0F, d[1] | (d[2] << 8) | (d[3] << 16)
        size = int.from_bytes(d[4:8], 'little')
        order = '>' if bits & 1 else '<'
        if cls == 0:
            signed = bool(bits & 0x08)
            return np.dtype(f'{order}{"i" if signed else "u"}{size}'), 12
        if cls == 1:
            if size not in (2, 4, 8):
                raise H5Error(f'float size {size} not supported')
            return np.dtype(f'{order}f{size}'), 20
        if cls == 3:
            return ('S', size), 8
        raise H5Error(f'datatype class {cls} not supported')

    def chunk_btree(self, addr, ndims, out):
        p = self.a(addr)
        if self.buf[p:p + 4] != b'TREE' or self.buf[p + 4] != 1:
            raise H5Error('bad chunk B-tree node')
        level, used = self.buf[p + 5], self.u(p + 6, 2)
        q = p + 8 + 2 * self.so
        ksz = 8 + 8 * ndims                           # size, filter mask, ndims offsets (rank + 1)
        for _ in range(used):
            size, mask = self.u(q, 4), self.u(q + 4, 4)
            offs = tuple(self.u(q + 8 + 8 * i, 8) for i in range(ndims))
            child = self.u(q + ksz, self.so)
            if level > 0:
                self.chunk_btree(child, ndims, out)
            else:
                out.append((offs, size, mask, child))
            q += ksz + self.so


class Dataset:
    def __init__(self, f, addr, name):
        self._f, self.addr, self.name = f, addr, name
        r = f._r
        self.shape, self.dtype, self._layout, self._filters = None, None, None, []
        self.attrs = {}
        for mtype, _, d in r.messages(addr):
            if mtype == 0x01:
                self.shape = r.dataspace(d)
            elif mtype == 0x03:
                self.dtype = r.datatype(d)[0]
            elif mtype == 0x08:
                self._layout = d
            elif mtype == 0x0B:
                self._filters = _filters(d)
            elif mtype == 0x0C:
                k, v = _attribute(r, d)
                self.attrs[k] = v

    def read(self):
        r = self._f._r
        d = self._layout
        shape = self.shape if self.shape is not None else ()
        if isinstance(self.dtype, tuple):
            raise H5Error('string datasets are not supported')
        n = int(np.prod(shape)) if shape else 1
        nbytes = n * self.dtype.itemsize
        ver = d[0]
        if ver == 3:
            cls = d[1]
            if cls == 0:
                raw = d[4:4 + int.from_bytes(d[2:4], 'little')]
            elif cls == 1:
                a = int.from_bytes(d[2:2 + r.so], 'little')
                raw = b'\0' * nbytes if a == (1 << (8 * r.so)) - 1 else bytes(r.buf[r.a(a):r.a(a) + nbytes])
            elif cls == 2:
                rank = d[2] - 1
                bt = int.from_bytes(d[3:3 + r.so], 'little')
                cdims = [int.from_bytes(d[3 + r.so + 4 * i:7 + r.so + 4 * i], 'little') for i in range(rank)]
                return self._read_chunked(bt, cdims, shape).reshape(shape)
            else:
                raise H5Error(f'layout class {cls} not supported')
        elif ver in (1, 2):
            rank, cls = d[1], d[2]
            q = 8
            if cls == 0:                               # compact: dims then size + data
                q += 4 * rank
                sz = int.from_bytes(d[q:q + 4], 'little')
                raw = d[q + 4:q + 4 + sz]
            else:
                a = int.from_bytes(d[q:q + r.so], 'little')
                if cls == 2:
                    cdims = [int.from_bytes(d[q + r.so + 4 * i:q + r.so + 4 * i + 4], 'little')
                             for i in range(rank - 1)]
                    return self._read_chunked(a, cdims, shape).reshape(shape)
                raw = bytes(r.buf[r.a(a):r.a(a) + nbytes])
        else:
            raise H5Error(f'layout message version {ver} not supported')
        return np.frombuffer(raw[:nbytes], dtype=self.dtype).reshape(shape).astype(self.dtype.newbyteorder('='))

    def _read_chunked(self, bt, cdims, shape):
        r = self._f._r
        out = np.zeros(shape, dtype=self.dtype.newbyteorder('='))
        chunks = []
        if bt != (1 << (8 * r.so)) - 1:
            r.chunk_btree(bt, len(shape) + 1, chunks)
        csz = int(np.prod(cdims)) * self.dtype.itemsize
        for offs, size, mask, addr in chunks:
            raw = bytes(r.buf[r.a(addr):r.a(addr) + size])
            for k, (fid, vals) in reversed(list(enumerate(self._filters))):
                if mask & (1 << k):
                    continue
                if fid == 1:
                    raw = zlib.decompress(raw)
                elif fid == 2:                          # shuffle
                    es = self.dtype.itemsize
                    raw = np.frombuffer(raw, np.uint8).reshape(es, -1).T.tobytes()
                elif fid == 3:                          # fletcher32: drop the checksum
                    raw = raw[:-4]
                else:
                    raise H5Error(f'filter {fid} not supported')
            block = np.frombuffer(raw[:csz], dtype=self.dtype).reshape(cdims)
            sl = tuple(slice(o, min(o + c, s)) for o, c, s in zip(offs, cdims, shape))
            out[sl] = block[tuple(slice(0, s.stop - s.start) for s in sl)]
        return out


def _filters(d):
    ver, n = d[0], d[1]
    q = 8 if ver == 1 else 2
    out = []
    for _ in range(n):
        fid = int.from_bytes(d[q:q + 2], 'little')
        q += 2
        nlen = 0
        if ver == 1 or fid >= 256:
            nlen = int.from_bytes(d[q:q + 2], 'little')
            q += 2
        q += 2                                            # flags
        nv = int.from_bytes(d[q:q + 2], 'little')
        q += 2
        if ver == 1:
            q += (nlen + 7) // 8 * 8
        else:
            q += nlen
        vals = [int.from_bytes(d[q + 4 * i:q + 4 * i + 4], 'little') for i in range(nv)]
        q += 4 * nv
        if ver == 1 and nv % 2:
            q += 4
        out.append((fid, vals))
    return out


def _attribute(r, d):
    ver = d[0]
    nsz, tsz, ssz = (int.from_bytes(d[k:k + 2], 'little') for k in (2, 4, 6))
    q = 8 if ver < 3 else 9
    pad = (lambda n: (n + 7) // 8 * 8) if ver == 1 else (lambda n: n)
    name = d[q:q + nsz].split(b'\0')[0].decode('utf-8')
    q += pad(nsz)
    dt = r.datatype(d[q:q + tsz])[0]
    q += pad(tsz)
    shape = r.dataspace(d[q:q + ssz])
    q += pad(ssz)
    n = int(np.prod(shape)) if shape else 1
    if isinstance(dt, tuple):
        vals = [d[q + i * dt[1]:q + (i + 1) * dt[1]].split(b'\0')[0].decode('utf-8', 'replace') for i in range(n)]
        return name, vals[0] if not shape else vals
    arr = np.frombuffer(d[q:q + n * dt.itemsize], dtype=dt).reshape(shape or ())
    return name, arr


class Group:
    def __init__(self, f, addr, name='/'):
        self._f, self.addr, self.name = f, addr, name
        self._links = None
        self._attrs = None

    def keys(self):
        if self._links is None:
            self._links = self._f._r.links(self.addr)
        return sorted(self._links)

    @property
    def attrs(self):
        if self._attrs is None:
            self._attrs = dict(_attribute(self._f._r, d) for t, _, d in self._f._r.messages(self.addr) if t == 0x0C)
        return self._attrs

    def __contains__(self, path):
        try:
            self[path]
            return True
        except KeyError:
            return False

    def __getitem__(self, path):
        node = self
        for comp in [c for c in path.split('/') if c]:
            if not isinstance(node, Group):
                raise KeyError(path)
            node.keys()
            if comp not in node._links:
                raise KeyError(f'{path}: no member {comp!r} in {node.name}')
            node = self._f._open(node._links[comp], (node.name.rstrip('/') + '/' + comp))
        return node

    def visit(self, fn, _prefix=''):
        """fn(path, obj) for every object below this group, depth first (sorted names)."""
        for k in self.keys():
            obj = self[k]
            p = _prefix + k
            fn(p, obj)
            if isinstance(obj, Group):
                obj.visit(fn, p + '/')


class File(Group):
    """Read-only HDF5 file: ``File(path)['a/b'].read()``."""

    def __init__(self, path):
        self._fh = open(path, 'rb')
        try:
            self._mm = mmap.mmap(self._fh.fileno(), 0, access=mmap.ACCESS_READ)
        except ValueError:
            raise H5Error('empty file')
        self._r = _Reader(self._mm)
        super().__init__(self, self._r.root, '/')

    def _open(self, addr, name):
        for mtype, _, _d in self._r.messages(addr):
            if mtype in (0x11, 0x06, 0x02):
                return Group(self, addr, name)
        return Dataset(self, addr, name)

    def close(self):
        self._mm.close()
        self._fh.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# ============================================================================ writer
class _Writer:
    """Superblock v0, object header v1, symbol-table groups, contiguous little-endian datasets."""
    LEAF_K, NODE_K = 4, 16

    def __init__(self):
        self.out = bytearray()

    def alloc(self, data, align=8):
        while len(self.out) % align:
            self.out += b'\0'
        p = len(self.out)
        self.out += data
        return p

    @staticmethod
    def _msg(mtype, data, flags=0):
        data = bytes(data) + b'\0' * (-len(data) % 8)
        return struct.pack('<HHB3x', mtype, len(data), flags) + data

    def object_header(self, msgs):
        body = b''.join(msgs)
        hdr = struct.pack('<BBHII', 1, 0, len(msgs), 1, len(body)) + b'\0' * 4
        return self.alloc(hdr + body)

    def dataset(self, arr):
        arr = np.ascontiguousarray(arr)
        dt = arr.dtype.newbyteorder('<')
        arr = arr.astype(dt, copy=False)
        data_addr = self.alloc(arr.tobytes()) if arr.nbytes else UNDEF
        space = struct.pack('<BBBx4x', 1, arr.ndim, 0) + b''.join(struct.pack('<Q', s) for s in arr.shape)
        if dt.kind == 'f':
            sz = dt.itemsize
            ebits, mbits, bias = {2: (5, 10, 15), 4: (8, 23, 127), 8: (11, 52, 1023)}[sz]
            # class bit field: little endian, mantissa normalisation 2 (implied MSB), sign at bit 8 * sz - 1
            cls_bits = (0x20 | ((sz * 8 - 1) << 8)).to_bytes(3, 'little')
            # properties: bit offset, precision, exponent location / size, mantissa location / size, bias
            dtype_msg = bytes([0x11]) + cls_bits + struct.pack('<I', sz) + \
                struct.pack('<HHBBBBI', 0, sz * 8, mbits, ebits, 0, mbits, bias)
        elif dt.kind in 'iu':
            sz = dt.itemsize
            dtype_msg = bytes([0x10, 0x08 if dt.kind == 'i' else 0, 0, 0]) + struct.pack('<I', sz) + \
                struct.pack('<HH', 0, sz * 8)
        else:
            raise H5Error(f'dtype {dt} not supported by the writer')
        layout = struct.pack('<BBQQ', 3, 1, data_addr, arr.nbytes)
        fill = bytes([2, 2, 2, 0])        # fill value message v2: late allocation, write-if-set, undefined
        return self.object_header([self._msg(0x01, space), self._msg(0x03, dtype_msg), self._msg(0x05, fill),
                                   self._msg(0x08, layout)])

    def group(self, children):
        """children: {name: object header address} -> object header address of the new group."""
        names = sorted(children)
        heap = bytearray(b'\0' * 8)                   # offset 0: the empty name (key 0)
        offs = {}
        for n in names:
            offs[n] = len(heap)
            heap += n.encode('utf-8') + b'\0'
            heap += b'\0' * (-len(heap) % 8)
        # one 16-B free block at the end of the data segment, as the HDF5 library lays out a new heap:
        # {offset of the next free block = 1 (H5HL_FREE_NULL, end of list), size of this block = 16}
        heap_data = self.alloc(bytes(heap) + struct.pack('<QQ', 1, 16))
        heap_hdr = self.alloc(b'HEAP' + bytes([0, 0, 0, 0]) + struct.pack('<QQQ', len(heap) + 16, len(heap),
                                                                         heap_data))
        per = 2 * self.LEAF_K
        groups = [names[i:i + per] for i in range(0, len(names), per)] or [[]]
        if len(groups) > 2 * self.NODE_K:
            raise H5Error('group too large for a single-level B-tree')
        snods = []
        for g in groups:
            ent = b''
            for n in g:
                ent += struct.pack('<QQII16x', offs[n], children[n], 0, 0)
            ent += b'\0' * ((per - len(g)) * 40)
            snods.append(self.alloc(b'SNOD' + struct.pack('<BBH', 1, 0, len(g)) + ent))
        keys = [0] + [offs[g[-1]] if g else 0 for g in groups]
        node = b'TREE' + struct.pack('<BBHQQ', 0, 0, len(snods) if names else 0, UNDEF, UNDEF)
        body = struct.pack('<Q', keys[0])
        for s, k in zip(snods if names else [], keys[1:]):
            body += struct.pack('<QQ', s, k)
        body += b'\0' * ((2 * self.NODE_K + 1) * 16 - len(body))
        tree = self.alloc(node + body)
        return self.object_header([self._msg(0x11, struct.pack('<QQ', tree, heap_hdr))]), tree, heap_hdr


def write(path, tree):
    """Write a nested dict {name: dict | ndarray} as an HDF5 file (groups and contiguous datasets)."""
    w = _Writer()
    w.alloc(b'\0' * 96)                               # superblock placeholder

    def emit(node):
        kids = {}
        for name, v in node.items():
            if '/' in name or not name:
                raise H5Error(f'bad member name {name!r}')
            kids[name] = emit(v) if isinstance(v, dict) else w.dataset(np.asarray(v))
        return w.group(kids)[0]

    root_children = {}
    for name, v in tree.items():
        root_children[name] = emit(v) if isinstance(v, dict) else w.dataset(np.asarray(v))
    root, tree_addr, heap_addr = w.group(root_children)
    eof = len(w.out)
    sb = SIGNATURE + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack('<HHI', w.LEAF_K, w.NODE_K, 0)
    sb += struct.pack('<QQQQ', 0, UNDEF, eof, UNDEF)
    sb += struct.pack('<QQII', 0, root, 1, 0) + struct.pack('<QQ', tree_addr, heap_addr)
    w.out[:len(sb)] = sb
    with open(path, 'wb') as f:
        f.write(bytes(w.out))


# ============================================================================ Keras weights layout
_SEQ = 'layer_with_weights-{}'


def unet_h5_paths(depth=4):
    """Our parameter name -> [(candidate group paths under the UnetConditional, var index)].

    Keras 3 saving_lib: a saveable's own variables go to ``<path>/vars/<i>`` (kernel 0, bias 1); attributes
    that hold layers add their name to the path; a list / dict of layers adds the snake-case class name of
    each item (``dense``, ``dense_1``, ...).  Plain Python lists nested in lists (UnetConditional's downs /
    ups / cond_mlp_* hold lists of layers, networks.py:908-991) are not KerasSaveable, and Keras 3 does not
    descend into them; this package's writer stores them under their list indices (``downs/0/0/...``), the
    first candidate below, so such files round-trip."""
    c = {}

    def dense(name, *paths):
        c[name + '.kernel'] = [(p, 0) for p in paths]
        c[name + '.bias'] = [(p, 1) for p in paths]

    dense('time_mlp', 'cond_mlp_down/0/0/layers/dense', 'cond_mlp_down/0/0/' + _SEQ.format(0))
    enc = ['dense', 'dense_1', 'dense_2']
    for i in range(3):
        dense(f'cond_enc.hidden{i}', f'encoder_cond/0/encoder/layer_{i}',
              f'encoder_cond/encoder_v3_noskip/encoder/{enc[i]}')
    dense('cond_enc.z', 'encoder_cond/0/dense_z/layer_0', 'encoder_cond/encoder_v3_noskip/dense_z/dense')
    for d in range(depth):
        dense(f'down{d}.time_proj', f'cond_mlp_down/{d}/0/layers/dense_1')
        dense(f'down{d}.label_proj', f'cond_mlp_down/{d}/1/layers/dense_1')
        dense(f'down{d}.conv', f'downs/{d}/0/conv_l/0', f'downs/{d}/0/conv_l/conv1d')
        dense(f'down{d}.res', f'downs/{d}/0/res_conv')
    for u in range(depth - 1):
        dense(f'up{u}.time_proj', f'cond_mlp_up/{u}/0/layers/dense_1')
        dense(f'up{u}.label_proj', f'cond_mlp_up/{u}/1/layers/dense_1')
        dense(f'up{u}.upconv', f'ups/{u}/1')
        dense(f'up{u}.conv', f'ups/{u}/3/conv_l/0', f'ups/{u}/3/conv_l/conv1d')
        dense(f'up{u}.res', f'ups/{u}/3/res_conv')
    dense('final', 'final_conv')
    return c


def load_unet_h5(path, spec, network_path=None, strict=True):
    """{our name: array} from a Keras ``.weights.h5`` of the ImprovedDDPM model (root group ``network``) or of
    the UnetConditional itself.  ``strict=False`` returns only the variables the file holds (Keras 3 files of
    the reference's network hold only what saving_lib reaches, see unet_h5_paths); missing names are listed
    in the KeyError otherwise."""
    cands = unet_h5_paths()
    out, missing = {}, []
    with File(path) as f:
        if network_path is None:
            network_path = 'network' if 'network' in f.keys() else ''
        root = f[network_path] if network_path else f
        for name, shape in spec:
            arr = None
            for p, k in cands.get(name, []):
                key = f'{p}/vars/{k}'
                if key in root:
                    arr = np.asarray(root[key].read(), dtype=np.float32)
                    break
            if arr is None:
                missing.append(name)
                continue
            if tuple(arr.shape) != tuple(shape):
                raise H5Error(f'{name}: shape {arr.shape} != {tuple(shape)}')
            out[name] = arr
    if missing and strict:
        raise KeyError(f'{len(missing)} variables not in {path}: {missing[:8]}...')
    return out


def save_unet_h5(path, weights, network_path='network'):
    """Write ``weights`` ({our name: array}) in the layout load_unet_h5 reads (first candidate paths)."""
    cands = unet_h5_paths()
    tree = {}
    for name, arr in weights.items():
        p, k = cands[name][0]
        node = tree
        for comp in ((network_path + '/') if network_path else '') .split('/') + p.split('/') + ['vars']:
            if comp:
                node = node.setdefault(comp, {})
        node[str(k)] = np.asarray(arr, dtype=np.float32)
    write(path, tree)
