"""Per-kernel ISA fingerprint of libpetdiff.so's U-Net code object (a CPU-side proof that a source
change leaves the machine code of the kernels it does not target unchanged).

  python scripts/isa_dump.py dump  out.json [lib.so]    # {kernel: sha256 of its normalised disassembly}
  python scripts/isa_dump.py compare a.json b.json       # kernels in both: equal / DIFFERENT

The disassembly of each function symbol is normalised before hashing: instruction addresses, encodings
and symbolic branch targets are dropped (branch immediates are PC-relative), so moving a kernel inside the
code object (another kernel removed before it) does not count as a change.
"""
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OBJDUMP = '/opt/rocm/lib/llvm/bin/llvm-objdump'


def code_object(path, symbol=b'conv_kernel'):
    import struct
    with open(path, 'rb') as f:
        b = f.read()
    shoff = struct.unpack_from('<Q', b, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from('<HHH', b, 0x3A)
    secs = [struct.unpack_from('<IIQQQQIIQQ', b, shoff + i * shentsize) for i in range(shnum)]
    stro = secs[shstrndx][4]
    fb = None
    for s in secs:
        if b[stro + s[0]:b.index(b'\0', stro + s[0])] == b'.hip_fatbin':
            fb = b[s[4]:s[4] + s[5]]
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
                return co
        i = fb.find(magic, i + 1)
    raise SystemExit(f'no gfx950 code object with {symbol!r} in {path}')


def functions(co):
    with tempfile.NamedTemporaryFile(suffix='.elf') as f:
        f.write(co)
        f.flush()
        txt = subprocess.run([OBJDUMP, '-d', '--no-show-raw-insn', '--mcpu=gfx950', f.name],
                             check=True, capture_output=True, text=True).stdout
    funcs, cur = {}, None
    head = re.compile(r'^([0-9a-f]+) <(.+)>:$')
    for line in txt.splitlines():
        m = head.match(line)
        if m:
            cur = m.group(2)
            funcs[cur] = []
            continue
        if cur is None or not line.strip():
            continue
        # branch immediates are PC-relative already; the comment (address, encoding, target) is dropped
        funcs[cur].append(line.split('//')[0].strip())
    return funcs


def dump(out, path=None):
    from pet_posterior_distribution_amd import _lib
    funcs = functions(code_object(path or _lib.LIB_PATH))
    res = {k: {'sha': hashlib.sha256('\n'.join(v).encode()).hexdigest()[:16], 'n': len(v)} for k, v in funcs.items()}
    with open(out, 'w') as f:
        json.dump(res, f, indent=0, sort_keys=True)
    print(f'{len(res)} functions -> {out}')


def compare(pa, pb):
    a, b = json.load(open(pa)), json.load(open(pb))
    both = sorted(set(a) & set(b))
    bad = [k for k in both if a[k]['sha'] != b[k]['sha']]
    for k in both:
        print(f"{'equal    ' if k not in bad else 'DIFFERENT'} {a[k]['n']:6d} {b[k]['n']:6d}  {k}")
    for k in sorted(set(a) - set(b)):
        print(f'only in {pa}: {k}')
    for k in sorted(set(b) - set(a)):
        print(f'only in {pb}: {k}')
    print(f'{len(both) - len(bad)} of {len(both)} common functions identical')
    return 1 if bad else 0


def regs(path=None, pattern='conv_kernel'):
    """Per-kernel register / LDS / scratch figures from the code object's AMDGPU metadata note."""
    from pet_posterior_distribution_amd import _lib
    co = code_object(path or _lib.LIB_PATH)
    with tempfile.NamedTemporaryFile(suffix='.elf') as f:
        f.write(co)
        f.flush()
        txt = subprocess.run([OBJDUMP.replace('objdump', 'readelf'), '--notes', f.name], check=True,
                             capture_output=True, text=True).stdout
    rows, cur = [], {}
    for line in txt.splitlines():
        m = re.match(r'\s*-?\s*\.(\w+):\s+(\S+)', line)
        if not m:
            continue
        k, v = m.groups()
        if k == 'agpr_count' and cur:     # a kernel's map starts with .agpr_count in this metadata layout
            rows.append(cur)
            cur = {}
        cur[k] = v
    rows.append(cur)
    out = []
    for r in rows:
        if pattern in r.get('name', ''):
            out.append((r['name'], int(r.get('vgpr_count', -1)), int(r.get('agpr_count', -1)),
                        int(r.get('sgpr_count', -1)), int(r.get('group_segment_fixed_size', -1)),
                        int(r.get('private_segment_fixed_size', -1)), int(r.get('vgpr_spill_count', -1))))
    for o in out:
        print(f'{o[0]:60s} vgpr {o[1]:4d} agpr {o[2]:4d} sgpr {o[3]:3d} lds {o[4]:6d} scratch {o[5]:4d} spill {o[6]}')
    return out


if __name__ == '__main__':
    if sys.argv[1] == 'regs':
        regs(sys.argv[2] if len(sys.argv) > 2 else None)
        sys.exit(0)
    if sys.argv[1] == 'dump':
        dump(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
