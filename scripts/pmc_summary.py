"""Summarise rocprofv3 --pmc passes: per-kernel mean counter value per dispatch.

FETCH_SIZE is doubled (gfx950 tallies 128-B requests at 64 B: MI355X_MICROARCH.md HBM);
FETCH_SIZE / WRITE_SIZE are in KB.  Usage: python scripts/pmc_summary.py gpurun_out/pmc1 [out.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


LAYERS = ['down1', 'down2', 'down3', 'up0.conv2', 'up0.block', 'up1.conv2', 'up1.block', 'up2.conv2', 'up2.block',
          'up0.fused', 'up1.fused', 'up2.fused', 'up2.fused']   # kind 12: the bf16x3 final level (LK_UP2_FX3)


def short(name):
    import re
    m = re.search(r'conv_kernelI(?:DF16b|DF16_|f)Li(\d+)E', name)
    if m:
        return LAYERS[int(m.group(1))]
    if 'down0_kernel' in name or 'down0_mfma_kernel' in name:
        return 'down0'
    # rocprofv3 demangles conv_kernel<__bf16, 1, XS> as 'conv_kernel<bool _Accum, int, E, XS>' (before the
    # XS parameter existed: 'conv_kernel<bool _Accum, int, E>'); of the 16-bit conv kinds a generate
    # launches (0, 1, 2, 9, 10, 11) only kind 1 (down2) comes out that way
    if re.search(r'conv_kernel<bool _Accum, int, E(, \d+)?>', name):
        return 'down2'
    if re.search(r'conv_kernel<bool _Accum, int, EL, int, E>', name):   # conv_kernel<bf16, 2, 1> (bf16x3 down3)
        return 'down3'
    return None


def main(d, out=None, update_traffic=False, dtype='bfloat16'):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, 'p*', 'run_counter_collection.csv')):
        for r in csv.DictReader(open(f)):
            k = short(r['Kernel_Name'])
            if k is None:
                continue
            vals[k][r['Counter_Name']].append(float(r['Counter_Value']))
    res = {}
    for k, cs in vals.items():
        res[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        if 'FETCH_SIZE' in res[k]:
            res[k]['hbm_read_bytes_corrected'] = res[k]['FETCH_SIZE'] * 2 * 1024
        if 'WRITE_SIZE' in res[k]:
            res[k]['hbm_write_bytes'] = res[k]['WRITE_SIZE'] * 1024
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from pet_posterior_distribution_amd import _lib
    code_hash = _lib.kernel_code_hash()       # the build these passes measured (same tree on the GPU box)
    for k in sorted(res):
        print(k, {c: round(v, 1) for c, v in res[k].items()})
    print('kernels:', sorted(res), 'code_hash:', code_hash)
    if out:
        json.dump(dict(res, _meta={'code_hash': code_hash, 'dtype': dtype}), open(out, 'w'), indent=1)
    if out and update_traffic:
        # bench.py's bf16 roofline reads these: update them only from passes over the default
        # (bf16, B = 1024) workload -- a --dtype bf16x3 run once overwrote them with its 3x bytes
        tp = os.path.join(root, 'profiles', 'pmc_traffic.json')
        tr = json.load(open(tp)) if os.path.exists(tp) else {}
        suf = {'bfloat16': '', 'bf16x3': '_bf16x3', 'float16': '_f16'}[dtype]
        for key, pre0 in (('up0.block', 'up0_block'), ('up0.fused', 'up0_fused')):
            pre = pre0 + suf
            if key in res:
                tr[pre + '_code_hash'] = code_hash
            ub = res.get(key, {})
            if 'hbm_read_bytes_corrected' in ub and 'hbm_write_bytes' in ub:
                tr[pre + '_bytes_per_launch'] = ub['hbm_read_bytes_corrected'] + ub['hbm_write_bytes']
                tr[pre + '_read_bytes'] = ub['hbm_read_bytes_corrected']
                tr[pre + '_write_bytes'] = ub['hbm_write_bytes']
                tr[pre + '_source'] = os.path.relpath(out, root)
            for c, name in (('SQ_VALU_MFMA_BUSY_CYCLES', '_mfma_busy_cycles'), ('GRBM_GUI_ACTIVE', '_grbm_gui_active')):
                if c in ub:
                    tr[pre + name] = ub[c]
        # every step kernel's counters (bench.py's per-kernel roofline table), stamped with the build
        ks = {}
        for key, ub in res.items():
            row = {}
            if 'hbm_read_bytes_corrected' in ub and 'hbm_write_bytes' in ub:
                row['bytes'] = ub['hbm_read_bytes_corrected'] + ub['hbm_write_bytes']
            for c, name in (('SQ_VALU_MFMA_BUSY_CYCLES', 'mfma_busy_cycles'), ('GRBM_GUI_ACTIVE', 'grbm_gui_active'),
                            ('SQ_LDS_BANK_CONFLICT', 'lds_bank_conflict_cycles'), ('SQ_WAIT_ANY', 'sq_wait_any'),
                            ('SQ_BUSY_CYCLES', 'sq_busy_cycles')):
                if c in ub:
                    row[name] = ub[c]
            ks[key] = row
        tr['kernels' + suf] = {'code_hash': code_hash, 'source': os.path.relpath(out, root), 'per_launch': ks}
        tr['method'] = 'rocprofv3 --pmc FETCH_SIZE (x2, gfx950 64-B tally) + WRITE_SIZE, KB->B, mean per dispatch'
        json.dump(tr, open(tp, 'w'), indent=1)
    return res


if __name__ == '__main__':
    # --traffic: update profiles/pmc_traffic.json (bench.py's PMC fields) from these passes;
    # --dtype=bf16x3|float16: the passes ran bench.py --dtype ... (keys get a dtype suffix)
    dt = next((x.split('=', 1)[1] for x in sys.argv[1:] if x.startswith('--dtype=')), 'bfloat16')
    args = [x for x in sys.argv[1:] if not x.startswith('--')]
    main(args[0], args[1] if len(args) > 1 else None, update_traffic='--traffic' in sys.argv[1:], dtype=dt)
