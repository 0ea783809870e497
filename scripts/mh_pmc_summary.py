"""Per-update PMC figures of the MH chain kernel (configs[2]) from scripts/gpu_r4.sh's mhpmc stage.

Usage: python scripts/mh_pmc_summary.py gpurun_out/<TAG>/mhpmc <chains> <steps_per_chain> out.json

Takes the largest mh_chain_kernel dispatch of every pass (the 10k-chain run; the warm-up and the 4-chain
protocol are smaller or run the batched kernel), divides each counter by its element updates
(chains x steps x 96) and writes the instruction mix, the wave-cycle split (issuing / waiting / stalled:
SQ_ACTIVE_INST_ANY + SQ_WAIT_ANY + SQ_WAIT_INST_ANY = SQ_WAVE_CYCLES, quad-cycles), the VALU pipe's
busy cycles (fp64 wave64 at 4 cycles, other VALU at 2: MI355X_MICROARCH.md cycle constants) and the
fabric bytes (FETCH_SIZE x 2, gfx950's 64-B tally, + WRITE_SIZE, KB).  bench.py's mh roofline reads it.
"""
import csv
import glob
import json
import os
import sys


def largest_dispatch(path):
    per, grid = {}, {}
    for r in csv.DictReader(open(path)):
        if 'mh_chain_kernel' not in r['Kernel_Name']:
            continue
        d = r['Dispatch_Id']
        grid[d] = int(r.get('Grid_Size', 0) or 0)
        per.setdefault(d, {})
        per[d][r['Counter_Name']] = per[d].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    if not per:
        return {}
    return per[max(per, key=lambda d: (grid[d], d))]


def kernel_hash():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from pet_posterior_distribution_amd import _lib
    return _lib.kernel_code_hash(b'mh_chain_kernel')


def main():
    root, chains, steps, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    c = {}
    for p in sorted(glob.glob(os.path.join(root, 'p*', 'run_counter_collection.csv'))):
        c.update(largest_dispatch(p))
    upd = chains * steps * 96
    f = {k: v / upd for k, v in c.items()}
    fp64 = sum(f.get(k, 0.0) for k in ('SQ_INSTS_VALU_FMA_F64', 'SQ_INSTS_VALU_MUL_F64', 'SQ_INSTS_VALU_ADD_F64',
                                        'SQ_INSTS_VALU_TRANS_F64'))
    valu = f.get('SQ_INSTS_VALU', 0.0)
    wave = c.get('SQ_WAVE_CYCLES', 0.0)
    res = {
        'element_updates': upd, 'chains': chains, 'steps_per_chain': steps,
        'per_update': {k.replace('SQ_INSTS_', '').lower(): round(v, 2) for k, v in f.items() if k.startswith('SQ_INSTS')},
        'fp64_valu_per_update': round(fp64, 2), 'valu_per_update': round(valu, 2),
        'valu_pipe_cycles_per_update': round(4 * fp64 + 2 * (valu - fp64), 1),
        'wave_cycle_split': {'issuing': round(c.get('SQ_ACTIVE_INST_ANY', 0) / wave, 4),
                             'waiting (s_waitcnt / barrier)': round(c.get('SQ_WAIT_ANY', 0) / wave, 4),
                             'issue-stalled': round(c.get('SQ_WAIT_INST_ANY', 0) / wave, 4)} if wave else None,
        'lds_bank_conflict_per_update': round(f.get('SQ_LDS_BANK_CONFLICT', 0.0), 3),
        'fabric_kb_per_launch': round((2 * c.get('FETCH_SIZE', 0.0) + c.get('WRITE_SIZE', 0.0)), 1),
        'source': root,
        'code_hash': kernel_hash(),
    }
    with open(out, 'w') as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
