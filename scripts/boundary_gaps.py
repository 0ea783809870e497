"""Launch-boundary gaps of the reverse loop from a rocprofv3 kernel trace.

Usage: python scripts/boundary_gaps.py <kernel_trace.csv> [min_calls]

For every pair of consecutive kernels on the same queue (sorted by start time) the gap is
start(next) - end(prev); the gaps are grouped by boundary (prev kernel -> next kernel) and the
boundaries seen at least min_calls times (default 20: the loop's, not set-up launches) are printed
with their count, median and mean gap in microseconds, plus the loop's median kernel durations.
"""
import csv
import sys
from collections import defaultdict

import numpy as np


def short(name):
    for key in ('conv_kernel', 'down0_kernel'):
        if key in name:
            # _ZN7petdiff11conv_kernelIDF16bLi9ELi0EEE... -> conv<9,0>
            import re
            m = re.search(r'Li(\d+)ELi(\d+)E', name)
            return f'{key.split("_")[0]}<{m.group(1)},{m.group(2)}>' if m else key
    return name.split('(')[0][:40]


def main():
    path = sys.argv[1]
    min_calls = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), short(r['Kernel_Name']),
                         r.get('Queue_Id', '0')))
    rows.sort()
    gaps, durs = defaultdict(list), defaultdict(list)
    last = {}
    for s, e, n, q in rows:
        durs[n].append(e - s)
        if q in last:
            ps, pe, pn = last[q]
            gaps[(pn, n)].append(s - pe)
        last[q] = (s, e, n)
    total = 0.0
    print(f'{"boundary":40s} {"count":>7s} {"median us":>10s} {"mean us":>9s}')
    for (a, b), g in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
        if len(g) < min_calls:
            continue
        g = np.asarray(g) / 1e3
        total += np.median(g)
        print(f'{a + " -> " + b:40s} {len(g):7d} {np.median(g):10.2f} {g.mean():9.2f}')
    print(f'sum of the loop boundaries\' median gaps: {total:.2f} us')
    print(f'{"kernel":40s} {"count":>7s} {"median us":>10s}')
    for n, d in sorted(durs.items(), key=lambda kv: -len(kv[1])):
        if len(d) >= min_calls:
            print(f'{n:40s} {len(d):7d} {np.median(d) / 1e3:10.2f}')


if __name__ == '__main__':
    main()
