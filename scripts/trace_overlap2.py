"""How much of two loops' kernel time overlaps (scripts/gpu_mptrace_r3.sh).

Reads rocprofv3 kernel traces: either several trace directories (one per process: the group is the
process) or one directory with two queues (the group is Queue_Id).  Prints, for the U-Net step kernels
(conv / down0 / seam), the busy time of each group, the time both groups have a kernel running, and the
union.  Usage: python scripts/trace_overlap2.py DIR [DIR ...]
"""
import csv
import glob
import os
import sys


def intervals(paths):
    groups = {}
    for i, p in enumerate(paths):
        for f in glob.glob(os.path.join(p, '**', '*kernel_trace.csv'), recursive=True):
            for r in csv.DictReader(open(f)):
                n = r['Kernel_Name']
                if not any(k in n for k in ('conv_kernel', 'down0_kernel', 'seam23')):
                    continue
                g = i if len(paths) > 1 else r['Queue_Id']
                groups.setdefault(g, []).append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    return groups


def merge(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def total(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    i = j = 0
    out = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def main(paths):
    g = intervals(paths)
    keys = sorted(g)
    print('groups:', {k: len(v) for k, v in g.items()})
    if len(keys) < 2:
        print('fewer than two groups')
        return
    a, b = merge(g[keys[0]]), merge(g[keys[1]])
    ov = intersect(a, b)
    un = total(merge(a + b))
    print(f'busy A {total(a) / 1e6:.2f} ms, busy B {total(b) / 1e6:.2f} ms, both {ov / 1e6:.2f} ms, '
          f'union {un / 1e6:.2f} ms, overlap / union {ov / un:.3f}')


if __name__ == '__main__':
    main(sys.argv[1:])
