"""Concurrency of conv kernels across HW queues in a rocprofv3 kernel trace (--kernel-trace CSV):
per queue the busy time, and the time during which conv kernels of two or more queues run at once.
Usage: python scripts/trace_overlap.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def main(path):
    iv = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if 'conv_kernel' not in r['Kernel_Name'] and 'conv_kernelI' not in r['Kernel_Name']:
            continue
        iv[r['Queue_Id']].append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    ev = []
    for q, lst in iv.items():
        for a, b in lst:
            ev.append((a, 1))
            ev.append((b, -1))
    ev.sort()
    busy = multi = 0
    depth, last = 0, None
    for t, d in ev:
        if last is not None and depth > 0:
            busy += t - last
            if depth > 1:
                multi += t - last
        depth += d
        last = t
    print({'queues': {q: len(v) for q, v in iv.items()}, 'busy_ms': round(busy / 1e6, 2),
           'overlap_ms': round(multi / 1e6, 2), 'overlap_frac': round(multi / max(busy, 1), 4)})


if __name__ == '__main__':
    main(sys.argv[1])
