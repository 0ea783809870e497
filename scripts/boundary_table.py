"""Reclaimable time at each of the reverse step's six launch boundaries, from seq_micro's per-workgroup stamps
(profiles/r05/seq/{bf16,x3}.txt: the chained step, S = serial launches, C = one captured graph).

For the boundary producer -> consumer the reclaimable time is what a perfect hand-off would remove:
  tail   the producer's last workgroup end - its median workgroup end (per-XCD speed, stragglers),
  gap    the consumer's first workgroup start - the producer's last end (dispatch / AQL barrier),
  ramp   the consumer's start skew (its last workgroup start - first; the start-up burst).
Medians over the files' rounds and both launch modes.  The up2.fused -> down1 boundary is the step's own
(the next reverse step's first layer): its gap is not in the one-step stamps, and the rocprofv3 trace's
timestamps cannot resolve it (rocprof_trace_gaps.txt: median 0, mean skewed by set-up launches), so the
median of the five measured gaps stands in for it (every boundary inside the captured graph is the same
kind of AQL-barrier hand-off).

Usage: python scripts/boundary_table.py profiles/r05/seq [out.txt]
"""
import os
import re
import sys
from collections import defaultdict

import numpy as np

LINE = re.compile(r'^\s+(\S+)\s+start\s+([\d.]+) ramp\s+([\d.]+) \| end median\s+([\d.]+) last\s+([\d.]+) tail\s+([\d.]+) '
                  r'\| gap to next\s+([\d.]+)')


def parse(path):
    """[(mode, [(layer, start, ramp, end_med, end_last, tail, gap)])] per stamp block."""
    blocks, cur, mode = [], None, None
    for line in open(path):
        if re.match(r'^\s+[SC] stamps', line):
            mode = line.strip()[0]
            cur = []
            blocks.append((mode, cur))
            continue
        m = LINE.match(line)
        if m and cur is not None:
            cur.append((m.group(1),) + tuple(float(x) for x in m.groups()[1:]))
    return blocks


def trace_loop_gap(seq_dir):
    p = os.path.join(seq_dir, 'rocprof_trace_gaps.txt')
    if not os.path.exists(p):
        return None
    for line in open(p):
        if line.startswith('conv<11,0> -> conv<0,0>'):
            return float(line.split()[-1])
    return None


def table(path, loop_gap):
    per = defaultdict(lambda: defaultdict(list))
    for mode, rows in parse(path):
        for a, b in zip(rows, rows[1:] + [None]):
            key = f'{a[0]} -> {b[0] if b else "down1 (next step)"}'
            per[key]['tail'].append(a[5])
            if b is not None:
                per[key]['gap'].append(a[6])
                per[key]['ramp'].append(b[2])
            else:   # the step's own boundary: down1's ramp of this step stands in for the next one's
                per[key]['ramp'].append(rows[0][2])
    measured = [g for d in per.values() for g in d['gap']]
    loop_gap = float(np.median(measured)) if measured else loop_gap
    out = []
    for key, d in per.items():
        tail = float(np.median(d['tail']))
        ramp = float(np.median(d['ramp']))
        gap = float(np.median(d['gap'])) if d['gap'] else (loop_gap if loop_gap is not None else float('nan'))
        out.append((key, tail, gap, ramp, tail + gap + ramp, len(d['tail'])))
    return out


def main():
    seq = sys.argv[1] if len(sys.argv) > 1 else 'profiles/r05/seq'
    loop_gap = trace_loop_gap(seq)
    lines = []
    for name, step_us in (('bf16', None), ('x3', None)):
        path = os.path.join(seq, f'{name}.txt')
        if not os.path.exists(path):
            continue
        rows = table(path, loop_gap)
        spans = [float(m.group(1)) for m in re.finditer(r'first start -> last end ([\d.]+) us', open(path).read())]
        step = float(np.median(spans)) if spans else float('nan')
        lines.append(f'== {name}: {len(spans)} stamped steps, median span {step:.2f} us (first start -> last end)')
        lines.append(f'{"boundary":34s} {"tail":>6s} {"gap":>6s} {"ramp":>6s} {"sum":>6s} {"% step":>7s}  n')
        tot = 0.0
        for key, tail, gap, ramp, s, n in rows:
            tot += s
            lines.append(f'{key:34s} {tail:6.2f} {gap:6.2f} {ramp:6.2f} {s:6.2f} {100 * s / step:6.2f}%  {n}')
        lines.append(f'{"all six boundaries":34s} {"":6s} {"":6s} {"":6s} {tot:6.2f} {100 * tot / step:6.2f}%')
        lines.append('')
    txt = '\n'.join(lines)
    print(txt)
    if len(sys.argv) > 2:
        with open(sys.argv[2], 'w') as f:
            f.write(txt + '\n')


if __name__ == '__main__':
    main()
