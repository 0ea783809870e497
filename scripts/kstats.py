"""Per-layer kernel averages (us) from rocprofv3 kernel_stats CSVs, side by side.
Usage: python scripts/kstats.py a/run_kernel_stats.csv [b/run_kernel_stats.csv ...]"""
import csv
import re
import sys

LAYERS = ['down1', 'down2', 'down3', 'up0.conv2', 'up0.block', 'up1.conv2', 'up1.block', 'up2.conv2', 'up2.block',
          'up0.fused', 'up1.fused', 'up2.fused', 'up2.fused']   # kind 12: the bf16x3 final level (LK_UP2_FX3)


def label(name):
    if 'down0_kernel' in name or 'down0_mfma_kernel' in name:
        return 'down0'
    # rocprofv3's demangler garbles the bf16 instances of kinds 1 and 2 (down2, down3):
    # conv_kernel<bf16, 1, XS> -> 'conv_kernel<bool _Accum, int, E, XS>',
    # conv_kernel<bf16, 2, 1> -> 'conv_kernel<bool _Accum, int, EL, int, E>'
    if re.search(r'conv_kernel<bool _Accum, int, EL, int, E>', name):
        return 'down3'
    if re.search(r'conv_kernel<bool _Accum, int, E(, \d+)?>', name):
        return 'down2'
    m = re.search(r'conv_kernel.*?Li(\d+)E', name) or re.search(r'conv_kernel<[^,]*, (\d+)>', name)
    if 'conv_kernel' in name and m:
        return LAYERS[int(m.group(1))]
    return None


def load(path):
    out = {}
    for r in csv.DictReader(open(path)):
        k = label(r['Name'])
        if k:
            out[k] = (int(r['Calls']), float(r['AverageNs']) / 1e3)
    return out


cols = [load(p) for p in sys.argv[1:]]
keys = ['down0'] + list(dict.fromkeys(LAYERS))
print('%-10s' % 'kernel' + ''.join('%18s' % ('calls / avg us',) for _ in cols))
for k in keys:
    print('%-10s' % k + ''.join('%8s %9.2f' % (c[k][0], c[k][1]) if k in c else '%18s' % '-' for c in cols))
tot = [sum(n * a for n, a in c.values()) for c in cols]
steps = [max(n for n, _ in c.values()) for c in cols]
print('%-10s' % 'us/step' + ''.join('%18.2f' % (t / s) for t, s in zip(tot, steps)))
