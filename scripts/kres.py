"""Register / LDS / scratch usage of the conv kernels from a device-only .s file.
Usage: hipcc --cuda-device-only -S unet_kernels.hip -o /tmp/u.s && python scripts/kres.py /tmp/u.s [filter]"""
import re
import sys

src = open(sys.argv[1]).read()
filt = sys.argv[2] if len(sys.argv) > 2 else 'conv_kernel'
for blk in src.split('- .agpr_count:')[1:]:
    name = re.search(r'\.name:\s+(\S+)', blk).group(1)
    if filt not in name:
        continue

    def g(k):
        return re.search(r'\.' + k + r':\s+(\d+)', blk).group(1)

    body = src[src.index(name + ':'):]
    body = body[:body.index('s_endpgm')]
    print(f"{name[:60]:60s} vgpr {g('vgpr_count'):>4} agpr {blk.split()[0]:>4} lds {g('group_segment_fixed_size'):>7} "
          f"scratch {g('private_segment_fixed_size'):>4} mfma {body.count('v_mfma'):>5} accmov {body.count('accvgpr_mov'):>4}")
