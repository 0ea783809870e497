#!/usr/bin/env python3
"""Benchmark: posterior samples/sec of the 1000-step iDDPM reverse process (48-ROI TAC).

Workload (BASELINE.json configs[1]): f128/d4 1-D conditional U-Net, 1000-step
iDDPM reverse (ImprovedDDPM.ddpm_loop, diffusion_model.py:670-715), n_posterior =
1024 samples per GPU, bf16 network / fp32 p_sample, one synthetic test TAC per
GPU, synthetic (identity-denoiser Glorot) weights of the shipped architecture.

A bench "step" = one whole posterior job through distributed.sample_posterior_sharded (the
configs[3] driver): x_T, one full generate() (1000 reverse steps, one replayed hipGraph) over
the rank's 1024 samples, the GPU Welford statistics and their all-gather over RCCL (the only
collective).  Weak scaling: every rank owns 1024 samples of its own TAC
(TAC-major shards); value = all ranks' samples / max-over-ranks time.

Launch: python bench.py --gpus N --steps K --warmup W  (N>1 via torch.distributed.run).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# algorithmic work
FLOP_PER_SAMPLE_STEP = 296_361_984          # x-dependent U-Net convs incl. 1x1 residuals
# dominant kernel = up0 ConvBlock: relu(conv6(1024->512) + conv1(1024->512)) at L=12 (App. A: 37.75+6.29 M MAC)
UP0_BLOCK_FLOP_PER_SAMPLE = 2 * 12 * 512 * 1024 * 7
UP0_BLOCK_EXEC_FLOP_PER_SAMPLE = 2 * 12 * 512 * 1024 * 6   # executed (residual folded into the centre tap)
# fused up0 level (16-bit default): up0's k2 conv (App. A: 13.20 M MAC, 1074 input channels) + the block
# in one kernel; executed = skip half (6 taps x 512 at 12 positions) + 2-phase composite (4 taps x 1024 at
# 6 coarse rows per phase) + the l = 0, 1 left-edge correction rows (1024 -> 512 each), less the (position,
# tap) products that read only padding, which the kernel skips (CONV_UP0_ZS): 63 of the 72 skip-half
# products and 20 of the 24 composite products per phase remain
UP0_CONV2_FLOP_PER_SAMPLE = 2 * 12 * 2 * 1074 * 512
UP0_FUSED_EXEC_FLOP_PER_SAMPLE = 2 * 512 * 512 * 63 + 2 * 2 * 1024 * 512 * 20 + 2 * 2 * 1024 * 512
PEAK_BF16_TFLOPS = 2500.0                   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0                       # HBM3E (MI355X_MICROARCH.md)
PEAK_CLOCK_HZ = 2.4e9                       # engine clock the dense MFMA peak is quoted at
N_SIMD = 256 * 4                            # 256 CUs x 4 SIMDs
# FLOP the kernels EXECUTE per sample-step: the label / time input channels of every concat are
# hoisted into per-level maps and the 1x1 residuals folded into the centre tap, so the convs multiply
# only the x channels: down0 (VALU) + down1..3 + the up levels' k2 convs and blocks (unfused, as the
# exact-f32 path runs them) + the final 1x1 conv
EXEC_FLOP_PER_SAMPLE_STEP_UNFUSED = 2 * (48 * 6 * 2 * 128 + 24 * 6 * 128 * 256 + 12 * 6 * 256 * 512 +
                                         6 * 6 * 512 * 1024 + 12 * 2 * 1024 * 512 + 12 * 6 * 1024 * 512 +
                                         24 * 2 * 512 * 256 + 24 * 6 * 512 * 256 + 48 * 2 * 256 * 128 +
                                         48 * 6 * 256 * 128 + 48 * 128 * 4)
# MFMA FLOP the 16-bit path executes per sample-step: down1, down2 / down3 with their zero taps skipped
# (position-major: 63 / 72 and 54 / 72 of the (fragment, tap) products), and the fused up levels
# (skip half 6 taps + 2-phase composite 4 taps + the two left-edge correction rows); down0 and the
# final 1x1 conv run on VALU and are not counted
EXEC_MFMA_FLOP_PER_SAMPLE_STEP_FUSED = int(
    2 * 24 * 6 * 128 * 256 + 2 * 12 * 6 * 256 * 512 * 63 / 72 + 2 * 6 * 6 * 512 * 1024 * 54 / 72 +
    sum(2 * L * 6 * cs * co + 2 * L * 4 * cb * co + 2 * 2 * cb * co
        for L, cs, cb, co in ((12, 512, 1024, 512), (24, 256, 512, 256), (48, 128, 256, 128))))
# Per-launch work of the step's kernels (SURVEY App. A MACs per sample-step; x2 = FLOP).  Each entry:
# (timing key, kernel, algorithmic MAC per sample, MFMA MAC the 16-bit kernel executes per sample).
# Executed: the label / time channels live in the hoisted maps, the 1x1 residual is folded into the
# centre tap, and the position-major down2 / down3 and up0 skip the (position, tap) products that read
# SAME padding (63 / 72, 54 / 72; up0: 63 of 72 skip-half and 20 of 24 composite products per phase).
# up2.fused also runs the final 1x1 conv, p_sample and the NEXT step's down0 (VALU, not in the MFMA count).
STEP_KERNELS = (
    ('down1', 'conv_kernel<down1> (L=24, 178->256 k6+res, MaxPool)', 24 * 7 * 178 * 256, 24 * 6 * 128 * 256),
    ('down2', 'conv_kernel<down2> (L=12, 306->512 k6+res, MaxPool)', 12 * 7 * 306 * 512, 12 * 6 * 256 * 512 * 63 // 72),
    ('down3', 'conv_kernel<down3> (L=6, 562->1024 k6+res)', 6 * 7 * 562 * 1024, 6 * 6 * 512 * 1024 * 54 // 72),
    ('up0.block', 'conv_kernel<up0 fused> (UpSampling1D + k2 1074->512 + ConvBlock 1024->512 k6+res, L=12)',
     12 * 2 * 1074 * 512 + 12 * 7 * 1024 * 512, UP0_FUSED_EXEC_FLOP_PER_SAMPLE // 2),
    ('up1.block', 'conv_kernel<up1 fused> (UpSampling1D + k2 562->256 + ConvBlock 512->256 k6+res, L=24)',
     24 * 2 * 562 * 256 + 24 * 7 * 512 * 256, 24 * 6 * 256 * 256 + 24 * 4 * 512 * 256 + 2 * 512 * 256),
    ('up2.block+final+p_sample', 'conv_kernel<up2 fused> (UpSampling1D + k2 306->128 + ConvBlock 256->128 k6+res, L=48) + final '
                  '1x1 128->4 + p_sample + next-step down0 (52->128 k6+res)',
     48 * 2 * 306 * 128 + 48 * 7 * 256 * 128 + 48 * 128 * 4 + 48 * 7 * 52 * 128,
     48 * 6 * 128 * 128 + 48 * 4 * 256 * 128 + 2 * 256 * 128),
)


def step_kernel_bytes(key, dtype):
    """Algorithmic HBM bytes per sample of a step kernel: its input activation rows read once, its
    output rows written once (16-bit: 2 B per value; bf16x3: [hi | lo] rows, 4 B), x_t / x_{t-1} fp32 for
    the final level.  The packed weights (read once per launch) are added by weight_bytes."""
    e = 4 if dtype in ('bf16x3', 'float32') else 2
    acts = {'down1': 24 * 128 + 24 * 256 + 12 * 256, 'down2': 12 * 256 + 12 * 512 + 6 * 512,
            'down3': 6 * 512 + 6 * 1024, 'up0.block': 12 * 512 + 6 * 1024 + 12 * 512,
            'up1.block': 24 * 256 + 12 * 512 + 24 * 256,
            'up2.block+final+p_sample': 48 * 128 + 24 * 256 + 48 * 128 + 24 * 128}[key]   # up2: + next s0 / p0
    return acts * e + (2 * 96 * 4 if key.startswith('up2') else 0)


def weight_bytes(key, dtype):
    """Packed weight bytes of a step kernel (x channels only; the fused levels' composite taps)."""
    e = 4 if dtype in ('bf16x3', 'float32') else 2
    w = {'down1': 6 * 128 * 256, 'down2': 6 * 256 * 512, 'down3': 6 * 512 * 1024,
         'up0.block': 6 * 512 * 512 + 8 * 1024 * 512, 'up1.block': 6 * 256 * 256 + 8 * 512 * 256,
         'up2.block+final+p_sample': 6 * 128 * 128 + 8 * 256 * 128}[key]
    return w * e


# per-layer timing: every timed launch runs TIMING_REPS times back to back between its two HIP events
# (ImprovedDDPM.set_kernel_timing), so one event's queue gap is shared by 8 launches and the mean launch
# time tracks rocprofv3's kernel duration
TIMING_REPS = 8

# training step: forward + data grad + weight grad of every layer, incl. the
# per-sample condition encoder / label projections / time MLP (6,002,304 FLOP per sample forward)
TRAIN_FLOP_PER_SAMPLE = 3 * (FLOP_PER_SAMPLE_STEP + 6_002_304)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--batch', type=int, default=1024, help='posterior samples per GPU')
    ap.add_argument('--tacs', type=int, default=1,
                    help='test TACs per GPU (samples split TAC-major; config 4 = 32 TACs x 8192 per GPU)')
    ap.add_argument('--chunk', type=int, default=0,
                    help='samples per launch (0 = PETDIFF_MAX_BATCH); larger batches run as chunks')
    ap.add_argument('--config4', action='store_true',
                    help='BASELINE configs[3] per-rank shard: 32 TACs x 8192 posterior samples per GPU')
    ap.add_argument('--reverse-steps', type=int, default=1000)
    ap.add_argument('--dtype', default='bfloat16', choices=['bfloat16', 'float16', 'float32', 'bf16x3'],
                    help='bf16x3: fp32-class accuracy on the bf16 kernels (3 MFMA products; peak = bf16 dense / 3)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-kernel-timing', action='store_true')
    ap.add_argument('--no-extras', action='store_true',
                    help='skip the exact-f32 and bf16x3 rates, the full MH configs[2] run and the reference-protocol ratio')
    ap.add_argument('--workload', default='iddpm', choices=['iddpm', 'mh', 'train'],
                    help='iddpm: BASELINE configs[1] (the metric); mh: configs[2] MH/SRTM2 baseline')
    ap.add_argument('--train-batch', type=int, default=256, help='training batch per GPU (main_script.py:169)')
    ap.add_argument('--mh-chains', type=int, default=10000)
    ap.add_argument('--mh-iters', type=int, default=10000, help='MH draws per chain (kept)')
    ap.add_argument('--mh-tune', type=int, default=10000, help='MH tuning steps per chain (config 3: 20k steps in total)')
    return ap.parse_args()


def init_dist():
    """One process per GPU (torch.distributed.run env).  Returns (world, rank, device).

    The collective backend is RCCL ('nccl').  PETDIFF_BENCH_BACKEND=gloo is a rehearsal mode for a
    box with fewer GPUs than ranks: ranks share devices round-robin (LOCAL_RANK mod device count)
    and the few small collectives (barrier, max of the timer, stats all-gather) go over gloo on host
    tensors.  RCCL refuses two ranks on one GPU, so this is how the N>1 code path of this file is
    exercised on a 1-GPU box; the timed region is the same either way."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        os.environ.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
        backend = os.environ.get('PETDIFF_BENCH_BACKEND', 'nccl')
        if backend == 'gloo':
            torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
            dist.init_process_group('gloo')
        else:
            torch.cuda.set_device(local)
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    else:
        torch.cuda.set_device(0)
    return world, rank, torch.device('cuda', torch.cuda.current_device())


def coll_device(dev):
    """Where collective operands live: the GPU for RCCL, the host for the gloo rehearsal."""
    import torch.distributed as dist
    return 'cpu' if dist.get_backend() == 'gloo' else dev


def max_over_ranks(elapsed, dev):
    import torch
    import torch.distributed as dist
    e = torch.tensor([elapsed], device=coll_device(dev), dtype=torch.float64)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    return float(e.item())


def host_threads():
    """CPU threads for the baseline leg: the job's CPU share (OMP_NUM_THREADS on the GPU
    box, 16 per GPU), never the whole machine's core count."""
    try:
        n = int(os.environ.get('OMP_NUM_THREADS', '0'))
    except ValueError:
        n = 0
    if n <= 0:
        n = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else (os.cpu_count() or 1)
    return max(1, min(n, 16))


def cpu_baseline(weights, cond, budget_s=15.0):
    """The oracle's p_sample on the host CPU, bounded: oracle/iddpm_torch_cpu.py (the NumPy oracle
    restated with torch's CPU conv1d, 2.4x its rate; checked against it in tests/test_cpu.py),
    fp32, B = 256 samples of configs[1]'s TAC, as many reverse steps as fit in ~budget_s, extrapolated
    to the 1000-step process.  Threads: the job's CPU share (host_threads)."""
    import torch
    from oracle import iddpm_ref as R
    from oracle import iddpm_torch_cpu as TC
    cores = host_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(cores)
    S = R.schedule_tables(R.get_beta_schedule('cosine', 1000))
    rng = np.random.default_rng(0)
    B = 256
    x = torch.as_tensor(rng.standard_normal((B, 48, 2)).astype(np.float32))
    c = torch.as_tensor(np.repeat(np.asarray(cond, np.float32)[None], B, 0))
    net = TC.TorchCpuUnet({k: v.astype(np.float32) for k, v in weights.items()})
    net.ddpm(S, x, np.full(B, 999, np.int32), c, torch.zeros_like(x))      # warm-up (oneDNN primitives)
    n, t0 = 0, time.perf_counter()
    for ti in R.loop_indices(1000):
        z = torch.as_tensor(rng.standard_normal((B, 48, 2)).astype(np.float32))
        m, _, vt = net.ddpm(S, x, np.full(B, ti, np.int32), c, z)
        x = m + vt
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    torch.set_num_threads(prev)
    per_step = dt / n
    return {'value': B / (per_step * 1000.0), 'unit': 'samples/s', 'cores': int(cores), 'kind': 'port',
            'sample': f'oracle/iddpm_torch_cpu.py (the oracle on torch CPU conv1d) fp32, B={B} samples x {n} '
                      f'reverse steps ({dt:.1f} s), extrapolated to 1000 steps'}


NO_PMC = {'traffic': None, 'mfma_busy': None, 'grbm': None, 'source': None}


def load_pmc(fused_up=False, dtype='bfloat16'):
    """Per-launch PMC figures of the dominant kernel from the committed rocprofv3 summary
    (profiles/pmc_traffic.json, written by scripts/pmc_summary.py --traffic): HBM bytes (FETCH_SIZE x2 +
    WRITE_SIZE), SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE.  The entries are stamped with the
    code-object hash of the U-Net kernels they were counted on (_lib.kernel_code_hash); when the
    loaded library's kernels differ, the counters belong to another build and every field is None
    (pmc_stale says so).  Missing entries are None."""
    from pet_posterior_distribution_amd import _lib
    pre = ('up0_fused' if fused_up else 'up0_block') + {'bfloat16': '', 'bf16x3': '_bf16x3',
                                                      'float16': '_f16'}.get(dtype, '_none')
    p = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    try:
        with open(p) as f:
            d = json.load(f)
    except Exception:
        d = {}
    have, now = d.get(pre + '_code_hash'), _lib.kernel_code_hash()
    out = dict(NO_PMC)
    if have is not None and have == now:
        out = {k: d.get(pre + suf) for k, suf in (('traffic', '_bytes_per_launch'), ('mfma_busy', '_mfma_busy_cycles'),
                                                  ('grbm', '_grbm_gui_active'), ('source', '_source'))}
    out['code_hash'] = now
    # no hash for this build (e.g. a code-object bundle the parser does not recognise): the counters
    # cannot be matched to it, so they are stale, not a match of two Nones
    out['stale'] = now is None or have != now
    out['counted_on'] = have
    return out


def pmc_fields(pmc, avg_s):
    """HBM GB/s and MFMA utilisation of the dominant kernel against chip peak.
    SQ_VALU_MFMA_BUSY_CYCLES = 32 cycles per 32x32x16 MFMA, 16 per 16x16x32 (the same per FLOP; MI355X_MICROARCH.md), summed over the
    1024 SIMDs.  mfma_util = busy / (1024 x 2.4 GHz x launch time): the MFMA pipes' share of the
    peak-clock cycles (the same ratio as executed FLOP/s / dense peak).  mfma_busy_vs_active divides
    by the kernel's own active cycles instead (GRBM_GUI_ACTIVE / 8 XCDs), which the guide notes
    reads high on dispatches this short, so that fraction reads low."""
    out = {'hbm_gbs': None, 'hbm_frac': None, 'mfma_util': None, 'mfma_busy_vs_active': None}
    if pmc['traffic']:
        out['hbm_gbs'] = round(pmc['traffic'] / avg_s / 1e9, 1)
        out['hbm_frac'] = round(pmc['traffic'] / avg_s / 1e9 / PEAK_HBM_GBS, 4)
    if pmc['mfma_busy']:
        out['mfma_util'] = round(pmc['mfma_busy'] / (N_SIMD * PEAK_CLOCK_HZ * avg_s), 4)
        if pmc['grbm']:
            out['mfma_busy_vs_active'] = round(pmc['mfma_busy'] / (N_SIMD * pmc['grbm'] / 8), 4)
    out['pmc_source'] = pmc['source']
    out['pmc_code_hash'] = pmc.get('code_hash')
    out['pmc_stale'] = pmc.get('stale')
    return out


def up0_roofline(layer_ms, bt, dtype, tflops_pipeline=None):
    """`roofline` of the dominant kernel (up0's fused level; up0.block when unfused) from per-layer HIP-event
    timing (ms, count) of one eager generate at bt samples per launch (each launch repeated TIMING_REPS times
    between its events): algorithmic FLOP per launch / mean
    launch time against the dtype's dense MFMA peak (fp16 dense = bf16 dense; bf16x3 runs 3 bf16 products
    per fp32 product, so its peak is bf16 dense / 3; f32: the fp32 MFMA peak), plus the PMC fields of the
    same kernel and dtype when the committed counters were taken on this build (load_pmc)."""
    peak = {'float32': PEAK_F32_TFLOPS, 'bf16x3': PEAK_BF16_TFLOPS / 3}.get(dtype, PEAK_BF16_TFLOPS)
    ms, cnt = layer_ms['up0.block']
    avg_s = ms / max(cnt, 1) / 1e3
    fused_up = layer_ms['up0.conv2'][1] == 0      # the k2 conv runs inside the block kernel
    alg = UP0_BLOCK_FLOP_PER_SAMPLE + (UP0_CONV2_FLOP_PER_SAMPLE if fused_up else 0)
    exe = UP0_FUSED_EXEC_FLOP_PER_SAMPLE if fused_up else UP0_BLOCK_EXEC_FLOP_PER_SAMPLE
    ach = alg * bt / avg_s / 1e12
    # the PMC passes are taken at B = 1024 (config 2), per dtype
    pmc = load_pmc(fused_up, dtype) if bt == 1024 else dict(NO_PMC)
    kname = ('conv_kernel<up0 fused> (UpSampling1D + k2 conv 1074->512 + ConvBlock 1024->512 k6+res, L=12)'
             if fused_up else 'conv_kernel<up0.block> (L=12, 1024->512, k6+res)')
    roof = {'bound': 'mfma', 'kernel': kname + (' [bf16x3: 3 bf16 MFMA products per fp32 product]'
                                               if dtype == 'bf16x3' else ''),
            'achieved': round(ach, 2), 'peak': round(peak, 2), 'unit': 'TFLOP/s', 'frac': round(ach / peak, 4),
            'traffic': pmc['traffic'], 'avg_launch_us': round(avg_s * 1e6, 2),
            'executed_tflops': round((3 if dtype == 'bf16x3' else 1) * exe * bt / avg_s / 1e12, 2)}
    if fused_up:
        ab = step_kernel_bytes('up0.block', dtype) * bt + weight_bytes('up0.block', dtype)
        roof['alg_bytes'] = int(ab)
        roof['traffic_ratio'] = round(pmc['traffic'] / ab, 2) if pmc['traffic'] else None
    if tflops_pipeline is not None:
        roof['pipeline_tflops'] = round(tflops_pipeline, 2)
        roof['pipeline_alg_over_peak'] = round(tflops_pipeline / peak, 4)
    roof.update(pmc_fields(pmc, avg_s))
    kt = kernel_table(layer_ms, bt, dtype)
    if kt is not None:
        roof['step_kernels'] = kt
    return roof


def load_pmc_kernels(dtype):
    """Per-kernel PMC counters of the step kernels (profiles/pmc_traffic.json 'kernels<suffix>', written by
    scripts/pmc_summary.py --traffic) when they were counted on this build's kernels, else None."""
    from pet_posterior_distribution_amd import _lib
    suf = {'bfloat16': '', 'bf16x3': '_bf16x3', 'float16': '_f16'}.get(dtype)
    try:
        with open(os.path.join(ROOT, 'profiles', 'pmc_traffic.json')) as f:
            d = json.load(f).get('kernels' + suf) if suf is not None else None
    except Exception:
        d = None
    now = _lib.kernel_code_hash()
    if not d or now is None or d.get('code_hash') != now:
        return None
    return d


def kernel_table(layer_ms, bt, dtype):
    """Every step kernel of the 16-bit path against the dtype's dense MFMA peak (bf16x3: bf16 / 3):
    mean launch time (HIP events, one eager generate at bt samples per launch), algorithmic GFLOP per
    launch and alg_over_peak (algorithmic FLOP/s / peak: the kernels execute fewer FLOPs
    than the reference's count -- hoisted label / time channels, folded residuals, skipped padding
    products -- so this ratio may exceed 1), exec_frac (the MFMA FLOPs the kernel executes / peak; <= 1),
    algorithmic bytes per launch (activations once + packed weights once) and, when the committed PMC
    passes were taken on this build, HBM-side traffic, its ratio to the algorithmic bytes, mfma_util
    (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x 2.4 GHz x launch time)) and LDS bank-conflict cycles."""
    if dtype == 'float32' or layer_ms['up0.conv2'][1] != 0:
        return None                                   # the unfused path: the up levels run as two launches
    peak = PEAK_BF16_TFLOPS / 3 if dtype == 'bf16x3' else PEAK_BF16_TFLOPS
    xm = 3 if dtype == 'bf16x3' else 1
    pk = load_pmc_kernels(dtype) if bt == 1024 else None
    rows = []
    for key, name, alg_mac, exe_mac in STEP_KERNELS:
        ms, cnt = layer_ms[key]
        if cnt == 0:
            continue
        avg = ms / cnt / 1e3
        alg = 2 * alg_mac * bt
        ab = (step_kernel_bytes(key, dtype)) * bt + weight_bytes(key, dtype)
        r = {'kernel': name, 'timing_key': key, 'launches_per_generate': cnt // TIMING_REPS, 'us': round(avg * 1e6, 2),
             'alg_gflop': round(alg / 1e9, 3), 'alg_over_peak': round(alg / avg / 1e12 / peak, 4),
             'exec_frac': round(xm * 2 * exe_mac * bt / avg / 1e12 / PEAK_BF16_TFLOPS, 4), 'alg_bytes': int(ab)}
        if pk is not None:
            c = pk['per_launch'].get(key.split('+')[0].replace('.block', '.fused'), {})
            if c.get('bytes'):
                r['traffic'] = int(c['bytes'])
                r['traffic_ratio'] = round(c['bytes'] / ab, 2)
                r['hbm_frac'] = round(c['bytes'] / avg / 1e9 / PEAK_HBM_GBS, 4)
            if c.get('mfma_busy_cycles'):
                r['mfma_util'] = round(c['mfma_busy_cycles'] / (N_SIMD * PEAK_CLOCK_HZ * avg), 4)
            if 'lds_bank_conflict_cycles' in c:
                r['lds_bank_conflict_cycles'] = int(c['lds_bank_conflict_cycles'])
        rows.append(r)
    return {'peak_tflops': round(peak, 2), 'samples_per_launch': bt,
            'pmc': None if pk is None else {'code_hash': pk['code_hash'], 'source': pk['source']},
            'kernels': rows}


def layer_us(layer_ms):
    return {k: round(v[0] / max(v[1], 1) * 1e3, 2) for k, v in layer_ms.items()}



# MH cost per element update (one ROI's SRTM2 + 54 truncated-normal terms), counted
# from mh_kernels.hip: 54x54 operator FMAs + per-frame exp/sqrt/div/log/erfc/log.
MH_FP64_FLOP_PER_UPDATE = 2 * 54 * 54 + 54 * 120


def mh_roofline(chain_steps_per_s, launch_chain_steps):
    """configs[2]'s chain kernel against the bound it hits (round 6).  The kernel is
    issue-bound, not fp64-FLOP-bound: its waves spend ~55 % of their cycles issuing, ~34 % waiting on LDS /
    wave barriers (PMC, SQ_ACTIVE_INST_ANY / SQ_WAIT_ANY / SQ_WAVE_CYCLES).  The committed PMC summary
    (profiles/mh_pmc.json, scripts/mh_pmc_summary.py, stamped with the MH code object's hash) gives the
    instruction mix per element update; the VALU pipe's cycles per update are fp64 wave64 instructions x 4 +
    the other VALU x 2 (MI355X_MICROARCH.md).  achieved = live updates/s x those cycles, peak = 1024 SIMDs x
    2.4 GHz; traffic = the counted fabric bytes of one 10k-chain launch scaled to this launch's chain-steps.
    The fp64 FLOP figure of earlier rounds stays as fp64_tflops / fp64_frac (an estimate, 12,312 FLOP per
    update).  Counters of another build: every counter-derived field None, pmc_stale True."""
    from pet_posterior_distribution_amd import _lib
    fl = chain_steps_per_s * 96 * MH_FP64_FLOP_PER_UPDATE / 1e12
    out = {'bound': 'valu-issue', 'achieved': None, 'peak': round(1024 * 2.4, 1), 'unit': 'G VALU-pipe cycles/s',
           'frac': None, 'traffic': None, 'fp64_tflops': round(fl, 2), 'fp64_frac': round(fl / 78.6, 4),
           'flop_per_update': MH_FP64_FLOP_PER_UPDATE}
    try:
        with open(os.path.join(ROOT, 'profiles', 'mh_pmc.json')) as f:
            d = json.load(f)
    except Exception:
        d = {}
    now = _lib.kernel_code_hash(b'mh_chain_kernel')
    out['pmc_stale'] = not d or d.get('code_hash') != now
    if not out['pmc_stale']:
        cyc = d['valu_pipe_cycles_per_update']
        ach = chain_steps_per_s * 96 * cyc / 1e9
        out.update({'achieved': round(ach, 1), 'frac': round(ach / out['peak'], 4),
                    'traffic': round(d['fabric_kb_per_launch'] * 1024 * launch_chain_steps /
                                     (d['chains'] * d['steps_per_chain'])),
                    'traffic_unit': 'bytes per launch (PMC FETCH_SIZE x 2 + WRITE_SIZE, scaled)',
                    'valu_per_update': d['valu_per_update'], 'fp64_valu_per_update': d['fp64_valu_per_update'],
                    'valu_pipe_cycles_per_update': cyc, 'wave_cycle_split': d['wave_cycle_split'],
                    'pmc_source': d.get('source')})
    return out


def mh_cpu_baseline(P, budget_s=12.0):
    """oracle/mh_ref.c (C restatement, OpenMP over chains) on a bounded sample."""
    from oracle import mh_c
    prob = mh_c.MHProblem(**P)
    threads = host_threads()
    chains, iters = threads * 2, 10
    t0 = time.perf_counter()
    prob.run(chains, iters, 0, seed=5, threads=threads)
    dt = time.perf_counter() - t0
    iters = max(10, int(iters * budget_s / max(dt, 1e-3)))
    t0 = time.perf_counter()
    prob.run(chains, iters, 0, seed=5, threads=threads)
    dt = time.perf_counter() - t0
    return {'value': chains * iters / dt, 'unit': 'chain-steps/s', 'cores': threads, 'kind': 'port',
            'sample': f'oracle/mh_ref.c (gcc -O3, OpenMP), {chains} chains x {iters} steps ({dt:.1f} s)'}


def main_mh(args):
    """BASELINE configs[2]: MH/SRTM2, 48 ROI x 10k chains x 20k steps on one GPU
    (weak scaling over ranks: every rank runs its own chains of its own TAC)."""
    import torch
    import torch.distributed as dist
    world, rank, dev = init_dist()
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    from pet_posterior_distribution_amd.sim_data import mh_problem
    P = mh_problem(seed=rank)
    mh = MetropolisSRTM2(**P)
    n, iters, tune = args.mh_chains, args.mh_iters, args.mh_tune
    mh.run(min(n, 2048), 2, 0, seed=1)                           # warm-up (module load)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    res = mh.run(n, iters, tune, seed=1 + rank)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, dev)
    # the reference's protocol per TAC (main_script.py:363-364; pymc default 4 chains):
    # 4 chains x (20k draws + 40k tune), timed on a 1/50 slice and scaled
    t1 = time.perf_counter()
    mh.run(4, 400, 800, seed=3)
    torch.cuda.synchronize()
    ref_protocol_s = (time.perf_counter() - t1) * 50
    if rank == 0:
        steps = world * n * (iters + tune)
        value = steps / elapsed
        line = {
            'metric': 'MH chain-steps/sec (48-ROI SRTM2, element-wise Metropolis)', 'value': round(value, 1),
            'unit': 'chain-steps/s', 'n_gpus': world, 'steps': 1, 'warmup': 1,
            'ms_per_step': round(elapsed * 1e3, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'f64', 'data': 'synthetic (SRTM2 TAC + noise model, reference prior prior_stats_nROI48)',
            'config': {'workload': 'mcmc.py Metropolis-Hastings, 48 ROI x 2 params, SRTM2', 'chains_per_gpu': n,
                       'steps_per_chain': iters + tune, 'tune': tune},
            'roofline': mh_roofline(steps / elapsed / world, n * (iters + tune)),
            'mean_accept_rate': round(float(res['accept_rate'].mean()), 4),
            'reference_protocol_per_tac_s': round(ref_protocol_s, 2),
        }
        line['cpu_baseline'] = None if (world > 1 or args.no_cpu_baseline) else mh_cpu_baseline(P)
        print(json.dumps(line), flush=True)
    mh.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def train_cpu_baseline(weights, x0, cond, budget_s=12.0):
    """oracle/train_ref.py (NumPy fp64 forward + backward) on a bounded sample."""
    from oracle import iddpm_ref as R
    from oracle import train_ref as TR
    S = R.schedule_tables(R.get_beta_schedule('cosine', 1000))
    P = {k: v.astype(np.float64) for k, v in weights.items()}
    rng = np.random.default_rng(0)
    B = 2
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s or n == 0:
        TR.train_loss_and_grads(P, S, x0[:B], cond[:B], rng.integers(0, 1000, B), rng.standard_normal((B, 48, 2)))
        n += 1
    dt = time.perf_counter() - t0
    return {'value': n * B / dt, 'unit': 'training samples/s', 'cores': host_threads(), 'kind': 'port',
            'sample': f'oracle/train_ref.py (NumPy fp64, loss + full backward, no optimizer), {n} batches of {B} '
                      f'({dt:.1f} s)'}


def main_train(args):
    """ImprovedDDPM.train_step at the reference's batch (256 per GPU), fp32.
    Data-parallel over ranks: the per-rank gradients are summed over RCCL, which is exactly the
    gradient of the global batch on one device (J = B*mse + sum vlb splits over shards;
    tests/test_cpu_train.py gloo test); training data = the GPU synthetic-TAC generator (row 3)."""
    import torch
    import torch.distributed as dist
    world, rank, dev = init_dist()
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional, Adam, ExponentialDecay
    from pet_posterior_distribution_amd.configs import shipped_net_args, shipped_diff_args
    from pet_posterior_distribution_amd.networks import glorot_uniform_init
    from pet_posterior_distribution_amd.sim_data import simulate_dataset
    net = UnetConditional(**shipped_net_args(), seed=1234)
    net.build((None, 48, 2))
    net.weights = glorot_uniform_init(net.spec(), seed=1234)
    model = ImprovedDDPM(network=net, dtype='float32', device=dev.index, **shipped_diff_args())
    B = args.train_batch
    n_data = B * 8
    # main_script.py:169-192, 233: Adam(ExponentialDecay(2e-4 -> 5e-5 over 500 epochs), clipnorm 1.5)
    sched = ExponentialDecay(2e-4, n_data // B, (5e-5 / 2e-4) ** (1 / 500))
    model.compile(optimizer=Adam(learning_rate=sched, clipnorm=1.5), loss='MeanSquaredError')
    data = simulate_dataset(n_data, seed=7, sample_offset=rank * n_data, device=dev.index)
    x0 = torch.stack([data['varDVR'], data['varR1']], -1).to(torch.float32).contiguous()
    cond = data['condition']
    tr = model._ensure_trainer()
    loss = torch.empty(B, dtype=torch.float32, device=dev)
    it = [0]

    def one():
        k = it[0] % 8
        it[0] += 1
        tr.compute_gradients(x0[k * B:(k + 1) * B], cond[k * B:(k + 1) * B], seed=11,
                             sample_offset=rank * B, loss=loss)
        if world > 1:
            g = tr.gradients()
            if coll_device(dev) == 'cpu':
                gh = g.cpu()
                dist.all_reduce(gh)
                g.copy_(gh)
            else:
                dist.all_reduce(g)
            tr.set_gradients(g)
        tr.apply_gradients(1.0)

    for _ in range(max(args.warmup, 1)):
        one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, dev)
    stats = tr.last_stats()
    if rank == 0:
        samples = world * B * args.steps
        value = samples / elapsed
        ach = TRAIN_FLOP_PER_SAMPLE * samples / elapsed / 1e12
        line = {
            'metric': 'training samples/sec (ImprovedDDPM.train_step, batch 256 per GPU)', 'value': round(value, 1),
            'unit': 'samples/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'f32',
            'data': 'synthetic (GPU SRTM2 generator: truncated-MVN reference prior + noise model; Glorot init)',
            'config': {'workload': 'iDDPM training step (q-sample, U-Net fwd/bwd, MSE + 0.1 VLB, clipped Adam)',
                       'batch_per_gpu': B, 'global_batch': world * B,
                       'parallelism': f'dp{world} (RCCL all-reduce of the fp32 gradient blob)'},
            'roofline': {'bound': 'mfma', 'scope': 'whole step (rocBLAS fp32 GEMMs + HIP glue)',
                         'achieved': round(ach, 2), 'peak': PEAK_F32_TFLOPS, 'unit': 'TFLOP/s',
                         'frac': round(ach / PEAK_F32_TFLOPS, 4), 'traffic': None,
                         'flop_per_sample': TRAIN_FLOP_PER_SAMPLE},
            'last_loss': [round(float(v), 6) for v in stats],
        }
        line['cpu_baseline'] = None if (world > 1 or args.no_cpu_baseline) else \
            train_cpu_baseline(net.weights, x0[:2].cpu().numpy(), cond[:2].cpu().numpy())
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def f32_exact_rate(cond, B, n_rev, dev):
    """The reference's own precision (diffusion_model.py:7-10, fp32): the same generate() on the
    exact-f32 MFMA network (v_mfma_f32_32x32x2_f32; the path the 1e-4 parity tests run), one graph
    warm-up + one timed run of B samples x n_rev steps."""
    import torch
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    from pet_posterior_distribution_amd.configs import shipped_net_args, shipped_diff_args
    net = UnetConditional(**shipped_net_args(), seed=1234)
    net.build((None, 48, 2))
    m = ImprovedDDPM(network=net, dtype='float32', device=dev.index, **shipped_diff_args())
    x = m.philox_normal(B, seed=5)
    m.ddpm_loop(x, cond[None], num_timesteps=n_rev, seed=2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = m.ddpm_loop(x, cond[None], num_timesteps=n_rev, seed=2)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tf = FLOP_PER_SAMPLE_STEP * n_rev * B / el / 1e12
    te = EXEC_FLOP_PER_SAMPLE_STEP_UNFUSED * n_rev * B / el / 1e12
    m.close()
    return {'value': round(B / el, 2), 'unit': 'samples/s', 'dtype': 'f32', 'n_posterior': B,
            'reverse_steps': n_rev, 'ms_per_generate': round(el * 1e3, 2),
            'pipeline_tflops': round(tf, 2), 'peak': PEAK_F32_TFLOPS, 'alg_over_peak': round(tf / PEAK_F32_TFLOPS, 4),
            'executed_tflops': round(te, 2), 'executed_frac': round(te / PEAK_F32_TFLOPS, 4),
            'finite': bool(torch.isfinite(out).all()),
            'note': 'alg_over_peak: algorithmic FLOP (SURVEY 8(d): every Conv1D incl. its label/time channels and 1x1 '
                    'residual) / peak; the kernels hoist the label/time channels into maps and fold the residual into '
                    'the centre tap, so they execute 0.82 of that (executed_frac, the roofline fraction) and '
                    'alg_over_peak can exceed 1'}


def bf16x3_rate(cond, B, n_rev, dev):
    """fp32-class accuracy on the bf16 MFMA path (PETDIFF_DTYPE_BF16X3: every fp32 operand split
    hi + lo into bf16, three products per pair, fp32 accumulate; tests/test_gpu_bf16x3.py holds it to
    the exact-f32 mode's 1e-4 parity bounds).  Same generate() as f32_exact_rate; frac counts the
    algorithmic FLOPs against the dense bf16 peak, executed_frac the 3 x executed bf16 MFMA FLOPs."""
    import torch
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    from pet_posterior_distribution_amd.configs import shipped_net_args, shipped_diff_args
    net = UnetConditional(**shipped_net_args(), seed=1234)
    net.build((None, 48, 2))
    m = ImprovedDDPM(network=net, dtype='bf16x3', device=dev.index, **shipped_diff_args())
    x = m.philox_normal(B, seed=5)
    m.ddpm_loop(x, cond[None], num_timesteps=n_rev, seed=2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = m.ddpm_loop(x, cond[None], num_timesteps=n_rev, seed=2)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tf = FLOP_PER_SAMPLE_STEP * n_rev * B / el / 1e12
    te = 3 * EXEC_MFMA_FLOP_PER_SAMPLE_STEP_FUSED * n_rev * B / el / 1e12
    # the dominant kernel of THIS network: per-layer HIP events over one eager generate on the launch stream
    m.set_kernel_timing(True, reps=TIMING_REPS)
    m.ddpm_loop(x, cond[None], num_timesteps=n_rev, seed=2, use_graph=False)
    lm = m.get_kernel_timing()
    m.set_kernel_timing(False)
    m.close()
    return {'value': round(B / el, 2), 'unit': 'samples/s', 'dtype': 'bf16x3 (fp32-class)', 'n_posterior': B,
            'reverse_steps': n_rev, 'ms_per_generate': round(el * 1e3, 2),
            'pipeline_tflops': round(tf, 2), 'alg_over_f32_peak': round(tf / PEAK_F32_TFLOPS, 4),
            'pipeline_alg_over_bf16x3_peak': round(tf / (PEAK_BF16_TFLOPS / 3), 4),
            'executed_bf16_tflops': round(te, 2), 'executed_frac': round(te / PEAK_BF16_TFLOPS, 4),
            'roofline': up0_roofline(lm, B, 'bf16x3'), 'layer_us': layer_us(lm),
            'finite': bool(torch.isfinite(out).all())}


def mh_config2_and_protocol(iddpm_10k_s, dev, cpu=True):
    """BASELINE configs[2] at full size -- 48 ROI x 10k chains x 20k steps (10k tune + 10k draws), fp64,
    about 16 s -- with its fp64 roofline and the oracle/mh_ref.c CPU baseline (rank 0, bounded sample); and
    the reference's per-TAC MCMC protocol (main_script.py:363-364, pymc's default 4 chains: 4 x (20k draws
    + 40k tune)), timed as a 1/10 slice x 10, against iDDPM's 10,000 posterior samples of one TAC
    (main_script.py:315-319) on the same GPU -- the README.md:12 '> 230x' claim, same silicon."""
    import torch
    from pet_posterior_distribution_amd.mcmc import MetropolisSRTM2
    from pet_posterior_distribution_amd.sim_data import mh_problem
    P = mh_problem(seed=0)
    mh = MetropolisSRTM2(**P)
    mh.run(512, 2, 0, seed=1)
    torch.cuda.synchronize()
    n, tune, draws = 10000, 10000, 10000
    t0 = time.perf_counter()
    res = mh.run(n, draws, tune, seed=7)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    steps = n * (tune + draws)
    fl = steps * 96 * MH_FP64_FLOP_PER_UPDATE / el / 1e12
    t1 = time.perf_counter()
    mh.run(4, 2000, 4000, seed=3)
    torch.cuda.synchronize()
    proto = (time.perf_counter() - t1) * 10
    mh.close()
    # the paper's own comparison (README.md:12): the network on the GPU against MCMC on CPU cores.  PyMC runs
    # its 4 chains in parallel processes, so the protocol takes one chain's 60k steps on 4 cores; here the
    # C restatement of the same sampler (oracle/mh_ref.c, 4 OpenMP threads, one chain each), timed on
    # 4 x (2000 + 4000) steps and scaled x 10 (about 1 s of CPU work)
    cpu_proto = None
    if cpu:
        from oracle import mh_c
        prob = mh_c.MHProblem(**P)
        t2 = time.perf_counter()
        prob.run(4, 2000, 4000, seed=3, threads=4)
        cpu_proto = (time.perf_counter() - t2) * 10
    cfg2 = {'value': round(steps / el, 1), 'unit': 'chain-steps/s', 'chains': n, 'steps_per_chain': tune + draws,
            'tune': tune, 'draws': draws, 'seconds': round(el, 3), 'dtype': 'f64',
            'roofline': mh_roofline(steps / el, steps),
            'mean_accept_rate': round(float(res['accept_rate'].mean()), 4),
            'cpu_baseline': mh_cpu_baseline(P) if cpu else None}
    return (cfg2,
            {'mh_protocol_s_per_tac': round(proto, 3), 'mh_protocol': '4 chains x (20000 draws + 40000 tune), '
             'timed as 4 x (2000 + 4000) x 10', 'iddpm_s_per_tac': round(iddpm_10k_s, 3),
             'iddpm_protocol': '10,000 posterior samples x 1000 reverse steps, bf16, one launch',
             'iddpm_speedup_over_mh': round(proto / iddpm_10k_s, 2), 'reference_claim': '> 230x (README.md:12)',
             'mh_cpu_protocol_s_per_tac': None if cpu_proto is None else round(cpu_proto, 3),
             'mh_cpu_protocol': 'oracle/mh_ref.c (gcc -O3, OpenMP), 4 threads = one chain each, as PyMC runs its '
                                '4 chains; 4 x (2000 + 4000) steps timed, x 10',
             'iddpm_gpu_over_mh_cpu': None if cpu_proto is None else round(cpu_proto / iddpm_10k_s, 2)})


def weights_sensitivity(net, cond, B, dev, reps=3):
    """The step's speed depends on the weight VALUES: the chip holds its clock by power under this load, and
    MFMA energy depends on operand bit activity.  The same workload as `value` (configs[1]: B samples x 1000
    steps, one generate() per rep) for bf16 and bf16x3 with:
      * glorot: the headline's own random-init weights (UnetConditional(seed=1234)), re-timed here beside the
        others so the ratios are same-process;
      * trained: the shipped network after 800 Adam steps on GPU-simulated training data
        (tests/helpers.quick_trained_weights: batch 256, lr 2e-4, clipnorm 1.5 as main_script.py:169-174,
        regenerated in-process, about 3 s), an eps-predictor whose reverse chain stays bounded;
      * zeros: all-zero weights (the power floor: MFMA operands toggle nothing);
      * trained_r02: scripts/train_protocol.py's longer-trained network, when weights/trained_r02.npz exists.
    Context for `value`, which uses the glorot weights."""
    import torch
    from pet_posterior_distribution_amd import ImprovedDDPM
    from pet_posterior_distribution_amd.configs import shipped_diff_args
    keep = net.weights
    variants = {'glorot': keep}
    try:
        from tests.helpers import quick_trained_weights
        variants['trained'] = quick_trained_weights()[0]
    except Exception as e:   # noqa: BLE001 -- reported, not fatal: the headline line must still print
        variants['trained_error'] = repr(e)
    variants['zeros'] = {k: np.zeros_like(v) for k, v in keep.items()}
    tw = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'weights', 'trained_r02.npz')
    if os.path.exists(tw):
        with np.load(tw) as z:
            variants['trained_r02'] = {k: z[k] for k in keep}
    out = {'reps': reps, 'n_posterior': B, 'reverse_steps': 1000}
    try:
        for dtype, tag in (('bfloat16', ''), ('bf16x3', 'bf16x3_')):
            for name, w in variants.items():
                if isinstance(w, str):
                    out[name] = w
                    continue
                net.weights = w
                m = ImprovedDDPM(network=net, dtype=dtype, device=dev.index, **shipped_diff_args())
                x = m.philox_normal(B, seed=1)
                m.ddpm_loop(x, cond[None], seed=2)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    y = m.ddpm_loop(x, cond[None], seed=2)
                torch.cuda.synchronize()
                out[tag + name + '_samples_per_s'] = round(reps * B / (time.perf_counter() - t0), 1)
                if name == 'trained':
                    out[tag + 'trained_outputs_finite'] = bool(torch.isfinite(y).all())
                m.close()
    finally:
        net.weights = keep
    for tag in ('', 'bf16x3_'):
        g, t = out.get(tag + 'glorot_samples_per_s'), out.get(tag + 'trained_samples_per_s')
        if g and t:
            out[tag + 'trained_over_glorot'] = round(t / g, 4)
    return out


def iddpm_10k_seconds(model, cond):
    """One TAC's posterior as the reference draws it: n_posterior = chunk_size = 10,000 samples in one
    ddpm_loop (main_script.py:315-319, 414-420), graph warm-up then one timed run."""
    import torch
    x = model.philox_normal(10000, seed=9)
    model.ddpm_loop(x, cond[None], seed=4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.ddpm_loop(x, cond[None], seed=4)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def main():
    args = parse()
    if args.workload == 'mh':
        return main_mh(args)
    if args.workload == 'train':
        return main_train(args)
    import torch
    import torch.distributed as dist
    world, rank, dev = init_dist()

    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    from pet_posterior_distribution_amd.sim_data import make_condition
    from pet_posterior_distribution_amd.configs import shipped_net_args, shipped_diff_args

    net = UnetConditional(**shipped_net_args(), seed=1234)
    net.build((None, 48, 2))
    model = ImprovedDDPM(network=net, dtype=args.dtype, device=dev.index, **shipped_diff_args())
    if args.config4:
        args.batch, args.tacs = 32 * 8192, 32
    from pet_posterior_distribution_amd import _lib
    if args.chunk:
        if not 0 < args.chunk <= _lib.MAX_BATCH:
            raise SystemExit(f'--chunk must be in [1, {_lib.MAX_BATCH}]')
        _lib.MAX_BATCH = args.chunk
    chunk = _lib.MAX_BATCH
    B = args.batch
    n_tac = args.tacs
    if n_tac < 1 or B % n_tac:
        raise SystemExit('--batch must be a multiple of --tacs')
    # BASELINE configs[3]'s product path (distributed.sample_posterior_sharded, tests/test_gpu_sharded.py):
    # world * n_tac synthetic test TACs (TAC k = make_condition(seed=k)) x B / n_tac posterior samples each,
    # sharded TAC-major, so rank r owns TACs r * n_tac .. r * n_tac + n_tac - 1 and global samples
    # r * B .. r * B + B - 1; x_T and z from the counter-based Philox stream keyed by the global sample index.
    # One bench step = one whole job: x_T, the 1000-step generate (one replayed hipGraph per launch of
    # <= PETDIFF_MAX_BATCH samples), the GPU Welford statistics and their all-gather + merge.
    from pet_posterior_distribution_amd.distributed import TacTable, sample_posterior_sharded, rank_tac_range
    n_per = B // n_tac
    table = TacTable(world * n_tac, lambda k: make_condition(seed=k))
    cond = table.rows(range(rank * n_tac, rank * n_tac + n_tac))          # this rank's TACs (built once)
    coll = coll_device(dev) if world > 1 else None
    n_rev = args.reverse_steps
    offset = rank * B
    ag = {'ms': 0.0}

    def one():
        return sample_posterior_sharded(model, table, n_per, seed=2, x_T_seed=1, num_timesteps=n_rev,
                                        return_samples=True, coll_device=coll)

    long_run = B > chunk                      # e.g. --config4: about a minute per step; say so on stderr
    for i in range(args.warmup):
        res = one()
        if long_run:
            torch.cuda.synchronize()
            print(f'[bench] warmup {i + 1}/{args.warmup} done', file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        res = one()
        if long_run:
            print(f'[bench] step {i + 1}/{args.steps} done', file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, dev)
    _, allst, (lo, hi, out) = res
    assert (lo, hi) == (offset, offset + B)
    if world > 1:                              # the all-gather alone, and the host merge, timed once after the loop
        from pet_posterior_distribution_amd.distributed import (allgather_stats, merge_gathered_tacs,
                                                                pad_own_tacs, rank_tac_range)
        t0r, t1r = rank_tac_range(len(allst), n_per, world, rank)
        pad = pad_own_tacs(allst[t0r:t1r], len(allst), n_per, world)
        torch.cuda.synchronize()
        ta = time.perf_counter()
        parts = allgather_stats(pad, device=coll)      # the collective on the padded own-TAC partials only
        torch.cuda.synchronize()
        ag['ms'] = (time.perf_counter() - ta) * 1e3
        tb = time.perf_counter()
        merge_gathered_tacs(parts, len(allst), n_per)
        ag['merge_ms'] = (time.perf_counter() - tb) * 1e3
    ag_ms = ag['ms']
    finite = bool(torch.isfinite(out).all())
    x_T = model.philox_normal(min(B, chunk), seed=1, sample_offset=offset)
    tac = torch.arange(n_tac, device=dev, dtype=torch.int32).repeat_interleave(n_per)

    # per-layer kernel timing (HIP events on the launch stream, one eager generate)
    layer_ms = None
    if not args.no_kernel_timing:
        model.set_kernel_timing(True, reps=TIMING_REPS)
        bt = min(B, chunk)   # one launch's worth of samples
        model.ddpm_loop(x_T[:bt], cond, num_timesteps=n_rev, seed=2, sample_offset=offset, use_graph=False,
                        tac=tac[:bt] if n_tac > 1 else None)
        layer_ms = model.get_kernel_timing()
        model.set_kernel_timing(False)

    if rank == 0:
        samples = world * B * args.steps
        value = samples / elapsed
        tflops_pipeline = FLOP_PER_SAMPLE_STEP * n_rev * samples / elapsed / 1e12
        roof = up0_roofline(layer_ms, bt, args.dtype, tflops_pipeline) if layer_ms is not None else None
        line = {
            'metric': 'posterior samples/sec (48-ROI TAC, 1000-step reverse) at 1/2/4/8 MI355X',
            'value': round(value, 2), 'unit': 'samples/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': {'bfloat16': 'bf16', 'float16': 'f16', 'float32': 'f32',
                                                    'bf16x3': 'bf16x3 (fp32-class)'}[args.dtype],
            'data': 'synthetic (test TACs drawn from the reference prior prior_stats_nROI48 + SRTM2 + noise model; '
                    'identity-denoiser Glorot weights of the shipped net)',
            'config': {'workload': 'iDDPM reverse process, f128/d4 1-D conditional U-Net, 48-ROI x 2 params',
                       'n_posterior_per_gpu': B, 'reverse_steps': n_rev, 'global_batch': world * B,
                       'tacs': world * n_tac, 'samples_per_launch': min(B, chunk),
                       'parallelism': f'dp{world} (TAC-major sample shards, RCCL all-gather of stats)',
                       'driver': 'distributed.sample_posterior_sharded',
                       'hipgraph': True},
            'roofline': roof,
            'outputs_finite': finite,
            'stats_allgather_ms': round(ag_ms, 3),
            # host placement + Chan merge of the gathered rows (gather_merge_own_tacs minus its all-gather)
            'stats_merge_ms': round(ag.get('merge_ms', 0.0), 3),
            # bytes each rank receives: world x the largest rank's TAC range x 2,304 B (own TACs only)
            'stats_allgather_bytes': world * max(t1 - t0 for t0, t1 in (rank_tac_range(world * n_tac, n_per, world, r)
                                                                        for r in range(world))) * 48 * 2 * 3 * 8,
        }
        if layer_ms is not None:
            line['layer_us'] = layer_us(layer_ms)
        if world == 1 and not args.no_cpu_baseline:
            line['cpu_baseline'] = cpu_baseline(net.weights, cond[0])
        else:
            line['cpu_baseline'] = None
        if world == 1 and not args.no_extras and args.dtype == 'bfloat16' and n_rev == 1000 and n_tac == 1:
            line['f32_exact'] = f32_exact_rate(cond[0], B, n_rev, dev)
            line['bf16x3'] = bf16x3_rate(cond[0], B, n_rev, dev)
            t10k = iddpm_10k_seconds(model, cond[0])
            line['mh_config2'], line['reference_protocol'] = mh_config2_and_protocol(t10k, dev,
                                                                                     not args.no_cpu_baseline)
            line['weights_sensitivity'] = weights_sensitivity(net, cond[0], B, dev)
        sm = allst[..., 1]
        line['posterior_mean_DVR_roi0'] = [round(float(v), 5) for v in sm[:, 0, 0]]
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
