"""In-process A/B of a handle switch read at creation (default PETDIFF_FUSE_DOWN1: the fused next-step down1
against the standalone down1 launch; AB_VAR=PETDIFF_SEAM23 etc.), per dtype: configs[1] workload (1 TAC x
1024 samples x 1000 steps, graph), rounds interleaved, plus per-layer HIP-event times of one eager generate
per variant and a bitwise check of a 20-step loop.  The library under test is PETDIFF_LIB (or the in-tree
build).  Usage: [AB_VAR=...] python scripts/ab_fd1.py OUT.jsonl [dtypes...]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))


VAR = os.environ.get('AB_VAR', 'PETDIFF_FUSE_DOWN1')


def main(out, dtypes):
    from pet_posterior_distribution_amd import ImprovedDDPM, UnetConditional
    from pet_posterior_distribution_amd.configs import shipped_net_args, shipped_diff_args
    from pet_posterior_distribution_amd.sim_data import make_condition
    torch.cuda.set_device(0)
    cond = make_condition(0)
    net = UnetConditional(**shipped_net_args(), seed=1234)
    net.build((None, 48, 2))
    B, reps, rounds = 1024, 4, 3
    f = open(out, 'a')
    for dt in dtypes:
        models = {}
        for fuse in ('1', '0'):
            os.environ[VAR] = fuse
            m = ImprovedDDPM(network=net, dtype=dt, **shipped_diff_args())
            m._ensure_handle()
            x = m.philox_normal(B, seed=1)
            m.ddpm_loop(x, cond[None], seed=2)
            models[fuse] = (m, x)
        res = {k: [] for k in models}
        for _ in range(rounds):
            for k, (m, x) in models.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    m.ddpm_loop(x, cond[None], seed=2)
                torch.cuda.synchronize()
                res[k].append(round(reps * B / (time.perf_counter() - t0), 1))
        lay = {}
        for k, (m, x) in models.items():
            m.set_kernel_timing(True)
            m.ddpm_loop(x, cond[None], seed=2, use_graph=False)
            t = m.get_kernel_timing()
            m.set_kernel_timing(False)
            lay[k] = {n: round(v[0] / max(v[1], 1) * 1e3, 2) for n, v in t.items() if v[1]}
        same = bool(torch.equal(models['1'][0].ddpm_loop(models['1'][1], cond[None], seed=3, num_timesteps=20),
                                models['0'][0].ddpm_loop(models['0'][1], cond[None], seed=3, num_timesteps=20)))
        rec = {'switch': VAR, 'dtype': dt, 'lib': os.environ.get('PETDIFF_LIB', 'in-tree'), 'samples_per_s_fused': res['1'],
               'samples_per_s_standalone': res['0'], 'layer_us_fused': lay['1'], 'layer_us_standalone': lay['0'],
               'bitwise_equal_20_steps': same}
        print(json.dumps(rec), flush=True)
        f.write(json.dumps(rec) + '\n')
        for m, _ in models.values():
            m.close()
    os.environ.pop(VAR, None)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2:] or ['bfloat16', 'bf16x3', 'float16'])
