"""Test/benchmark infrastructure, NOT the product: a torch-CPU fp32 restatement of the iDDPM
p_sample (ImprovedDDPM.ddpm, diffusion_model.py:651-663) and of UnetConditional.call
(networks.py:994-1093), for bench.py's cpu_baseline leg only.  It follows oracle/iddpm_ref.py
operation for operation (Keras SAME padding (2, 3) for k = 6 and (0, 1) for k = 2, a separate
1x1 residual conv, concat order [label | time | x], the raw Reshape of the label projection,
the condition encoder recomputed every call as the reference does), with the convolutions on
torch's CPU conv1d (oneDNN) instead of NumPy per-tap matmuls: about 2.4x the NumPy oracle's
rate on the same cores.  tests/test_cpu.py checks it against oracle/iddpm_ref.py."""
import math

import numpy as np
import torch
import torch.nn.functional as F

from oracle import iddpm_ref as R


class TorchCpuUnet:
    """Weights (the oracle's dict of Keras-layout arrays) converted once to torch CPU tensors."""

    def __init__(self, P, dtype=torch.float32):
        self.dt = dtype
        self.P = {}
        for k, v in P.items():
            t = torch.as_tensor(np.asarray(v), dtype=dtype)
            if k.endswith('.kernel') and t.dim() == 3:      # Keras Conv1D (k, Cin, Cout) -> (Cout, Cin, k)
                t = t.permute(2, 1, 0).contiguous()
            self.P[k] = t

    def conv(self, x, name):
        """Conv1D(padding='same') on channels-last x (B, L, C)."""
        w, b = self.P[name + '.kernel'], self.P[name + '.bias']
        k = w.shape[2]
        pl = (k - 1) // 2
        y = F.conv1d(F.pad(x.transpose(1, 2), (pl, k - 1 - pl)), w, b)
        return y.transpose(1, 2)

    def dense(self, x, name):
        return x @ self.P[name + '.kernel'] + self.P[name + '.bias']

    def forward(self, x, t, cond, depth=4):
        P = self.P
        B, n_roi = x.shape[0], x.shape[1]
        down_L, up_L = R.level_lengths(n_roi, depth)
        emb = torch.as_tensor(R.sinusoidal_pos_emb(np.asarray(t), dt=np.float32), dtype=self.dt)
        a = self.dense(emb, 'time_mlp')
        h_t = 0.5 * a * (1.0 + torch.erf(a / math.sqrt(2.0)))             # GELU(approximate=False)
        e = cond
        for i in range(3):
            e = torch.relu(self.dense(e, f'cond_enc.hidden{i}'))
        z_lab = self.dense(e, 'cond_enc.z')

        def cond_inputs(prefix, L):
            tim = self.dense(h_t, prefix + '.time_proj').reshape(B, L, -1)
            lab = self.dense(z_lab, prefix + '.label_proj').reshape(B, L, -1)
            return lab, tim

        skips, h = [], x
        for d in range(depth):
            lab, tim = cond_inputs(f'down{d}', down_L[d])
            h = torch.cat([lab, tim, h], dim=-1)
            h = torch.relu(self.conv(h, f'down{d}.conv') + self.conv(h, f'down{d}.res'))
            skips.append(h)
            if d < depth - 1:
                h = h.reshape(B, h.shape[1] // 2, 2, h.shape[2]).amax(dim=2)
        for u in range(depth - 1):
            lab, tim = cond_inputs(f'up{u}', up_L[u])
            h = torch.cat([lab, tim, h], dim=-1).repeat_interleave(2, dim=1)
            h = self.conv(h, f'up{u}.upconv')
            h = torch.cat([skips[depth - 2 - u], h], dim=-1)
            h = torch.relu(self.conv(h, f'up{u}.conv') + self.conv(h, f'up{u}.res'))
        return self.conv(h, 'final')

    def ddpm(self, S, x_t, t, cond, z):
        """ImprovedDDPM.ddpm, learn_ranged + eps (the shipped config): (mean, var, var_tilde)."""
        with torch.no_grad():
            out = self.forward(x_t, t, cond)
            eps, v = out[..., :2], out[..., 2:]
            ti = torch.as_tensor(np.asarray(t), dtype=torch.long)

            def ex(name):
                return torch.as_tensor(np.asarray(S[name], dtype=np.float32))[ti].reshape(-1, 1, 1)
            min_log = ex('posterior_log_variance_clipped')
            max_log = torch.log(ex('beta'))
            frac = (v + 1) / 2
            logvar = frac * max_log + (1 - frac) * min_log
            x0 = 1.0 / ex('sqrt_alpha_bar') * x_t - torch.sqrt(1.0 / ex('alpha_bar') - 1) * eps
            mean = ex('posterior_mean_coef1') * x0 + ex('posterior_mean_coef2') * x_t
            mask = (ti != 0).to(self.dt).reshape(-1, 1, 1)
            var = mask * torch.exp(0.5 * logvar) * z
            return mean, var, var
