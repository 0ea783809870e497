"""Multi-GPU sharding of posterior sampling.

Posterior samples and test TACs are independent units: every rank (one process
per GPU, torch.distributed over RCCL) samples a contiguous block of the global
(TAC, sample) index space with no per-step communication.  The noise of global
sample g is Philox(seed, g, step), so the result is independent of the world
size.  The only collective is one all-gather of per-(TAC, ROI, parameter)
Welford partials {count, mean, M2} (fp64, 2,304 B per TAC) of each rank's OWN TAC
range (padded to the largest range), merged on the host with Chan's parallel
formula into the population mean / std of main_script.py:433-436.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_total, world, rank):
    """Contiguous block [lo, hi) of n_total units owned by `rank` (sizes differ by <= 1)."""
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def tac_major_shards(n_tac, n_per_tac, world, rank):
    """Global sample indices of `rank` for n_tac TACs x n_per_tac samples, TAC-major
    (whole TACs per rank when n_tac >= world).  Returns (lo, hi) over g = tac*n_per_tac + s."""
    return shard_range(n_tac * n_per_tac, world, rank)


def rank_tac_range(n_tac, n_per_tac, world, rank):
    """TACs [t0, t1) that rank `rank`'s sample block touches (t0 == t1: an empty block).  Consecutive
    ranks' ranges overlap in at most one TAC (the TAC their blocks split)."""
    lo, hi = tac_major_shards(n_tac, n_per_tac, world, rank)
    if hi <= lo:
        return lo // max(n_per_tac, 1), lo // max(n_per_tac, 1)
    return lo // n_per_tac, (hi - 1) // n_per_tac + 1


def merge_stats(parts):
    """Chan et al. pairwise merge of [..., 3] {count, mean, M2} partials along axis 0."""
    parts = np.asarray(parts, dtype=np.float64)
    n, mean, m2 = parts[0, ..., 0].copy(), parts[0, ..., 1].copy(), parts[0, ..., 2].copy()
    for p in parts[1:]:
        nb, mb, m2b = p[..., 0], p[..., 1], p[..., 2]
        tot = n + nb
        with np.errstate(invalid='ignore', divide='ignore'):
            delta = mb - mean
            w = np.where(tot > 0, nb / np.where(tot > 0, tot, 1), 0.0)
            mean = mean + delta * w
            m2 = m2 + m2b + delta * delta * np.where(tot > 0, n * nb / np.where(tot > 0, tot, 1), 0.0)
        n = tot
    return np.stack([n, mean, m2], axis=-1)


def local_stats_numpy(x, tac=None, n_tac=1):
    """Reference {count, mean, M2} of samples x (B, 48, 2) per condition (host, for tests)."""
    x = np.asarray(x, dtype=np.float64)
    tac = np.zeros(x.shape[0], dtype=np.int64) if tac is None else np.asarray(tac)
    out = np.zeros((n_tac,) + x.shape[1:] + (3,))
    for k in range(n_tac):
        xs = x[tac == k]
        if xs.shape[0]:
            out[k, ..., 0] = xs.shape[0]
            out[k, ..., 1] = xs.mean(0)
            out[k, ..., 2] = ((xs - xs.mean(0)) ** 2).sum(0)
    return out


def allgather_stats(stats, group=None, device=None):
    """All-gather this rank's [n_local, ...,3] partials (every rank's array the same shape); returns
    [world, n_local, ..., 3] on the host.

    Uses the process group's backend (nccl = RCCL over xGMI on MI355X, gloo on CPU)."""
    import torch
    import torch.distributed as dist
    t = torch.as_tensor(np.ascontiguousarray(stats), dtype=torch.float64)
    if device is not None:
        t = t.to(device)
    world = dist.get_world_size(group)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    return np.stack([o.cpu().numpy() for o in out])


def gather_merge_own_tacs(local, n_tac, n_per_tac, group=None, device=None):
    """SURVEY 8(e) payload: each rank contributes only the partials of its own TAC range (``local``:
    [t1 - t0, 48, 2, 3] for rank_tac_range), zero-padded to the largest range over the ranks; the host
    scatters every rank's rows to their TACs and Chan-merges (zero-count rows are neutral, and a TAC split
    between two ranks is merged from both).  Returns the merged [n_tac, 48, 2, 3] statistics.  Each rank
    receives world x max-range x 2,304 B (configs[3]: 8 x 32 TACs = 590 KB, not 8 x 256)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    return merge_gathered_tacs(allgather_stats(pad_own_tacs(local, n_tac, n_per_tac, world), group=group,
                                               device=device), n_tac, n_per_tac)


def pad_own_tacs(local, n_tac, n_per_tac, world):
    """This rank's [t1 - t0, ...] partials zero-padded to the widest rank range (the all-gather payload)."""
    width = max(max(t1 - t0 for t0, t1 in (rank_tac_range(n_tac, n_per_tac, world, r) for r in range(world))), 1)
    local = np.asarray(local, dtype=np.float64)
    pad = np.zeros((width,) + local.shape[1:])
    pad[:local.shape[0]] = local
    return pad


def merge_gathered_tacs(parts, n_tac, n_per_tac):
    """[world, width, ...] gathered payloads -> every rank's rows placed at their TACs, Chan-merged."""
    world = parts.shape[0]
    placed = np.zeros((world, n_tac) + parts.shape[2:])
    for r in range(world):
        t0, t1 = rank_tac_range(n_tac, n_per_tac, world, r)
        placed[r, t0:t1] = parts[r, :t1 - t0]
    return merge_stats(placed)


def summarize(stats):
    """{count, mean, M2} -> mean / population std (ddof=0) per ROI for DVR (ch 0) and R1 (ch 1)."""
    cnt, mean, m2 = stats[..., 0], stats[..., 1], stats[..., 2]
    std = np.sqrt(m2 / np.maximum(cnt, 1))
    return {'mean_DVR': mean[..., 0], 'mean_R1': mean[..., 1], 'std_DVR': std[..., 0], 'std_R1': std[..., 1]}


def sample_posterior_sharded(model, cond_all, n_per_tac, seed=0, x_T_seed=1, group=None, use_graph=True,
                             return_samples=False, coll_device=None, num_timesteps=None):
    """BASELINE configs[3] driver (main_script.py:414-436 for many test TACs at once): n_tac TACs x
    n_per_tac posterior samples, sharded TAC-major over the ranks (global sample g = tac * n_per_tac + s).

    Each rank generates its block [lo, hi) -- x_T and z from counter-based Philox keyed by g, so the
    samples do not depend on the world size or on how ddpm_loop chunks the block -- reduces it on
    the GPU to per-TAC Welford partials {count, mean, M2} (fp64), and the partials of all ranks are
    all-gathered (RCCL over xGMI, or gloo) and merged with Chan's formula; a TAC that spans two ranks
    is merged from its two partials.  ``cond_all`` is the (n_tac, 49, 54) table of every TAC, or a
    TacTable (below) that builds only this rank's rows.

    ``num_timesteps`` is ddpm_loop's (None = all T steps, as main_script.py:418-420 runs it).
    Returns (summary dict of (n_tac, 48) arrays, merged stats (n_tac, 48, 2, 3)); with
    ``return_samples`` also (lo, hi, this rank's samples x_0 (hi - lo, 48, 2) on the device)."""
    import torch.distributed as dist
    dist_on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if dist_on else 1
    rank = dist.get_rank(group) if dist_on else 0
    n_tac = len(cond_all)
    lo, hi = tac_major_shards(n_tac, n_per_tac, world, rank)
    t0, t1 = rank_tac_range(n_tac, n_per_tac, world, rank)
    local = np.zeros((t1 - t0, 48, 2, 3))          # this rank's TACs only (the all-gather payload)
    x0 = None
    if hi > lo:
        g = np.arange(lo, hi)
        tac_g = g // n_per_tac
        tacs = np.arange(t0, t1)                    # contiguous: every TAC of the range has samples here
        cond = cond_all.rows(tacs) if hasattr(cond_all, 'rows') else np.asarray(cond_all)[tacs]
        local_tac = (tac_g - t0).astype(np.int32)
        x_T = model.philox_normal(hi - lo, seed=x_T_seed, sample_offset=lo)
        x0 = model.ddpm_loop(x_T, cond, num_timesteps=num_timesteps, seed=seed, sample_offset=lo, use_graph=use_graph,
                             tac=local_tac if len(tacs) > 1 else None)
        local[:] = model.posterior_stats(x0, local_tac if len(tacs) > 1 else None, n_tac=len(tacs))
    if world > 1:
        if coll_device is None:
            coll_device = 'cpu' if dist.get_backend(group) == 'gloo' else model.device
        stats = gather_merge_own_tacs(local, n_tac, n_per_tac, group=group, device=coll_device)
    else:
        stats = np.zeros((n_tac, 48, 2, 3))
        stats[t0:t1] = local
    if return_samples:
        return summarize(stats), stats, (lo, hi, x0)
    return summarize(stats), stats


class TacTable:
    """Lazily built condition table for sample_posterior_sharded: ``len`` = number of TACs, ``rows(idx)``
    builds only the requested TACs (make(k) -> (49, 54)), so a rank never synthesises the others'."""

    def __init__(self, n_tac, make):
        self.n_tac, self.make = int(n_tac), make
        self._rows = {}                       # built rows are kept: repeated calls reuse them

    def __len__(self):
        return self.n_tac

    def rows(self, idx):
        for k in idx:
            if int(k) not in self._rows:
                self._rows[int(k)] = np.asarray(self.make(int(k)), dtype=np.float32)
        return np.stack([self._rows[int(k)] for k in idx])
