"""GAE-style advantages + discounted returns on device (C ABI d2d_gae_scan et al.).

Replaces compute_gae / discount_rewards (/root/reference/algorithms/ippo.py:92-116
== algorithms/d2d_ppo.py:100-124) for a [T][E] batch of envs, with the
normalisation statistics optionally all-reduced over a torch.distributed
process group (data-parallel shards of envs), so every rank normalises with
the global column mean/std exactly as one big rollout would.
"""
import torch
import torch.distributed as dist

from . import _lib


def _all_reduce(t, group):
    if group is not None and dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, group=group)
    return t


def normalize_columns_(x2d, ddof, group=None, n_total=None):
    """In place: x = (x - mean) / std per column iff every column's std > 0.
    x2d: contiguous float32 [rows][cols] on the GPU.  Returns the gate tensor."""
    lib = _lib.require_gpu()
    rows, cols = x2d.shape
    dev = x2d.device
    st = _lib.stream_ptr()
    ws = torch.empty(int(lib.d2d_colstats_workspace(rows, cols)), dtype=torch.float64, device=dev)
    s1 = torch.empty(cols, dtype=torch.float64, device=dev)
    m2 = torch.empty(cols, dtype=torch.float64, device=dev)
    mean = torch.empty(cols, dtype=torch.float64, device=dev)
    scale = torch.empty(cols, dtype=torch.float64, device=dev)
    gate = torch.zeros(1, dtype=torch.int32, device=dev)
    n = float(rows if n_total is None else n_total)
    _lib.check(lib.d2d_colstats(rows, cols, x2d.data_ptr(), None, ws.data_ptr(), s1.data_ptr(), st), "d2d_colstats")
    _all_reduce(s1, group)
    _lib.check(lib.d2d_colstats_finalize(cols, s1.data_ptr(), None, n, ddof, mean.data_ptr(), None, None, st),
               "d2d_colstats_finalize")
    _lib.check(lib.d2d_colstats(rows, cols, x2d.data_ptr(), mean.data_ptr(), ws.data_ptr(), m2.data_ptr(), st),
               "d2d_colstats")
    _all_reduce(m2, group)
    _lib.check(lib.d2d_colstats_finalize(cols, s1.data_ptr(), m2.data_ptr(), n, ddof, mean.data_ptr(),
                                         scale.data_ptr(), gate.data_ptr(), st), "d2d_colstats_finalize")
    _lib.check(lib.d2d_normalize_columns(rows, cols, x2d.data_ptr(), mean.data_ptr(), scale.data_ptr(),
                                         gate.data_ptr(), st), "d2d_normalize_columns")
    return gate


def gae_returns(rewards, values, dones, gamma, lam=0.97, normalize_adv=True, normalize_ret=True, group=None,
                last_shard=True, n_envs_total=None):
    """rewards [T][E] or [T][E][cols] float32, values [T][E][cols] float32, dones [T] (bool/uint8).

    Returns (adv, ret), both [T][E][cols] float32:
      adv = the reference's compute_gae output (lambda-returns, ippo.py:92-102), normalised with ddof 0;
      ret = discount_rewards (ippo.py:104-116), normalised with ddof 1.
    """
    lib = _lib.require_gpu()
    if values.dim() != 3:
        raise ValueError("values must be [T][E][cols]")
    T, E, cols = values.shape
    values = values.contiguous().float()
    rewards = rewards.contiguous().float()
    if rewards.dim() == 2:
        rcols = 1
        if tuple(rewards.shape) != (T, E):
            raise ValueError("rewards must be [T][E] or [T][E][cols]")
    else:
        rcols = rewards.shape[2]
        if tuple(rewards.shape[:2]) != (T, E) or rcols not in (1, cols):
            raise ValueError("rewards must be [T][E] or [T][E][cols]")
    d = dones.to(device=values.device, dtype=torch.uint8).contiguous()
    if d.numel() != T:
        raise ValueError("dones must have T entries")
    adv = torch.empty_like(values)
    ret = torch.empty_like(values)
    _lib.check(lib.d2d_gae_scan(T, E, cols, rcols, rewards.data_ptr(), values.data_ptr(), d.data_ptr(), float(gamma),
                                float(lam), 1 if last_shard else 0, adv.data_ptr(), ret.data_ptr(),
                                _lib.stream_ptr()), "d2d_gae_scan")
    n_total = None if n_envs_total is None else T * int(n_envs_total)
    if normalize_adv:
        normalize_columns_(adv.view(T * E, cols), 0, group, n_total)
    if normalize_ret:
        normalize_columns_(ret.view(T * E, cols), 1, group, n_total)
    return adv, ret
