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


def two_pass_column_stats(colsum, finalize, group=None):
    """The cross-rank protocol behind normalize_columns_ (data-parallel shards of envs normalise with
    the GLOBAL column mean / std):
        s1 = Σ x per column (local)            -> all-reduce -> mean = finalize(s1, None)
        m2 = Σ (x - mean)^2 per column (local) -> all-reduce -> (mean, scale, gate) = finalize(s1, m2)
    colsum(center) returns a fresh float64 [cols] tensor of local sums (center None: plain sums);
    finalize(s1, m2) returns (mean, scale, gate).  Two deterministic passes instead of a one-pass
    Σx / Σx² keep the variance of large-mean columns exact to float64."""
    s1 = colsum(None)
    _all_reduce(s1, group)
    mean = finalize(s1, None)[0]
    m2 = colsum(mean)
    _all_reduce(m2, group)
    return finalize(s1, m2)


def normalize_columns_(x2d, ddof, group=None, n_total=None, tce=None):
    """In place: x = (x - mean) / std per column iff every column's std > 0.
    x2d: contiguous float32 [rows][cols] on the GPU, or (tce = (T, cols, E)) a contiguous
    [T][cols][E] tensor whose column c is the T*E elements (t, c, e).  Returns the gate tensor."""
    lib = _lib.require_gpu()
    if tce is None:
        rows, cols = x2d.shape
    else:
        T, cols, E = tce
        rows = T * E
    dev = x2d.device
    st = _lib.stream_ptr()
    ws = torch.empty(int(lib.d2d_colstats_workspace(rows, cols)), dtype=torch.float64, device=dev)
    mean = torch.empty(cols, dtype=torch.float64, device=dev)
    scale = torch.empty(cols, dtype=torch.float64, device=dev)
    gate = torch.zeros(1, dtype=torch.int32, device=dev)
    n = float(rows if n_total is None else n_total)

    def colsum(center):
        out = torch.empty(cols, dtype=torch.float64, device=dev)
        c = None if center is None else center.data_ptr()
        if tce is None:
            _lib.check(lib.d2d_colstats(rows, cols, x2d.data_ptr(), c, ws.data_ptr(), out.data_ptr(), st),
                       "d2d_colstats")
        else:
            _lib.check(lib.d2d_colstats_tce(T, cols, E, x2d.data_ptr(), c, ws.data_ptr(), out.data_ptr(), st),
                       "d2d_colstats_tce")
        return out

    def finalize(s1, m2):
        _lib.check(lib.d2d_colstats_finalize(cols, s1.data_ptr(), None if m2 is None else m2.data_ptr(), n, ddof,
                                             mean.data_ptr(), None if m2 is None else scale.data_ptr(),
                                             None if m2 is None else gate.data_ptr(), st), "d2d_colstats_finalize")
        return mean, scale, gate

    two_pass_column_stats(colsum, finalize, group)
    if tce is None:
        _lib.check(lib.d2d_normalize_columns(rows, cols, x2d.data_ptr(), mean.data_ptr(), scale.data_ptr(),
                                             gate.data_ptr(), st), "d2d_normalize_columns")
    else:
        _lib.check(lib.d2d_normalize_columns_tce(T, cols, E, x2d.data_ptr(), mean.data_ptr(), scale.data_ptr(),
                                                 gate.data_ptr(), st), "d2d_normalize_columns_tce")
    return gate


def moments_colsum(moments, multi_rank):
    """two_pass_column_stats' colsum(center) from one rank's moments [3][cols] = (n, sum, M2 about the
    local mean): Σx, and Σ(x - center)² = M2 + n (mean_local - center)²."""
    n_loc, s_loc, m2_loc = moments[0], moments[1], moments[2]

    def colsum(center):
        if center is None:
            return s_loc.clone()
        if not multi_rank:
            return m2_loc.clone()  # one rank: the local mean IS the mean (the correction is 0 up to rounding)
        mean_loc = torch.where(n_loc > 0, s_loc / n_loc.clamp(min=1), center)
        return m2_loc + n_loc * (mean_loc - center) ** 2
    return colsum


def moments_stats(moments, ddof, n, group=None):
    """(mean, scale, gate) of one output from the scan's fused moments [3][cols] (n, sum, M2) of this
    rank's elements, through the two_pass_column_stats protocol: Σx all-reduced, then
    Σ(x - mean)² = M2 + n (mean_local - mean)² all-reduced -- the same sums a second pass over the data
    would produce, from [cols] vectors."""
    lib = _lib.require_gpu()
    cols = moments.shape[1]
    dev = moments.device
    st = _lib.stream_ptr()
    mean = torch.empty(cols, dtype=torch.float64, device=dev)
    scale = torch.empty(cols, dtype=torch.float64, device=dev)
    gate = torch.zeros(1, dtype=torch.int32, device=dev)
    colsum = moments_colsum(moments, group is not None)

    def finalize(s1, m2):
        _lib.check(lib.d2d_colstats_finalize(cols, s1.data_ptr(), None if m2 is None else m2.data_ptr(), float(n),
                                             ddof, mean.data_ptr(), None if m2 is None else scale.data_ptr(),
                                             None if m2 is None else gate.data_ptr(), st), "d2d_colstats_finalize")
        return mean, scale, gate

    two_pass_column_stats(colsum, finalize, group)
    return mean, scale, gate


def gae_returns(rewards, values, dones, gamma, lam=0.97, normalize_adv=True, normalize_ret=True, group=None,
                last_shard=True, n_envs_total=None, layout="tec"):
    """rewards [T][E] or [T][E][cols] float32, values [T][E][cols] float32, dones [T] (bool/uint8).
    layout "tce": values / per-column rewards / outputs are [T][cols][E] instead (the policy
    kernel's value layout; the update kernels read it coalesced).

    Returns (adv, ret), in the values' layout, float32:
      adv = the reference's compute_gae output (lambda-returns, ippo.py:92-102), normalised with ddof 0;
      ret = discount_rewards (ippo.py:104-116), normalised with ddof 1.
    Normalised outputs take two scans (ABI 9): the first only accumulates both outputs' column moments
    (d2d_gae_scan_moments with no outputs: 4 B read per element), the statistics are finalised (and
    all-reduced across ranks), and the second recomputes the recursion and writes the normalised
    values (d2d_gae_scan_normalized: 4 B read + 8 B written) -- bitwise the scan + separate
    normalisation pass (d2d_normalize_pair), at 16 instead of 28 B of HBM traffic per element.
    """
    lib = _lib.require_gpu()
    if values.dim() != 3:
        raise ValueError("values must be 3-D")
    tce = layout == "tce"
    if tce:
        T, cols, E = values.shape
    else:
        T, E, cols = values.shape
    values = values.contiguous().float()
    rewards = rewards.contiguous().float()
    if rewards.dim() == 2:
        rcols = 1
        if tuple(rewards.shape) != (T, E):
            raise ValueError("rewards must be [T][E] or shaped like values")
    else:
        rcols = rewards.shape[1] if tce else rewards.shape[2]
        lead = (rewards.shape[0], rewards.shape[2]) if tce else tuple(rewards.shape[:2])
        if tuple(lead) != (T, E) or rcols not in (1, cols):
            raise ValueError("rewards must be [T][E] or shaped like values")
    d = dones.to(device=values.device, dtype=torch.uint8).contiguous()
    if d.numel() != T:
        raise ValueError("dones must have T entries")
    dev = values.device
    adv = torch.empty_like(values)
    ret = torch.empty_like(values)
    lay = 1 if tce else 0
    scan = (T, E, cols, rcols, rewards.data_ptr(), values.data_ptr(), d.data_ptr(), float(gamma), float(lam),
            1 if last_shard else 0, lay)
    if not (normalize_adv or normalize_ret):
        _lib.check(lib.d2d_gae_scan(*scan[:10], adv.data_ptr(), ret.data_ptr(), _lib.stream_ptr()) if not tce else
                   lib.d2d_gae_scan_tce(*scan[:10], adv.data_ptr(), ret.data_ptr(), _lib.stream_ptr()), "d2d_gae_scan")
        return adv, ret
    moments = torch.empty((2, 3, cols), dtype=torch.float64, device=dev)
    ws = torch.empty(int(lib.d2d_gae_moments_workspace(E, cols, lay)), dtype=torch.float64, device=dev)
    _lib.check(lib.d2d_gae_scan_moments(*scan, None, None, moments.data_ptr(), ws.data_ptr(), ws.numel(),
                                        _lib.stream_ptr()), "d2d_gae_scan_moments")
    n = T * E if n_envs_total is None else T * int(n_envs_total)
    args, keep = [], []
    for do, k, ddof in ((normalize_adv, 0, 0), (normalize_ret, 1, 1)):
        if do:
            mean, scale, gate = moments_stats(moments[k], ddof, n, group)
            args.append((mean.data_ptr(), scale.data_ptr(), gate.data_ptr()))
            keep.append((mean, scale, gate))  # alive until the launch is queued
        else:
            args.append((None, None, None))
    _lib.check(lib.d2d_gae_scan_normalized(*scan, adv.data_ptr(), *args[0], ret.data_ptr(), *args[1],
                                           _lib.stream_ptr()), "d2d_gae_scan_normalized")
    return adv, ret
