"""TEST INFRASTRUCTURE ONLY — numpy restatement of the reference's
compute_gae / discount_rewards (/root/reference/algorithms/ippo.py:92-116,
identical in algorithms/d2d_ppo.py:100-124), extended to a [T][E][cols]
batch whose sequence order is env-major (env 0's T steps, then env 1's, ...),
i.e. exactly what the reference computes on np.concatenate over envs.
Pinned to the reference by tests/test_gae_oracle.py (golden vectors).
"""
import numpy as np


def compute_gae_seq(rewards, dones, values, gamma, lbda):
    """Reference semantics on a (L, cols) sequence, float64, vectorised over columns (ippo.py:92-102)."""
    r = np.asarray(rewards, dtype=np.float64)
    v = np.asarray(values, dtype=np.float64)
    d = np.asarray(dones, dtype=np.float64)
    L = r.shape[0]
    adv = np.zeros_like(v)
    adv[L - 1] = r[L - 1] - v[L - 1]
    gae = np.zeros_like(v[0])
    for step in range(L - 2, -1, -1):
        delta = r[step] + gamma * v[step + 1] * (1 - d[step]) - v[step]
        gae = delta + gamma * lbda * (1 - d[step]) * gae
        adv[step] = gae + v[step]
    if (adv.std(0) > 0).all():
        adv = (adv - adv.mean(0)) / adv.std(0)
    return adv.astype(np.float32)


def discount_rewards_seq(rewards, gamma, dones, normalize=True, exact_stats=False):
    """Reference semantics (ippo.py:104-116): float64 recursion, float32 cast, ddof=1 normalisation.
    exact_stats: take mean/std in float64 instead of the reference's float32 (at 1e5+ rows the
    reference's own float32 reduction noise exceeds 1e-5; the batched checks compare exact values)."""
    r = np.asarray(rewards, dtype=np.float64)
    d = np.asarray(dones, dtype=np.float64)
    out = np.zeros_like(r)
    R = np.zeros_like(r[0])
    for i in range(r.shape[0] - 1, -1, -1):
        R = r[i] + R * gamma * (1 - d[i])
        out[i] = R
    out = out.astype(np.float32)
    if normalize:
        x = out.astype(np.float64) if exact_stats else out
        sd = x.std(0, ddof=1)
        if (sd > 0).all():
            out = ((x - x.mean(0)) / sd).astype(np.float32)
    return out


def gae_returns_batched(rewards, values, dones, gamma, lbda):
    """rewards [T][E] (broadcast) or [T][E][cols]; values [T][E][cols]; dones [T].
    Returns (adv, ret) [T][E][cols] float32 for the env-major concatenated sequence."""
    v = np.asarray(values, dtype=np.float64)
    T, E, cols = v.shape
    r = np.asarray(rewards, dtype=np.float64)
    if r.ndim == 2:
        r = np.repeat(r[:, :, None], cols, axis=2)
    seq = lambda x: np.transpose(x, (1, 0, 2)).reshape(E * T, cols)  # noqa: E731
    d = np.tile(np.asarray(dones, dtype=np.float64), E)
    adv = compute_gae_seq(seq(r), d, seq(v), gamma, lbda)
    ret = discount_rewards_seq(seq(r), gamma, d, True, exact_stats=True)
    back = lambda x: np.transpose(x.reshape(E, T, cols), (1, 0, 2))  # noqa: E731
    return back(adv), back(ret)


def colstats_finalize(s1, m2, n, ddof):
    """Restatement of d2d_colstats_finalize (csrc/gae_kernels.hip): mean = Σx / n; with the centred
    sums m2: scale = 1 / std (std with ddof, as np.std / torch.std in ippo.py:100, 114), gate = every
    column's std > 0 (the reference normalises only then, quirk Q2).  torch float64 in and out."""
    import torch
    mean = s1 / n
    if m2 is None:
        return mean, None, None
    sd = torch.sqrt(m2 / (n - ddof))
    gate = torch.tensor([int(bool((sd > 0).all()))], dtype=torch.int32)
    return mean, 1.0 / sd, gate
