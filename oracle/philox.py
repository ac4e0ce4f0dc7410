"""TEST INFRASTRUCTURE ONLY — never imported by the product path.

Philox4x32-10 counter-based generator (Salmon, Moraes, Dror, Shaw, SC'11,
"Parallel random numbers: as easy as 1, 2, 3"), restated in numpy so the
oracle can check the HIP kernels' production-mode draws bit for bit.

The reference draws from NumPy's legacy global MT19937 stream
(envs/combinatorial_env.py:68,117,180; envs/channel_selection_env.py:105,161);
that stream is not replicated — parity against the reference is pinned by
replaying recorded draws.  Philox is this framework's documented production
RNG; its counter layout is:

    key     = (seed & 0xffffffff, seed >> 32)
    counter = (env_global_index, agent | 0xffffffff for per-env draws,
               rng_step, stream << 24 | block)
    streams : 0 = channel flips, 1 = arrivals, 2 = synthetic actions
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)

STREAM_FLIP, STREAM_ARRIVAL, STREAM_ACTION = 0, 1, 2
PER_ENV = 0xFFFFFFFF


def philox4x32_10(c0, c1, c2, c3, seed):
    """Vectorised Philox4x32-10.  c* are broadcastable uint32-valued arrays."""
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint64) & MASK32 for x in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = int(seed) & 0xFFFFFFFF
    k1 = (int(seed) >> 32) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + W0) & 0xFFFFFFFF
            k1 = (k1 + W1) & 0xFFFFFFFF
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0)
    return c0, c1, c2, c3


def words(env_idx, agent, rng_step, stream, n_words, seed):
    """n_words uint32 draws for each (env, agent): shape broadcast(env, agent) + (n_words,)."""
    nblk = (n_words + 3) // 4
    out = []
    for b in range(nblk):
        r = philox4x32_10(env_idx, agent, rng_step, (stream << 24) | b, seed)
        out.extend(r)
    return np.stack(out[:n_words], axis=-1).astype(np.uint64)


def threshold(p):
    """Bernoulli(p) from one uint32 word r: success iff r < floor(p * 2**32)."""
    p = np.clip(np.asarray(p, dtype=np.float64), 0.0, 1.0)
    return np.floor(p * 4294967296.0).astype(np.uint64)


def poisson_inversion(u32, lam, p0):
    """Poisson(lam) by sequential CDF inversion of u = r * 2**-32, capped at 255.
    Same IEEE double operation order as the C oracle and the HIP kernel."""
    u = np.asarray(u32, dtype=np.float64) * (1.0 / 4294967296.0)
    lam = np.broadcast_to(np.asarray(lam, dtype=np.float64), u.shape)
    p = np.broadcast_to(np.asarray(p0, dtype=np.float64), u.shape).copy()
    F = p.copy()
    x = np.zeros(u.shape, dtype=np.int64)
    live = (u >= F) & (x < 255)
    while live.any():
        x = np.where(live, x + 1, x)
        p = np.where(live, (p * lam) / np.maximum(x, 1), p)
        F = np.where(live, F + p, F)
        live = live & (u >= F) & (x < 255)
    return x
