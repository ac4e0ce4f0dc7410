"""Python entry to the GRU window-policy kernels (C ABI d2d_policy_gru / d2d_gru_grad,
csrc/gru_kernels.hip): the reference's RNN module (algorithms/ippo.py:14-51 == d2d_ppo.py:24-59)
for every agent at once, windows rebuilt in-kernel from the rollout buffer."""
import ctypes

import torch

from . import _lib
from .record import set_format

KIND = {"sigmoid": 0, "softmax": 1, None: 2}


def desc(params, n_envs, kind, history_len, episode_length, seed=0, env_base=0, rng_offset=None):
    """d2d_gru_desc of agent-stacked RNN params (StackedNets kind 'rnn': w_ih, w_hh, b_ih, b_hh, w1, b1, w2, b2)."""
    p = params
    N, threeH, F = p["w_ih"].shape
    H = threeH // 3
    A = p["w2"].shape[1]
    for t in p.values():
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("GRU params must be contiguous float32")
    d = _lib.GruDesc(N, int(n_envs), F, H, A, int(kind), int(history_len), int(episode_length),
                     *(p[n].data_ptr() for n in ("w_ih", "w_hh", "b_ih", "b_hh", "w1", "b1", "w2", "b2")),
                     int(seed) & 0xFFFFFFFFFFFFFFFF, int(env_base), None if rng_offset is None else rng_offset)
    return d


def carry_floats(params, n_envs, history_len, episode_length):
    """Floats of the carried-state scratch of one policy over n_envs envs (d2d_gru_carry_floats)."""
    lib = _lib.require_gpu()
    n = lib.d2d_gru_carry_floats(ctypes.byref(desc(params, n_envs, 2, history_len, episode_length)))
    if n < 0:
        raise ValueError("d2d_gru_carry_floats: unsupported shape")
    return n


def policy(params, obs, kind, history_len, episode_length, slot0, n_slots, padded=False, forced=None, rng_step=0,
           deterministic=False, seed=0, env_base=0, rng_offset=None, actions_out=None, out=None, hcarry=None,
           carry_in=False, want_actions=True):
    """obs [T][E][N][F] (the rollout buffer: fp32, or the env kernel's ObsRecord).  kind 'sigmoid' / 'softmax' (actors): returns
    (actions [n_slots][E][N], logp [N][n_slots * E]); kind None (value): returns values [N][n_slots * E].
    hcarry (one unpadded slot per launch, slots in order: d2d_policy_gru_carry): float32 scratch of carry_floats()
    elements holding h after the previous slot's window; carry_in: the previous launch on it was slot0 - 1 and
    slot0's episode position is in [1, history_len - 1] (its window extends that one by one step).
    want_actions=False with forced: actions = NULL to the C ABI (only the log-probs are stored; returns (None, logp))."""
    lib = _lib.require_gpu()
    T, E, N, F = obs.shape
    k = KIND[kind]
    d = desc(params, E, k, history_len, episode_length, seed, env_base, rng_offset)
    optr = set_format(d, obs)
    dev = obs.device
    if out is None:
        out = torch.empty((N, n_slots * E), dtype=torch.float32, device=dev)
    act = None
    if k != 2 and (want_actions or forced is None):
        A = params["w2"].shape[1]
        mb = 1 if (k == 1 or A <= 8) else 2 if A <= 16 else 4
        dt = {1: torch.uint8, 2: torch.int16, 4: torch.int32}[mb]
        act = actions_out if actions_out is not None else torch.empty((n_slots, E, N), dtype=dt, device=dev)
    if hcarry is not None:
        if n_slots != 1 or padded:
            raise ValueError("the carried state serves one unpadded slot per launch")
        if hcarry.dtype != torch.float32 or hcarry.device != dev or hcarry.numel() < lib.d2d_gru_carry_floats(
                ctypes.byref(d)):
            raise ValueError("hcarry must be a float32 device tensor of d2d_gru_carry_floats elements")
        rc = lib.d2d_policy_gru_carry(ctypes.byref(d), T, optr, int(slot0), None if forced is None else forced.data_ptr(),
                                      int(rng_step) & 0xFFFFFFFF, 1 if deterministic else 0,
                                      None if act is None else act.data_ptr(), out.data_ptr(), hcarry.data_ptr(),
                                      1 if carry_in else 0, _lib.stream_ptr())
        _lib.check(rc, "d2d_policy_gru_carry")
        return (act, out) if k != 2 else out
    rc = lib.d2d_policy_gru(ctypes.byref(d), T, optr, int(slot0), int(n_slots), 1 if padded else 0,
                            None if forced is None else forced.data_ptr(), int(rng_step) & 0xFFFFFFFF,
                            1 if deterministic else 0, None if act is None else act.data_ptr(), out.data_ptr(),
                            _lib.stream_ptr())
    _lib.check(rc, "d2d_policy_gru")
    return (act, out) if k != 2 else out


def _strides3(t, T, E, N):
    if t.dim() == 3:
        assert tuple(t.shape) == (T, E, N)
        return t.stride(0), t.stride(1), t.stride(2)
    assert t.dim() == 2 and tuple(t.shape) == (N, E * T), tuple(t.shape)
    return t.stride(1), T * t.stride(1), t.stride(0)


def _arr(st):
    return (ctypes.c_int64 * 3)(*[int(v) for v in st])


class _Workspace:
    def __init__(self):
        self.buf = None

    def get(self, floats, device):
        if self.buf is None or self.buf.numel() < floats or self.buf.device != device:
            self.buf = torch.empty((max(int(floats), 1),), dtype=torch.float32, device=device)
        return self.buf


_ws = _Workspace()


def grads(params, obs, kind, history_len, episode_length, weight, actions=None, logp_old=None, clip=0.1, beta=0.01,
          scale=None, grads=None, stats=None):
    """Gradients of every agent's loss w.r.t. its RNN params (what autograd leaves in .grad):
    actors (kind 'sigmoid' / 'softmax'): -mean min(r W, clip(r) W) - beta mean entropy over the padded
    training windows of every sample; value (kind None): mean (V - R)^2, weight = R.
    weight / logp_old: [T][E][N] or [N][E*T] (env-major), any strides.  Returns (grads, stats [N][2])."""
    lib = _lib.require_gpu()
    T, E, N, F = obs.shape
    k = KIND[kind]
    d = desc(params, E, k, history_len, episode_length)
    optr = set_format(d, obs)
    dev = obs.device
    grads = grads if grads is not None else {n: torch.empty_like(v) for n, v in params.items()}
    if stats is None:
        stats = torch.empty((N, 2), dtype=torch.float32, device=dev)
    scale = 1.0 / (T * E) if scale is None else scale
    ws = _ws.get(lib.d2d_gru_grad_workspace(ctypes.byref(d), T), dev)
    lo_st = _arr(_strides3(logp_old, T, E, N)) if logp_old is not None else None
    rc = lib.d2d_gru_grad(ctypes.byref(d), T, optr, None if actions is None else actions.data_ptr(),
                          None if logp_old is None else logp_old.data_ptr(), lo_st, weight.data_ptr(),
                          _arr(_strides3(weight, T, E, N)), float(clip), float(beta), float(scale),
                          *(grads[n].data_ptr() for n in ("w_ih", "w_hh", "b_ih", "b_hh", "w1", "b1", "w2", "b2")),
                          stats.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_ptr())
    _lib.check(rc, "d2d_gru_grad")
    return grads, stats
