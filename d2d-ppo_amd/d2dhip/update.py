"""Python entry to the fused PPO-update kernels (C ABI d2d_ppo_actor_grad / d2d_ppo_critic_grad).

The kernels return the gradients torch autograd would leave in `.grad` for every agent's
loss (ippo.py:194-217, d2d_ppo.py:198-216); the optimizer step stays in torch.
"""
import ctypes

import torch

from . import _lib
from .record import set_format


def _strides3(t, T, E, N):
    """Element strides (t, e, k) of a per-sample tensor given as [T][E][N] (any strides) or
    [N][T*E] env-major (sample index e*T + t, the learners' _seq layout)."""
    if t.dim() == 3:
        assert tuple(t.shape) == (T, E, N)
        return t.stride(0), t.stride(1), t.stride(2)
    assert t.dim() == 2 and tuple(t.shape) == (N, E * T), tuple(t.shape)
    return t.stride(1), T * t.stride(1), t.stride(0)


def _arr(strides):
    return (ctypes.c_int64 * 3)(*[int(s) for s in strides])


class UpdateWorkspace:
    """Device scratch of the partial-gradient sums, grown on demand and reused."""

    def __init__(self):
        self.buf = None

    def get(self, floats, device):
        if self.buf is None or self.buf.numel() < floats or self.buf.device != device:
            self.buf = torch.empty((max(int(floats), 1),), dtype=torch.float32, device=device)
        return self.buf


_ws = UpdateWorkspace()


def _desc(net, E, kind, critic=False):
    p = net
    N, H, F = p["w1"].shape
    A = 1 if critic else p["w2"].shape[1]
    return _lib.MlpDesc(N, E, F, H, A, kind, p["w1"].data_ptr(), p["b1"].data_ptr(), p["w2"].data_ptr(),
                        p["b2"].data_ptr(), None, None, None, None, 0, 0)


def _grads_like(net, grads):
    if grads is None:
        return {k: torch.empty_like(v) for k, v in net.items()}
    return grads


def actor_grads(net, obs, actions, logp_old, weight, kind, clip=0.1, beta=0.01, scale=None, grads=None,
                stats=None, workspace=None):
    """net: dict w1 [N][H][F], b1 [N][H], w2 [N][A][H], b2 [N][A] (fp32, contiguous).
    obs [T][E][N][F] fp32 or an ObsRecord of that shape; actions [T][E][N] masks (kind 'comb') or uint8 ids ('chsel');
    logp_old / weight: [T][E][N] or [N][E*T] (env-major), any strides.
    Returns (grads dict like net, stats [N][2] = (sum min-surrogate, sum entropy))."""
    lib = _lib.require_gpu()
    T, E, N, F = obs.shape
    dev = obs.device
    assert obs.is_contiguous()
    assert actions.shape == (T, E, N) and actions.is_contiguous()
    for t in net.values():
        assert t.dtype == torch.float32 and t.is_contiguous() and t.device == dev
    assert net["w1"].shape[:1] == (N,) and net["w1"].shape[2] == F
    assert logp_old.dtype == torch.float32 and weight.dtype == torch.float32
    k = 0 if kind == "comb" else 1
    B = T * E
    scale = 1.0 / B if scale is None else scale
    grads = _grads_like(net, grads)
    if stats is None:
        stats = torch.empty((N, 2), dtype=torch.float32, device=dev)
    H, A = net["w1"].shape[1], net["w2"].shape[1]
    need = lib.d2d_ppo_workspace(N, T, E, F, H, A)
    ws = (workspace or _ws).get(need, dev)
    desc = _desc(net, E, k)
    optr = set_format(desc, obs)
    rc = lib.d2d_ppo_actor_grad(desc, T, optr, actions.data_ptr(), logp_old.data_ptr(),
                                _arr(_strides3(logp_old, T, E, N)), weight.data_ptr(),
                                _arr(_strides3(weight, T, E, N)), float(clip), float(beta), float(scale),
                                grads["w1"].data_ptr(), grads["b1"].data_ptr(), grads["w2"].data_ptr(),
                                grads["b2"].data_ptr(), stats.data_ptr(), ws.data_ptr(), ws.numel(),
                                _lib.stream_ptr())
    _lib.check(rc, "d2d_ppo_actor_grad")
    return grads, stats


def critic_grads(net, obs, returns, scale=None, grads=None, stats=None, workspace=None, values=None):
    """net: dict w1 [N][H][F], b1 [N][H], w2 [N][1][H], b2 [N][1].  returns [T][E][N] or [N][E*T].
    values: None, or an fp32 tensor viewed as [T][E][N] (or [N][E*T]) that receives V(obs) of every sample
    (d2d_ppo_critic_grad_values: iPPO's rollout values from the first epoch's critic pass).
    Returns (grads, stats [N][2] = (sum (V - R)^2, 0))."""
    lib = _lib.require_gpu()
    T, E, N, F = obs.shape
    dev = obs.device
    assert obs.is_contiguous()
    for t in net.values():
        assert t.dtype == torch.float32 and t.is_contiguous() and t.device == dev
    B = T * E
    scale = 1.0 / B if scale is None else scale
    grads = _grads_like(net, grads)
    if stats is None:
        stats = torch.empty((N, 2), dtype=torch.float32, device=dev)
    H = net["w1"].shape[1]
    need = lib.d2d_ppo_workspace(N, T, E, F, H, 1)
    ws = (workspace or _ws).get(need, dev)
    desc = _desc(net, E, 0, critic=True)
    optr = set_format(desc, obs)
    if values is not None:
        assert values.dtype == torch.float32 and values.device == dev
    rc = lib.d2d_ppo_critic_grad_values(desc, T, optr, returns.data_ptr(), _arr(_strides3(returns, T, E, N)),
                                        float(scale), grads["w1"].data_ptr(), grads["b1"].data_ptr(),
                                        grads["w2"].data_ptr(), grads["b2"].data_ptr(), stats.data_ptr(),
                                        ws.data_ptr(), ws.numel(),
                                        None if values is None else values.data_ptr(),
                                        None if values is None else _arr(_strides3(values, T, E, N)), _lib.stream_ptr())
    _lib.check(rc, "d2d_ppo_critic_grad_values")
    return grads, stats
