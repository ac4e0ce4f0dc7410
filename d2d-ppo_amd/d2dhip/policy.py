"""Python entry to the fused behaviour-policy kernel (C ABI d2d_policy_mlp_step)."""
import torch

from . import _lib
from .record import set_format


def policy_mlp_step(actor, obs, kind, critic=None, forced=None, rng_step=0, deterministic=False, seed=0,
                    env_base=0, actions=None, logp=None, value=None, want_value=True, want_actions=True):
    """actor/critic: dicts of agent-stacked fp32 tensors w1 [N][H][F], b1 [N][H], w2 [N][A][H], b2 [N][A]
    (critic: A = 1).  obs [E][N][F] fp32, or the env kernel's ObsRecord of that shape.  kind 'comb' (Bernoulli, masks out) or 'chsel' (Categorical, ids out).
    want_value=False with critic weights passes value = NULL to the C ABI (valid usage: the value is skipped);
    want_actions=False with forced passes actions = NULL (only the log-probs are stored; actions returned as None).
    Returns (actions [E][N], logp [N][E], value [N][E] or None)."""
    lib = _lib.require_gpu()
    N, H, F = actor["w1"].shape
    A = actor["w2"].shape[1]
    E = obs.shape[0]
    dev = obs.device
    assert tuple(obs.shape) == (E, N, F) and obs.is_contiguous()
    for t in list(actor.values()) + (list(critic.values()) if critic else []):
        assert t.dtype == torch.float32 and t.is_contiguous() and t.device == dev
    k = 0 if kind == "comb" else 1
    store_actions = want_actions or forced is None
    if actions is None and store_actions:
        if k == 0:
            dt = torch.uint8 if A <= 8 else torch.int16
            actions = torch.zeros((E, N), dtype=dt, device=dev)
        else:
            actions = torch.zeros((E, N), dtype=torch.uint8, device=dev)
    if logp is None:
        logp = torch.empty((N, E), dtype=torch.float32, device=dev)
    if critic is not None and value is None and want_value:
        value = torch.empty((N, E), dtype=torch.float32, device=dev)
    p = lambda t: t.data_ptr()  # noqa: E731
    desc = _lib.MlpDesc(N, E, F, H, A, k, p(actor["w1"]), p(actor["b1"]), p(actor["w2"]), p(actor["b2"]),
                        p(critic["w1"]) if critic else None, p(critic["b1"]) if critic else None,
                        p(critic["w2"]) if critic else None, p(critic["b2"]) if critic else None, int(seed),
                        int(env_base))
    optr = set_format(desc, obs)
    rc = lib.d2d_policy_mlp_step(desc, optr, None if forced is None else forced.contiguous().data_ptr(),
                                 int(rng_step), 1 if deterministic else 0,
                                 actions.data_ptr() if store_actions else None, logp.data_ptr(),
                                 None if value is None else value.data_ptr(), _lib.stream_ptr())
    _lib.check(rc, "d2d_policy_mlp_step")
    return (actions if store_actions else None), logp, (value if critic is not None and want_value else None)
