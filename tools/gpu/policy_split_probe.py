"""Timing probe: the rollout policy kernel at the headline slot (64 agents x 8 channels x 65,536 envs, compact
record) with the iPPO critic fused (the default) vs the actor alone -- the critic's weight fragments are what hold
the fused kernel at two waves per SIMD (224 VGPRs; 137 without them).
usage: python tools/gpu/policy_split_probe.py [--envs 65536] [--reps 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]

import torch  # noqa: E402

from bench import config3_params  # noqa: E402


def timed(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from algorithms.ippo import iPPO
    from d2dhip.policy import policy_mlp_step
    from envs.combinatorial_env import CombinatorialEnv
    env = CombinatorialEnv(**config3_params(200), n_envs=a.envs, device="cuda", seed=7)
    torch.manual_seed(1)
    lr = iPPO(env, hidden_size=64, gamma=0.6, device="cuda", combinatorial=True)
    b = env.batch()
    ring = b.record_buffer((1,))
    b.reset(want_obs=True, out_obs=ring[0])
    x = ring[0]
    pp = {k: v.data for k, v in lr.policy.params.items()}
    vp = {k: v.data for k, v in lr.value.params.items()}
    from d2dhip import _lib
    lib = _lib.require_gpu()
    out = {"envs": a.envs}
    res = {}
    for split in (0, 1, 0, 1):
        _lib.check(lib.d2d_set_option(_lib.D2D_OPT_POLICY_CRITIC_SPLIT, split), "set_option")
        key = "actor_critic_split_us" if split else "actor_critic_fused_us"
        out.setdefault(key, []).append(1e3 * timed(lambda: policy_mlp_step(pp, x, "comb", vp, rng_step=3), a.reps))
        res[split] = [t.clone() for t in policy_mlp_step(pp, x, "comb", vp, rng_step=3)]
    out["actor_only_us"] = 1e3 * timed(lambda: policy_mlp_step(pp, x, "comb", None, rng_step=3), a.reps)
    out["split_bitwise_equal"] = all(torch.equal(u, v) for u, v in zip(res[0], res[1]))
    _lib.check(lib.d2d_set_option(_lib.D2D_OPT_POLICY_CRITIC_SPLIT, 0), "set_option")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
