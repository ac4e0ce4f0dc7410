"""Timing probe: the actor-only rollout policy kernel at the headline slot (64 agents x 8 channels x 65,536 envs,
compact record) in its three modes -- sampled (training rollouts), deterministic (test()) and forced (D2D-PPO's
epoch-start log-prob pass, the `chain` phase) -- for A/B of policy_kernels.hip builds (D2D_LIB_VARIANT).  With --save
the log-probs of each mode go to a .pt file, so two builds' outputs can be compared offline.
usage: python tools/gpu/policy_mode_probe.py [--envs 65536] [--reps 30] [--save PATH]"""
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
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--save", default=None)
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
    act = b.action_buffer()
    for _ in range(5):  # a few steps so the buffers and ACKs are not all zero
        b.sample_actions(0.3, out=act)
        b.step(act, want_obs=True, out_obs=ring[0])
    x = ring[0]
    pp = {k: v.data for k, v in lr.policy.params.items()}
    act_s, lp_s, _ = policy_mlp_step(pp, x, "comb", None, rng_step=3)
    forced = act_s.clone()
    out = {"envs": a.envs, "lib_variant": os.environ.get("D2D_LIB_VARIANT", "")}
    for _ in range(2):
        out.setdefault("sample_us", []).append(1e3 * timed(lambda: policy_mlp_step(pp, x, "comb", None, rng_step=3), a.reps))
        out.setdefault("forced_us", []).append(
            1e3 * timed(lambda: policy_mlp_step(pp, x, "comb", None, forced=forced), a.reps))
        out.setdefault("forced_noact_us", []).append(
            1e3 * timed(lambda: policy_mlp_step(pp, x, "comb", None, forced=forced, want_actions=False), a.reps))
        out.setdefault("deterministic_us", []).append(
            1e3 * timed(lambda: policy_mlp_step(pp, x, "comb", None, deterministic=True), a.reps))
    _, lp_f, _ = policy_mlp_step(pp, x, "comb", None, forced=forced)
    _, lp_f2, _ = policy_mlp_step(pp, x, "comb", None, forced=forced, want_actions=False)
    out["forced_noact_equals"] = bool(torch.equal(lp_f2, lp_s))
    act_d, lp_d, _ = policy_mlp_step(pp, x, "comb", None, deterministic=True)
    out["forced_equals_sampled"] = bool(torch.equal(lp_f, lp_s))
    if a.save:
        torch.save({"act_s": act_s.cpu(), "lp_s": lp_s.cpu(), "lp_f": lp_f.cpu(), "act_d": act_d.cpu(),
                    "lp_d": lp_d.cpu()}, a.save)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
