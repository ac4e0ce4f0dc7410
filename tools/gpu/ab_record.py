"""A/B timing of the MLP gradient kernels and the policy kernel on the compact obs record vs the
fp32 obs rows of the same rollout (the record decoded once on the device).
usage: python tools/gpu/ab_record.py [--envs 2048] [--reps 10]"""
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
    ap.add_argument("--envs", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from algorithms.ippo import iPPO
    from d2dhip.policy import policy_mlp_step
    from d2dhip.update import actor_grads, critic_grads
    from envs.combinatorial_env import CombinatorialEnv
    env = CombinatorialEnv(**config3_params(200), n_envs=a.envs, device="cuda", seed=7)
    torch.manual_seed(1)
    lr = iPPO(env, hidden_size=64, gamma=0.6, device="cuda", combinatorial=True)
    ro = lr._rollout(a.envs)
    rec = ro.obs
    f32 = ro.obs_f32.contiguous()
    pp = {k: v.data for k, v in lr.policy.params.items()}
    vp = {k: v.data for k, v in lr.value.params.items()}
    ga = {k: torch.empty_like(v) for k, v in pp.items()}
    gv = {k: torch.empty_like(v) for k, v in vp.items()}
    lo, adv, ret = ro.logp.permute(0, 2, 1), ro.adv_tne.permute(0, 2, 1), ro.ret_tne.permute(0, 2, 1)
    out = {}
    for name, obs in (("record", rec), ("fp32", f32)):
        out[name] = {
            "actor_ms": timed(lambda: actor_grads(pp, obs, ro.actions, lo, adv, "comb", grads=ga), a.reps),
            "critic_ms": timed(lambda: critic_grads(vp, obs, ret, grads=gv), a.reps),
            "policy_slot_us": 1e3 * timed(lambda: policy_mlp_step(pp, obs[5], "comb", vp, rng_step=3), a.reps * 10),
        }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
