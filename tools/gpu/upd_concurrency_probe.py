"""Timing probe: the MLP actor and critic update kernels back to back on one stream vs concurrently on two streams
(the critic on a side stream), at a 2,048-env and a 16,384-env rollout of the headline 64 x 8 configuration.
usage: python tools/gpu/upd_concurrency_probe.py [--reps 10]"""
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
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from algorithms.ippo import iPPO
    from d2dhip.update import actor_grads, critic_grads
    from envs.combinatorial_env import CombinatorialEnv
    out = {}
    for E in (2048, 16384):
        env = CombinatorialEnv(**config3_params(200), n_envs=E, device="cuda", seed=7)
        torch.manual_seed(1)
        lr = iPPO(env, hidden_size=64, gamma=0.6, device="cuda", combinatorial=True)
        ro = lr._rollout(E)
        pp = {k: v.data for k, v in lr.policy.params.items()}
        vp = {k: v.data for k, v in lr.value.params.items()}
        ga = {k: torch.empty_like(v) for k, v in pp.items()}
        gv = {k: torch.empty_like(v) for k, v in vp.items()}
        lo, adv, ret = ro.logp.permute(0, 2, 1), ro.adv_tne.permute(0, 2, 1), ro.ret_tne.permute(0, 2, 1)
        s2 = torch.cuda.Stream()
        actor = lambda: actor_grads(pp, ro.obs, ro.actions, lo, adv, "comb", grads=ga)  # noqa: E731
        critic = lambda: critic_grads(vp, ro.obs, ret, grads=gv)  # noqa: E731

        def seq():
            actor()
            critic()

        def conc():
            cur = torch.cuda.current_stream()
            s2.wait_stream(cur)
            with torch.cuda.stream(s2):
                critic()
            actor()
            cur.wait_stream(s2)

        out[E] = {"actor_ms": timed(actor, a.reps), "critic_ms": timed(critic, a.reps),
                  "sequential_ms": timed(seq, a.reps), "concurrent_ms": timed(conc, a.reps)}
        del lr, env, ro
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
