"""The fused env + policy rollout slot prototype (ippo.py:293-330;
d2d_comb_policy_fused_step) measured against the two-launch slot it replaces, at the headline batch
(64 agents x 8 channels x 65,536 envs, the compact record, the actor-only policy of iPPO training rollouts,
H = 64):
  * slot time: the two-launch slot (policy kernel then env kernel, HIP events per kernel and the slot's wall
    time) and the fused launch at 32- and 64-env slices (D2D_OPT_FUSED_SLICE), 40 slots each after 8 warm-up;
  * bit-exactness of the fused slots at this size (records, env state, rewards, actions, log-probs) over the
    timed slots;
  * a whole 200-slot iPPO training rollout (graph-replayed) with D2D_FUSED_SLOT off / on.
usage (GPU box): python3 tools/gpu/fused_slot.py [E]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]
import torch  # noqa: E402


def make(E, seed=42):
    import bench
    from algorithms.ippo import iPPO
    from envs.combinatorial_env import CombinatorialEnv
    env = CombinatorialEnv(**bench.config3_params(200), n_envs=E, device="cuda:0", seed=seed)
    torch.manual_seed(0)
    return iPPO(env, hidden_size=64, gamma=0.6, policy_lr=3e-4, value_lr=1e-3, device="cuda:0", combinatorial=True)


def main():
    from d2dhip import _lib
    from d2dhip.record import set_format
    lib = _lib.require_gpu()
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    K, W = 40, 8
    res = {"workload": f"64 agents x 8 channels x {E} envs, compact record (32 B/agent-step), iPPO MLP actor H = 64",
           "slots_timed": K}

    def run(mode, se=32):
        lr = make(E)
        b = lr.env.batch()
        ring = b.record_buffer((2,))
        acts = [b.action_buffer() for _ in range(2)]
        logp = [torch.empty((b.spec.N, b.E), dtype=torch.float32, device="cuda:0") for _ in range(2)]
        rew = torch.empty(E, dtype=torch.int32, device="cuda:0")
        b.reset(want_obs=True, out_obs=ring[0])
        lr._policy_slot(ring, 0, 0, True, acts[0], logp[0], None, None, b)
        desc = lr._mlp_desc(E, b.desc.env_base, critic=False)
        desc.rng_offset = b.rng_off.data_ptr()
        set_format(desc, ring[0])
        lib.d2d_set_option(_lib.D2D_OPT_FUSED_SLICE, se)
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)]
        snaps = []

        def slot(k, e=None):
            cur, nxt = k % 2, (k + 1) % 2
            if e is not None:
                e[0].record()
            if mode == "two_launch":
                b.step(acts[cur], want_obs=True, out_obs=ring[nxt], out_reward=rew)
                if e is not None:
                    e[1].record()
                lr._policy_slot(ring, 0, nxt, True, acts[nxt], logp[nxt], None, None, b)
            else:
                b.step_policy_fused(acts[cur], ring[nxt], rew, desc, False, acts[nxt], logp[nxt])
                if e is not None:
                    e[1].record()
            if e is not None:
                e[2].record()

        for k in range(W):
            slot(k)
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for k in range(K):
            slot(W + k, ev[k])
        t1.record()
        torch.cuda.synchronize()
        # the last slot's outputs (for the bit-exactness check)
        nxt = (W + K) % 2
        snaps = [ring[nxt].data.clone(), acts[nxt].clone(), logp[nxt].clone(), rew.clone(), b.buffers.clone(),
                 b.channels.clone(), b.received.clone(), b.discarded.clone()]
        lib.d2d_set_option(_lib.D2D_OPT_FUSED_SLICE, 0)
        out = {"slot_us": t0.elapsed_time(t1) / K * 1e3}
        if mode == "two_launch":
            out["env_us"] = sum(e[0].elapsed_time(e[1]) for e in ev) / K * 1e3
            out["policy_us"] = sum(e[1].elapsed_time(e[2]) for e in ev) / K * 1e3
        else:
            out["fused_us"] = sum(e[0].elapsed_time(e[1]) for e in ev) / K * 1e3
        del lr, b, ring
        torch.cuda.empty_cache()
        return out, snaps

    base, ref = run("two_launch")
    res["two_launch"] = base
    for se in (32, 64):
        r, snap = run("fused", se)
        r["bit_exact"] = all(torch.equal(x, y) for x, y in zip(ref, snap))
        r["vs_two_launch"] = base["slot_us"] / r["slot_us"]
        res[f"fused_slice{se}"] = r
        print(f"[fused_slot] slice {se}: {r}", file=sys.stderr, flush=True)
    print(f"[fused_slot] two-launch: {base}", file=sys.stderr, flush=True)

    # whole training rollouts, graph-replayed (the second of each is timed)
    roll = {}
    for fused in (False, True):
        lr = make(E, seed=3)
        lr.fused_slot = fused
        lr._rollout(E, defer_values=True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        ro = lr._rollout(E, defer_values=True)
        torch.cuda.synchronize()
        roll["fused" if fused else "two_launch"] = {"rollout_s": time.perf_counter() - t}
        roll["fused" if fused else "two_launch"]["_digest"] = [int(ro.actions.sum()), float(ro.logp.double().sum())]
        del lr, ro
        torch.cuda.empty_cache()
        print(f"[fused_slot] rollout fused={fused}: {roll}", file=sys.stderr, flush=True)
    roll["same_rollout"] = roll["fused"]["_digest"] == roll["two_launch"]["_digest"]
    res["rollout_200_slots"] = roll
    res["fused_best_slot_us"] = min(res["fused_slice32"]["slot_us"], res["fused_slice64"]["slot_us"])
    res["verdict"] = ("fused faster" if res["fused_best_slot_us"] < base["slot_us"] else "two-launch faster")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
