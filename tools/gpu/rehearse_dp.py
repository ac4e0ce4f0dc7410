"""Multi-rank rehearsal of the data-parallel PRODUCT path on one GPU.

    [D2D_REHEARSE_N=64] python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29541 tools/gpu/rehearse_dp.py

Both ranks share cuda:0 over gloo (a 1-GPU box cannot run RCCL between two ranks).  Each rank
owns an env shard (env_base = rank * E), rolls out, computes GAE with the cross-rank
normalisation statistics and runs one update epoch with the all-reduced gradients, for iPPO
and for D2D-PPO (fused HIP kernels).  Rank 0 then tears the group down and repeats the same on
ONE process with the concatenated batch (2E envs, same seeds): the sharded run must reproduce
  * the rollout (obs, actions, log-probs) bit for bit (Philox counters are global env indices),
  * the normalised advantages / returns (1e-5: float64 statistics, different summation order),
  * the all-reduced, clipped gradients (2e-5 of max|g|) and the post-Adam weights (2 % of lr).
One JSON line with the measured differences is printed; exit status 1 on any violation.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "d2d-ppo_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# batch shape: 8 agents by default; D2D_REHEARSE_N=64 rehearses the benched 64 x 8 agent count
E, N, C, L = (int(os.environ.get(f"D2D_REHEARSE_{k}", v)) for k, v in (("E", 96), ("N", 8), ("C", 8), ("L", 20)))
ALGOS = ("ippo", "d2d", "ippo_gru", "d2d_gru")
# the ranks' tensors (hundreds of MB at 64 agents) go to a scratch directory outside gpurun_out/
OUT = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"d2d_rehearse_dp_{os.environ.get('MASTER_PORT', '0')}")


def make_env(n_envs):
    from envs.combinatorial_env import CombinatorialEnv
    return CombinatorialEnv(N, C, np.array([7, 14] * (N // 2)), np.full(N, 0.4), episode_length=L,
                            channel_switch=np.full((N, C), 0.3), homogeneous_size=True, n_envs=n_envs,
                            device="cuda:0", seed=7)


def run(algo, n_envs):
    from algorithms.d2d_ppo import D2DPPO
    from algorithms.ippo import iPPO
    torch.manual_seed(0)
    np.random.seed(0)
    env = make_env(n_envs)
    kw = dict(hidden_size=64, gamma=0.6, policy_lr=3e-3, value_lr=1e-3, device="cuda:0", combinatorial=True,
              early_stopping=False)
    if algo.endswith("_gru"):  # the GRU window kernels (xp_load.py's learner shape, short window)
        kw.update(useRNN=True, history_len=4)
    lr = iPPO(env, **kw) if algo.startswith("ippo") else D2DPPO(env, beta_entropy=0.02, **kw)
    assert lr._fused_update_ok()
    ro = lr._rollout(n_envs)
    out = {"obs": ro.obs_f32, "actions": ro.actions, "logp": ro.logp}
    if algo.startswith("ippo"):
        out["adv"], out["ret"] = ro.adv_tne, ro.ret_tne
    else:
        out["ret_mean"] = ro.ret_mean.view(n_envs, L)
    np.random.seed(5)
    lr._update_epoch(ro, lr._update_state(ro))
    params = lr.policy.params
    for k, p in params.items():
        out[f"grad/{k}"] = p.grad
        out[f"w/{k}"] = p.data
    if algo.startswith("d2d"):
        for k, p in lr.value_network.named_parameters():
            out[f"cgrad/{k}"] = p.grad
    return {k: v.detach().cpu().clone() for k, v in out.items()}


def main():
    rank = int(os.environ.get("RANK", "0"))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    torch.cuda.set_device(0)
    os.makedirs(OUT, exist_ok=True)
    dist.init_process_group("gloo")
    for algo in ALGOS:
        torch.save(run(algo, E), os.path.join(OUT, f"{algo}_rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()
    if rank != 0:
        return 0
    rep, bad = {}, []
    for algo in ALGOS:
        full = run(algo, E * ws)
        shards = [torch.load(os.path.join(OUT, f"{algo}_rank{r}.pt")) for r in range(ws)]
        for r in range(ws):
            os.remove(os.path.join(OUT, f"{algo}_rank{r}.pt"))
        d = {}
        for k in ("obs", "actions"):          # [T][E]...: env axis 1
            ok = torch.equal(torch.cat([s[k] for s in shards], 1), full[k])
            d[k + "_exact"] = ok
            bad += [] if ok else [f"{algo} {k}"]
        for k in ("logp", "adv", "ret"):      # [T][N][E]: env axis 2
            if k in full:
                err = (torch.cat([s[k] for s in shards], 2) - full[k]).abs().max().item()
                d[k] = err
                tol = 0.0 if k == "logp" else 1e-5
                bad += [] if err <= tol else [f"{algo} {k} {err:.2e}"]
        if "ret_mean" in full:                # [E][T]
            err = (torch.cat([s["ret_mean"] for s in shards], 0) - full["ret_mean"]).abs().max().item()
            d["ret_mean"] = err
            bad += [] if err <= 1e-5 else [f"{algo} ret_mean {err:.2e}"]
        for k in full:
            if k.startswith(("grad/", "cgrad/")):
                g = full[k]
                errs = [(s[k] - g).abs().max().item() for s in shards]
                rel = max(errs) / max(g.abs().max().item(), 1e-30)
                d[k + "_rel"] = rel
                bad += [] if rel <= 2e-5 else [f"{algo} {k} {rel:.2e}"]
                same = all(torch.equal(s[k], shards[0][k]) for s in shards)
                d[k + "_ranks_identical"] = same
                bad += [] if same else [f"{algo} {k} differs across ranks"]
            if k.startswith("w/"):
                err = max((s[k] - full[k]).abs().max().item() for s in shards)
                d[k + "_over_lr"] = err / 3e-3
                bad += [] if err <= 0.02 * 3e-3 else [f"{algo} {k} {err / 3e-3:.2e} lr"]
        rep[algo] = d
    print(json.dumps({"rehearse_dp": rep, "world_size": ws, "envs_per_rank": E, "agents": N, "channels": C,
                      "violations": bad}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
