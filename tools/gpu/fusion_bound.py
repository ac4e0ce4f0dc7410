"""Measured bound of SURVEY §8(f) rank 1, the fused env + policy rollout slot (ippo.py:293-330), at the headline
batch (64 agents x 8 channels x 65,536 envs, the compact record, H = 64): what a kernel that runs the env step and
the next slot's policy together could save at most is (i) the policy kernel's read of the slot's record, which
the env kernel has just written (the record must still be written: it is the rollout buffer the update reads),
and (ii) the launch boundary between the two kernels.  Measured here:
  * the training slot as iPPO runs it (actor-only policy kernel, then the env kernel), per-kernel HIP events and
    the slot's wall time per step (the boundary = slot - policy - env);
  * the same policy launches with every record DMA aimed outside the buffer (libd2dhip_noread.so, run in a child
    process: the same instructions, no memory traffic for the obs) -- policy_us - noread_us bounds (i).
usage (GPU box, after bash tools/gpu/build_fusion_bound.sh): python3 tools/gpu/fusion_bound.py"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]

CHILD = r'''
import json, sys, os, torch
sys.path[:0] = [{root!r}, os.path.join({root!r}, "d2d-ppo_amd")]
import bench
from algorithms.ippo import iPPO
from envs.combinatorial_env import CombinatorialEnv
E = 65536
env = CombinatorialEnv(**bench.config3_params(200), n_envs=E, device="cuda:0", seed=42)
torch.manual_seed(0)
lr = iPPO(env, hidden_size=64, gamma=0.6, policy_lr=3e-4, value_lr=1e-3, device=env.batch().device, combinatorial=True)
b = env.batch()
ring = b.record_buffer((2,))
act = b.action_buffer()
logp = torch.empty((b.spec.N, b.E), dtype=torch.float32, device=b.device)
val = torch.empty_like(logp)
b.reset(want_obs=True, out_obs=ring[0])
res = {{}}
for name, vslot, with_env in (("actor", None, True), ("actor+critic", val, True), ("actor_only_policy", None, False)):
    K = 40
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)]
    def slot(k, e=None):
        if b.timestep >= env.episode_length:
            b.reset(want_obs=True, out_obs=ring[k % 2])
        if e is not None: e[0].record()
        lr._policy_slot(ring, 0, k % 2, True, act, logp, vslot, None, b)
        if e is not None: e[1].record()
        if with_env:
            b.step(act, want_obs=True, out_obs=ring[(k + 1) % 2])
        if e is not None: e[2].record()
    for k in range(8): slot(k)
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    for k in range(K): slot(k, ev[k])
    t1.record(); torch.cuda.synchronize()
    pol = sum(e[0].elapsed_time(e[1]) for e in ev) / K * 1e3
    envk = sum(e[1].elapsed_time(e[2]) for e in ev) / K * 1e3
    res[name] = {{"policy_us": pol, "env_us": envk, "slot_us": t0.elapsed_time(t1) / K * 1e3}}
print(json.dumps(res))
'''


def run(variant):
    env = dict(os.environ)
    if variant:
        env.update({"D2D_LIB_VARIANT": variant, "D2D_ALLOW_ABLATION": "1"})
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], env=env, capture_output=True, text=True,
                       timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if not lines:
        raise RuntimeError(r.stderr[-2000:])
    return json.loads(lines[-1])


if __name__ == "__main__":
    base, noread = run(None), run("noread")
    rec_bytes = 65536 * 64 * 32
    a, n = base["actor"], noread["actor"]
    out = {"workload": "64 agents x 8 channels x 65,536 envs, compact record (32 B/agent-step), iPPO MLP H = 64",
           "base": base, "noread": noread,
           "record_read_us": a["policy_us"] - n["policy_us"],
           "record_bytes_per_slot": rec_bytes,
           "record_read_GBps": rec_bytes / max(a["policy_us"] - n["policy_us"], 1e-9) / 1e3,
           "boundary_us": a["slot_us"] - a["policy_us"] - a["env_us"],
           "fusion_saves_at_most_us": (a["policy_us"] - n["policy_us"]) + (a["slot_us"] - a["policy_us"] - a["env_us"]),
           "slot_us": a["slot_us"]}
    out["fusion_saves_at_most_frac"] = out["fusion_saves_at_most_us"] / a["slot_us"]
    print(json.dumps(out, indent=1))
