"""Time the GRU kernels with phases removed (A/B builds of libd2dhip; timing only, the ablated
kernels compute wrong gradients).  Build on the CPU host first:
    bash tools/gpu/build_ablate_gru.sh
then on the GPU box:  python3 tools/gpu/ablate_gru.py [variant ...]   (default: base gab1 .. gab4)
Shapes = bench.py's GRU leg (xp_load: D2D-PPO GRU, H = 64, history_len = 64, 64 agents x 8 channels):
the update over a 256-env x 200-slot rollout on the compact record, the policy slot 63 at 65,536 envs
(fp32 rows).  Prints ms per launch."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CODE = r'''
import sys, os, json, torch, numpy as np
sys.path[:0] = [{root!r}, os.path.join({root!r}, "d2d-ppo_amd")]
import bench
from algorithms.d2d_ppo import D2DPPO
from d2dhip import gru
from envs.combinatorial_env import CombinatorialEnv
params = bench.config3_params(200)
N, H, L = 64, 64, 64
res = {{}}
def timed(fn, reps):
    fn(); torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps): fn()
    ev[1].record(); torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps
env = CombinatorialEnv(**params, n_envs=256, device="cuda", seed=52)
torch.manual_seed(6); np.random.seed(6)
lr = D2DPPO(env, hidden_size=H, gamma=0.6, policy_lr=3e-4, value_lr=1e-3, device="cuda", useRNN=True,
            combinatorial=True, history_len=L, early_stopping=False)
ro = lr._rollout(256)
pp = {{k: v.data for k, v in lr.policy.params.items()}}
W = torch.randn((ro.T, 256, N), device="cuda")
gbuf = {{k: torch.empty_like(v) for k, v in pp.items()}}
res["grad_ms"] = timed(lambda: gru.grads(pp, ro.obs, "sigmoid", L, ro.L, W, actions=ro.actions,
                                         logp_old=ro.logp.permute(0, 2, 1), grads=gbuf), 2)
if {policy!r}:
    E = 65536
    env = CombinatorialEnv(**params, n_envs=E, device="cuda", seed=51)
    b = env.batch()
    buf = torch.empty((L, E, N, b.spec.F), dtype=torch.float32, device="cuda")
    act = b.action_buffer()
    b.reset(want_obs=True, out_obs=buf[0])
    for i in range(1, L):
        b.sample_actions(0.1, out=act)
        b.step(act, want_obs=True, out_obs=buf[i])
    logp = torch.empty((N, E), dtype=torch.float32, device="cuda")
    acts = torch.empty((1, E, N), dtype=act.dtype, device="cuda")
    res["policy_ms"] = timed(lambda: gru.policy(pp, buf, "sigmoid", L, 200, L - 1, 1, rng_step=7, seed=3,
                                                actions_out=acts, out=logp), 3)
print(json.dumps(res))
'''

if __name__ == "__main__":
    out = {}
    variants = sys.argv[1:] or ["", "gab1", "gab2", "gab3", "gab4"]
    for n, v in enumerate(variants):
        env = dict(os.environ)
        if v:
            env["D2D_LIB_VARIANT"] = v
            env["D2D_ALLOW_ABLATION"] = "1"
        code = CODE.format(root=ROOT, policy=(v in ("", "prev") or v.startswith("pol")))
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        out[f"{n}:{v or 'base'}"] = json.loads(line[-1]) if line else r.stderr[-800:]
        print(json.dumps({f"{n}:{v or 'base'}": out[f"{n}:{v or 'base'}"]}), flush=True)
    print(json.dumps(out, indent=1))
