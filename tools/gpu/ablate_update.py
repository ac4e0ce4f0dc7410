"""Time the actor update kernel with phases removed (A/B builds of libd2dhip; timing only, the
ablated kernels compute wrong gradients).  Build on the CPU host first:
    bash tools/gpu/build_ablate.sh
then on the GPU box:  python3 tools/gpu/ablate_update.py
Prints ms per actor-gradient launch at 2,048 envs x 200 slots x 64 agents (F 30, H 64, A 8)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CODE = r'''
import sys, os, torch, json
sys.path[:0] = [{root!r}, os.path.join({root!r}, "d2d-ppo_amd")]
from d2dhip.update import actor_grads
from d2dhip.envbatch import pack_masks_torch
T, E, N, F, H, A = 200, 2048, 64, 30, 64, 8
g = torch.Generator(device="cuda").manual_seed(0)
net = {{"w1": torch.randn(N, H, F, device="cuda", generator=g) * 0.1, "b1": torch.zeros(N, H, device="cuda"),
       "w2": torch.randn(N, A, H, device="cuda", generator=g) * 0.1, "b2": torch.zeros(N, A, device="cuda")}}
obs = torch.randint(0, 3, (T, E, N, F), device="cuda", generator=g).float()
acts = pack_masks_torch(torch.randint(0, 2, (T, E, N, A), device="cuda", generator=g)).contiguous()
lo = -torch.rand(T, E, N, device="cuda", generator=g)
W = torch.randn(T, E, N, device="cuda", generator=g)
for _ in range(2):
    actor_grads(net, obs, acts, lo, W, "comb")
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for _ in range(5):
    actor_grads(net, obs, acts, lo, W, "comb")
ev[1].record()
torch.cuda.synchronize()
print(json.dumps({{"ms": ev[0].elapsed_time(ev[1]) / 5}}))
'''

if __name__ == "__main__":
    out = {}
    for v in ["", "abl1", "abl2", "abl3", "lf32"]:
        env = dict(os.environ)
        if v:
            env["D2D_LIB_VARIANT"] = v
        r = subprocess.run([sys.executable, "-c", CODE.format(root=ROOT)], env=env, capture_output=True, text=True,
                           timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        out[v or "base"] = json.loads(line[-1])["ms"] if line else r.stderr[-500:]
    print(json.dumps(out, indent=1))
