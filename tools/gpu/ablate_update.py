"""Time the actor update kernel with phases removed (A/B builds of libd2dhip; timing only, the
ablated kernels compute wrong gradients).  Build on the CPU host first:
    bash tools/gpu/build_ablate.sh
then on the GPU box:  python3 tools/gpu/ablate_update.py
Prints ms per actor / critic gradient launch at 2,048 envs x 200 slots x 64 agents (F 30, H 64, A 8), on
fp32 obs rows and on the compact record (the learners' rollout format)."""
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
# per-sample scalars in the learner's [T][N][E] layout, viewed as [T][E][N] (coalesced over envs)
lo = -torch.rand(T, N, E, device="cuda", generator=g).permute(0, 2, 1)
W = torch.randn(T, N, E, device="cuda", generator=g).permute(0, 2, 1)
from d2dhip.update import critic_grads
vnet = {{"w1": net["w1"].clone(), "b1": net["b1"].clone(), "w2": torch.randn(N, 1, H, device="cuda", generator=g) * 0.1,
        "b2": torch.zeros(N, 1, device="cuda")}}
R = torch.randn(T, N, E, device="cuda", generator=g).permute(0, 2, 1)
# the same inputs as the compact record the learners roll out (bias byte 1 at column F, no int8 columns)
from d2dhip.record import ObsRecord
from d2dhip import _lib
RB = _lib.record_bytes(F)
rdata = torch.zeros((T, E, N, RB), dtype=torch.uint8, device="cuda")
rdata[..., :F] = obs.to(torch.uint8)
rdata[..., F] = 1
rec = ObsRecord(rdata, F, torch.zeros((N, RB // 32), dtype=torch.int32, device="cuda"))
res = {{}}
for name, fn in (("actor", lambda: actor_grads(net, obs, acts, lo, W, "comb")),
                 ("critic", lambda: critic_grads(vnet, obs, R)),
                 ("actor_rec", lambda: actor_grads(net, rec, acts, lo, W, "comb")),
                 ("critic_rec", lambda: critic_grads(vnet, rec, R))):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(5):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    res[name] = ev[0].elapsed_time(ev[1]) / 5
print(json.dumps(res))
'''

if __name__ == "__main__":
    out = {}
    variants = sys.argv[1:] or ["", "abl1", "abl2", "abl3", "abl4", "abl5", "lf32"]
    for n, v in enumerate(variants):
        env = dict(os.environ)
        if v:
            env["D2D_LIB_VARIANT"] = v
            env["D2D_ALLOW_ABLATION"] = "1"
        r = subprocess.run([sys.executable, "-c", CODE.format(root=ROOT)], env=env, capture_output=True, text=True,
                           timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        out[f"{n}:{v or 'base'}"] = json.loads(line[-1]) if line else r.stderr[-500:]
    print(json.dumps(out, indent=1))
