"""Interleaved in-process ablation of the env-step kernel (64 x 8 x 65536 envs).

Variants (timed with HIP events around each env-step launch, median of rounds):
  base      obs emitted, Philox draws, plain stores          (the product default)
  nt        same with non-temporal obs stores
  noobs     no obs emission (diagnostic: cost of the obs write stream)
  replay    obs, draws read from pre-generated buffers (diagnostic: Philox cost)
  state     obs + D2D state emission
  rec       the compact obs record instead of fp32 rows (the learners' and the bench's default)
  rec_replay  record, draws read from pre-generated buffers (Philox cost on the record path)
  rec_none    record path without any obs output (state / counters only)
plus torch fill_/copy_ of comparable sizes as write / copy bandwidth anchors.
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import config3_params  # noqa: E402


def main():
    from envs.combinatorial_env import CombinatorialEnv
    from d2dhip import _lib
    E = int(os.environ.get("ABL_ENVS", 65536))
    params = config3_params()
    env = CombinatorialEnv(**params, n_envs=E, device="cuda", seed=1)
    b = env.batch()
    lib = b.lib
    act = b.action_buffer()
    g = torch.Generator(device="cuda").manual_seed(0)
    flips = torch.randint(0, 256, (E, 64), device="cuda", dtype=torch.int32, generator=g).to(torch.uint8)
    arrs = torch.randint(0, 2, (E, 64), device="cuda", dtype=torch.int32, generator=g).to(torch.uint8)
    rec = b.record
    b.reset(want_obs=True)

    def run(variant, n=40):
        lib.d2d_set_option(_lib.D2D_OPT_NT_STORES, 1 if variant == "nt" else 0)
        evs = []
        for _ in range(n):
            if b.timestep >= 200:
                b.reset(want_obs=True)
            b.sample_actions(0.1, out=act)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if variant == "noobs":
                b.step(act, want_obs=False)
            elif variant == "replay":
                b.step(act, want_obs=True, replay=(flips, arrs))
            elif variant == "state":
                b.step(act, want_obs=True, want_state=True)
            elif variant == "rec":
                b.step(act, out_obs=rec)
            elif variant == "rec_replay":
                b.step(act, out_obs=rec, replay=(flips, arrs))
            elif variant == "rec_none":
                b.step(act, want_obs=False, replay=(flips, arrs))
            else:
                b.step(act, want_obs=True)
            e1.record()
            evs.append((e0, e1))
        torch.cuda.synchronize()
        return statistics.median(a.elapsed_time(c) for a, c in evs) * 1e3

    variants = ["base", "nt", "noobs", "replay", "state", "rec", "rec_replay", "rec_none"]
    res = {v: [] for v in variants}
    for v in variants:
        run(v, 10)
    for r in range(7):
        for v in variants:
            res[v].append(run(v))
    lib.d2d_set_option(_lib.D2D_OPT_NT_STORES, 0)
    # bandwidth anchors: write-only and copy of the obs-sized buffer
    x = torch.empty(E * 64 * 30, dtype=torch.float32, device="cuda")
    y = torch.empty_like(x)
    fill, copy = [], []
    for _ in range(20):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(); x.fill_(1.0); e1.record(); y.copy_(x); e2.record()
        torch.cuda.synchronize()
        fill.append(e0.elapsed_time(e1) * 1e3)
        copy.append(e1.elapsed_time(e2) * 1e3)
    nbytes = x.numel() * 4
    out = {v: {"median_us": statistics.median(t), "min_us": min(t)} for v, t in res.items()}
    alg = 172.0 * 64 * E
    for v in out:
        a_v = (alg - 120.0 * 64 * E + (32.0 * 64 * E if v.startswith("rec") and v != "rec_none" else 0.0)
               if v.startswith("rec") or v == "noobs" else alg)
        out[v]["alg_GBps"] = a_v / (out[v]["median_us"] * 1e-6) / 1e9
    out["torch_fill_obs_sized"] = {"us": statistics.median(fill), "GBps": nbytes / statistics.median(fill) / 1e3}
    out["torch_copy_obs_sized"] = {"us": statistics.median(copy), "GBps": 2 * nbytes / statistics.median(copy) / 1e3}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
