"""A/B timing of the MLP update kernels on the learners' rollout format (compact record), 64 agents x 8 channels,
F = 30, H = 64 (or argv[2]), at E envs x 200 slots (argv[1], default 2,048): the actor kernel, and the critic on the
hidden-on-rows kernel (default) vs the sample-on-rows kernel of rounds 2-4 (D2D_OPT_CRITIC_GRAD_ROWS = 1), with the
two critics' gradient difference relative to max|g| (fp32 rounding only).
usage (GPU box): python3 tools/gpu/upd_ab.py [E] [H] [reps] [real]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]
import torch  # noqa: E402


def main():
    from d2dhip import _lib
    from d2dhip.envbatch import pack_masks_torch
    from d2dhip.record import ObsRecord
    from d2dhip.update import actor_grads, critic_grads
    lib = _lib.require_gpu()
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    T, N, F, A = 200, 64, 30, 8
    g = torch.Generator(device="cuda").manual_seed(0)
    net = {"w1": torch.randn(N, H, F, device="cuda", generator=g) * 0.1, "b1": torch.randn(N, H, device="cuda", generator=g) * 0.05,
           "w2": torch.randn(N, A, H, device="cuda", generator=g) * 0.1, "b2": torch.zeros(N, A, device="cuda")}
    vnet = {"w1": torch.randn(N, H, F, device="cuda", generator=g) * 0.1, "b1": torch.randn(N, H, device="cuda", generator=g) * 0.05,
            "w2": torch.randn(N, 1, H, device="cuda", generator=g) * 0.1, "b2": torch.zeros(N, 1, device="cuda")}
    RB = _lib.record_bytes(F)
    rdata = torch.zeros((T, E, N, RB), dtype=torch.uint8, device="cuda")
    rdata[..., :F] = torch.randint(0, 3, (T, E, N, F), device="cuda", generator=g, dtype=torch.uint8)
    rdata[..., F] = 1
    rec = ObsRecord(rdata, F, torch.zeros((N, RB // 32), dtype=torch.int32, device="cuda"))
    acts = pack_masks_torch(torch.randint(0, 2, (T, E, N, A), device="cuda", generator=g)).contiguous()
    lo = -torch.rand(T, N, E, device="cuda", generator=g).permute(0, 2, 1)
    W = torch.randn(T, N, E, device="cuda", generator=g).permute(0, 2, 1)
    R = torch.randn(T, N, E, device="cuda", generator=g).permute(0, 2, 1)

    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(reps):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / reps

    if "real" in sys.argv[4:]:  # a real iPPO rollout of the bench's c3 config instead of random inputs
        import bench
        from algorithms.ippo import iPPO
        from envs.combinatorial_env import CombinatorialEnv
        env = CombinatorialEnv(**bench.config3_params(200), n_envs=E, device="cuda:0", seed=7)
        torch.manual_seed(1)
        lr = iPPO(env, hidden_size=H, gamma=0.6, policy_lr=3e-4, value_lr=1e-3, device="cuda:0", combinatorial=True)
        ro = lr._rollout(E)
        net = {k: v.data for k, v in lr.policy.params.items()}
        vnet = {k: v.data for k, v in lr.value.params.items()}
        rec, acts = ro.obs, ro.actions
        lo, W, R = ro.logp.permute(0, 2, 1), ro.adv_tne.permute(0, 2, 1), ro.ret_tne.permute(0, 2, 1)
    res = {"E": E, "T": T, "N": N, "F": F, "H": H, "agent_samples": T * E * N, "inputs": "real" if "real" in sys.argv[4:] else "random"}
    res["actor_ms"] = timed(lambda: actor_grads(net, rec, acts, lo, W, "comb"))
    grads = {}
    for name, opt in (("critic_t", 0), ("critic_rows", 1)):
        lib.d2d_set_option(_lib.D2D_OPT_CRITIC_GRAD_ROWS, opt)
        try:
            res[f"{name}_ms"] = timed(lambda: critic_grads(vnet, rec, R))
            gr, st = critic_grads(vnet, rec, R)
            grads[name] = {k: v.double().clone() for k, v in gr.items()}
        finally:
            lib.d2d_set_option(_lib.D2D_OPT_CRITIC_GRAD_ROWS, 0)
    for k in grads["critic_t"]:
        a, b = grads["critic_t"][k], grads["critic_rows"][k]
        res[f"t_vs_rows/{k}"] = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
