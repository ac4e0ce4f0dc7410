"""Does the D2D central critic's second read of the bf16 state operand (the split-K dW1 GEMM after the fused
forward) come from the 256 MB MALL when forward and dW1 run chunk by chunk?  Times, at configs[4]'s widest
state (N agents, default 256, 4,096 envs x 200 slots, a real rollout), the fused forward + dW1 over the whole
batch against the same two calls per sample chunk (chunk operand <= a few x 10 MB .. 500 MB), and checks the
chunked dW1 against the whole-batch one.
usage (GPU box): python3 tools/gpu/critic_chunk_probe.py [N] [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from algorithms.d2d_ppo import D2DPPO
    from d2dhip import _lib
    from envs.combinatorial_env import CombinatorialEnv
    lib = _lib.require_gpu()
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    E = 4096
    p5 = dict(n_agents=N, n_channels=8, deadlines=np.full(N, 7), lbdas=np.full(N, 1 / 14), period=None,
              arrival_probs=None, offsets=None, episode_length=200, traffic_model="aperiodic",
              periodic_devices=[], channel_switch=np.ones((N, 8)) * 0.8)
    env = CombinatorialEnv(**p5, n_envs=E, device="cuda:0", seed=22)
    torch.manual_seed(3)
    lr = D2DPPO(env, hidden_size=64, gamma=0.4, policy_lr=3e-4, value_lr=1e-3, beta_entropy=0.01,
                device=env.batch().device, useRNN=False, combinatorial=True)
    ro = lr._rollout(E)
    lr._update_state(ro)
    xb = ro.state_bf16
    B, S8 = xb.shape
    S = ro.state_dim if "state_dim" in ro.__dict__ else S8
    l1, l2 = lr.value_network.linear1, lr.value_network.linear2
    H = l1.weight.shape[0]
    dev = xb.device
    nimg = int(lib.d2d_central_critic_image_bytes(H, S))
    img = torch.empty((nimg // 16, 4), dtype=torch.int32, device=dev)
    w1 = l1.weight.detach().contiguous()
    ret = ro.ret_mean.contiguous()
    v = torch.empty(B, dtype=torch.float32, device=dev)
    dhm = torch.empty((B, 3 * H), dtype=torch.bfloat16, device=dev)

    def fwd(b0, b1):
        Bc = b1 - b0
        G = int(lib.d2d_central_critic_blocks(H, Bc))
        part = torch.empty((max(G, 1), 2 * H + 2), dtype=torch.float32, device=dev)
        _lib.check(lib.d2d_central_critic_fwd(H, Bc, S, S8, xb[b0:b1].data_ptr(), w1.data_ptr(),
                                              l1.bias.detach().data_ptr(), l2.weight.detach().data_ptr(),
                                              l2.bias.detach().data_ptr(), ret[b0:b1].data_ptr(), img.data_ptr(),
                                              v[b0:b1].data_ptr(), dhm[b0:b1].data_ptr(), part.data_ptr(), G,
                                              _lib.stream_ptr()), "fwd")
        return part

    def whole():
        fwd(0, B)
        return lr._dw1_gemm_bm(dhm, xb)

    def chunked(C):
        acc = None
        for b0 in range(0, B, C):
            b1 = min(B, b0 + C)
            fwd(b0, b1)
            g = lr._dw1_gemm_bm(dhm[b0:b1], xb[b0:b1])
            acc = g if acc is None else acc.add_(g)
        return acc

    def timed(fn):
        out = fn()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(reps):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / reps, out

    t_whole, g_ref = timed(whole)
    res = {"agents": N, "samples": B, "state_dim": S, "operand_bytes": B * S8 * 2, "whole_ms": t_whole, "chunks": []}
    scale = g_ref.abs().max().item()
    for C in (8192, 16384, 32768, 65536, 131072):
        t, g = timed(lambda: chunked(C))
        res["chunks"].append({"chunk_samples": C, "chunk_operand_MB": C * S8 * 2 / 1e6, "ms": t,
                              "max_rel_diff_vs_whole": (g - g_ref).abs().max().item() / scale})
        print(json.dumps(res["chunks"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
