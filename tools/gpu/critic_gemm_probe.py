"""Timing probe: the D2D central critic's first-layer GEMM at configs[4]'s 256 agents (S = 3,848 -> 3,848 padded to
a multiple of 8, H = 64, B = 4,096 envs x 200 slots) on bf16 operands with fp32 output, in the orientations hipBLASLt
may serve differently: [3H][S] x [S][B] (the learner's), [B][S] x [S][3H], and the fp32 output with a bias epilogue.
usage: python tools/gpu/critic_gemm_probe.py"""
import json

import torch


def timed(fn, reps=10):
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
    B, S, H = 4096 * 200, 3848, 64
    g = torch.Generator(device="cuda").manual_seed(0)
    xb = torch.randint(0, 8, (B, S), device="cuda", generator=g).to(torch.bfloat16)
    w3 = (torch.randn(3 * H, S, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    w3t = w3.t().contiguous()
    out = {"B": B, "S": S, "3H": 3 * H, "tflop": 2 * B * S * 3 * H / 1e12}
    out["w3_x_xbT_ms"] = timed(lambda: torch.mm(w3, xb.t(), out_dtype=torch.float32))
    out["xb_x_w3T_ms"] = timed(lambda: torch.mm(xb, w3.t(), out_dtype=torch.float32))
    out["xb_x_w3t_contig_ms"] = timed(lambda: torch.mm(xb, w3t, out_dtype=torch.float32))
    out["bf16_out_xb_x_w3T_ms"] = timed(lambda: torch.mm(xb, w3.t()))
    for k in list(out):
        if k.endswith("_ms"):
            out[k.replace("_ms", "_tflops")] = out["tflop"] / (out[k] / 1e3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
