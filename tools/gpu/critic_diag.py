"""Diagnostic of d2d_central_critic_fwd against float64 on random integer states: values, dpre = the sum of dhm's
three parts, and the partial sums, per hidden tile.  usage: python3 tools/gpu/critic_diag.py [H] [S] [B]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]
import torch  # noqa: E402


def main():
    from d2dhip import _lib
    lib = _lib.require_gpu()
    H = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 3848
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 1280
    S8 = -(-S // 8) * 8
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.zeros((B, S8), device="cuda")
    x[:, :S] = torch.randint(-1, 3, (B, S), device="cuda", generator=g).float()
    xb = x.to(torch.bfloat16).contiguous()
    w1 = torch.randn((H, S), device="cuda", generator=g) * 0.05
    b1 = torch.randn(H, device="cuda", generator=g) * 0.1
    w2 = torch.randn(H, device="cuda", generator=g) * 0.1
    b2 = torch.randn(1, device="cuda", generator=g) * 0.1
    ret = torch.randn(B, device="cuda", generator=g)
    G = int(lib.d2d_central_critic_blocks(H, B))
    img = torch.empty((int(lib.d2d_central_critic_image_bytes(H, S)) // 16, 4), dtype=torch.int32, device="cuda")
    v = torch.empty(B, device="cuda")
    dhm = torch.empty((B, 3 * H), dtype=torch.bfloat16, device="cuda")
    part = torch.empty((G, 2 * H + 2), device="cuda")
    _lib.check(lib.d2d_central_critic_fwd(H, B, S, S8, xb.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                                          b2.data_ptr(), ret.data_ptr(), img.data_ptr(), v.data_ptr(), dhm.data_ptr(),
                                          part.data_ptr(), G, _lib.stream_ptr()), "d2d_central_critic_fwd")
    torch.cuda.synchronize()
    X = x[:, :S].double()
    pre = X @ w1.double().t() + b1.double()
    v64 = torch.relu(pre) @ w2.double() + b2.double()
    d = v64 - ret.double()
    dv = d * 2.0 / B
    dpre = (pre > 0).double() * w2.double() * dv[:, None]
    got = dhm[:, :H].double() + dhm[:, H:2 * H].double() + dhm[:, 2 * H:].double()
    sums = part.double().sum(0)
    res = {"H": H, "S": S, "B": B, "G": G, "v_err": float((v.double() - v64).abs().max()),
           "dpre_err_by_tile": [float((got[:, 16 * t:16 * t + 16] - dpre[:, 16 * t:16 * t + 16]).abs().max())
                                for t in range(H // 16)],
           "dpre_max": float(dpre.abs().max()),
           "db1_err": float((sums[:H] - dpre.sum(0)).abs().max()), "db1_max": float(dpre.sum(0).abs().max()),
           "dw2_err": float((sums[H:2 * H] - (torch.relu(pre) * dv[:, None]).sum(0)).abs().max()),
           "db2_err": float(sums[2 * H] - dv.sum()), "loss_err": float(sums[2 * H + 1] - (d * d).sum())}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
