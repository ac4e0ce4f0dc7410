"""Accuracy of the fused PPO gradient kernels at the headline batch (parity at the sizes the
bench times): iPPO, 64 agents x 8 channels, E envs (default 65,536) x 200 slots on the compact record,
the actor and critic gradients of agents 0..K-1 against float64 autograd of the reference losses
(ippo.py:194-216: clipped surrogate + 0.01 entropy with Bernoulli(softmax) per channel; MSE value loss),
accumulated over sample chunks.  Prints max |kernel - f64| / max |g| per tensor, and the same for fp32 torch autograd over the same
chunks (the fp32 band the kernels are held to).
The kernels' accumulation chains are long here: at 65,536 envs 409,600 32-sample tiles per agent, at
most 256 per wave since round 3 (update_blocks); tests/test_update_gpu.py runs the comparison at 8,192 envs.
usage (GPU box): python3 tools/gpu/ppo_grads_full_batch.py [E] [K | a:b] [reversed] [envelope] [noemu]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def split2(v):
    """v rounded to the kernels' two-way round-to-nearest bf16 split h + m (update_kernels.hip split2_4)."""
    h = v.float().to(torch.bfloat16).to(v.dtype)
    return h + (v.float() - h.float()).to(torch.bfloat16).to(v.dtype)


U32 = 2.0 ** -24   # fp32 unit roundoff


def _flip_envelope(x, pre, absum, F, env):
    """Accumulate the relu-mask flip envelope of one float64 forward chunk.  A (sample, hidden) pair is
    ambiguous when |pre| <= 2 (F + 2) u sum_j |w_j x_j| + |b|: within twice the standard fp32 dot-product
    error bound (Higham gamma_K, K = F + 1 products plus the bias), so any fp32 evaluation of the
    pre-activation -- the kernels' split-bf16 MFMA sums, torch's GEMM -- may land on either side of 0
    and take the other relu mask.  A flipped mask at (s, h) moves dW1[h, :] by dA[s, h] x_s and db1[h]
    by dA[s, h] (dA = dL/drelu(pre)), so |g_fp32 - g64| <= band + sum over ambiguous s of |dA| |x_s|
    elementwise.  Returns a hook that adds the chunk's part once dA is known."""
    amb = (pre.detach().abs() <= 2 * (F + 2) * U32 * absum)
    env["n_amb"] = env.get("n_amb", 0) + int(amb.sum())

    def hook(dA):
        a = (dA.detach().abs() * amb)                 # [B][H]
        env["w1"] = env.get("w1", 0) + a.t() @ x.detach().abs()
        env["b1"] = env.get("b1", 0) + a.sum(0)
    return hook


def grads_vs_float64(E, agents, emulate=True, seed=11, reversed_fp32=False, envelope=False):
    """Relative errors {"<net>/<agent>/<param>": max |g - g64| / max |g64|} of the kernels ("actor",
    "critic"), of torch fp32 autograd ("actor_torch32", "critic_torch32") and, with emulate, of float64
    with one kernel rounding emulated ("actor_emu_dh": dH on the two-way split of the dW1 operand;
    "actor_emu_h": relu(H) on the two-way split in the logits); with reversed_fp32, torch fp32 autograd
    with the layer-1 inputs summed in reverse column order ("actor_torch32r": another, equally valid
    fp32 rounding) and the number of (sample, hidden) relu masks each fp32 forward gets wrong against
    float64 ("mask_flips32/<k>", "mask_flips32r/<k>"); with envelope, the relu-mask flip envelope of
    _flip_envelope for both nets' layer 1 and, per tensor, "excess/<net>/<k>/<n>" = max over elements of
    (|g - g64| - envelope) / max |g64| for the kernels ("excess32/..." for torch fp32), and
    "ambiguous_<net>/<k>" = the number of ambiguous (sample, hidden) pairs."""
    import bench
    from algorithms.ippo import iPPO
    from d2dhip.update import actor_grads, critic_grads
    from envs.combinatorial_env import CombinatorialEnv
    env = CombinatorialEnv(**bench.config3_params(200), n_envs=E, device="cuda:0", seed=seed)
    torch.manual_seed(3)
    np.random.seed(3)
    lr = iPPO(env, hidden_size=64, gamma=0.6, policy_lr=3e-4, value_lr=1e-3, device=env.batch().device,
              combinatorial=True, early_stopping=False)
    ro = lr._rollout(E)
    pp = {k: v.data.contiguous() for k, v in lr.policy.params.items()}
    vp = {k: v.data.contiguous() for k, v in lr.value.params.items()}
    ga, _ = actor_grads(pp, ro.obs, ro.actions, ro.logp.permute(0, 2, 1), ro.adv_tne.permute(0, 2, 1), "comb",
                        clip=0.1, beta=0.01)
    ga = {k: v.double().clone() for k, v in ga.items()}
    gc, _ = critic_grads(vp, ro.obs, ro.ret_tne.permute(0, 2, 1))
    gc = {k: v.double().clone() for k, v in gc.items()}
    torch.cuda.synchronize()
    T = ro.T
    B = T * E
    C = env.batch().spec.C
    rec = ro.obs
    F = rec.obs_dim
    sg = (rec.signed.to(torch.int64) & 0xFFFFFFFF)
    out = {"E": E, "T": T, "samples_per_agent": B}
    for k in agents:
        print(f"[ppo_grads_full_batch] E {E}: agent {k}", file=sys.stderr, flush=True)  # progress (long runs)
        cols = torch.arange(F, device="cuda")
        neg = ((sg[k, cols // 32] >> (cols % 32)) & 1).bool()
        q = {n: v[k].double().clone().requires_grad_() for n, v in pp.items()}
        qv = {n: v[k].double().clone().requires_grad_() for n, v in vp.items()}
        q32 = {n: v[k].clone().requires_grad_() for n, v in pp.items()}
        qv32 = {n: v[k].clone().requires_grad_() for n, v in vp.items()}
        qe1 = {n: v[k].double().clone().requires_grad_() for n, v in pp.items()}
        qe2 = {n: v[k].double().clone().requires_grad_() for n, v in pp.items()}
        q32r = {n: v[k].clone().requires_grad_() for n, v in pp.items()}
        runs = [(torch.float64, q, qv, 0), (torch.float32, q32, qv32, 0)]
        if reversed_fp32:
            runs += [(torch.float32, q32r, None, 3)]
        flips = [0, 0]
        envs = {"actor": {}, "critic": {}}
        if emulate:
            runs += [(torch.float64, qe1, None, 1), (torch.float64, qe2, None, 2)]
        chunk = max(1, (1 << 21) // E)
        for t0 in range(0, T, chunk):
            sl = slice(t0, min(T, t0 + chunk))
            d = rec.data[sl, :, k, :F]
            for dt, qa, qc, emu in runs:
                x = torch.where(neg, d.view(torch.int8).to(dt), d.to(dt)).reshape(-1, F)
                bits = ((ro.actions[sl, :, k].to(torch.int64).unsqueeze(-1) >> torch.arange(C, device="cuda")) & 1)
                bits = bits.reshape(-1, C).to(dt)
                lo = ro.logp[sl, k, :].to(dt).reshape(-1)
                adv = ro.adv_tne[sl, k, :].to(dt).reshape(-1)
                ret = ro.ret_tne[sl, k, :].to(dt).reshape(-1)
                if emu == 3:  # fp32 with the input columns summed in reverse order
                    pre = x.flip(-1) @ qa["w1"].flip(-1).t() + qa["b1"]
                else:
                    pre = x @ qa["w1"].t() + qa["b1"]
                if reversed_fp32 and dt == torch.float32:
                    with torch.no_grad():
                        ref_pre = x.double() @ pp["w1"][k].double().t() + pp["b1"][k].double()
                        flips[emu == 3] += int(((pre > 0) != (ref_pre > 0)).sum())
                if envelope and dt == torch.float64 and emu == 0:
                    with torch.no_grad():
                        xa = x.abs()
                        ab = xa @ qa["w1"].detach().abs().t() + qa["b1"].detach().abs()
                    hk = _flip_envelope(x, pre, ab, F, envs["actor"])
                if emu == 1:  # dH on the kernel's two-way RNE bf16 split (the dW1 / db1 operand)
                    pre.register_hook(split2)
                h = torch.relu(pre)
                if envelope and dt == torch.float64 and emu == 0:
                    h.register_hook(hk)
                if emu == 2:  # relu(H) on the two-way split in the logits (before round 3's three-way split)
                    h = h + (split2(h) - h).detach()
                probs = torch.softmax(h @ qa["w2"].t() + qa["b2"], -1)
                dist = torch.distributions.Bernoulli(probs=probs, validate_args=False)
                ratio = torch.exp(dist.log_prob(bits).mean(-1) - lo)
                surr = torch.min(ratio * adv, torch.clamp(ratio, 0.9, 1.1) * adv)
                (-(surr.sum() / B) - 0.01 * dist.entropy().mean(-1).sum() / B).backward()
                if qc is None:
                    continue
                prev = x @ qc["w1"].t() + qc["b1"]
                hv = torch.relu(prev)
                if envelope and dt == torch.float64:
                    with torch.no_grad():
                        abv = x.abs() @ qc["w1"].detach().abs().t() + qc["b1"].detach().abs()
                    hv.register_hook(_flip_envelope(x, prev, abv, F, envs["critic"]))
                v = (hv @ qc["w2"].t() + qc["b2"])[:, 0]
                (((v - ret) ** 2).sum() / B).backward()
        tags = [("actor_torch32", q32)] + ([("actor_emu_dh", qe1), ("actor_emu_h", qe2)] if emulate else [])
        if reversed_fp32:
            tags += [("actor_torch32r", q32r)]
            out[f"mask_flips32/{k}"], out[f"mask_flips32r/{k}"] = flips
        for n in q:
            ref = q[n].grad
            out[f"actor/{k}/{n}"] = float((ga[n][k] - ref).abs().max() / ref.abs().max())
            for tag, qq in tags:
                out[f"{tag}/{k}/{n}"] = float((qq[n].grad.double() - ref).abs().max() / ref.abs().max())
        for n in qv:
            ref = qv[n].grad
            out[f"critic/{k}/{n}"] = float((gc[n][k] - ref).abs().max() / ref.abs().max())
            out[f"critic_torch32/{k}/{n}"] = float((qv32[n].grad.double() - ref).abs().max() / ref.abs().max())
        if envelope:
            for net, ref_p, got, p32 in (("actor", q, ga, q32), ("critic", qv, gc, qv32)):
                e = envs[net]
                out[f"ambiguous_{net}/{k}"] = e.get("n_amb", 0)
                for n in ref_p:
                    ref = ref_p[n].grad
                    sc = ref.abs().max()
                    env_n = e.get(n, 0)
                    env_n = env_n if torch.is_tensor(env_n) else torch.zeros_like(ref)
                    env_n = env_n.reshape(ref.shape)   # dA carries the loss's 1 / B already
                    out[f"excess/{net}/{k}/{n}"] = float(((got[n][k] - ref).abs() - env_n).max() / sc)
                    out[f"excess32/{net}/{k}/{n}"] = float(((p32[n].grad.double() - ref).abs() - env_n).max() / sc)
    return out


if __name__ == "__main__":
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    ks = sys.argv[2] if len(sys.argv) > 2 else "2"   # K (agents 0..K-1) or a:b (agents a..b-1)
    agents = range(*map(int, ks.split(":"))) if ":" in ks else range(int(ks))
    K = len(agents)
    out = grads_vs_float64(E, agents, reversed_fp32="reversed" in sys.argv[3:], envelope="envelope" in sys.argv[3:],
                           emulate="noemu" not in sys.argv[3:])
    print(json.dumps(out), flush=True)
    summ = {}
    for kk, vv in out.items():
        if kk.count("/") == 2:
            tag, _, n = kk.split("/")
            summ.setdefault(f"{tag}/{n}", []).append(vv)
        elif kk.count("/") == 3:
            tag, net, _, n = kk.split("/")
            summ.setdefault(f"{tag}/{net}/{n}", []).append(vv)
    res = {"E": E, "T": out["T"], "agents": K, "agent_range": ks, "samples_per_agent": out["samples_per_agent"]}
    res.update({kk: {"max": max(vv), "median": float(np.median(vv))} for kk, vv in sorted(summ.items())})
    print(json.dumps(res), flush=True)
