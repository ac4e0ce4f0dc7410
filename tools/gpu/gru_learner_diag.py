"""First-step gradient of a GRU learner fixture (tests/golden/learner_*.npz) on the kernels against the
reference's recorded gradient, beside the torch agent-stacked fp32 path, per tensor, with the location of
the largest kernel error (the input column, for weight_ih).  Run once per library variant
(D2D_LIB_VARIANT=gdw0 / gdh0 with D2D_ALLOW_ABLATION=1: the fp32-MFMA weight-gradient / dh builds).
usage (GPU box): python3 tools/gpu/gru_learner_diag.py learner_ippo_rnn_cat_ep4 [E]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_learner_gpu as T  # noqa: E402
from conftest import GOLDEN  # noqa: E402

if __name__ == "__main__":
    name = sys.argv[1]
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    algo = name.split("_")[1]
    n_ep = int(z["episodes"]) if "episodes" in z.files else 2
    teacher = dict(actions=z["ro/actions"], reset_arrivals=z["draws/reset_arrivals"], flips=z["draws/flips"],
                   arrivals=z["draws/arrivals"])
    recs = {}
    for path in ("kernel", "torch"):
        env, kind, common, iPPO, D2DPPO = T.build(z, n_envs=E)
        lr = iPPO(env, **common) if algo == "ippo" else D2DPPO(env, beta_entropy=0.02, **common)
        for i, ag in enumerate(lr.agents):
            ag.policy_network.load_state_dict(T._sd(z, f"init/agent{i}/policy"))
            if algo == "ippo":
                ag.value_network.load_state_dict(T._sd(z, f"init/agent{i}/value"))
        if algo == "d2d":
            lr.value_network.load_state_dict(T._sd(z, "init/critic"))
        if path == "torch":
            lr._fused_upd = False
        ro = lr._rollout(n_ep, teacher=teacher)
        np.random.seed(21)  # the D2D agent permutation of the first epoch, as train() seeds it in the test
        rec = T.GradRecorder(lr)
        lr._update_epoch(ro, lr._update_state(ro))  # train()'s first epoch (train() refuses A/B builds)
        rec.learner = lr
        recs[path] = rec
        if path == "kernel":
            obs0 = ro.obs_f32[:, :, 0, :].reshape(-1, ro.obs_f32.shape[-1]).cpu().numpy()
            vals, counts = np.unique(obs0[:, -1], return_counts=True)
            print("agent 0 last obs column values:", dict(zip(np.round(vals, 4).tolist(), counts.tolist())))
    for (msg, pre, net), (_, _, nt) in zip(T._nets(recs["kernel"].learner, algo), T._nets(recs["torch"].learner, algo)):
        steps = T.ref_grads(z, pre[len("final/"):])
        for (k, v), (_, vt) in zip(net.named_parameters(), nt.named_parameters()):
            g = recs["kernel"].grad_at(v.detach(), 0).numpy()
            gt = recs["torch"].grad_at(vt.detach(), 0).numpy()
            r = steps[0][k].astype(np.float64)
            sc = np.abs(r).max()
            d = np.abs(g - r)
            loc = np.unravel_index(np.argmax(d), d.shape)
            print(f"{msg:16s} {k:22s} kernel {d.max() / sc:.2e} at {tuple(int(x) for x in loc)} (g {g[loc]:+.6e} "
                  f"ref {r[loc]:+.6e})  torch {np.abs(gt - r).max() / sc:.2e}")
