"""The D2D central critic's passes at configs[4]'s widest state (N agents, default 256: S = 7 N + 8 (N + 1), 4,096 envs
x 200 slots), timed one by one with HIP events on a real rollout: the fp32 -> bf16 state conversion
(d2d_states_to_bf16_padded, once per rollout), the fused forward (d2d_central_critic_fwd: W1 image + forward +
backward glue, every epoch) and the split-K dW1 GEMM (hipBLASLt bmm, every epoch); each with its bytes and rate.
usage (GPU box): python3 tools/gpu/critic_probe.py [N] [reps]"""
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
    D2DPPO.state_bf16_rollout = False  # fp32 state rows, so that the conversion pass can be timed
    torch.manual_seed(3)
    lr = D2DPPO(env, hidden_size=64, gamma=0.4, policy_lr=3e-4, value_lr=1e-3, beta_entropy=0.01,
                device=env.batch().device, useRNN=False, combinatorial=True)
    ro = lr._rollout(E)
    lr._update_state(ro)
    st = ro.__dict__["states"]
    S = ro.state_dim if "state_dim" in ro.__dict__ else st.shape[2]
    T_, E_ = st.shape[0], st.shape[1]
    S8 = -(-S // 8) * 8
    B = T_ * E_
    xb = torch.empty((B, S8), dtype=torch.bfloat16, device="cuda:0")
    flag = torch.empty(1, dtype=torch.int32, device="cuda:0")

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(reps):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / reps

    conv = timed(lambda: _lib.check(lib.d2d_states_to_bf16_padded(T_, E_, S, st.shape[2], st.data_ptr(), xb.data_ptr(),
                                                                   S8, flag.data_ptr(), _lib.stream_ptr()), "conv"))
    ro.state_bf16 = xb
    crit = [None]

    def fwd():
        crit[0] = lr._critic_fused_forward(ro, xb, S)

    f = timed(fwd)
    dhm = crit[0][3]
    g = timed(lambda: lr._dw1_gemm_bm(dhm, xb))
    xbytes = B * S8 * 2
    res = {"agents": N, "envs": E, "samples": B, "state_dim": S, "operand_bytes": xbytes,
           "convert_ms": conv, "convert_GBps": (B * st.shape[2] * 4 + xbytes) / conv / 1e6,
           "fwd_ms": f, "fwd_operand_GBps": xbytes / f / 1e6,
           "dw1_ms": g, "dw1_operand_GBps": xbytes / g / 1e6,
           "iteration_5_epochs_ms": conv + 5 * (f + g)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
