"""The data-parallel PRODUCT path across ranks on the GPU.

Two fresh child ranks (torch.distributed.run, gloo: a one-GPU box cannot run RCCL between two ranks; both
ranks on cuda:0, each initialising the GPU itself) run tools/gpu/rehearse_dp.py at the benched agent count
(64 agents x 8 channels): every rank owns an env shard (env_base = rank * E), rolls out on the HIP policy and
env kernels, normalises advantages / returns with the cross-rank column statistics, and runs one update epoch
of iPPO and D2D-PPO (MLP and GRU policies) on the fused gradient kernels with the bucketed gradient all-reduce
(algorithms/data_parallel.py; the per-agent updates of ippo.py:418-426 and d2d_ppo.py:429-446).  Rank 0 then
repeats each case in one process on the concatenated batch.  Bars (the script exits 1 on any violation):
  * rollouts (obs, actions, log-probs) bit-exact: the Philox counters are global env indices;
  * normalised advantages / returns within 1e-5;
  * all-reduced gradients within 2e-5 of max|g| of the one-process batch and identical on every rank;
  * post-Adam weights within 2 % of the learning rate.
The nccl branch of the same code is bench.py --gpus N under the driver (8-GPU nodes only)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(420)
def test_two_rank_product_path_equals_one_process_batch(tmp_path):
    env = dict(os.environ)
    env.update({"D2D_REHEARSE_N": "64", "D2D_REHEARSE_C": "8", "TMPDIR": str(tmp_path), "PYTHONUNBUFFERED": "1",
                "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tools", "gpu", "rehearse_dp.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400, cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"rehearse_dp"')]
    assert lines, f"no result line (rc {r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    res = json.loads(lines[-1])
    print(json.dumps({"violations": res["violations"], "world_size": res["world_size"], "agents": res["agents"],
                      "worst_grad_rel": max(v for d in res["rehearse_dp"].values() for k, v in d.items()
                                            if k.endswith("_rel"))}))
    assert res["world_size"] == 2 and res["agents"] == 64 and res["channels"] == 8
    assert set(res["rehearse_dp"]) == {"ippo", "d2d", "ippo_gru", "d2d_gru"}
    for algo, d in res["rehearse_dp"].items():
        assert d["obs_exact"] and d["actions_exact"] and d["logp"] == 0.0, algo
    assert res["violations"] == [], res["violations"]
    assert r.returncode == 0, r.stderr[-3000:]
