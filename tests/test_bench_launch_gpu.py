"""bench.py --gpus N on one node without an external launcher.

The driver's scaling run is `bench.py --gpus N`; bench.py starts the N rank processes itself when no
WORLD_SIZE is set (bench.self_launch) before anything touches the GPU, and every rank reports the group it
joined: `n_gpus` (WORLD_SIZE), `ranks_seen` (an all-reduce of ones over the group) and `dist_backend`.  On a
one-GPU box two ranks cannot run RCCL against each other, so the GPU test uses the rehearsal switches
(D2D_BENCH_BACKEND=gloo, D2D_BENCH_SHARE_GPU=1: both ranks on cuda:0); the nccl branch is the default of the
same code.  The PPO leg's update runs the bucketed gradient all-reduce (algorithms/data_parallel.py, the
per-agent updates of ippo.py:418-426), so its "allreduce" phase must be present and non-zero."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

LAUNCH_VARS = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_ADDR", "MASTER_PORT")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_VARS}
    env.update({"PYTHONUNBUFFERED": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    env.update(kw)
    return env


def test_bench_refuses_world_size_mismatch():
    """WORLD_SIZE from a launcher that disagrees with --gpus: exit 2 before any GPU call (runs on CPU)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu-baseline"],
                       env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "refusing" in r.stderr


@pytest.mark.gpu
@pytest.mark.timeout(420)
def test_bench_self_launch_two_ranks(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--legs", "env,ppo", "--steps", "10",
           "--warmup", "3", "--envs", "8192", "--ppo-envs", "256", "--ppo-epochs", "2", "--env-mode", "record",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=_env(D2D_BENCH_BACKEND="gloo", D2D_BENCH_SHARE_GPU="1", TMPDIR=str(tmp_path)),
                       capture_output=True, text=True, timeout=400, cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert r.returncode == 0, f"rc {r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    assert len(lines) == 1, r.stdout[-3000:]  # rank 0 alone prints the line
    res = json.loads(lines[0])
    ph = res["ppo"]["phase_ms_per_update"]
    print(json.dumps({"n_gpus": res["n_gpus"], "ranks_seen": res["ranks_seen"], "backend": res["dist_backend"],
                      "value": res["value"], "ppo_phase_ms": ph}))
    assert res["n_gpus"] == res["ranks_seen"] == 2
    assert res["dist_backend"] == "gloo"
    assert res["config"]["global_envs"] == 2 * 8192
    assert ph.get("allreduce", 0.0) > 0.0, ph
    assert res["value"] > 0 and res["ppo_updates_per_s"] > 0
