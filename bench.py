"""Benchmark: the D2D-PPO env-step hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

Workload (BASELINE.json configs[2]): combinatorial_env, 64 agents x 8 channels,
channel_switch_8 tiled to 64 rows, deadlines [7,14]x32, heterogeneous traffic
(periodic = {k : k mod 6 < 3}, load 1/2), 65,536 envs per GPU (weak scaling:
rank r owns envs [r*E, (r+1)*E) with its own Philox counters, no data-path
collective).  One step = one slot for every env: the env-step kernel on synthetic
actions (Philox Bernoulli(0.1) per agent-channel, generated on the device before the
timed region: inputs resident in HBM) emitting the observation to HBM as the learners
consume it: the compact obs record (32 B per agent-step,
d2dhip/record.py, bit-exact decode to the fp32 obs).  The same K steps with fp32 obs
rows (the reference-API layout, 120 B per agent-step) are reported as `fp32_obs`.
Every episode_length slots the envs reset (inside the timed loop).  Inputs are
HBM-resident before timing starts.

More legs are reported in the same JSON line (they do not change `value`):
  rollout : the iPPO behaviour-policy slot at the same 65,536 envs — agent-stacked
            actor + critic forward (H=64), Bernoulli sampling, log-probs, action
            packing and the env kernel (ippo.py:293-330 batched);
  ppo     : PPO updates/s — one update = one epoch of the iPPO clipped-surrogate
            + value update for all 64 actors and 64 critics (ippo.py:194-217,
            418-426) over a full-episode rollout of --ppo-envs envs per GPU
            (200 slots), incl. the RCCL gradient all-reduce when N > 1;
  train   : one whole iPPO training iteration (rollout + GAE + --train-epochs PPO epochs)
            at the full 65,536 envs per GPU (ippo.py:406-441);
  configs : BASELINE.json configs[1] (chsel 16x4, 4,096 envs, D2D-PPO) and configs[4]
            (agent sweep 8..256 x 8 channels, 4,096 envs/GPU, D2D-PPO): env-step rates and
            one D2D-PPO training iteration each;
  d2denv  : the single-channel D2DEnv (envs/env.py): 64 agents with ring
            neighbourhoods, env-step rate, its kernel's HBM fraction, one iPPO iteration;
  gru     : xp_load.py's learner (D2D-PPO, GRU, history_len 64): policy slot, BPTT update, iteration;
  gru_c5  : configs[4] as xp_n_agents.py writes its learner (GRU, history_len = n_agents = 64/128/256).
The line ends with the metric's second half (ppo_updates_per_s, train_s_per_iteration,
train_env_steps_per_s_end_to_end) so that a truncated record still shows it.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "d2d-ppo_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "env-steps/sec (agents×envs) + PPO updates/sec, 64 agents × 8 ch, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA peak of one MI355X (MI355X_MICROARCH.md; no sparsity)
BYTES_PER_AGENT_STEP = 172.0   # B_as = 6D + 11C at D=14, C=8 (fp32 obs: 4F = 120 B of it)
RECORD_BYTES_PER_AGENT_STEP = BYTES_PER_AGENT_STEP - 120.0 + 32.0  # the 120 B of fp32 obs -> a 32 B record row


def config3_params(episode_length=200):
    cs8 = np.array(json.load(open(os.path.join(PKG, "combinatorial_load", "channel_switch_8.json")))["__nd__"])
    N = 64
    return dict(n_agents=N, n_channels=8, deadlines=np.array([7, 14] * (N // 2)), lbdas=np.full(N, 0.5),
                period=np.full(N, 2), arrival_probs=np.resize(np.array([.2, .4, .8, 1, 1, 1]), N),
                offsets=np.zeros(N), episode_length=episode_length, traffic_model="heterogeneous",
                homogeneous_size=True, periodic_devices=[k for k in range(N) if k % 6 < 3],
                channel_switch=np.resize(cs8, (N, 8)))


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n):
    """`bench.py --gpus N` (N > 1) started without a launcher: start N fresh rank processes (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in their env, one per GPU) and wait for them.  This parent never touches the GPU (no
    HIP call before or after the fork: the children initialise their own devices); it forwards the ranks'
    output, kills the remaining ranks when one fails (a rank left alone would block in its next collective) and
    returns the worst child exit status."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                    "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                    "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")})
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))

    def stop(signum, _frame):  # the launcher's own time limit: take the ranks down with it
        for p in procs:
            if p.poll() is None:
                p.kill()
        sys.exit(128 + signum)

    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    rcs = [None] * n
    failed_at = None
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
                if rcs[r] not in (None, 0) and failed_at is None:
                    failed_at = time.monotonic()
                    print(f"[bench] rank {r} exited with {rcs[r]}; stopping the other ranks", file=sys.stderr,
                          flush=True)
        if failed_at is not None and time.monotonic() - failed_at > 10:
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    p.kill()
        time.sleep(0.2)
    bad = [rc for rc in rcs if rc != 0]
    return max(bad, key=abs) if bad else 0


def setup_dist(n_gpus):
    """One process per GPU over RCCL ("nccl").  The world comes from the launcher's env (WORLD_SIZE; bench.py
    starts the ranks itself when run without one, self_launch) and must equal --gpus: a mismatch exits non-zero
    instead of silently benchmarking another GPU count.  Rehearsal switches for a 1-GPU box (never set by the
    driver): D2D_BENCH_BACKEND=gloo and D2D_BENCH_SHARE_GPU=1 (every rank on cuda:0).
    Returns (rank, world, local, ranks_seen): ranks_seen = an all-reduce of one per rank over the group."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        print(f"[bench] WORLD_SIZE={world} but --gpus {n_gpus}: refusing to report a {world}-rank run as "
              f"{n_gpus} GPUs", file=sys.stderr, flush=True)
        sys.exit(2)
    if os.environ.get("D2D_BENCH_SHARE_GPU") == "1":
        local = 0
    ranks_seen = 1
    if world > 1:
        torch.cuda.set_device(local)
        backend = os.environ.get("D2D_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        one = torch.ones((1,), dtype=torch.int64, device=f"cuda:{local}" if backend == "nccl" else "cpu")
        dist.all_reduce(one)
        ranks_seen = int(one.item())
        if ranks_seen != world:
            print(f"[bench] all-reduce of ones saw {ranks_seen} ranks, WORLD_SIZE {world}", file=sys.stderr)
            sys.exit(3)
    else:
        torch.cuda.set_device(0)
    return rank, world, local, ranks_seen


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(x, world):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def host_cores():
    """CPUs this process may run on: the affinity set, capped by a cgroup CPU quota when one is set
    (a container's share of a large host).  Returns (cores, affinity, quota or None)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // period)
        except (OSError, ValueError):
            pass
    return (min(aff, quota) if quota else aff), aff, quota


def cpu_baseline_c(params, seconds=8.0, max_envs=16384):  # bounded: ~`seconds` of host work
    """C oracle ("port") on every host core (OpenMP), Philox mode, same workload, bounded sample."""
    from oracle.c_oracle import COracle
    threads, aff, quota = host_cores()
    E = max_envs
    c = COracle("comb", params, n_envs=E, seed=42, nthreads=threads)
    c.reset(rng_step=0, want_state=False)
    rs, steps = 1, 0
    t0 = time.perf_counter()
    while True:
        a = c.sample_actions(rs, p=0.1)
        c.step(a, rng_step=rs + 1, want_state=False)
        rs += 2
        steps += 1
        if c.timestep >= params["episode_length"]:
            c.reset(rng_step=rs, want_state=False)
            rs += 1
        el = time.perf_counter() - t0
        if el >= seconds or steps >= 4000:
            break
    v = E * steps / el
    return {"value": v, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "agent_steps_per_s": v * params["n_agents"],
            "sample": f"oracle/c/d2d_oracle.c (OpenMP, {threads} threads = affinity {aff}"
                      f"{'' if quota is None else f', cgroup quota {quota}'}): {E} envs x {steps} slots of the same "
                      f"64x8 workload incl. action sampling and fp32 obs, {el:.1f} s"}


def _numpy_worker(args):
    """One host process of the NumPy leg: the oracle's per-env restatement of the reference step
    (oracle/env_oracle.py, one env at a time like CombinatorialEnv.step) for `seconds`."""
    params, proc, seconds, E = args
    from oracle.env_oracle import EnvOracle
    o = EnvOracle("comb", params, n_envs=E, seed=42, env_base=proc * E)
    rng = np.random.default_rng(proc)
    o.reset(rng_step=0)
    rs, steps = 1, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        a = (rng.random((E, params["n_agents"], params["n_channels"])) < 0.1).astype(np.int64)
        o.step(a, rng_step=rs)
        rs += 1
        steps += 1
        if o.timestep >= params["episode_length"]:
            o.reset(rng_step=rs)
            rs += 1
    return E * steps, time.perf_counter() - t0


def cpu_baseline_numpy(params, seconds=8.0, E=4):
    """The NumPy restatement, one process per host core.  Runs BEFORE the GPU is
    touched (fork of a process without a HIP context).  Aggregate env-steps/s = sum over processes."""
    import multiprocessing as mp
    cores, aff, quota = host_cores()
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(cores) as pool:
        res = pool.map(_numpy_worker, [(params, p, seconds, E) for p in range(cores)])
    wall = time.perf_counter() - t0
    v = sum(n / el for n, el in res)
    return {"value": v, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "agent_steps_per_s": v * params["n_agents"],
            "sample": f"oracle/env_oracle.py (NumPy, per-env loop mirroring CombinatorialEnv.step), {cores} processes "
                      f"(affinity {aff}{'' if quota is None else f', cgroup quota {quota}'}) x {E} envs x ~{seconds:.0f} s "
                      f"of the same 64x8 workload, fp32 obs; {wall:.1f} s wall"}


class PhaseTimer:
    """Splits learner work into phases with HIP events on the current stream (the learners call
    _phase(name) after each phase; the time since the previous mark is charged to `name`)."""

    def __init__(self):
        self.marks = []
        self.start()

    def start(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.prev = e

    def mark(self, name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.marks.append((name, self.prev, e))
        self.prev = e

    def totals_ms(self):
        torch.cuda.synchronize()
        out = {}
        for name, a, b in self.marks:
            out[name] = out.get(name, 0.0) + a.elapsed_time(b)
        return out


def load_profile_json(name):
    """A committed measurement under profiles/ (rocprofv3 PMC summaries made by tools/gpu/*.sh on the GPU
    box from a committed tree; each records the commit and the rocprofv3 output it came from).  Returns
    (dict, repo-relative path) or (None, path)."""
    rel = os.path.join("profiles", name)
    try:
        return json.load(open(os.path.join(ROOT, rel))), rel
    except (OSError, ValueError):
        return None, rel


def load_pmc_traffic(mode="fp32"):
    return load_profile_json("pmc_traffic.json" if mode == "fp32" else f"pmc_traffic_{mode}.json")


def pmc_mfma(kernel_prefix, leg=None):
    """PMC-measured MFMA pipe utilisation of a kernel (tools/pmc_mfma.py: SQ_VALU_MFMA_BUSY_CYCLES / (kernel
    cycles x 1024 SIMDs) over rocprofv3 --pmc passes), with its source.  leg: the per-leg profile
    profiles/pmc_mfma_<leg>.json (tools/gpu/pmc_legs.sh runs the bench with that leg alone, so every dispatch of
    the row is one of the leg's launches -- the row's dispatch count is reported beside it); else the mixed
    profiles/pmc_mfma.json."""
    d, rel = load_profile_json(f"pmc_mfma_{leg}.json" if leg else "pmc_mfma.json")
    if not d:
        return None
    for k in d.get("kernels", []):
        name = k.get("kernel", "")
        if name.startswith("void "):  # rocprofv3 prints template kernels with their return type
            name = name[5:]
        if name.startswith(kernel_prefix):
            pd = k.get("per_dispatch", {})
            valu, mfma = pd.get("SQ_INSTS_VALU"), pd.get("SQ_INSTS_MFMA")
            # SQ_INSTS_VALU counts the MFMAs too: non-MFMA vector instructions per MFMA
            vpm = (valu - mfma) / mfma if valu is not None and mfma else None
            return {"mfma_busy_frac_pmc": k.get("mfma_busy_frac"), "valu_per_mfma_pmc": vpm,
                    "wave_time_split": k.get("wave_time_split"), "dispatches": k.get("dispatches", {}).get("SQ_WAVES"),
                    "source": rel, "commit": d.get("commit"), "workload": d.get("workload"),
                    "pmc_kernel": k.get("kernel"), "avg_duration_us": k.get("avg_duration_us")}
    return None


def env_kernel_name(spec, record):
    """The env-step kernel instantiation a step of this spec launches (csrc/env_kernels.hip dispatch_*),
    as rocprofv3 names it."""
    dw = {1: 1, 2: 2, 3: 3, 4: 4}.get(int(spec.DW), int(spec.DW))
    large = "true" if spec.N > 64 else "false"
    if spec.kind == "chsel":
        return f"d2d::chsel_kernel<{dw}, {large}>"
    if spec.kind == "single":
        return f"d2d::single_kernel<{dw}, {large}>"
    mask = "unsigned char" if spec.C <= 8 else "unsigned short" if spec.C <= 16 else "unsigned int"
    ct = spec.C if spec.C in (4, 8, 16) else 0
    return f"d2d::comb_kernel<{mask}, {dw}, {large}, {ct}, false>" + (" (record)" if record else "")


def rollout_leg(env, args, world):
    """iPPO behaviour-policy slots at the full env batch (policy in the loop)."""
    from algorithms.ippo import iPPO
    torch.manual_seed(0)
    lr = iPPO(env, hidden_size=64, gamma=0.6, policy_lr=3e-4, value_lr=1e-3, device=env.batch().device,
              useRNN=False, combinatorial=True)
    b = env.batch()
    # the rollout buffer format the learner runs on (the compact record by default)
    ring = b.record_buffer((2,)) if lr._record_ok() else torch.empty((2,) + tuple(b.obs.shape), dtype=torch.float32,
                                                                       device=b.device)
    rew = torch.empty((b.E,), dtype=torch.int32, device=b.device)
    act = b.action_buffer()
    logp = torch.empty((b.spec.N, b.E), dtype=torch.float32, device=b.device)
    val = torch.empty_like(logp)
    b.reset(want_obs=True, out_obs=ring[0])

    K = args.rollout_steps
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)]

    # the training slot as iPPO.train runs it: actor-only when the values are deferred to the first epoch's
    # critic pass (iPPO.defer_values), else actor + critic
    vslot = None if lr._defer_values_ok() else val

    def slot(k, e=None):
        if b.timestep >= env.episode_length:
            b.reset(want_obs=True, out_obs=ring[k % 2])
        with torch.no_grad():
            if e is not None:
                e[0].record()
            lr._policy_slot(ring, 0, k % 2, True, act, logp, vslot, None, b)
            if e is not None:
                e[1].record()
            b.step(act, want_obs=True, out_obs=ring[(k + 1) % 2], out_reward=rew)
            if e is not None:
                e[2].record()

    for k in range(10):
        slot(k)
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    for k in range(K):
        slot(k, ev[k])
    torch.cuda.synchronize()
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world)
    v = b.E * world * K / el
    path = ("fused HIP policy kernel (exact 3-way bf16 split MFMA, fp32-accurate)" if lr._fused_ok()
            else "torch agent-stacked bmm")
    pol_ms = max_over_ranks(float(np.mean([e[0].elapsed_time(e[1]) for e in ev])), world)
    env_ms = max_over_ranks(float(np.mean([e[1].elapsed_time(e[2]) for e in ev])), world)
    F, H, A = lr.policy.F, lr.policy.H, lr.policy.A
    # actor (+ critic when the slot computes values) forward per agent-step
    flop = 2 * (F * H + H * A) + (2 * (F * H + H) if vslot is not None else 0)
    # the products run as exact bf16 splits: an fp32-equivalent rate is no roofline (it can
    # exceed the fp32 MFMA peak); the roofline figure is the executed MFMA pipe's busy fraction (PMC, with
    # its source file and commit), beside the algorithmic rate in GFLOP/s
    return {"env_steps_per_s": v, "agent_steps_per_s": v * b.spec.N, "ms_per_step": el / K * 1e3, "steps": K,
            "policy": (f"iPPO MLP H=64 {'actor+critic' if vslot is not None else 'actor'}, 64 agents, Bernoulli "
                       f"sampling, fp32; {path}"),
            "values": ("per slot (actor + critic kernel)" if vslot is not None else
                       "deferred: V(obs) of every sample from the first epoch's critic-gradient pass "
                       "(d2d_ppo_critic_grad_values), GAE after it"),
            "obs_format": "compact record (u8)" if lr._record_ok() else "fp32",
            "policy_kernel_us": pol_ms * 1e3, "env_kernel_us": env_ms * 1e3,
            "policy_flop_per_agent_step": flop,
            "policy_algorithmic_gflops": flop * b.E * b.spec.N / (pol_ms / 1e3) / 1e9,
            "policy_mfma_pmc": pmc_mfma("d2d::policy_split_kernel", "rollout")}


def ppo_leg(args, rank, world, local):
    """PPO updates/s of iPPO on a full-episode rollout of --ppo-envs envs per GPU."""
    from algorithms.ippo import iPPO
    from envs.combinatorial_env import CombinatorialEnv
    params = config3_params(args.episode_length)
    E2 = args.ppo_envs
    env2 = CombinatorialEnv(**params, n_envs=E2, device=f"cuda:{local}", seed=7)
    torch.manual_seed(1)
    lr = iPPO(env2, hidden_size=64, gamma=0.6, policy_lr=3e-4, value_lr=1e-3, device=f"cuda:{local}",
              useRNN=False, combinatorial=True)
    ro = lr._rollout(E2)
    upd = lr._update_state(ro)
    lr._update_epoch(ro, upd)  # warm-up (allocator, hipBLASLt heuristics)
    torch.cuda.synchronize()
    barrier(world)
    lr.phase_timer = PhaseTimer()
    t0 = time.perf_counter()
    P = args.ppo_epochs
    for _ in range(P):
        lr._update_epoch(ro, upd)
    torch.cuda.synchronize()
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world)
    # per-update phase split (HIP events at the learner's marks), max over ranks; "allreduce" is the bucketed
    # gradient all-reduce (algorithms/data_parallel.py), absent at N = 1
    phases = {k: max_over_ranks(v / P, world) for k, v in lr.phase_timer.totals_ms().items()}
    lr.phase_timer = None
    N = params["n_agents"]
    samples = ro.T * E2 * world
    F, H, A = lr.policy.F, lr.policy.H, lr.policy.A
    out = {"updates_per_s": P / el, "ms_per_update": el / P * 1e3, "epochs": P,
           "batch": f"{E2} envs/GPU x {ro.T} slots x {N} agents (actor+critic, one Adam step each)",
           "agent_samples_per_update": samples * N, "agent_samples_per_s": samples * N * P / el,
           "phase_ms_per_update": phases}
    if upd is None:
        out["path"] = "fused HIP update kernels (actor + critic gradients) + torch Adam"
        out["kernels"] = update_kernel_roofline(lr, ro, F, H, A, reps=P)
    else:
        out["path"] = "torch agent-stacked bmm autograd + Adam"
    return out


def update_kernel_roofline(lr, ro, F, H, A, reps=4):
    """Live HIP-event timing of the two gradient kernels (each incl. its partial-sum reduce) on
    the leg's rollout, and their algorithmic FLOPs per agent-sample (SURVEY §8d MFMA roofline):
      actor  fwd 2(FH + HA), bwd dW2 2HA + dH 2AH + dW1 2FH (no input gradient)
      critic fwd 2(FH + H),  bwd dV2 2H + dHv 2H + dV1 2FH
    The products run as exact bf16 splits, so the algorithmic rate can exceed the
    dense fp32 matrix peak; the roofline figure is the MFMA pipe's busy fraction."""
    from d2dhip.update import actor_grads, critic_grads
    pp, vp = lr.policy.params, lr.value.params
    N = lr.policy.N
    agent_samples = ro.T * ro.E * N
    f_actor = 2 * (F * H + H * A) + 2 * H * A + 2 * A * H + 2 * F * H
    f_critic = 2 * (F * H + H) + 2 * H + 2 * H + 2 * F * H
    ga = {k: torch.empty_like(v) for k, v in pp.items()}
    gv = {k: torch.empty_like(v) for k, v in vp.items()}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ta = tc = 0.0
    for _ in range(reps):
        ev[0].record()
        actor_grads({k: v.data for k, v in pp.items()}, ro.obs, ro.actions, ro.logp.permute(0, 2, 1),
                    ro.adv_tne.permute(0, 2, 1), "comb", grads=ga)
        ev[1].record()
        critic_grads({k: v.data for k, v in vp.items()}, ro.obs, ro.ret_tne.permute(0, 2, 1), grads=gv)
        ev[2].record()
        torch.cuda.synchronize()
        ta += ev[0].elapsed_time(ev[1]) / reps
        tc += ev[1].elapsed_time(ev[2]) / reps
    # MFMA pipe time per 32-sample tile from the kernels' static instruction mix (F + 1 <= 32,
    # H <= 64, A <= 8: csrc/update_kernels.hip, bf16 logits): 104 (actor on the compact record: no
    # HN recompute) or 128 (fp32 rows) / 40 (critic, either orientation; PMC-confirmed,
    # profiles/r05/pmc_upd_r05c.json) v_mfma_f32_16x16x32_bf16 at 16 cycles/SIMD
    # (MI355X_MICROARCH.md cycle table), 2.4 GHz peak clock
    from d2dhip.record import ObsRecord
    pipe = {"actor": (104 if isinstance(ro.obs, ObsRecord) else 128) * 16, "critic": 40 * 16}
    simds, clock = 1024, 2.4e9
    tiles = ro.T * ((ro.E + 31) // 32) * N
    res = {}
    for name, ms, fl in (("actor", ta, f_actor), ("critic", tc, f_critic)):
        busy = tiles * pipe[name] / simds / clock / (ms / 1e3)
        # executed bf16 MFMA work (16 x 16 x 32 x 2 flop per instruction, pipe cycles / 16) over the dense
        # bf16 peak: <= 1 by construction; the algorithmic fp32 rate is reported in GFLOP/s, not as a fraction
        executed = tiles * pipe[name] / 16 * 16384 / (ms / 1e3) / 1e12
        res[name] = {"ms": ms, "flop_per_agent_sample": fl,
                     "algorithmic_gflops": agent_samples * fl / (ms / 1e3) / 1e9,
                     "executed_bf16_tflops": executed, "executed_over_bf16_dense_peak": executed / BF16_PEAK_TFLOPS,
                     "mfma_cycles_per_tile": pipe[name], "mfma_pipe_busy_frac_static": busy,
                     # (the critic at H <= 64 runs the hidden-on-rows ppo_critic_grad_t_kernel since round 5)
                     "mfma_pmc": (pmc_mfma("d2d::ppo_critic_grad_t_kernel", "ppo") if name == "critic" else None)
                     or pmc_mfma(f"d2d::ppo_{name}_grad_kernel", "ppo"), "bound": "mfma"}
    return res


def train_leg(env, args, rank, world, local):
    """One full iPPO training iteration at the bench's env batch (the north-star scale): a
    200-slot rollout of every env (policy kernel + env kernel per slot), GAE/returns, and n_epoch
    fused PPO epochs over all T*E*N agent-samples (the loop body of iPPO.train, ippo.py:410-426,
    without its periodic test()).  Reported: seconds per iteration and end-to-end env-steps/s."""
    from algorithms.ippo import iPPO
    torch.manual_seed(2)
    lr = iPPO(env, hidden_size=64, gamma=0.6, policy_lr=3e-4, value_lr=1e-3, device=env.batch().device,
              useRNN=False, combinatorial=True)
    E = env.batch().E

    def iteration(n_epoch):
        # the body of iPPO.train for one iteration (ippo.py:410-426) without the test(50) calls
        # the reference makes when iter % test_freq == 0 (always true at iter 0); as train() does, the rollout's
        # values come from the first epoch's critic pass (iPPO.defer_values)
        ro = lr._rollout(E, defer_values=True)
        upd = lr._update_state(ro)
        for _ in range(n_epoch):
            lr._update_epoch(ro, upd)
        del ro, upd

    iteration(1)  # warm-up: allocations, kernels
    torch.cuda.synchronize()
    barrier(world)
    lr.phase_timer = PhaseTimer()
    t0 = time.perf_counter()
    iteration(args.train_epochs)
    torch.cuda.synchronize()
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world)
    phases = {k: max_over_ranks(v, world) for k, v in lr.phase_timer.totals_ms().items()}
    lr.phase_timer = None
    T = env.episode_length
    epoch_ms = sum(v for k, v in phases.items() if k not in ("rollout", "gae")) / args.train_epochs
    return {"s_per_iteration": el, "n_epoch": args.train_epochs, "envs_per_gpu": E, "slots": T,
            "agent_samples_per_epoch": E * world * T * env.n_agents,
            "env_steps_per_s_end_to_end": E * world * T / el,
            "phase_ms": phases,
            "ppo_ms_per_update": epoch_ms,
            "ppo_updates_per_s": 1e3 / epoch_ms,
            "ppo_batch": f"{E} envs/GPU x {T} slots x {env.n_agents} agents (the headline batch; one update = "
                         f"one epoch: actor + critic gradients, all-reduce, Adam)",
            "path": "fused policy kernel + env kernel rollout, HIP GAE, fused PPO gradient kernels + Adam"}


def _env_rate(env, steps=40, bytes_per_agent_step=None):
    """Env-step throughput of a batched env (device-sampled actions + env kernel, fp32 obs emitted)
    and the env kernel's own HBM roofline: its average HIP-event time against SURVEY §8(d)'s
    algorithmic bytes per agent-step."""
    b = env.batch()
    act = b.action_buffer()
    b.reset(want_obs=True)
    for _ in range(5):
        b.sample_actions(0.1, out=act)
        b.step(act, want_obs=True)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        if b.timestep >= env.episode_length:
            b.reset(want_obs=True)
        b.sample_actions(0.1, out=act)
        evs[i][0].record()
        b.step(act, want_obs=True)
        evs[i][1].record()
    torch.cuda.synchronize()
    rate = b.E * steps / (time.perf_counter() - t0)
    kern_us = float(np.mean([x.elapsed_time(y) for x, y in evs])) * 1e3
    roof = {"kernel": env_kernel_name(b.spec, False), "kernel_avg_us": kern_us,
            "step_us": 1e6 * b.E / rate}
    if bytes_per_agent_step:
        launch = bytes_per_agent_step * b.spec.N * b.E
        roof.update({"bytes_per_agent_step": bytes_per_agent_step, "bytes_per_launch": launch,
                     "achieved_GBps": launch / (kern_us / 1e6) / 1e9,
                     "hbm_frac": launch / (kern_us / 1e6) / 1e9 / HBM_PEAK_GBS})
    return rate, roof


def _env_rate_graph(env, reps=5):
    """The same env steps replayed as one captured HIP graph per episode (reset + episode_length x
    (synthetic-action sampling + env kernel)), as the learners' training rollouts run: the device-side rate
    of the small configurations, whose eager step loop is bound by Python and launch overhead.  The replays
    advance the env kernel's Philox counters through the rng_offset word (fresh channel flips and arrivals
    every replay); the synthetic actions repeat per replay."""
    b = env.batch()
    act = b.action_buffer()
    L = env.episode_length

    def episode():
        b.reset(want_obs=True)
        for _ in range(L):
            b.sample_actions(0.1, out=act)
            b.step(act, want_obs=True)

    side = torch.cuda.Stream(device=b.device)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        episode()  # warm-up (allocations, kernel attributes)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    base = b.rng_step
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        episode()
    delta = b.rng_step - base
    b.rng_step = base
    g.replay()  # first replay (graph upload) untimed
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(reps):
        b.rng_off.fill_(delta * (r + 1))
        g.replay()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    b.rng_off.zero_()
    b.rng_step = base + delta * (reps + 1)
    return b.E * L * reps / el


def _d2d_iteration(env, n_epoch, combinatorial):
    """One D2D-PPO training iteration (d2d_ppo.py:405-448 loop body without test()): rollout of
    every env, returns, n_epoch epochs (critic values, GAE, chain over a random agent cycle,
    fused actor gradients, clip + Adam, central critic).  Seconds after one warm-up iteration, the
    fused-update flag and the iteration's phase split (HIP events at the learner's phase marks, ms)."""
    from algorithms.d2d_ppo import D2DPPO
    torch.manual_seed(3)
    np.random.seed(3)
    lr = D2DPPO(env, hidden_size=64, gamma=0.4, policy_lr=3e-4, value_lr=1e-3, beta_entropy=0.01,
                device=env.batch().device, useRNN=False, combinatorial=combinatorial)
    E = env.batch().E

    def it(ne):
        ro = lr._rollout(E)
        upd = lr._update_state(ro)
        for _ in range(ne):
            lr._update_epoch(ro, upd)

    it(1)
    torch.cuda.synchronize()
    lr.phase_timer = PhaseTimer()
    t0 = time.perf_counter()
    it(n_epoch)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    phases = lr.phase_timer.totals_ms()
    lr.phase_timer = None
    return el, lr._fused_update_ok(), phases


def configs_leg(args, rank, world, local):
    """The other BASELINE.json GPU configs, per GPU (weak scaling shards):
      c2  channel_selection_env 16 agents x 4 channels, 4,096 envs, D2D-PPO (categorical);
      c5  xp_n_agents sweep: combinatorial N in {8..256} x 8 channels, deadlines 7, switch 0.8,
          lambda 1/14 aperiodic, 32,768 envs over 8 GPUs = 4,096 per GPU, D2D-PPO.
    Env-step rates and one training iteration each (MLP policies, H = 64, n_epoch = 5 as in
    xp_load.py:106)."""
    from envs.channel_selection_env import ChannelSelectionEnv
    from envs.combinatorial_env import CombinatorialEnv
    dev = f"cuda:{local}"
    out = {}
    N = 16
    p2 = dict(n_agents=N, n_channels=4, deadlines=np.full(N, 7), lbdas=np.full(N, 1 / 3.5), period=np.full(N, 2),
              arrival_probs=np.full(N, 0.5), offsets=np.zeros(N), episode_length=args.episode_length,
              traffic_model="aperiodic", periodic_devices=[], channel_switch=np.full(5, 0.8))
    env = ChannelSelectionEnv(**p2, n_envs=4096, device=dev, seed=21)
    env.shard(rank, world)
    # chsel B_as = 1 + 2D + 4(D + C + 1) + 2(C + 1)/N = 63.6 B at D = 7, C = 4, N = 16
    rate, roof = _env_rate(env, bytes_per_agent_step=1 + 2 * 7 + 4 * (7 + 4 + 1) + 2 * 5 / N)
    rate_g = _env_rate_graph(env)
    it_s, fused, phases = _d2d_iteration(env, 5, combinatorial=False)
    out["c2"] = {"envs_per_gpu": 4096, "agents": N, "channels": 4, "env_steps_per_s": rate * world,
                 "env_steps_per_s_graph": rate_g * world,
                 "env_kernel": roof, "d2d_iteration_s": it_s, "fused_update": fused, "phase_ms": phases,
                 "d2d_env_steps_per_s_end_to_end": 4096 * world * args.episode_length / it_s}
    del env
    sweep = []
    for N in (8, 16, 32, 64, 128, 256):
        p5 = dict(n_agents=N, n_channels=8, deadlines=np.full(N, 7), lbdas=np.full(N, 1 / 14), period=None,
                  arrival_probs=None, offsets=None, episode_length=args.episode_length, traffic_model="aperiodic",
                  periodic_devices=[], channel_switch=np.ones((N, 8)) * 0.8)
        env = CombinatorialEnv(**p5, n_envs=4096, device=dev, seed=22)
        env.shard(rank, world)
        # comb B_as = 6D + 11C = 130 B at D = 7, C = 8 (fp32 obs rows)
        rate, roof = _env_rate(env, bytes_per_agent_step=6 * 7 + 11 * 8)
        rate_g = _env_rate_graph(env)
        it_s, fused, phases = _d2d_iteration(env, 5, combinatorial=True)
        sweep.append({"agents": N, "env_steps_per_s": rate * world, "agent_steps_per_s": rate * world * N,
                      "env_steps_per_s_graph": rate_g * world,
                      "env_kernel": roof, "d2d_iteration_s": it_s, "fused_update": fused, "phase_ms": phases})
        del env
        torch.cuda.empty_cache()
    out["c5"] = {"envs_per_gpu": 4096, "channels": 8, "sweep": sweep}
    return out


def d2denv_leg(args, rank, world, local):
    """D2DEnv (envs/env.py): 64 agents on one shared channel, ring
    neighbourhoods {k-1, k, k+1} (obs = 3 buffers + 3 channel bits + ack = 25 floats), deadlines 7,
    lambda 1/14 aperiodic, switch 0.2, `--envs` envs per GPU.  Env-step rate with device-sampled
    Bernoulli(0.05) attempts, the single_kernel's HIP-event time against its algorithmic bytes, and
    one iPPO iteration (4 epochs) at 4,096 envs."""
    from envs.env import D2DEnv
    N, d = 64, 7
    nb = [[(k - 1) % N, k, (k + 1) % N] for k in range(N)]
    p = dict(n_agents=N, deadlines=np.full(N, d), lbdas=np.full(N, 1 / 14), episode_length=args.episode_length,
             channel_switch=0.2, neighbourhoods=nb)
    env = D2DEnv(**p, n_envs=args.envs, device=f"cuda:{local}", seed=31)
    env.shard(rank, world)
    b = env.batch()
    s = b.spec
    act = b.action_buffer()
    from d2dhip._lib import record_bytes
    rec = b.record_buffer(())

    def run(record):
        out_obs = rec if record else None
        b.reset(want_obs=True, out_obs=out_obs)
        for _ in range(10):
            b.sample_actions(0.05, out=act)
            b.step(act, want_obs=True, out_obs=out_obs)
        steps = 100
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            if b.timestep >= env.episode_length:
                b.reset(want_obs=True, out_obs=out_obs)
            b.sample_actions(0.05, out=act)
            evs[i][0].record()
            b.step(act, want_obs=True, out_obs=out_obs)
            evs[i][1].record()
        torch.cuda.synchronize()
        wall = max_over_ranks(time.perf_counter() - t0, world)
        kern_ms = max_over_ranks(float(np.mean([a.elapsed_time(bb) for a, bb in evs])), world)
        # algorithmic bytes of one launch: per agent row r+w (buffers 4*DW, channel 1, received 4, discarded 4),
        # the action byte and the obs row (fp32: 4F; the record: record_bytes(F)); per env the reward and the two
        # counters (r+w)
        per_agent = 2 * (4 * s.DW + 1 + 8) + 1 + (record_bytes(s.F) if record else 4 * s.F)
        per_env = 4 + 16
        bytes_launch = (per_agent * N + per_env) * b.E
        achieved = bytes_launch / (kern_ms / 1e3) / 1e9
        return {"env_steps_per_s": args.envs * world * steps / wall, "kernel_avg_us": kern_ms * 1e3,
                "bytes_per_launch": bytes_launch, "achieved_GBps": achieved, "hbm_frac": achieved / HBM_PEAK_GBS}

    # --d2denv-env-only with --env-mode fp32 / record: one obs format only, so that every single_kernel dispatch of a
    # PMC pass is that format's --envs launch (tools/gpu/profile_single.sh)
    only = args.env_mode if args.d2denv_env_only and args.env_mode != "both" else None
    f32 = run(False) if only != "record" else {}
    recd = run(True) if only != "fp32" else {}
    del env, b, act, rec
    torch.cuda.empty_cache()
    out = {"agents": N, "envs_per_gpu": args.envs, "obs_dim": s.F, "neighbourhood": "ring {k-1,k,k+1}",
           "kernel": "d2d::single_kernel<2, false>", **f32,
           "record": dict(recd, what="the same steps emitting the compact obs record the learners consume (ABI 14: "
                                     f"{record_bytes(s.F)} B per agent-step instead of {4 * s.F} B of fp32 rows)")}

    def traffic(name):
        pmc, rel = load_profile_json(name)
        if pmc and pmc.get("envs") == args.envs and pmc.get("agents") == N:
            return {"bytes_per_launch": pmc.get("bytes_per_launch"),
                    "traffic_over_algorithmic": pmc.get("traffic_over_algorithmic"), "file": rel,
                    "commit": pmc.get("commit")}
        return None
    t32, trec = traffic("pmc_traffic_single.json"), traffic("pmc_traffic_single_record.json")
    if t32:
        out["traffic"] = t32
    if trec:
        out["record"]["traffic"] = trec
    if args.d2denv_env_only:  # PMC passes: every single_kernel dispatch is a --envs launch
        return out
    from algorithms.ippo import iPPO
    env = D2DEnv(**p, n_envs=4096, device=f"cuda:{local}", seed=32)
    env.shard(rank, world)
    torch.manual_seed(3)
    lr = iPPO(env, hidden_size=64, gamma=0.4, policy_lr=3e-4, value_lr=1e-3, device=env.batch().device,
              early_stopping=False)

    def it(ne):
        ro = lr._rollout(4096)
        upd = lr._update_state(ro)
        for _ in range(ne):
            lr._update_epoch(ro, upd)

    it(1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    it(4)
    torch.cuda.synchronize()
    it_s = max_over_ranks(time.perf_counter() - t1, world)
    out.update({"ippo_iteration_s_4096_envs": it_s, "fused_update": bool(lr._fused_update_ok()),
                "ippo_env_steps_per_s_end_to_end": 4096 * world * args.episode_length / it_s})
    del env, lr
    torch.cuda.empty_cache()
    return out


def gru_leg(args, rank, world, local):
    """xp_load.py's learner (D2D-PPO with GRU policies, hidden 64, history_len = n_agents = 64,
    xp_load.py:78-89) on the configs[2] env (64 agents x 8 channels):
      (1) one behaviour-policy slot at the full --envs batch: the GRU window kernel over a full 64-step
          window (slot 63 of the episode) for every agent of every env, sampling + log-probs;
      (2) the BPTT update kernel (PPO.train_step's evaluate + loss + backward through the padded
          training windows) over a 200-slot rollout of --gru-envs envs;
      (3) one whole D2D-PPO iteration (rollout + 5 epochs) at --gru-envs envs.
    Roofline: the update kernel computes in v_mfma_f32_16x16x4_f32 (fraction of the fp32 MFMA
    peak); the policy kernel's step runs v_mfma_f32_16x16x32_bf16 on exact three-way splits, so its
    algorithmic rate is reported beside the MFMA pipe's busy fraction (its static instruction mix:
    per 16-sample tile and window step 12 gate tiles x (3 input + 2 chunks x 6 recurrent) bf16 MFMAs
    of 16 cycles, plus the head's 80 fp32 MFMAs of 32 cycles once per window).  Algorithmic FLOP per
    agent-sample and window step: GRU cell 2*3H*(F+1) + 2*3H*H (input + recurrent products); the
    update counts the forward and the two backward products (dW, dh) of every step: 3x that."""
    from algorithms.d2d_ppo import D2DPPO
    from d2dhip import gru
    from envs.combinatorial_env import CombinatorialEnv
    params = config3_params(args.episode_length)
    N, H, L = params["n_agents"], 64, params["n_agents"]
    dev = f"cuda:{local}"
    E = args.envs
    env = CombinatorialEnv(**params, n_envs=E, device=dev, seed=51)
    env.shard(rank, world)
    b = env.batch()
    torch.manual_seed(5)
    lr = D2DPPO(env, hidden_size=H, gamma=0.6, policy_lr=3e-4, value_lr=1e-3, device=dev, useRNN=True,
                combinatorial=True, history_len=L, early_stopping=False)
    assert lr._gru_ok()
    F = b.spec.F
    # 64 real env slots of obs (random attempts) = the window of slot 63
    buf = torch.empty((L, E, N, F), dtype=torch.float32, device=dev)
    act = b.action_buffer()
    b.reset(want_obs=True, out_obs=buf[0])
    for i in range(1, L):
        b.sample_actions(0.1, out=act)
        b.step(act, want_obs=True, out_obs=buf[i])
    pp = {k: v.data for k, v in lr.policy.params.items()}
    logp = torch.empty((N, E), dtype=torch.float32, device=dev)
    acts = torch.empty((1, E, N), dtype=act.dtype, device=dev)

    def slot():
        gru.policy(pp, buf, "sigmoid", L, args.episode_length, L - 1, 1, rng_step=7, seed=3, actions_out=acts,
                   out=logp)

    slot()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record()
    for _ in range(3):
        slot()
    ev[1].record()
    torch.cuda.synchronize()
    pol_ms = max_over_ranks(ev[0].elapsed_time(ev[1]) / 3, world)
    cell = 2 * 3 * H * (F + 1) + 2 * 3 * H * H
    head = 2 * (H * H + H * 8)
    pol_flop = (L * cell + head) * E * N
    pol_tiles = (E + 15) // 16 * N
    pol_pipe = pol_tiles * (L * 12 * (3 + 2 * 6) * 16 + 80 * 32) / (1024 * 2.4e9) / (pol_ms / 1e3)
    del buf, lr, env, b
    torch.cuda.empty_cache()
    slot_out = {"envs_per_gpu": E, "window": L, "ms": pol_ms, "agent_steps_per_s": E * world * N / (pol_ms / 1e3),
                "env_steps_per_s": E * world / (pol_ms / 1e3), "flop": pol_flop,
                "algorithmic_gflops": pol_flop / (pol_ms / 1e3) / 1e9, "mfma_pipe_busy_frac_static": pol_pipe}
    if args.gru_slot_only:
        return {"policy_slot": slot_out}
    # (2) + (3) at --gru-envs envs
    E2 = args.gru_envs
    env = CombinatorialEnv(**params, n_envs=E2, device=dev, seed=52)
    env.shard(rank, world)
    torch.manual_seed(6)
    np.random.seed(6)
    lr = D2DPPO(env, hidden_size=H, gamma=0.6, policy_lr=3e-4, value_lr=1e-3, device=dev, useRNN=True,
                combinatorial=True, history_len=L, early_stopping=False)
    ro = lr._rollout(E2)
    pp = {k: v.data for k, v in lr.policy.params.items()}
    W = torch.randn((ro.T, E2, N), device=dev)
    gbuf = {k: torch.empty_like(v) for k, v in pp.items()}
    args_g = (pp, ro.obs, "sigmoid", L, ro.L, W)
    gru.grads(*args_g, actions=ro.actions, logp_old=ro.logp.permute(0, 2, 1), grads=gbuf)
    torch.cuda.synchronize()
    ev[2].record()
    gru.grads(*args_g, actions=ro.actions, logp_old=ro.logp.permute(0, 2, 1), grads=gbuf)
    ev[3].record()
    torch.cuda.synchronize()
    grad_ms = max_over_ranks(ev[2].elapsed_time(ev[3]), world)
    samples = ro.T * E2 * N
    grad_flop = 3 * L * cell * samples + 3 * head * samples
    # one untimed iteration first: the first update epochs of a process pay one-time host costs
    # (kernel loads, hipBLASLt solution lookup for the central critic, allocator growth) of ~0.5-1 s
    ro = lr._rollout(E2)
    for _ in range(5):
        lr._update_epoch(ro, lr._update_state(ro))
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    ro = lr._rollout(E2)
    for _ in range(5):
        lr._update_epoch(ro, lr._update_state(ro))
    torch.cuda.synchronize()
    it_s = max_over_ranks(time.perf_counter() - t0, world)
    it_ = 1 if F + 1 <= 16 else 2 if F + 1 <= 32 else 3 if F + 1 <= 48 else 4
    # the policy step runs bf16 MFMAs on exact splits (its fp32-equivalent rate is no roofline: the
    # roofline figure is the executed MFMA pipe's busy fraction); the update's products are fp32 MFMAs
    out = {"config": f"xp_load.py learner: D2D-PPO, GRU H={H}, history_len={L}, {N} agents x 8 channels",
           "policy_slot": {"envs_per_gpu": E, "window": L,
                           "kernel": f"d2d::gru_policy_kernel<4, {2 if it_ <= 2 else 4}, 0, 0, {'true' if it_ <= 2 else 'false'}>",
                           "ms": pol_ms, "agent_steps_per_s": E * world * N / (pol_ms / 1e3),
                           "env_steps_per_s": E * world / (pol_ms / 1e3),
                           "flop": pol_flop, "algorithmic_gflops": pol_flop / (pol_ms / 1e3) / 1e9,
                           "mfma_pipe_busy_frac_static": pol_pipe, "mfma_pmc": pmc_mfma("d2d::gru_policy_kernel", "gru_slot"),
                           "bound": "mfma"},
           "update": {"envs_per_gpu": E2, "slots": ro.T, "agent_samples": samples,
                      "kernel": (f"d2d::gru_grad_kernel<4, {it_}, 0, true, true, {'true' if L > 64 else 'false'}>" if it_ <= 3
                                 else f"d2d::gru_grad_kernel<4, {it_}, 0, true, false, false>"),
                      "weight_gradients": "cooperative LDS exchange" if it_ <= 3 else "per-wave global row history",
                      "ms": grad_ms,
                      "agent_samples_per_s": samples * world / (grad_ms / 1e3), "flop": grad_flop,
                      # the products run as bf16 MFMAs on exact / two-way splits: an fp32-equivalent rate is
                      # no headroom figure (it is not bounded by the fp32 MFMA peak) -- the executed pipe's
                      # utilisation is mfma_pmc.mfma_busy_frac_pmc; the algorithmic rate is in GFLOP/s
                      "algorithmic_gflops": grad_flop / (grad_ms / 1e3) / 1e9,
                      "mfma_pmc": pmc_mfma("d2d::gru_grad_kernel", "gru")},
           "d2d_iteration_s": it_s, "d2d_iteration_envs_per_gpu": E2, "n_epoch": 5,
           "d2d_env_steps_per_s_end_to_end": E2 * world * ro.T / it_s,
           "flop_per_agent_step_cell": cell}
    del lr, env, ro
    torch.cuda.empty_cache()
    return out


def gru_c5_leg(args, rank, world, local):
    """configs[4] as xp_n_agents.py writes its learner (xp_n_agents.py:98-112): D2D-PPO with GRU policies,
    hidden 64, gamma 0.4, history_len = n_agents, on the c5 env (N agents x 8 channels, deadlines 7, switch 0.8,
    lambda 1/14 aperiodic) at --gru-c5-envs envs per GPU.  Per N: one 200-slot training rollout (GRU window
    kernel per slot + env kernel), one D2D-PPO epoch (central critic, GAE, the forced log-prob pass over the
    padded training windows, the chain, the GRU BPTT update of all N actors, Adam) and one whole iteration
    with n_epoch = 1; iteration_s = rollout + GAE + 5 epochs is the n_epoch = 5 iteration (xp_n_agents.py:110)
    assembled from the measured parts (an epoch's cost does not depend on the epoch index after the first)."""
    from algorithms.d2d_ppo import D2DPPO
    from envs.combinatorial_env import CombinatorialEnv
    dev = f"cuda:{local}"
    E = args.gru_c5_envs
    sweep = []
    for N in [int(x) for x in args.gru_c5_agents.split(",") if x]:
        p5 = dict(n_agents=N, n_channels=8, deadlines=np.full(N, 7), lbdas=np.full(N, 1 / 14), period=None,
                  arrival_probs=None, offsets=None, episode_length=args.episode_length, traffic_model="aperiodic",
                  periodic_devices=[], channel_switch=np.ones((N, 8)) * 0.8)
        env = CombinatorialEnv(**p5, n_envs=E, device=dev, seed=60 + N)
        env.shard(rank, world)
        torch.manual_seed(7)
        np.random.seed(7)
        lr = D2DPPO(env, hidden_size=64, gamma=0.4, policy_lr=3e-4, value_lr=1e-3, beta_entropy=0.01, device=dev,
                    useRNN=True, combinatorial=True, history_len=N, early_stopping=False)
        gru_ok = bool(lr._gru_ok())
        # warm-up: one rollout and one epoch (kernel loads, hipBLASLt heuristics, allocator growth)
        tw = time.perf_counter()
        ro = lr._rollout(E)
        lr._update_epoch(ro, lr._update_state(ro))
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench gru_c5] N={N} E={E}: warm-up rollout + epoch {time.perf_counter() - tw:.1f} s",
                  file=sys.stderr, flush=True)
        barrier(world)
        t0 = time.perf_counter()
        ro = lr._rollout(E)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        upd = lr._update_state(ro)
        lr._update_epoch(ro, upd)     # epoch 1 (its forced log-prob pass included: no first-epoch shortcut on GRU)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        lr.phase_timer = PhaseTimer()
        lr._update_epoch(ro, upd)     # epoch 2 (with its phase split: the forced pass is in "chain")
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        ep_phases = {k: max_over_ranks(v, world) for k, v in lr.phase_timer.totals_ms().items()}
        lr.phase_timer = None
        barrier(world)
        if rank == 0:
            print(f"[bench gru_c5] N={N}: rollout {t1 - t0:.2f} s, epochs {t2 - t1:.2f} / {t3 - t2:.2f} s",
                  file=sys.stderr, flush=True)
        roll = max_over_ranks(t1 - t0, world)
        ep1 = max_over_ranks(t2 - t1, world)
        ep = max_over_ranks(t3 - t2, world)
        samples = ro.T * E * world * N
        sweep.append({"agents": N, "history_len": N, "envs_per_gpu": E, "gru_kernels": gru_ok,
                      "rollout_s": roll, "rollout_env_steps_per_s": E * world * ro.T / roll,
                      "epoch_s": ep, "epoch_phase_ms": ep_phases, "first_epoch_s": ep1, "agent_samples_per_epoch": samples,
                      "update_agent_samples_per_s": samples / ep,
                      "iteration_s": roll + ep1 + 4 * ep,
                      "iteration_env_steps_per_s_end_to_end": E * world * ro.T / (roll + ep1 + 4 * ep)})
        del lr, env, ro, upd
        torch.cuda.empty_cache()
    return {"config": "xp_n_agents.py learner: D2D-PPO, GRU H=64, history_len = n_agents, gamma 0.4, "
                      "beta_entropy 0.01 (xp_n_agents.py:98-112), n_epoch = 5",
            "what": "per N: measured rollout (200 slots), first and second epoch; iteration_s = rollout + first epoch "
                    "+ 4 x second epoch (the n_epoch = 5 iteration from its measured parts)",
            "sweep": sweep}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--episode-length", type=int, default=200)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--legs", default="env,rollout,ppo,train,configs,d2denv,gru,gru_c5")
    ap.add_argument("--gru-c5-envs", type=int, default=512,
                    help="envs per GPU of the c5 GRU leg (512 x 256 agents = 131,072 GRU windows per slot fill the "
                         "chip; the O(L H^2) BPTT at L = 256 makes a 4,096-env epoch minutes long)")
    ap.add_argument("--gru-c5-agents", default="64,128,256", help="agent counts of the c5 GRU leg")
    ap.add_argument("--gru-envs", type=int, default=256, help="envs per GPU in the GRU update / iteration")
    ap.add_argument("--gru-slot-only", action="store_true", help="gru leg: the 65,536-env policy slot only (PMC passes)")
    ap.add_argument("--d2denv-env-only", action="store_true", help="d2denv leg: the env steps only (PMC passes)")
    ap.add_argument("--rollout-steps", type=int, default=60)
    ap.add_argument("--ppo-envs", type=int, default=2048, help="envs per GPU in the PPO-update rollout")
    ap.add_argument("--ppo-epochs", type=int, default=6)
    ap.add_argument("--train-epochs", type=int, default=4, help="n_epoch of the train leg")
    ap.add_argument("--action-ring", type=int, default=2, help="distinct pre-generated synthetic action slots")
    ap.add_argument("--env-mode", default="both", choices=["both", "record", "fp32"],
                    help="obs output of the headline env steps (value = the first of record, fp32)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the ranks here, before anything touches the GPU
        sys.exit(self_launch(args.gpus))

    params = config3_params(args.episode_length)
    world0 = int(os.environ.get("WORLD_SIZE", "1"))
    cpu = None
    if not args.no_cpu_baseline and world0 == 1:
        # before any GPU call: the NumPy leg forks one worker per host core
        cpu = cpu_baseline_numpy(params, seconds=args.cpu_seconds)
        cpu["c_openmp"] = cpu_baseline_c(params, seconds=args.cpu_seconds)

    rank, world, local, ranks_seen = setup_dist(args.gpus)
    from envs.combinatorial_env import CombinatorialEnv

    E = args.envs
    env = CombinatorialEnv(**params, n_envs=E, device=f"cuda:{local}", seed=42)
    env.shard(rank, world)
    b = env.batch()
    N, C = params["n_agents"], params["n_channels"]
    act = b.action_buffer()
    K = args.steps

    # The synthetic actions are inputs of the env step (the policy's output in a rollout): generated
    # on the device BEFORE the timed region (Philox Bernoulli(0.1) per agent-channel, a ring of
    # --action-ring distinct slots, 4 MB each at 65,536 envs), so the timed region is the env step alone
    # with its inputs resident in HBM.  The in-loop variant (sampler + env kernel per step, rounds 1-2)
    # is reported beside it as `with_inloop_action_sampling`.
    ring = max(1, min(K, args.action_ring))
    acts = torch.empty((ring,) + tuple(act.shape), dtype=act.dtype, device=act.device)
    for i in range(ring):
        b.sample_actions(0.1, out=acts[i])
    torch.cuda.synchronize()

    def env_phase(mode, inloop=False):
        """warmup + K timed steps emitting the record ('record') or fp32 obs rows ('fp32')."""
        out = b.record if mode == "record" else b.obs
        step_i = [0]

        def one_step(ev=None):
            if b.timestep >= params["episode_length"]:
                b.reset(want_obs=True, out_obs=out)
            if inloop:
                b.sample_actions(0.1, out=act)
                a_t = act
            else:
                a_t = acts[step_i[0] % ring]
                step_i[0] += 1
            if ev is not None:
                ev[0].record()
            b.step(a_t, want_obs=True, out_obs=out)
            if ev is not None:
                ev[1].record()

        b.reset(want_obs=True, out_obs=out)
        for _ in range(args.warmup):
            one_step()
        step_i[0] = 0
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        t_start, t_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        barrier(world)
        torch.cuda.synchronize()
        w0 = time.perf_counter()
        t_start.record()
        for i in range(K):
            one_step(evs[i])
        t_end.record()
        torch.cuda.synchronize()
        barrier(world)
        wall = time.perf_counter() - w0
        gpu_s = t_start.elapsed_time(t_end) / 1e3
        kern_ms = np.array([a.elapsed_time(bb) for a, bb in evs])
        t = max_over_ranks(max(wall, gpu_s), world)
        kern_avg_ms = max_over_ranks(float(kern_ms.mean()), world)
        bpas = RECORD_BYTES_PER_AGENT_STEP if mode == "record" else BYTES_PER_AGENT_STEP
        bytes_per_launch = bpas * N * E
        achieved = bytes_per_launch / (kern_avg_ms / 1e3) / 1e9
        pmc, pmc_rel = load_pmc_traffic(mode)
        traffic = src = None
        # the committed PMC profile applies only to the very workload it measured
        if pmc and pmc.get("kernel_prefix") and pmc.get("envs") == E and pmc.get("agents") == N:
            traffic = pmc.get("bytes_per_launch")
            src = {"file": pmc_rel, "commit": pmc.get("commit"), "rocprofv3": pmc.get("source"),
                   "traffic_over_algorithmic": pmc.get("traffic_over_algorithmic")}
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
                "kernel": env_kernel_name(b.spec, mode == "record"), "kernel_avg_us": kern_avg_ms * 1e3,
                "bytes_per_launch": bytes_per_launch, "bytes_per_agent_step": bpas}
        return total_envs * K / t, t, roof

    total_envs = E * world
    modes = ["record", "fp32"] if args.env_mode == "both" else [args.env_mode]
    env_res = {m: env_phase(m) for m in modes}
    env_steps_per_s, t, roofline = env_res[modes[0]]
    vi, ti, _ = env_phase(modes[0], inloop=True)
    inloop = {"env_steps_per_s": vi, "ms_per_step": ti / K * 1e3,
              "what": "the same K steps with the synthetic actions sampled on the device inside the timed loop "
                      "(sample_actions_kernel + env kernel per step; the rounds 1-2 `value` definition)"}
    fp32_obs = None
    if len(modes) > 1:
        v32, t32, r32 = env_res["fp32"]
        fp32_obs = {"env_steps_per_s": v32, "agent_steps_per_s": v32 * N, "ms_per_step": t32 / K * 1e3,
                    "roofline": r32,
                    "what": "the same K steps emitting fp32 obs rows [E][N][F] (the reference-API layout)"}

    legs = set(args.legs.split(","))
    rollout = ppo = None
    if "rollout" in legs:
        rollout = rollout_leg(env, args, world)
    if "ppo" in legs:
        ppo = ppo_leg(args, rank, world, local)
    train = train_leg(env, args, rank, world, local) if "train" in legs else None
    configs = configs_leg(args, rank, world, local) if "configs" in legs else None
    d2denv = d2denv_leg(args, rank, world, local) if "d2denv" in legs else None
    gru_res = gru_leg(args, rank, world, local) if "gru" in legs else None
    gru_c5 = gru_c5_leg(args, rank, world, local) if "gru_c5" in legs else None

    if rank == 0:
        res = {
            "metric": METRIC,
            "value": env_steps_per_s,
            "unit": "env-steps/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "dist_backend": dist.get_backend() if world > 1 else None,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": t / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "obs_format": modes[0],
            "data": "synthetic (Philox actions/channels/arrivals; reference channel_switch_8 tiled to 64 agents)",
            "config": {"workload": f"combinatorial_env {N} agents x {C} channels, {E} envs per GPU"
                                   + (" (BASELINE.json configs[2])" if (N, C, E) == (64, 8, 65536) else
                                      " (NOT the BASELINE.json configs[2] batch)")
                                   + "; step = one env-step kernel launch (reset when the episode ends) on "
                                   + "pre-generated synthetic actions, emitting "
                                   + ("the compact obs record" if modes[0] == "record" else "fp32 obs rows")
                                   + " (in-loop action sampling: with_inloop_action_sampling)",
                       "agents": N, "channels": C, "envs_per_gpu": E, "global_envs": total_envs,
                       "episode_length": args.episode_length, "parallelism": f"dp{world} (env shards, no collective)",
                       "actions": f"synthetic Bernoulli(0.1) per agent-channel, {ring} device-resident slots generated "
                                  "before the timed region"},
            "agent_steps_per_s": env_steps_per_s * N,
            "roofline": roofline,
        }
        res["with_inloop_action_sampling"] = inloop
        if fp32_obs is not None:
            res["fp32_obs"] = fp32_obs
        if rollout is not None:
            res["rollout"] = rollout
        if ppo is not None:
            res["ppo"] = ppo
        if train is not None:
            res["train"] = train
        if configs is not None:
            res["configs"] = configs
        if d2denv is not None:
            res["d2denv"] = d2denv
        if gru_res is not None:
            res["gru"] = gru_res
        if gru_c5 is not None:
            res["gru_c5"] = gru_c5
        if cpu is not None:
            res["cpu_baseline"] = cpu
        # the metric's second half at the END of the line (the driver's record keeps the line's tail): PPO
        # updates/s at the --ppo-envs batch and at the headline batch, the whole training iteration
        if ppo is not None:
            res["ppo_updates_per_s"] = ppo["updates_per_s"]
            res["ppo_updates_per_s_batch"] = ppo["batch"]
        if train is not None:
            res["ppo_updates_per_s_headline_batch"] = train["ppo_updates_per_s"]
            res["train_s_per_iteration"] = train["s_per_iteration"]
            res["train_env_steps_per_s_end_to_end"] = train["env_steps_per_s_end_to_end"]
            res["train_phase_ms"] = train["phase_ms"]
        if gru_c5 is not None:
            res["c5_gru_summary"] = [{k: r[k] for k in ("agents", "rollout_s", "epoch_s", "iteration_s")}
                                     for r in gru_c5["sweep"]]
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
