"""Generate the golden fixtures in tests/golden/ from the reference itself.

Runs ONLY in the build container (it imports /root/reference through
tools/ref_import.py).  The outputs are plain .npz data: inputs (params,
actions), the random draws the reference made (recovered from its state
diffs, not by re-implementing its RNG), and every output of reset/step.

  python tools/gen_fixtures.py            # all fixtures
  python tools/gen_fixtures.py env gae    # subsets

Env fixtures record, per step s (reference envs/combinatorial_env.py:127-242,
envs/channel_selection_env.py:116-214):
  flips[s]     channel flip draw  = |H_after - H_before|      (comb: N x C, chsel: C+1)
  arrivals[s]  arrival draw       = B_after[k, d_k-1]          (0 when agent k drew nothing)
  obs[s]       per-agent obs, zero-padded to max length (obs_len holds the true lengths)
  state[s]     concatenated state vector
  rewards, done, ack, buffers, chan, received, discarded (+ chsel counters)
Each episode starts with a reset whose draws/outputs are in reset_* arrays.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from ref_import import ref_module  # noqa: E402
import safe_pickle  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")
DATA = "/root/reference/combinatorial_load"


def _jsonable(v):
    if isinstance(v, np.ndarray):
        return {"__nd__": v.tolist(), "dtype": str(v.dtype)}
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    return v


def env_configs():
    setup8 = safe_pickle.load(f"{DATA}/setup_8_channels.p")
    cs8 = safe_pickle.load(f"{DATA}/channel_switch_8.p")
    cfgs = []
    # (i) xp_load.py:60-75 plumbing, load 1/2
    load = 0.5
    cfgs.append(("comb_6x8_setup8", "comb", dict(
        n_agents=6, n_channels=8, deadlines=setup8["deadlines"], lbdas=np.array([load] * 6),
        period=np.array([int(1 / load)] * 6), arrival_probs=setup8["arrival_probs"],
        offsets=setup8["offsets"], episode_length=200, traffic_model="heterogeneous",
        homogeneous_size=True, periodic_devices=list(setup8["periodic_devices"]),
        channel_switch=setup8["channel_switch"]), 2, 0.15))
    # (ii) run_ippo_combinatorial.py:58-76 plumbing at 8 agents, 1-D channel_switch broadcast
    cfgs.append(("comb_8x8_ippo", "comb", dict(
        n_agents=8, n_channels=8, deadlines=np.array([7, 14] * 4), lbdas=np.array([1.0] * 8),
        period=np.array([1 / 1.0] * 8), arrival_probs=np.array([0.4, 0.8] * 4), offsets=np.zeros(8),
        episode_length=50, traffic_model="heterogeneous", periodic_devices=[0, 1],
        channel_switch=np.array([0.8] * 8)), 2, 0.2))
    # (iii) config-3 shape: 64 x 8, channel_switch_8 tiled (agent k uses row k mod 6)
    N = 64
    cfgs.append(("comb_64x8_tiled", "comb", dict(
        n_agents=N, n_channels=8, deadlines=np.array([7, 14] * (N // 2)), lbdas=np.array([0.5] * N),
        period=np.array([2] * N), arrival_probs=np.resize(np.array([.2, .4, .8, 1, 1, 1]), N),
        offsets=np.zeros(N), episode_length=50, traffic_model="heterogeneous", homogeneous_size=True,
        periodic_devices=[k for k in range(N) if k % 6 < 3], channel_switch=np.resize(cs8, (N, 8))), 1, 0.1))
    # (iv) xp_n_agents.py:62-83 (4 channels, deadlines 7, switch 0.8, lambda 1/14), plus a busier 16x8
    for n in (4, 12):
        cfgs.append((f"comb_{n}x4_xpnagents", "comb", dict(
            n_agents=n, n_channels=4, deadlines=np.array([7] * n), lbdas=np.array([1 / 14] * n),
            period=None, arrival_probs=None, offsets=None, episode_length=200, traffic_model="aperiodic",
            collision_type="pessimistic", periodic_devices=[], channel_switch=np.ones((n, 4)) * 0.8), 1, 0.3))
    cfgs.append(("comb_16x8_aperiodic", "comb", dict(
        n_agents=16, n_channels=8, deadlines=np.array([7] * 16), lbdas=np.array([0.6] * 16),
        episode_length=100, traffic_model="aperiodic", channel_switch=np.ones((16, 8)) * 0.8), 1, 0.12))
    # (vii) 'periodic' traffic model with a scalar period and staggered offsets; default channel_switch
    cfgs.append(("comb_4x3_periodic", "comb", dict(
        n_agents=4, n_channels=3, deadlines=np.array([3, 5, 4, 5]), lbdas=np.array([1.0] * 4), period=3,
        arrival_probs=np.array([1.0, 0.7, 0.5, 0.9]), offsets=np.array([0, 1, 2, 0]), episode_length=40,
        traffic_model="periodic"), 2, 0.5))
    # (viii) edge: single agent, single channel, heavy Poisson load (multi-packet cells)
    cfgs.append(("comb_1x1_heavy", "comb", dict(
        n_agents=1, n_channels=1, deadlines=np.array([3]), lbdas=np.array([2.5]), episode_length=30,
        traffic_model="aperiodic", channel_switch=np.array([[0.3]])), 2, 0.7))
    # (v) config-2 shape: channel selection 16 x 4, lambda 1/3.5, switch 0.8 on all 5 entries
    cfgs.append(("chsel_16x4", "chsel", dict(
        n_agents=16, n_channels=4, deadlines=np.array([7] * 16), lbdas=np.array([1 / 3.5] * 16),
        episode_length=100, traffic_model="aperiodic", channel_switch=np.array([0.8] * 5)), 2, None))
    # (vi) xp_gamma.py:33-54 parameters (5 x 16) with the heterogeneous model turned on
    cfgs.append(("chsel_5x16_het", "chsel", dict(
        n_agents=5, n_channels=16, deadlines=np.array([7] * 5), lbdas=np.array([1 / 3.5] * 5),
        period=np.array([7] * 5), arrival_probs=np.array([1] * 5), offsets=np.array([0, 2, 4, 0, 2]),
        episode_length=120, traffic_model="heterogeneous", periodic_devices=[2, 4],
        channel_switch=np.array([0.8] * 17)), 1, None))
    # edge: heterogeneous deadlines + heavy load on 2 channels
    cfgs.append(("chsel_6x2_mixed", "chsel", dict(
        n_agents=6, n_channels=2, deadlines=np.array([2, 5, 3, 7, 4, 6]), lbdas=np.array([0.9] * 6),
        episode_length=60, traffic_model="aperiodic", channel_switch=np.array([0.5, 0.3, 0.7])), 2, None))
    return cfgs


def run_env(name, kind, params, episodes, p_act, seed=42):
    mod = ref_module("envs.combinatorial_env" if kind == "comb" else "envs.channel_selection_env")
    cls = mod.CombinatorialEnv if kind == "comb" else mod.ChannelSelectionEnv
    env = cls(**params)
    N, C = env.n_agents, env.n_channels
    d = np.asarray(env.deadlines)
    D = int(d.max())
    homog = bool(params.get("homogeneous_size", False)) and kind == "comb"
    w = np.full(N, D) if homog else d.copy()
    F = (D + 2 * C) if kind == "comb" else (D + C + 1)
    obs_len = (w + 2 * C) if kind == "comb" else (d + C + 1)
    act_rng = np.random.default_rng(1234)
    np.random.seed(seed)

    def pad_obs(obs):
        out = np.zeros((N, F))
        for k in range(N):
            assert obs[k].shape[0] == obs_len[k]
            out[k, :obs_len[k]] = obs[k]
        return out

    rec = {k: [] for k in ["actions", "flips", "arrivals", "obs", "state", "rewards", "done", "ack", "buffers",
                           "chan", "received", "discarded", "sel_q", "sel_n", "success"]}
    rrec = {k: [] for k in ["arrivals", "obs", "state", "buffers", "chan", "received"]}
    metrics = {k: [] for k in ["jains", "urllc", "channel_score", "successful_transmissions"]}
    for ep in range(episodes):
        obs, state = env.reset()
        rrec["arrivals"].append(np.array([env.current_buffers[k, d[k] - 1] for k in range(N)]))
        rrec["obs"].append(pad_obs(obs))
        rrec["state"].append(np.concatenate(state))
        rrec["buffers"].append(env.current_buffers.copy())
        rrec["chan"].append(np.array(env.channel_state, dtype=np.float64).copy())
        rrec["received"].append(env.received_packets.copy())
        done = False
        t = 0
        while not done:
            if kind == "comb":
                p = p_act if t % 17 else 1.0  # every 17th step: everyone attempts every channel
                a = (act_rng.random((N, C)) < p).astype(np.float32)
                if t % 23 == 5:
                    a[:] = 0  # nobody attempts
            else:
                a = act_rng.integers(0, C + 1, size=N)
            H0 = np.array(env.channel_state, dtype=np.float64).copy()
            ltt0 = env.last_time_transmitted.copy()
            obs, state, rew, done, info = env.step(a)
            H1 = np.array(env.channel_state, dtype=np.float64).copy()
            rec["actions"].append(np.array(a))
            rec["flips"].append(np.abs(H1 - H0).astype(np.uint8))
            rec["arrivals"].append(np.array([env.current_buffers[k, d[k] - 1] for k in range(N)]))
            rec["obs"].append(pad_obs(obs))
            rec["state"].append(np.concatenate(state))
            rec["rewards"].append(np.asarray(rew))
            rec["done"].append(done)
            rec["ack"].append(np.array(env.last_feedback, dtype=np.float64))
            rec["buffers"].append(env.current_buffers.copy())
            rec["chan"].append(H1)
            rec["received"].append(env.received_packets.copy())
            rec["discarded"].append(env.discarded_packets.copy())
            rec["sel_q"].append(env.selected_channel_qualities)
            rec["sel_n"].append(env.number_selected_channel)
            rec["success"].append((env.last_time_transmitted == 1.0) & (ltt0 + 1 != 1.0))
            t += 1
        metrics["jains"].append(env.compute_jains())
        metrics["urllc"].append(env.compute_urllc())
        metrics["channel_score"].append(env.compute_channel_score())
        metrics["successful_transmissions"].append(env.successful_transmissions)
    out = {"params_json": json.dumps({k: _jsonable(v) for k, v in params.items()}), "kind": kind,
           "episodes": episodes, "obs_len": obs_len, "state_dim": env.state_space.shape[0],
           "obs_dims": np.array([env.observation_space[k].shape[0] for k in range(N)]),
           "action_n": np.array([env.action_space[k].n for k in range(N)])}
    for k, v in rec.items():
        out[k] = np.array(v)
    for k, v in rrec.items():
        out["reset_" + k] = np.array(v)
    for k, v in metrics.items():
        out["metric_" + k] = np.array(v)
    # compact dtypes (values are small integers except obs/state/ack in chsel)
    for k in ("buffers", "reset_buffers"):
        assert out[k].max() < 256
        out[k] = out[k].astype(np.uint8)
    for k in ("arrivals", "reset_arrivals"):
        out[k] = out[k].astype(np.uint8)
    out["actions"] = out["actions"].astype(np.uint8 if kind == "comb" else np.int64)
    out["chan"] = out["chan"].astype(np.uint8)
    out["reset_chan"] = out["reset_chan"].astype(np.uint8)
    if kind == "comb":
        out["obs"] = out["obs"].astype(np.float32)
        out["reset_obs"] = out["reset_obs"].astype(np.float32)
        out["state"] = out["state"].astype(np.float32)
        out["reset_state"] = out["reset_state"].astype(np.float32)
        assert np.all(out["ack"] == np.round(out["ack"]))
        out["ack"] = out["ack"].astype(np.int8)
    np.savez_compressed(os.path.join(OUT, f"env_{name}.npz"), **out)
    print(f"env_{name}: steps={len(rec['done'])} reward_sum={out['rewards'][:, 0].sum()} "
          f"urllc={metrics['urllc']}")


def gen_env():
    for name, kind, params, episodes, p_act in env_configs():
        run_env(name, kind, params, episodes, p_act)


def d2denv_configs():
    """D2DEnv (envs/env.py) cases: test.ipynb cell 5, a busier one with full neighbourhoods and
    channel flips, ring neighbourhoods with mixed deadlines, the heterogeneous and periodic
    traffic models, a single agent."""
    ring = lambda n: [[(k - 1) % n, k, (k + 1) % n] for k in range(n)]  # noqa: E731
    return [
        ("4_notebook", dict(n_agents=4, deadlines=np.array([7] * 4), lbdas=np.array([1 / 14] * 4), period=None,
                            arrival_probs=None, offsets=None, episode_length=200, traffic_model="aperiodic",
                            periodic_devices=[], reward_type=0, channel_switch=0, channel_decoding=1.,
                            neighbourhoods=[[i] for i in range(4)]), 2, 0.3),
        ("6_full_nbr", dict(n_agents=6, deadlines=np.array([4, 7, 5, 7, 3, 6]), lbdas=np.array([0.4] * 6),
                            episode_length=80, traffic_model="aperiodic", channel_switch=0.3,
                            neighbourhoods=[list(range(6)) for _ in range(6)]), 2, 0.25),
        ("8_ring_het", dict(n_agents=8, deadlines=np.array([7, 3, 5, 7, 2, 6, 7, 4]), lbdas=np.array([0.6] * 8),
                            period=np.array([2, 3, 2, 3, 2, 3, 2, 3]), arrival_probs=np.array([0.9, 0.5] * 4),
                            offsets=np.array([0, 1, 0, 2, 1, 0, 0, 1]), episode_length=60,
                            traffic_model="heterogeneous", periodic_devices=[1, 3, 5],
                            channel_switch=np.array([0.1, 0.5, 0.2, 0.3, 0.05, 0.4, 0.25, 0.15]),
                            neighbourhoods=ring(8)), 2, 0.2),
        ("5_periodic", dict(n_agents=5, deadlines=np.array([5] * 5), lbdas=np.array([1.0] * 5), period=3,
                            arrival_probs=np.array([1.0, 0.7, 0.5, 0.9, 0.8]), offsets=np.array([0, 1, 2, 0, 1]),
                            episode_length=40, traffic_model="periodic", channel_switch=0.2,
                            neighbourhoods=[[0, 4], [1, 0], [2], [3, 2, 1], [4, 3]]), 2, 0.35),
        ("1_single", dict(n_agents=1, deadlines=np.array([3]), lbdas=np.array([1.5]), episode_length=30,
                          traffic_model="aperiodic", channel_switch=0.4), 2, 0.6),
    ]


def run_d2denv(name, params, episodes, p_act, seed=42):
    """Record a D2DEnv trace (envs/env.py).  Draws recovered from state diffs: the channel flip
    mask |H_after - H_before| and the arrivals B_after[k, d_k - 1]; the decode draw needs no
    record (the channel state is 0/1, so binomial(1, state) is the state, env.py:101-103)."""
    mod = ref_module("envs.env")
    env = mod.D2DEnv(**params)
    N = env.n_agents
    d = np.asarray(env.deadlines)
    nbr = env.neighbourhoods
    obs_len = np.array([int(d[nb].sum()) + len(nb) + 1 for nb in nbr])
    F = int(obs_len.max())
    act_rng = np.random.default_rng(4321)
    np.random.seed(seed)

    def pad_obs(obs):
        out = np.zeros((N, F))
        for k in range(N):
            assert obs[k].shape[0] == obs_len[k]
            out[k, :obs_len[k]] = obs[k]
        return out

    rec = {k: [] for k in ["actions", "flips", "arrivals", "obs", "state", "rewards", "done", "ack", "buffers",
                           "chan", "received", "discarded", "channel_errors", "n_collisions", "success"]}
    rrec = {k: [] for k in ["arrivals", "obs", "state", "buffers", "chan", "received"]}
    metrics = {k: [] for k in ["jains", "urllc", "successful_transmissions", "channel_errors", "n_collisions"]}
    for ep in range(episodes):
        obs, state = env.reset()
        rrec["arrivals"].append(np.array([env.current_buffers[k, d[k] - 1] for k in range(N)]))
        rrec["obs"].append(pad_obs(obs))
        rrec["state"].append(np.asarray(state, dtype=np.float64))
        rrec["buffers"].append(env.current_buffers.copy())
        rrec["chan"].append(np.array(env.channel_state, dtype=np.float64).copy())
        rrec["received"].append(env.received_packets.copy())
        done = False
        t = 0
        while not done:
            p = p_act if t % 13 else 1.0        # every 13th step: everyone attempts (collisions)
            a = (act_rng.random(N) < p).astype(np.int64)
            if t % 19 == 4:
                a[:] = 0                         # nobody attempts
            if t % 7 == 3:
                a[:] = 0
                a[act_rng.integers(0, N)] = 1    # exactly one attempt (decode / channel error)
            H0 = np.array(env.channel_state, dtype=np.float64).copy()
            ltt0 = env.last_time_transmitted.copy()
            obs, state, rew, done, info = env.step(a)
            H1 = np.array(env.channel_state, dtype=np.float64).copy()
            rec["actions"].append(a)
            rec["flips"].append(np.abs(H1 - H0).astype(np.uint8))
            rec["arrivals"].append(np.array([env.current_buffers[k, d[k] - 1] for k in range(N)]))
            rec["obs"].append(pad_obs(obs))
            rec["state"].append(np.asarray(state, dtype=np.float64))
            rec["rewards"].append(np.asarray(rew, dtype=np.float64))
            rec["done"].append(done)
            rec["ack"].append(float(env.last_feedback))
            rec["buffers"].append(env.current_buffers.copy())
            rec["chan"].append(H1)
            rec["received"].append(env.received_packets.copy())
            rec["discarded"].append(env.discarded_packets.copy())
            rec["channel_errors"].append(env.channel_errors)
            rec["n_collisions"].append(env.n_collisions)
            rec["success"].append((env.last_time_transmitted == 1.0) & (ltt0 + 1 != 1.0))
            t += 1
        metrics["jains"].append(env.compute_jains())
        metrics["urllc"].append(env.compute_urllc())
        metrics["successful_transmissions"].append(env.successful_transmissions)
        metrics["channel_errors"].append(env.channel_errors)
        metrics["n_collisions"].append(env.n_collisions)
    out = {"params_json": json.dumps({k: _jsonable(v) for k, v in params.items()}), "kind": "single",
           "episodes": episodes, "obs_len": obs_len, "state_dim": env.state_space.shape[0],
           "obs_dims": np.array([env.observation_space[k].shape[0] for k in range(N)]),
           "action_n": np.array([env.action_space[k].n for k in range(N)])}
    for k, v in rec.items():
        out[k] = np.array(v)
    for k, v in rrec.items():
        out["reset_" + k] = np.array(v)
    for k, v in metrics.items():
        out["metric_" + k] = np.array(v)
    for k in ("buffers", "reset_buffers", "arrivals", "reset_arrivals"):
        assert out[k].max() < 256
        out[k] = out[k].astype(np.uint8)
    for k in ("chan", "reset_chan", "actions"):
        out[k] = out[k].astype(np.uint8)
    for k in ("obs", "reset_obs", "state", "reset_state"):
        out[k] = out[k].astype(np.float32)
    assert np.all(np.isin(out["ack"], (-1.0, 0.0, 1.0)))
    out["ack"] = out["ack"].astype(np.int8)
    np.savez_compressed(os.path.join(OUT, f"d2denv_{name}.npz"), **out)
    print(f"d2denv_{name}: steps={len(rec['done'])} acks(+1/0/-1)="
          f"{[(out['ack'] == v).sum() for v in (1, 0, -1)]} urllc={metrics['urllc']} "
          f"chan_err={metrics['channel_errors']}")


def gen_d2denv():
    for name, params, episodes, p_act in d2denv_configs():
        run_d2denv(name, params, episodes, p_act)


def gen_baselines():
    """act() of the four reference baselines (baselines.py) on seeded buffer matrices: EDF's
    earliest-deadline choice (ties, empty rows, the random pick when nobody has a packet) and the
    global-numpy-stream draws of GF / RandomAccess / CombinatorialRandomAccess, re-seeded per case."""
    bl = ref_module("algorithms.baselines")

    class _Env:
        def __init__(self, n, c, d):
            self.n_agents, self.n_channels, self.deadlines = n, c, np.asarray(d)

    rng = np.random.default_rng(11)
    out = {}
    cases = []
    for i in range(40):
        n = int(rng.integers(1, 9))
        D = int(rng.integers(1, 9))
        dens = [0.0, 0.05, 0.2, 0.6][i % 4]
        buf = (rng.random((n, D)) < dens) * rng.integers(1, 4, (n, D))
        if i % 5 == 0 and n > 1:          # ties on the earliest column
            buf[:, :] = 0
            buf[[0, n - 1], min(1, D - 1)] = 1
        cases.append(buf.astype(np.float64))
    for i, buf in enumerate(cases):
        n, D = buf.shape
        env = _Env(n, 3, np.full(n, D))
        out[f"case{i}/buffers"] = buf
        np.random.seed(1000 + i)
        out[f"case{i}/edf"] = bl.EarliestDeadlineFirstScheduler(env).act(buf)
        np.random.seed(2000 + i)
        out[f"case{i}/gf"] = bl.GFAccess(env, transmission_prob=0.4).act(buf)
        np.random.seed(3000 + i)
        out[f"case{i}/ra"] = bl.RandomAccess(env).act(buf.reshape(-1))
        np.random.seed(4000 + i)
        out[f"case{i}/cra"] = bl.CombinatorialRandomAccess(env, transmission_prob=0.3).act(buf)
    out["n_cases"] = np.array(len(cases))
    np.savez_compressed(os.path.join(OUT, "baselines_act.npz"), **out)
    print(f"baselines_act: {len(cases)} cases")


def gen_gae():
    ippo = ref_module("algorithms.ippo")
    d2d = ref_module("algorithms.d2d_ppo")
    rng = np.random.default_rng(7)
    out = {}
    cases = [("small", 6, 2, 3), ("mid", 400, 8, 200), ("big", 1000, 32, 200)]
    for name, T, N, L in cases:
        rew = rng.integers(0, 4, size=(T, 1)).repeat(N, 1).astype(np.int64)  # broadcast reward, like the envs
        vals = rng.normal(size=(T, N))
        dones = [((t + 1) % L == 0) for t in range(T)]
        # D2D path: 1-D mean reward, float32 values from the critic (d2d_ppo.py:425-426)
        v32 = rng.normal(size=T).astype(np.float32)
        out.update({f"{name}_rew": rew, f"{name}_val": vals, f"{name}_done": np.array(dones), f"{name}_v32": v32})
        for gamma in (0.6, 0.99):
            adv = ippo.compute_gae(rew, dones, vals, gamma, 0.97).numpy()
            ret = ippo.discount_rewards(rew, gamma, dones, True).numpy()
            adv2 = d2d.compute_gae(rew, dones, vals, gamma, 0.97).numpy()
            assert np.array_equal(adv, adv2)
            adv1d = d2d.compute_gae(rew.mean(1), dones, v32, gamma, 0.97).numpy()
            ret1d = d2d.discount_rewards(rew, gamma, dones, True).mean(1).numpy()
            key = f"{name}_g{gamma}"
            out.update({f"{key}_adv": adv, f"{key}_ret": ret, f"{key}_adv1d": adv1d, f"{key}_ret1d": ret1d})
    # edge: one all-zero column -> adv std 0 -> NO column normalised (quirk Q2)
    T, N = 50, 3
    rew = np.zeros((T, N), dtype=np.int64); rew[:, 1:] = rng.integers(0, 3, size=(T, 1))
    vals = rng.normal(size=(T, N)); vals[:, 0] = 0.0
    dones = [((t + 1) % 25 == 0) for t in range(T)]
    out["zerostd_rew"], out["zerostd_val"], out["zerostd_done"] = rew, vals, np.array(dones)
    out["zerostd_adv"] = ippo.compute_gae(rew, dones, vals, 0.9, 0.97).numpy()
    out["zerostd_ret"] = ippo.discount_rewards(rew, 0.9, dones, True).numpy()
    # edge: every step done
    T, N = 20, 2
    rew = rng.integers(0, 3, size=(T, 1)).repeat(N, 1).astype(np.int64)
    vals = rng.normal(size=(T, N))
    dones = [True] * T
    out["alldone_rew"], out["alldone_val"], out["alldone_done"] = rew, vals, np.array(dones)
    out["alldone_adv"] = ippo.compute_gae(rew, dones, vals, 0.8, 0.97).numpy()
    out["alldone_ret"] = ippo.discount_rewards(rew, 0.8, dones, True).numpy()
    np.savez_compressed(os.path.join(OUT, "gae_returns.npz"), **out)
    print("gae_returns:", len(out), "arrays")


def gen_data():
    """Re-serialise the reference's data pickles as JSON (read with tools/safe_pickle.py)."""
    dst = os.path.join(os.path.dirname(HERE), "d2d-ppo_amd", "combinatorial_load")
    os.makedirs(dst, exist_ok=True)
    for f in ("channel_switch_8", "setup_8_channels", "setup"):
        obj = safe_pickle.load(f"{DATA}/{f}.p")
        if isinstance(obj, dict):
            j = {k: _jsonable(v) for k, v in obj.items()}
        else:
            j = _jsonable(obj)
        with open(os.path.join(dst, f + ".json"), "w") as fh:
            json.dump(j, fh, indent=1)
    print("data json written to", dst)




# ----------------------------------------------------------------- learners
def _sd_np(module):
    return {k: v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


def _put(out, prefix, sd):
    for k, v in sd.items():
        out[f"{prefix}/{k}"] = v


class RecordingEnv:
    """Forwards to a reference env and records the actions it is given and the
    random draws it makes (flip masks / arrivals recovered from state diffs)."""

    def __init__(self, env):
        self.__dict__["_env"] = env
        self.__dict__["rec"] = {"reset_arrivals": [], "actions": [], "flips": [], "arrivals": []}

    def __getattr__(self, k):
        return getattr(self._env, k)

    def __setattr__(self, k, v):
        setattr(self._env, k, v)

    def reset(self):
        out = self._env.reset()
        d = np.asarray(self._env.deadlines)
        self.rec["reset_arrivals"].append([self._env.current_buffers[k, d[k] - 1] for k in range(self._env.n_agents)])
        return out

    def step(self, actions):
        if not hasattr(self._env, "homogeneous_size"):
            # ChannelSelectionEnv: the reference learners pass (N, 1) categorical actions, which the env
            # broadcasts to (N, N) (a crash/miscount bug); parity is defined on (N,) actions
            actions = np.asarray(actions).reshape(-1)
        H0 = np.array(self._env.channel_state, dtype=np.float64).copy()
        out = self._env.step(actions)
        H1 = np.array(self._env.channel_state, dtype=np.float64)
        d = np.asarray(self._env.deadlines)
        self.rec["actions"].append(np.array(actions, dtype=np.float64))
        self.rec["flips"].append(np.abs(H1 - H0).astype(np.uint8))
        self.rec["arrivals"].append([self._env.current_buffers[k, d[k] - 1] for k in range(self._env.n_agents)])
        return out


LEARNER_VARIANTS = {
    # name: (env kind, useRNN, combinatorial, history_len)
    "mlp_comb": ("comb", False, True, 4),
    "rnn_comb": ("comb", True, True, 4),
    "mlp_cat": ("chsel", False, False, 3),
    "rnn_cat": ("chsel", True, False, 3),
    "mlp_d2denv": ("single", False, False, 3),   # iPPO only: the reference D2DPPO cannot run on D2DEnv
    "rnn_d2denv": ("single", True, False, 3),
}

# The reference drivers' own GRU shapes (gen_learner_drivers): hidden_size = 64 with a long window
# (xp_load.py:78-89 runs D2D-PPO with history_len = n_agents), and run_ippo_combinatorial.py:29-89's
# 6 agents x 16 channels (obs up to 14 + 2 * 16 = 46 inputs) with history_len = 6.
# name: (env kind, useRNN, combinatorial, history_len, hidden, episode_length, algos, episodes)
DRIVER_VARIANTS = {
    "rnn_comb_h64L16": ("comb_xpload", True, True, 16, 64, 24, ("d2d", "ippo"), 1),
    "rnn_comb16_h64": ("comb16", True, True, 6, 64, 20, ("ippo", "d2d"), 1),
}


# The learners' default hidden_size 128 (ippo.py:225, d2d_ppo.py:222: what a user gets without the drivers'
# explicit 64), MLP policies, on the kernels' 8-hidden-tile path (gen_learner_defaults)
DEFAULT_VARIANTS = {
    "mlp_comb_h128": ("comb", False, True, 4, 128, 20, ("ippo", "d2d"), 2),
    "mlp_cat_h128": ("chsel", False, False, 3, 128, 20, ("ippo", "d2d"), 2),
}


def _learner_env(kind, episode_length=20):
    if kind == "comb_xpload":
        # xp_load.py:60-75 on setup_8_channels at load 1/2, homogeneous obs (14 + 2 * 8 = 30 inputs)
        mod = ref_module("envs.combinatorial_env")
        setup8 = safe_pickle.load(f"{DATA}/setup_8_channels.p")
        p = dict(n_agents=6, n_channels=8, deadlines=setup8["deadlines"], lbdas=np.array([0.5] * 6),
                 period=np.array([2] * 6), arrival_probs=setup8["arrival_probs"], offsets=setup8["offsets"],
                 episode_length=episode_length, traffic_model="heterogeneous", homogeneous_size=True,
                 periodic_devices=[0, 1, 2], channel_switch=setup8["channel_switch"])
        return mod.CombinatorialEnv(**p), p
    if kind == "comb16":
        # run_ippo_combinatorial.py:29-76 at load 1 (1-D channel_switch broadcast over agents)
        mod = ref_module("envs.combinatorial_env")
        p = dict(n_agents=6, n_channels=16, deadlines=np.array([7, 14] * 3), lbdas=np.array([1.0] * 6),
                 period=np.array([1.0] * 6), arrival_probs=np.array([0.4, 0.8] * 3), offsets=np.zeros(6),
                 episode_length=episode_length, traffic_model="heterogeneous", periodic_devices=[0, 1],
                 channel_switch=np.array([0.8] * 16))
        return mod.CombinatorialEnv(**p), p
    if kind == "comb":
        mod = ref_module("envs.combinatorial_env")
        setup8 = safe_pickle.load(f"{DATA}/setup_8_channels.p")
        return mod.CombinatorialEnv(
            n_agents=6, n_channels=8, deadlines=setup8["deadlines"], lbdas=np.array([0.5] * 6),
            period=np.array([2] * 6), arrival_probs=setup8["arrival_probs"], offsets=setup8["offsets"],
            episode_length=episode_length, traffic_model="heterogeneous", homogeneous_size=False,
            periodic_devices=[0, 1, 2], channel_switch=setup8["channel_switch"]), dict(
            n_agents=6, n_channels=8, deadlines=setup8["deadlines"], lbdas=np.array([0.5] * 6),
            period=np.array([2] * 6), arrival_probs=setup8["arrival_probs"], offsets=setup8["offsets"],
            episode_length=episode_length, traffic_model="heterogeneous", homogeneous_size=False,
            periodic_devices=[0, 1, 2], channel_switch=setup8["channel_switch"])
    if kind == "single":
        mod = ref_module("envs.env")
        p = dict(n_agents=5, deadlines=np.array([3, 5, 4, 3, 4]), lbdas=np.array([0.5] * 5),
                 episode_length=episode_length, traffic_model="aperiodic", channel_switch=0.3,
                 neighbourhoods=[[0, 1], [1, 2, 0], [2], [3, 4, 2], [4, 0]])
        return mod.D2DEnv(**p), p
    mod = ref_module("envs.channel_selection_env")
    p = dict(n_agents=4, n_channels=3, deadlines=np.array([4, 6, 4, 5]), lbdas=np.array([0.6] * 4),
             episode_length=episode_length, traffic_model="aperiodic", channel_switch=np.array([0.5, 0.3, 0.7, 0.2]))
    return mod.ChannelSelectionEnv(**p), p


def _tap_grads(out, tag, opt, net):
    """Record the .grad of every parameter of `net` each time `opt` steps (before the step runs)."""
    step = opt.step
    count = [0]

    def rec(*a, **kw):
        for n, prm in net.named_parameters():
            if prm.grad is not None:
                out[f"grads/{tag}/step{count[0]}/{n}"] = prm.grad.detach().numpy().copy()
        count[0] += 1
        return step(*a, **kw)
    opt.step = rec


def gen_learner(only=None, episodes=2, suffix="", algos=("ippo", "d2d"), variants=None):
    import torch
    ippo = ref_module("algorithms.ippo")
    d2d = ref_module("algorithms.d2d_ppo")
    import sys as _sys
    if only is None:
        only = [a for a in _sys.argv[2:]]
    if variants is None:
        variants = {k: v + (16, 20, algos, episodes) for k, v in LEARNER_VARIANTS.items()}
    for vname, (kind, useRNN, comb, hl, hidden, ep_len, v_algos, episodes) in variants.items():
        if only and vname not in only:
            continue
        for algo in (("ippo",) if kind == "single" else v_algos):
            out = {"kind": "comb" if kind.startswith("comb") else kind, "useRNN": useRNN, "combinatorial": comb,
                   "history_len": hl, "hidden": hidden, "gamma": 0.6, "episode_length": ep_len, "episodes": episodes}
            env, params = _learner_env(kind, ep_len)
            out["params_json"] = json.dumps({k: _jsonable(v) for k, v in params.items()})
            torch.manual_seed(3)
            np.random.seed(5)
            if algo == "ippo":
                lr = ippo.iPPO(env, hidden_size=hidden, gamma=0.6, policy_lr=3e-3, value_lr=1e-2, device="cpu",
                               useRNN=useRNN, combinatorial=comb, history_len=hl, early_stopping=False)
            else:
                lr = d2d.D2DPPO(env, hidden_size=hidden, gamma=0.6, policy_lr=3e-3, value_lr=1e-2, beta_entropy=0.02,
                                device="cpu", useRNN=useRNN, combinatorial=comb, history_len=hl,
                                early_stopping=False)
                _put(out, "init/critic", _sd_np(lr.value_network))
            for i, ag in enumerate(lr.agents):
                _put(out, f"init/agent{i}/policy", _sd_np(ag.policy_network))
                if algo == "ippo":
                    _put(out, f"init/agent{i}/value", _sd_np(ag.value_network))
            # --- teacher-forced rollout: record actions + env draws of a real create_rollouts
            rec_env = RecordingEnv(env)
            lr.env = rec_env
            torch.manual_seed(11)
            ro = lr.create_rollouts(episodes)
            lr.env = env
            for k, v in rec_env.rec.items():
                out[f"draws/{k}"] = np.array(v)
            if algo == "ippo":
                obs_t, acts, logp, rets, vals, advs, scores, dones = ro
                out["ro/values"] = np.asarray(vals)
                out["ro/advantages"] = advs.numpy()
            else:
                obs_t, states, acts, logp, rew_mean, rets, scores, dones = ro
                out["ro/states"] = states.numpy()
                out["ro/rewards_mean"] = np.asarray(rew_mean)
            for i, o in enumerate(obs_t):
                out[f"ro/obs{i}"] = o.numpy()
            out["ro/actions"] = np.asarray(acts, dtype=np.float64)
            out["ro/log_probs"] = logp.numpy()
            out["ro/returns"] = rets.numpy()
            out["ro/scores"] = np.array(scores)
            out["ro/dones"] = np.array(dones)
            # --- one training iteration on exactly that rollout (create_rollouts patched; the
            # iteration-0 evaluation is stubbed: it only reads the env, it does not change weights)
            if not comb:
                # Categorical actions come back as (T, N, 1) (ippo.py:318); actions[:, i] is then (T, 1)
                # and Categorical.log_prob broadcasts it against (T,) to (T, T) inside train_step
                # (SURVEY Q4).  Parity is defined on the flattened (T,) actions, so train on those.
                ro = list(ro)
                ai = 1 if algo == "ippo" else 2
                ro[ai] = np.asarray(ro[ai]).reshape(len(dones), env.n_agents)
                ro = tuple(ro)
            lr.create_rollouts = lambda num_episodes=4, _ro=ro: _ro
            lr.test = lambda num_episodes: (0.5, 1.0, 0, 0.0)
            # the gradient every Adam step consumes (grads/<net>/step<j>/<param>): the final-weight check
            # of tests/test_learner_gpu.py derives its Adam-aware bound from these reference gradients
            taps = [(f"agent{i}/policy", ag.policy_optimizer, ag.policy_network) for i, ag in enumerate(lr.agents)]
            if algo == "ippo":
                taps += [(f"agent{i}/value", ag.value_optimizer, ag.value_network) for i, ag in enumerate(lr.agents)]
            else:
                taps.append(("critic", lr.value_optimizer, lr.value_network))
            for tag, opt, net in taps:
                _tap_grads(out, tag, opt, net)
            np.random.seed(21)  # D2D agent permutation stream (d2d_ppo.py:421-422)
            if algo == "ippo":
                res = lr.train(1, n_epoch=2, num_episodes=episodes, test_freq=10 ** 9)
                out["train/policy_loss"] = np.array(res[2])
                out["train/value_loss"] = np.array(res[3])
            else:
                res = lr.train(1, num_episodes=episodes, n_epoch=2, test_freq=10 ** 9)
                out["train/policy_loss"] = np.array(res[2])          # [epoch][agent in sigma order]
                out["train/value_loss"] = np.array([float(v) for v in res[3]])
                np.random.seed(21)
                perms = []
                for _ in range(2):
                    c = np.arange(env.n_agents)
                    np.random.shuffle(c)
                    perms.append(c)
                out["train/perms"] = np.array(perms)
                _put(out, "final/critic", _sd_np(lr.value_network))
            for i, ag in enumerate(lr.agents):
                _put(out, f"final/agent{i}/policy", _sd_np(ag.policy_network))
                if algo == "ippo":
                    _put(out, f"final/agent{i}/value", _sd_np(ag.value_network))
            # preprocess_input_for_rnn on agent 0's obs (ippo.py:390-403)
            if useRNN:
                out["rnnwin/agent0"] = lr.preprocess_input_for_rnn(obs_t[0]).numpy()
            np.savez_compressed(os.path.join(OUT, f"learner_{algo}_{vname}{suffix}.npz"), **out)
            print(f"learner_{algo}_{vname}{suffix}: T={len(dones)} scores={np.round(scores, 3)}")


def gen_learner4():
    """4-episode traces (run on 2 envs x 2 waves, or 4 envs x 1 wave) for the multi-env sample order."""
    gen_learner(only=["mlp_comb", "rnn_cat", "mlp_d2denv"], episodes=4, suffix="_ep4")


def gen_learner_defaults():
    """MLP traces at the learners' default hidden_size 128 (DEFAULT_VARIANTS)."""
    gen_learner(only=[], variants=DEFAULT_VARIANTS)


def gen_learner_drivers():
    """GRU traces at the reference drivers' own network shapes (DRIVER_VARIANTS): hidden 64 with a
    16-step window, and the 6 x 16-channel env with 46 inputs."""
    gen_learner(only=[], variants=DRIVER_VARIANTS)


def gen_evaltest():
    """The reference's deterministic evaluation `test(num_episodes)` (ippo.py:345-388,
    d2d_ppo.py:341-383) for every learner variant: fixed weights, 4 episodes.  Recorded: the
    weights, the env draws of every reset / step, the actions test() took (argmax / p > 0.5) and
    its return tuple (mean URLLC score, mean Jain's index, summed channel errors, mean episode
    reward).  The MLP actors' last layer is scaled x4 before recording so that the softmax is
    peaked enough for p > 0.5 / argmax decisions to vary (the weights stored are the scaled ones)."""
    import torch
    ippo = ref_module("algorithms.ippo")
    d2d = ref_module("algorithms.d2d_ppo")
    n_ep = 4
    for vname, (kind, useRNN, comb, hl) in LEARNER_VARIANTS.items():
        for algo in (("ippo",) if kind == "single" else ("ippo", "d2d")):
            out = {"kind": kind, "useRNN": useRNN, "combinatorial": comb, "history_len": hl, "hidden": 16,
                   "gamma": 0.6, "episode_length": 20, "episodes": n_ep}
            env, params = _learner_env(kind)
            out["params_json"] = json.dumps({k: _jsonable(v) for k, v in params.items()})
            torch.manual_seed(17)
            np.random.seed(19)
            if algo == "ippo":
                lr = ippo.iPPO(env, hidden_size=16, gamma=0.6, device="cpu", useRNN=useRNN, combinatorial=comb,
                               history_len=hl, early_stopping=False)
            else:
                lr = d2d.D2DPPO(env, hidden_size=16, gamma=0.6, device="cpu", useRNN=useRNN, combinatorial=comb,
                                history_len=hl, early_stopping=False)
            for i, ag in enumerate(lr.agents):
                if not useRNN:
                    with torch.no_grad():
                        ag.policy_network.linear2.weight.mul_(4.0)
                _put(out, f"weights/agent{i}/policy", _sd_np(ag.policy_network))
            rec_env = RecordingEnv(env)
            lr.env = rec_env
            np.random.seed(23)
            res = lr.test(n_ep)
            for k, v in rec_env.rec.items():
                out[f"draws/{k}"] = np.array(v)
            out["result"] = np.array([float(x) for x in res], dtype=np.float64)
            np.savez_compressed(os.path.join(OUT, f"evaltest_{algo}_{vname}.npz"), **out)
            acts = np.array(rec_env.rec["actions"])
            print(f"evaltest_{algo}_{vname}: result={np.round(out['result'], 5)} mean action={acts.mean():.3f}")


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    table = {"data": gen_data, "env": gen_env, "d2denv": gen_d2denv, "gae": gen_gae, "learner": gen_learner,
             "baselines": gen_baselines, "evaltest": gen_evaltest, "learner4": gen_learner4,
             "learner_drivers": gen_learner_drivers, "learner_defaults": gen_learner_defaults}
    # `learner <variant> ...` regenerates only the named learner variants
    which = sys.argv[1:2] if sys.argv[1:2] == ["learner"] else sys.argv[1:]
    for w in which or list(table):
        table[w]()
