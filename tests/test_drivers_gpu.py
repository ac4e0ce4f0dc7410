"""The reference drivers' construction and call sequences, end to end on the GPU (pytest -m gpu).

Not copies of the drivers: each test performs the calls a driver makes, in the same order with the
same keyword arguments and input types, at a tiny iteration count:
  xp_load.py:31,63-108      setup pickle read from cwd -> CombinatorialEnv(periodic_devices = the
                            pickle's ndarray, quirk Q8) -> D2DPPO(useRNN=True, history_len=n_agents,
                            save_path, early_stopping=True) -> train(num_iter, n_epoch, num_episodes,
                            test_freq) -> load(save_path) -> test(n); results dict as at :154-162
  xp_load.py:92-104         the commented-out MCA-iPPO variant (same env, iPPO, gamma 0.4)
  xp_n_agents.py:71-83,137-140  aperiodic env -> CombinatorialRandomAccess(env) ->
                            get_best_transmission_probs -> run
  run_ippo_combinatorial.py:65-91  1-D channel_switch broadcast, iPPO with GRU
The setup pickles are written by tools/make_setup_pickles.py (our own files, from the JSON
settings), exactly where xp_load.py looks for them."""
import os
import pickle
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def xp_dir(tmp_path, monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_setup_pickles
    make_setup_pickles.main(str(tmp_path))
    monkeypatch.chdir(tmp_path)
    return tmp_path


def _xp_load_env(setup, load):
    from envs.combinatorial_env import CombinatorialEnv
    n_agents = setup["n_agents"]
    return CombinatorialEnv(n_agents=n_agents, n_channels=8, deadlines=setup["deadlines"],
                            lbdas=np.array([load] * n_agents), period=np.array([int(1 / load)] * n_agents),
                            arrival_probs=setup["arrival_probs"], offsets=setup["offsets"],
                            episode_length=setup["episode_length"], traffic_model="heterogeneous",
                            homogeneous_size=True, periodic_devices=setup["periodic_devices"],
                            channel_switch=setup["channel_switch"], verbose=False)


@pytest.mark.parametrize("algo", ["d2d", "ippo"])
def test_xp_load_sequence(xp_dir, algo):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm GPU")
    from algorithms.d2d_ppo import D2DPPO
    from algorithms.ippo import iPPO
    from algorithms.irdqn import iRDQN  # noqa: F401  (xp_load.py:6 imports it)
    np.random.seed(42)
    setup = pickle.load(open("combinatorial_load/setup_8_channels.p", "rb"))  # written by our tool
    assert isinstance(setup["periodic_devices"], np.ndarray)                    # quirk Q8
    n_agents = setup["n_agents"]
    xp_name = "combinatorial_load"
    os.mkdir(f"{xp_name}/results")
    results = {"scores": [], "jains": [], "channel_errors": [], "average_rewards": [], "training": []}
    for load in setup["loads_list"][:2]:
        model_folder = f"models_mcappo{setup['n_channels']}_seed_0_load_{load}"
        os.mkdir(f"{xp_name}/{model_folder}")
        env = _xp_load_env(setup, load)
        common = dict(hidden_size=64, policy_lr=3e-4, value_lr=1e-3, device=None, useRNN=True,
                      save_path=f"{xp_name}/{model_folder}", combinatorial=True, history_len=n_agents,
                      early_stopping=True)
        ppo = D2DPPO(env, gamma=0.6, **common) if algo == "d2d" else iPPO(env, gamma=0.4, **common)
        # xp_load.py:106 passes keywords, so the two learners' positional orders do not matter here
        res = ppo.train(num_iter=2, n_epoch=2, num_episodes=3, test_freq=1)
        assert os.path.exists(f"{xp_name}/{model_folder}/agent_{n_agents - 1}.pth")
        ppo.load(f"{xp_name}/{model_folder}")
        score, jains, ch_err, rewards = ppo.test(6)
        assert 0.0 <= score <= 1.0 and 0.0 < jains <= 1.0 + 1e-12 and ch_err == 0 and rewards >= 0
        scores_episode, score_test_list, policy_loss_list, value_loss_list = res
        assert len(scores_episode) == 2 * 3 and len(score_test_list) == 2 * 2
        if algo == "d2d":   # per-epoch lists of per-agent losses (sigma order), critic losses as tensors
            assert len(policy_loss_list) == 4 and all(len(p) == n_agents for p in policy_loss_list)
            assert all(torch.is_tensor(v) for v in value_loss_list)
        else:               # the last agent's losses per epoch (ippo.py:425-426)
            assert len(policy_loss_list) == 4 and all(np.isfinite(policy_loss_list))
        results["training"].append(res)
        for k, v in zip(("scores", "jains", "channel_errors", "average_rewards"), (score, jains, ch_err, rewards)):
            results[k].append(v)
    with open(f"{xp_name}/results/mcappo_8_channels.p", "wb") as fh:   # xp_load.py:154-162
        pickle.dump({k: (v if k == "training" else [np.array(v)]) for k, v in results.items()}, fh)


def test_xp_n_agents_baseline_sequence(xp_dir):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm GPU")
    from algorithms.baselines import CombinatorialRandomAccess
    from envs.combinatorial_env import CombinatorialEnv
    np.random.seed(13)
    for n_agents in (4, 8):
        n_channels = 4
        env = CombinatorialEnv(n_agents=n_agents, n_channels=n_channels, deadlines=np.array([7] * n_agents),
                               lbdas=np.array([1 / 14 for _ in range(n_agents)]), period=None, arrival_probs=None,
                               offsets=None, episode_length=200, traffic_model="aperiodic",
                               collision_type="pessimistic", periodic_devices=[],
                               channel_switch=np.ones((n_agents, n_channels)) * 0.8, verbose=False)
        gf = CombinatorialRandomAccess(env)
        cv = gf.get_best_transmission_probs(3)
        assert len(cv) == len(gf.transmission_prob_list)
        gf.transmission_prob = gf.transmission_prob_list[np.argmax(cv)]
        score, jains, ch, rewards = gf.run(5)
        assert 0.0 <= score <= 1.0 and 0.0 < jains <= 1.0 + 1e-12 and rewards >= 0


def test_run_ippo_combinatorial_sequence(xp_dir):
    """run_ippo_combinatorial.py:58-91 plumbing: 1-D channel_switch (broadcast over agents),
    heterogeneous traffic with an ndarray periodic_devices, iPPO with a GRU policy."""
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm GPU")
    from algorithms.ippo import iPPO
    from envs.combinatorial_env import CombinatorialEnv
    n_agents, n_channels = 6, 16
    env = CombinatorialEnv(n_agents=n_agents, n_channels=n_channels, deadlines=np.array([7, 14] * 3),
                           lbdas=np.array([1 / 3] * n_agents), period=np.array([3] * n_agents),
                           arrival_probs=np.array([1.0] * n_agents), offsets=np.zeros(n_agents),
                           episode_length=40, traffic_model="heterogeneous", periodic_devices=np.array([0, 1, 2]),
                           channel_switch=np.array([0.8] * n_channels), verbose=False)
    ippo = iPPO(env, hidden_size=64, gamma=0.4, policy_lr=3e-4, value_lr=1e-3, device=None, useRNN=True,
                save_path=None, combinatorial=True, history_len=10, early_stopping=False)
    # 46 inputs (14 + 2 * 16): the GRU rollout / update kernels with three input tiles and the compact
    # record (64-byte rows), not the torch fallback
    assert env.observation_space[1].shape[0] == 46
    assert ippo._gru_ok() and ippo._fused_update_ok() and ippo._record_ok()
    res = ippo.train(2, 2, 2, 100)   # positional: (num_iter, n_epoch, num_episodes, test_freq), ippo.py:406
    assert len(res[0]) == 4 and len(res[1]) == 2
    score, jains, ch, rew = ippo.test(4)
    assert 0.0 <= score <= 1.0 and ch == 0
