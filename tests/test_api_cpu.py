"""The reference's experiment drivers import these names (xp_load.py:4-7,
xp_n_agents.py:4-8, run_ippo_combinatorial.py, xp_gamma.py); they must all
resolve from d2d-ppo_amd/ with the reference's import paths."""
import inspect


def test_driver_imports_resolve():
    from envs.combinatorial_env import CombinatorialEnv  # noqa: F401
    from envs.channel_selection_env import ChannelSelectionEnv  # noqa: F401
    from algorithms.d2d_ppo import D2DPPO  # noqa: F401
    from algorithms.irdqn import iRDQN  # noqa: F401
    from algorithms.ippo import iPPO  # noqa: F401
    from algorithms.baselines import CombinatorialRandomAccess  # noqa: F401
    from algorithms.ippo import compute_gae, discount_rewards, Policy, Value, RNN, PPO, init_weights  # noqa: F401
    from algorithms.d2d_ppo import compute_gae as cg2, PPO as PPO2  # noqa: F401


def test_signatures_match_reference():
    from algorithms.d2d_ppo import D2DPPO
    from algorithms.ippo import iPPO
    from envs.channel_selection_env import ChannelSelectionEnv
    from envs.combinatorial_env import CombinatorialEnv
    p = lambda f: list(inspect.signature(f).parameters)  # noqa: E731
    assert p(iPPO.__init__)[:12] == ["self", "env", "hidden_size", "gamma", "policy_lr", "value_lr", "device",
                                     "useRNN", "save_path", "combinatorial", "history_len", "early_stopping"]
    assert p(D2DPPO.__init__)[:13] == ["self", "env", "hidden_size", "gamma", "policy_lr", "value_lr",
                                       "beta_entropy", "device", "useRNN", "save_path", "combinatorial",
                                       "history_len", "early_stopping"]
    # positional orders differ between the two reference trainers (ippo.py:406 vs d2d_ppo.py:401)
    assert p(iPPO.train) == ["self", "num_iter", "n_epoch", "num_episodes", "test_freq"]
    assert p(D2DPPO.train) == ["self", "num_iter", "num_episodes", "n_epoch", "test_freq"]
    assert p(CombinatorialEnv.__init__)[:16] == [
        "self", "n_agents", "n_channels", "deadlines", "lbdas", "period", "arrival_probs", "offsets",
        "episode_length", "traffic_model", "periodic_devices", "reward_type", "collision_type", "homogeneous_size",
        "channel_switch", "verbose"]
    assert p(ChannelSelectionEnv.__init__)[:14] == [
        "self", "n_agents", "n_channels", "deadlines", "lbdas", "period", "arrival_probs", "offsets",
        "episode_length", "traffic_model", "periodic_devices", "reward_type", "channel_switch", "verbose"]
    for m in ("reset", "step", "compute_jains", "compute_urllc", "compute_channel_score"):
        assert hasattr(CombinatorialEnv, m) and hasattr(ChannelSelectionEnv, m)
    for m in ("train", "test", "save", "load", "create_rollouts", "preprocess_input_for_rnn"):
        assert hasattr(iPPO, m) and hasattr(D2DPPO, m)
