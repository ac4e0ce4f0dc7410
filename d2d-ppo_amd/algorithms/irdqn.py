"""iRDQN — importable placeholder for /root/reference/algorithms/irdqn.py.

The independent recurrent DQN baseline is outside this build's hot path
(value-based baseline, not PPO).  xp_load.py:6 and
xp_n_agents.py:7 import the name, so it exists; constructing it raises.
"""


class ReplayBuffer:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("iRDQN's replay buffer is not part of the MI355X hot path (SURVEY.md §2)")


class iRDQN:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("iRDQN is not part of the MI355X hot path (SURVEY.md §2); "
                                  "use algorithms.ippo.iPPO or algorithms.d2d_ppo.D2DPPO")
