"""The heuristic baselines' act() against the reference's own outputs
(tests/golden/baselines_act.npz, tools/gen_fixtures.py gen_baselines): same
inputs, same global-numpy seeds -> identical actions (baselines.py:10-14,
61-74, 121-125, 181-183)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


class _Env:
    def __init__(self, n, c, d):
        self.n_agents, self.n_channels, self.deadlines = n, c, np.asarray(d)
        self.n_envs = 1


def _cases():
    z = np.load(os.path.join(GOLDEN, "baselines_act.npz"))
    return z, int(z["n_cases"])


@pytest.mark.parametrize("i", range(40))
def test_act_matches_reference(i):
    from algorithms import baselines as bl
    z, n = _cases()
    assert n == 40
    buf = z[f"case{i}/buffers"]
    N, D = buf.shape
    env = _Env(N, 3, np.full(N, D))
    np.random.seed(1000 + i)
    assert np.array_equal(bl.EarliestDeadlineFirstScheduler(env).act(buf), z[f"case{i}/edf"])
    np.random.seed(2000 + i)
    assert np.array_equal(bl.GFAccess(env, transmission_prob=0.4).act(buf), z[f"case{i}/gf"])
    np.random.seed(3000 + i)
    assert np.array_equal(bl.RandomAccess(env).act(buf.reshape(-1)), z[f"case{i}/ra"])
    np.random.seed(4000 + i)
    assert np.array_equal(bl.CombinatorialRandomAccess(env, transmission_prob=0.3).act(buf), z[f"case{i}/cra"])


def test_edf_choice_rule():
    """Earliest non-empty column wins, lowest agent index on ties; nobody -> one random agent."""
    from algorithms import baselines as bl
    env = _Env(4, 1, np.full(4, 5))
    edf = bl.EarliestDeadlineFirstScheduler(env)
    b = np.zeros((4, 5))
    b[2, 3] = b[1, 1] = b[3, 1] = 1
    assert np.array_equal(edf.act(b), [0, 1, 0, 0])
    a = edf.act(np.zeros((4, 5)))
    assert a.sum() == 1
