"""Minimal shape-only spaces (the reference uses gym.spaces only for shapes:
envs/combinatorial_env.py:49-58, envs/channel_selection_env.py:41-46).  gym is
not a dependency; callers read .shape / .n and index the Tuple."""


class Box:
    def __init__(self, low=None, high=None, shape=None, dtype=None):
        self.low, self.high = low, high
        self.shape = tuple(int(s) for s in shape)

    def __repr__(self):
        return f"Box{self.shape}"


class Discrete:
    def __init__(self, n):
        self.n = int(n)

    def __repr__(self):
        return f"Discrete({self.n})"


class MultiBinary:
    def __init__(self, n):
        self.n = int(n)
        self.shape = (self.n,)

    def __repr__(self):
        return f"MultiBinary({self.n})"


class Tuple(tuple):
    def __new__(cls, spaces):
        return tuple.__new__(cls, list(spaces))

    @property
    def spaces(self):
        return tuple(self)
