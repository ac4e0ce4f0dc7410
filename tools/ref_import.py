"""Import the read-only reference (/root/reference) in THIS container only.

The reference does `from gym import spaces` (envs/combinatorial_env.py:2,
envs/channel_selection_env.py:2); gym is not installed, so a minimal in-memory
stand-in for the four attributes the reference reads (Box.shape,
Discrete.n, MultiBinary.n, Tuple indexing) is registered in sys.modules.
Bytecode writing is disabled because the reference tree is read-only.

Only tools/ uses this, to generate the committed golden fixtures under
tests/golden/.  Nothing on the GPU box imports it.
"""
import importlib
import os
import sys
import types

REF = "/root/reference"


def _install_gym_stub():
    if "gym" in sys.modules:
        return
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")

    class Box:
        def __init__(self, low=None, high=None, shape=None, dtype=None):
            self.shape = tuple(shape)

    class Discrete:
        def __init__(self, n):
            self.n = int(n)

    class MultiBinary:
        def __init__(self, n):
            self.n = int(n)

    class Tuple(tuple):
        def __new__(cls, spaces_):
            return tuple.__new__(cls, list(spaces_))

    spaces.Box, spaces.Discrete, spaces.MultiBinary, spaces.Tuple = Box, Discrete, MultiBinary, Tuple
    gym.spaces = spaces
    sys.modules["gym"] = gym
    sys.modules["gym.spaces"] = spaces


def ref_module(name):
    """Import `name` (e.g. 'envs.combinatorial_env') from the reference tree."""
    if not os.path.isdir(REF):
        raise RuntimeError("/root/reference is not present (fixture generation runs only in the build container)")
    sys.dont_write_bytecode = True
    _install_gym_stub()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    return importlib.import_module(name)
