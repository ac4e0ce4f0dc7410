"""d2dhip — MI355X (gfx950) HIP implementation of the D2D-PPO hot path.

C ABI: include/d2d_hip.h, built into d2d-ppo_amd/lib/libd2dhip.so.
"""
from ._lib import D2DHipError, EXPORTED, LIB_PATH, load, require_gpu  # noqa: F401
from .spec import EnvSpec  # noqa: F401


def __getattr__(name):
    # lazy: importing EnvBatch pulls torch.cuda state only when asked for
    if name in ("EnvBatch", "pack_masks", "pack_masks_torch"):
        from . import envbatch
        return getattr(envbatch, name)
    if name in ("gae",):
        import importlib
        return importlib.import_module(".gae", __name__)
    raise AttributeError(name)
