"""Write combinatorial_load/{setup_8_channels,setup,channel_switch_8}.p for the
reference drivers (xp_load.py:31 reads setup_8_channels.p) from the JSON
settings shipped in d2d-ppo_amd/combinatorial_load/.  These pickles are
written by this script (plain dicts / ndarrays), not copied from the reference.

usage: python tools/make_setup_pickles.py OUT_DIR
"""
import json
import os
import pickle
import sys

import numpy as np

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "d2d-ppo_amd", "combinatorial_load")


def _decode(v):
    if isinstance(v, dict) and "__nd__" in v:
        return np.array(v["__nd__"], dtype=v["dtype"])
    return v


def main(out_dir):
    dst = os.path.join(out_dir, "combinatorial_load")
    os.makedirs(dst, exist_ok=True)
    for name in ("setup_8_channels", "setup", "channel_switch_8"):
        obj = json.load(open(os.path.join(SRC, name + ".json")))
        obj = {k: _decode(v) for k, v in obj.items()} if "__nd__" not in obj else _decode(obj)
        with open(os.path.join(dst, name + ".p"), "wb") as fh:
            pickle.dump(obj, fh)
    print("wrote", dst)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else ".")
