"""GRU update gradients at the bench's batch (xp_load shapes: 64 agents, H = 64, L = 64, 200-slot episode,
E envs, default 96: the float64 reference of 256 envs exceeds the 288 GB) on the compact record: the cooperative LDS weight-gradient path and the row-history
path (D2D_OPT_GRU_GRAD_HISTORY), each against float64 autograd, with torch fp32's own distance to
float64 (the band) beside them -- tests/test_gru_gpu.py's xp_grads_check without its assertions.
usage (GPU box): python3 tools/gpu/gru_coop_vs_history.py [E]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd"), os.path.join(ROOT, "tests")]

if __name__ == "__main__":
    import test_gru_gpu as t
    from d2dhip import _lib
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    lib = _lib.require_gpu()
    out = {"E": E}
    for kind in ("sigmoid", None):
        for name, hist in (("coop", 0), ("history", 1)):
            lib.d2d_set_option(_lib.D2D_OPT_GRU_GRAD_HISTORY, hist)
            errs = t.xp_grads_check(kind, "record", E, check=False)
            out[f"{kind}/{name}"] = {k: {"err64_over_max": e / s, "band_over_max": b / s} for k, (e, b, s) in errs.items()}
        lib.d2d_set_option(_lib.D2D_OPT_GRU_GRAD_HISTORY, 0)
    print(json.dumps(out))
