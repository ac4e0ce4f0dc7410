"""GRU update kernel vs float64 at long windows (tests/test_gru_gpu.py xp_grads_check without assertions): every
gradient tensor's error for the value (MSE) and sigmoid kinds at (N, L) in {(256, 256), (256, 128), (128, 256)},
and, for w_ih / w_hh, the error per column (the location of the largest errors).
usage (GPU box): python3 tools/gpu/gru_long_diag.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "d2d-ppo_amd"), os.path.join(ROOT, "tests")]
import test_gru_gpu as TG  # noqa: E402

if __name__ == "__main__":
    out = {}
    for N, L in ((256, 256), (256, 128), (128, 256)):
        for kind in (None, "sigmoid"):
            c = dict(N=N, F=23, H=64, A=8, L=L, ep=200, T=200, E=4)
            errs = TG.xp_grads_check(kind, "record", 4, check=False, cfg=c)
            key = f"{kind or 'value'}/N{N}/L{L}"
            out[key] = {n: {"err64_rel": e / s, "band_rel": b / s} for n, (e, b, s) in errs.items()}
            print(key, json.dumps({n: (round(v["err64_rel"], 8), round(v["band_rel"], 8)) for n, v in out[key].items()}),
                  flush=True)
            got, r64, r32 = TG.LAST
            for name in ("w_ih", "w_hh", "b_ih"):
                d = (got[name].double() - r64[name]).abs()[0] if got[name].dim() > 1 else None
                d = (got[name].double() - r64[name]).abs()
                # error by agent, by gate row block (r, z, n) and by column: where the large ones sit
                per_agent = d.reshape(d.shape[0], -1).max(1).values
                worst = int(per_agent.argmax())
                dw = d[worst]
                rows = dw.reshape(3, -1, *dw.shape[1:]).amax(dim=tuple(range(1, dw.dim() + 1))) if dw.dim() >= 1 else dw
                cols = dw.amax(0) if dw.dim() == 2 else None
                print(f"   {name}: worst agent {worst} ({float(per_agent[worst]):.3e}; median over agents "
                      f"{float(per_agent.median()):.3e}); by gate r/z/n {[f'{float(x):.2e}' for x in rows]}"
                      + (f"; by column {[f'{float(x):.1e}' for x in cols]}" if cols is not None else ""), flush=True)
