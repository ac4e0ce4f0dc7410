"""Print the headline and the main legs of a bench.py JSON line (file with the line among other output).
usage: python tools/bench_summary.py BENCH.json"""
import json
import sys


def main(path):
    txt = open(path).read()
    d = json.loads([ln for ln in txt.splitlines() if ln.startswith("{")][-1])
    print("value", round(d["value"] / 1e6, 1), "M", d["unit"], "ms/step", round(d["ms_per_step"], 4))
    r = d["roofline"]
    print("roofline", r["kernel"], "frac", round(r["frac"], 3), "kernel_avg_us", round(r["kernel_avg_us"], 1))
    ro = d["rollout"]
    print("rollout policy_us", round(ro["policy_kernel_us"], 1), "env_us", round(ro["env_kernel_us"], 1),
          "env_steps/s", round(ro["env_steps_per_s"] / 1e6, 1), "M")
    p = d["ppo"]
    k = p["kernels"]
    print("ppo updates/s", round(p["updates_per_s"], 1), "actor_ms", round(k["actor"]["ms"], 3), "critic_ms",
          round(k["critic"]["ms"], 3))
    t = d["train"]
    print("train s/iter", round(t["s_per_iteration"], 4), {a: round(b, 1) for a, b in t["phase_ms"].items()})
    g = d["gru"]
    print("gru policy_slot_ms", round(g["policy_slot"]["ms"], 1), "update_ms", round(g["update"]["ms"], 1),
          "d2d_iteration_s", round(g["d2d_iteration_s"], 3))
    c = d["configs"]
    print("c2 ms", round(c["c2"]["d2d_iteration_s"] * 1e3, 1), "c5 ms",
          [(s["agents"], round(s["d2d_iteration_s"] * 1e3, 1)) for s in c["c5"]["sweep"]])
    print("d2denv", round(d["d2denv"]["env_steps_per_s"] / 1e6, 1), "M", "cpu_baseline",
          round(d["cpu_baseline"]["value"]), d["cpu_baseline"]["kind"])


if __name__ == "__main__":
    main(sys.argv[1])
