"""Merge the summary lines of tools/gpu/ppo_grads_full_batch.py runs over agent ranges into one profile:
per tensor the max over the ranges and each range's median; the worst kernel / torch-fp32 excess over the
relu-mask flip envelope.
usage: python3 tools/merge_envelope.py out.json range1.json range2.json ..."""
import json
import sys


def summary(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


def main():
    out, srcs = sys.argv[1], sys.argv[2:]
    runs = [summary(p) for p in srcs]
    res = {"E": runs[0]["E"], "T": runs[0]["T"], "agents": sum(int(r["agents"]) for r in runs),
           "samples_per_agent": runs[0]["samples_per_agent"], "source": srcs,
           "bar": "excess over the relu-mask flip envelope, relative to max|g| "
                  "(tools/gpu/ppo_grads_full_batch.py envelope noemu)"}
    keys = [k for k, v in runs[0].items() if isinstance(v, dict) and "max" in v]
    for k in keys:
        res[k] = {"max": max(r[k]["max"] for r in runs), "median_of_ranges": [r[k]["median"] for r in runs]}
    res["worst_kernel_excess"] = max(res[k]["max"] for k in keys if k.startswith("excess/"))
    res["worst_torch32_excess"] = max(res[k]["max"] for k in keys if k.startswith("excess32/"))
    json.dump(res, open(out, "w"), indent=1)
    print(out, "worst kernel excess", res["worst_kernel_excess"], "torch fp32", res["worst_torch32_excess"])


if __name__ == "__main__":
    main()
