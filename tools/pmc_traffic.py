"""Turn rocprofv3 --pmc CSVs (separate FETCH_SIZE and WRITE_SIZE passes) into
profiles/pmc_traffic.json: HBM bytes per launch of the env-step kernel.

Correction (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE
and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide
(16 B/lane) coalesced reads -> read bytes = 2 * FETCH_SIZE * 1024 (our reads
are 16-B/lane buffer rows plus narrow mask/counter reads, so this is an upper
bound for the narrow part); WRITE_SIZE is exact for 16-B/lane streaming stores
(obs/state/buffer rows).  Both raw and corrected values are recorded.

usage: python tools/pmc_traffic.py FETCH.csv WRITE.csv OUT.json --kernel comb_kernel --envs 65536 --agents 64
"""
import argparse
import csv
import json
import statistics


def per_dispatch(path, counter, kernel):
    vals = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")
            if kernel not in name or row.get("Counter_Name") != counter:
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--kernel", default="comb_kernel")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--agents", type=int, default=64)
    ap.add_argument("--algorithmic-bytes", type=float, default=172.0 * 64 * 65536)
    ap.add_argument("--commit", default=None, help="the commit the profiled tree was built from")
    a = ap.parse_args()
    f = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    w = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    if not f or not w:
        raise SystemExit(f"no {a.kernel} rows (fetch {len(f)}, write {len(w)})")
    # the median dispatch (reset launches are a few of many)
    fk, wk = statistics.median(f), statistics.median(w)
    read_b = 2.0 * fk * 1024
    write_b = wk * 1024
    out = {"kernel_prefix": a.kernel, "envs": a.envs, "agents": a.agents,
           "fetch_size_kib_median": fk, "write_size_kib_median": wk, "dispatches": [len(f), len(w)],
           "read_bytes_corrected": read_b, "write_bytes": write_b,
           "bytes_per_launch": read_b + write_b,
           "bytes_per_launch_raw": (fk + wk) * 1024,
           "algorithmic_bytes_per_launch": a.algorithmic_bytes,
           "traffic_over_algorithmic": (read_b + write_b) / a.algorithmic_bytes,
           "commit": a.commit, "source": {"fetch": a.fetch, "write": a.write}}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
