"""MFMA pipe utilisation of kernels from rocprofv3 PMC passes -> profiles/<tag>/pmc_mfma.json
(copied to profiles/pmc_mfma.json for bench.py).

Inputs: the counter CSVs of tools/gpu/pmc_mfma.sh (pass 1: SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_MFMA,
SQ_INSTS_VALU, SQ_INSTS_LDS, SQ_INSTS_SALU, SQ_WAVES; pass 2: SQ_WAVE_CYCLES, SQ_BUSY_CYCLES,
SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE) and the
kernel-trace stats CSV of the same workload (average duration per kernel).

MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (average duration x clock x 1024 SIMDs): the counter counts
MFMA-pipe cycles summed over every SIMD (MI355X_MICROARCH.md: 32 per 32x32x16 bf16 MFMA, i.e. its
pass count x 4), so the ratio is the mean fraction of time each SIMD's matrix pipe was busy.  The
clock is the one the box ran at: derived from GRBM_GUI_ACTIVE (GPU cycles the kernel was active, per
XCD, summed over the 8 XCDs) over the same average duration.

usage: python tools/pmc_mfma.py --stats STATS.csv --pmc P1.csv P2.csv --kernel REGEX ... --out OUT.json
       [--commit HASH] [--workload TEXT]
"""
import argparse
import collections
import csv
import json
import re

SIMDS, XCDS = 1024, 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", required=True)
    ap.add_argument("--pmc", nargs="+", required=True)
    ap.add_argument("--kernel", nargs="+", required=True, help="regexes of the kernels to report")
    ap.add_argument("--out", required=True)
    ap.add_argument("--commit", default=None)
    ap.add_argument("--workload", default=None)
    a = ap.parse_args()
    dur = {}
    for r in csv.DictReader(open(a.stats)):
        dur[r["Name"]] = (float(r["AverageNs"]), int(r["Calls"]))
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for path in a.pmc:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    names = sorted({k for k, _ in tot})
    out = []
    for rx in a.kernel:
        for name in names:
            if not re.search(rx, name):
                continue
            c = {cn: tot[(name, cn)] / max(1, len(disp[(name, cn)])) for (kn, cn) in tot if kn == name}
            d = dur.get(name)
            row = {"kernel": name, "per_dispatch": c, "dispatches": {cn: len(disp[(name, cn)]) for (kn, cn) in tot if kn == name}}
            if d:
                avg_ns, calls = d
                row["avg_duration_us"] = avg_ns / 1e3
                gui = c.get("GRBM_GUI_ACTIVE")
                clock = gui / XCDS / (avg_ns * 1e-9) if gui else 2.4e9
                row["clock_hz"] = clock
                busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
                if busy is not None:
                    row["mfma_busy_frac"] = busy / (avg_ns * 1e-9 * clock * SIMDS)
            if c.get("SQ_INSTS_MFMA"):
                row["valu_per_mfma"] = c.get("SQ_INSTS_VALU", 0.0) / c["SQ_INSTS_MFMA"]
            if c.get("SQ_WAVE_CYCLES"):
                w = c["SQ_WAVE_CYCLES"]
                row["wave_time_split"] = {"issuing": c.get("SQ_ACTIVE_INST_ANY", 0) / w,
                                          "issue_stalled": c.get("SQ_WAIT_INST_ANY", 0) / w,
                                          "waiting": c.get("SQ_WAIT_ANY", 0) / w}
            out.append(row)
    res = {"commit": a.commit, "workload": a.workload, "source": {"stats": a.stats, "pmc": a.pmc},
           "formula": "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (avg duration x clock x 1024 SIMDs); "
                      "clock = GRBM_GUI_ACTIVE / 8 XCDs / avg duration",
           "kernels": out}
    json.dump(res, open(a.out, "w"), indent=1)
    for r in out:
        print(f"{r['kernel'][:90]:90s} busy {r.get('mfma_busy_frac', float('nan')):.3f} "
              f"valu/mfma {r.get('valu_per_mfma', float('nan')):.2f} avg {r.get('avg_duration_us', 0):.1f} us")


if __name__ == "__main__":
    main()
