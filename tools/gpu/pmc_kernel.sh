# SQ counter passes (one counter set per rocprofv3 run, no tracing domains) for the kernels
# matching a regex, over a bench.py leg.
# usage: bash tools/gpu/pmc_kernel.sh <tag> <kernel-regex> <bench args...>
R="$GRAFT_REPO_ROOT"; TAG="$1"; RX="$2"; shift 2
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/pmc_$TAG"; mkdir -p "$OUT"
run() {
  timeout -k 10 300 rocprofv3 --pmc $2 --kernel-include-regex "$RX" -d "$OUT/$1" -o run --output-format csv -- \
    python3 "$R/bench.py" --no-cpu-baseline "${BENCH_ARGS[@]}" > "$OUT/$1.log" 2>&1
}
BENCH_ARGS=("$@")
run p1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" && \
run p2 "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
rc=$?
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"][:60], r["Counter_Name"])
        tot[key] += float(r["Counter_Value"]); n[key] += 1
for k in sorted(tot):
    print(f"{k[0]:60s} {k[1]:26s} total {tot[k]:.4g}  rows {n[k]}")
PY
exit $rc
