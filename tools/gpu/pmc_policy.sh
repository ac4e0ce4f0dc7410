# SQ counter passes for the fused policy kernel (one counter set per rocprofv3 run, no tracing domains)
R="$GRAFT_REPO_ROOT"; TAG="${1:-policy}"
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/pmc_$TAG"; mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
run() {
  timeout -k 10 300 rocprofv3 --pmc $2 --kernel-include-regex "policy_" -d "$OUT/$1" -o run --output-format csv -- \
    python3 "$R/bench.py" --legs rollout --steps 3 --warmup 1 --rollout-steps 6 --no-cpu-baseline > "$OUT/$1.log" 2>&1
}
run p1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" && \
run p2 "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
rc=$?
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
disp = max(1, max(n.values()) if n else 1)
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:.4g}  (per dispatch ~{tot[k] / max(1, n[k] / (n[k] and 1)):.4g}, rows {n[k]})")
PY

exit $rc
