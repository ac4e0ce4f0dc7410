# PMC passes (one counter group per run) over the GRU kernels.  usage: bash tools/gpu/pmc_gru.sh <tag> [grad|policy]
R="$GRAFT_REPO_ROOT"; TAG="${1:-gru}"; W="${2:-grad}"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$R/gpurun_out/pmc_${TAG}_$i" -o run --output-format csv -- \
    python3 "$R/tools/gpu/gru_probe.py" "$W" > "$R/gpurun_out/pmc_${TAG}_$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - "$R/gpurun_out" "$TAG" <<'PY'
import csv, glob, os, sys, collections
out, tag = sys.argv[1], sys.argv[2]
tot = collections.defaultdict(float)
for f in glob.glob(os.path.join(out, f"pmc_{tag}_*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "gru_" in r.get("Kernel_Name", ""):
            key = (r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])
            tot[key] += float(r["Counter_Value"])
for (k, c), v in sorted(tot.items()):
    print(f"{k:42s} {c:28s} {v:.4g}")
PY
