# PMC of the MLP update kernels alone (tools/gpu/upd_ab.py workload: 2,048 envs x 200 slots x 64 agents on the
# record): a kernel-trace stats pass and two SQ counter passes, each its own rocprofv3 run, summarised by
# tools/pmc_mfma.py.  usage (GPU box): bash tools/gpu/pmc_upd.sh <tag> <commit> [E] [H]
R="$GRAFT_REPO_ROOT"; TAG="$1"; COMMIT="$2"; E="${3:-2048}"; H="${4:-64}"
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/pmcu_$TAG"; mkdir -p "$OUT"
RX='ppo_actor_grad|ppo_critic_grad'
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 "$R/tools/gpu/upd_ab.py" $E $H 5 > "$OUT/stats.log" 2>&1 || exit 11
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE \
  --kernel-include-regex "$RX" -d "$OUT/p1" -o run --output-format csv -- \
  python3 "$R/tools/gpu/upd_ab.py" $E $H 5 > "$OUT/p1.log" 2>&1 || exit 12
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS \
  --kernel-include-regex "$RX" -d "$OUT/p2" -o run --output-format csv -- \
  python3 "$R/tools/gpu/upd_ab.py" $E $H 5 > "$OUT/p2.log" 2>&1 || exit 13
S=$(ls "$OUT"/stats/*kernel_stats.csv | head -1)
P1=$(ls "$OUT"/p1/*counter_collection.csv | head -1)
P2=$(ls "$OUT"/p2/*counter_collection.csv | head -1)
python3 "$R/tools/pmc_mfma.py" --stats "$S" --pmc "$P1" "$P2" --kernel "$RX" --out "$OUT/pmc_mfma.json" \
  --commit "$COMMIT" --workload "tools/gpu/upd_ab.py $E $H 5"
