# Per-leg PMC of the MFMA kernels (a row's dispatches are all the leg's own launches): each leg of the
# bench run alone under a kernel-trace stats pass and two SQ counter passes (each its own rocprofv3 run, no tracing
# domains), summarised by tools/pmc_mfma.py into gpurun_out/pmcl_<tag>/pmc_mfma_<leg>.json.
# usage (GPU box): bash tools/gpu/pmc_legs.sh <tag> <commit> [legs]
R="$GRAFT_REPO_ROOT"; TAG="$1"; COMMIT="$2"; LEGS="${3:-rollout ppo gru_slot gru}"
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/pmcl_$TAG"; mkdir -p "$OUT"
for leg in $LEGS; do
  case $leg in
    rollout) RX='policy_split_kernel'; BARGS=(--legs rollout --rollout-steps 20) ;;
    ppo) RX='ppo_actor_grad|ppo_critic_grad'; BARGS=(--legs ppo --ppo-epochs 3) ;;
    gru_slot) RX='gru_policy_kernel'; BARGS=(--legs gru --gru-slot-only) ;;
    gru) RX='gru_grad_kernel'; BARGS=(--legs gru) ;;
  esac
  BARGS+=(--steps 5 --warmup 2 --no-cpu-baseline)
  D="$OUT/$leg"; mkdir -p "$D"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$D/stats" -o run --output-format csv -- \
    python3 "$R/bench.py" "${BARGS[@]}" > "$D/stats.log" 2>&1 || exit 11
  timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE \
    --kernel-include-regex "$RX" -d "$D/p1" -o run --output-format csv -- \
    python3 "$R/bench.py" "${BARGS[@]}" > "$D/p1.log" 2>&1 || exit 12
  timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS \
    --kernel-include-regex "$RX" -d "$D/p2" -o run --output-format csv -- \
    python3 "$R/bench.py" "${BARGS[@]}" > "$D/p2.log" 2>&1 || exit 13
  S=$(ls "$D"/stats/*kernel_stats.csv | head -1)
  P1=$(ls "$D"/p1/*counter_collection.csv | head -1)
  P2=$(ls "$D"/p2/*counter_collection.csv | head -1)
  python3 "$R/tools/pmc_mfma.py" --stats "$S" --pmc "$P1" "$P2" --kernel "$RX" --out "$OUT/pmc_mfma_$leg.json" \
    --commit "$COMMIT" --workload "bench.py ${BARGS[*]}" || exit 14
done
