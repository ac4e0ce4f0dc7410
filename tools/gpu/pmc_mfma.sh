# MFMA pipe utilisation of the update / policy kernels from PMC: a kernel-trace
# stats pass and two SQ counter passes (each its own rocprofv3 run, no tracing domains) over the same
# bench legs, summarised by tools/pmc_mfma.py.
# usage: bash tools/gpu/pmc_mfma.sh <tag> <commit> [bench legs]
R="$GRAFT_REPO_ROOT"; TAG="$1"; COMMIT="$2"; LEGS="${3:-rollout,ppo,gru}"
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/pmcm_$TAG"; mkdir -p "$OUT"
RX='ppo_actor_grad|ppo_critic_grad|policy_split|gru_policy|gru_grad_kernel|gae_scan|normalize_pair|comb_kernel'
BARGS=(--legs "$LEGS" --steps 20 --warmup 5 --no-cpu-baseline --rollout-steps 20 --ppo-epochs 3)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 "$R/bench.py" "${BARGS[@]}" > "$OUT/stats.log" 2>&1 || exit 11
timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE \
  --kernel-include-regex "$RX" -d "$OUT/p1" -o run --output-format csv -- \
  python3 "$R/bench.py" "${BARGS[@]}" > "$OUT/p1.log" 2>&1 || exit 12
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS \
  --kernel-include-regex "$RX" -d "$OUT/p2" -o run --output-format csv -- \
  python3 "$R/bench.py" "${BARGS[@]}" > "$OUT/p2.log" 2>&1 || exit 13
S=$(ls "$OUT"/stats/*kernel_stats.csv | head -1)
P1=$(ls "$OUT"/p1/*counter_collection.csv | head -1)
P2=$(ls "$OUT"/p2/*counter_collection.csv | head -1)
python3 "$R/tools/pmc_mfma.py" --stats "$S" --pmc "$P1" "$P2" --kernel "$RX" --out "$OUT/pmc_mfma.json" \
  --commit "$COMMIT" --workload "bench.py ${BARGS[*]}"
