# round 6: the hand-written critic dW1 kernel (tests + the c5 configs leg), single_kernel A/B (plain / NT stores /
# flat emission) and its SQ counters.
# usage (GPU box): bash tools/gpu/run_r06c.sh <commit>
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06c"; mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_critic_dw1_gpu.py tests/test_learner_gpu.py -k "dw1 or central_critic or d2d" -m gpu -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$O/pytest_gpu.log" | tail -3
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 300 python3 -u bench.py --legs d2denv --d2denv-env-only --steps 5 --warmup 2 --no-cpu-baseline --env-mode record > "$O/single_plain_$k.json" 2>&1 || exit 11
  D2D_NT_STORES=1 timeout -k 10 300 python3 -u bench.py --legs d2denv --d2denv-env-only --steps 5 --warmup 2 --no-cpu-baseline --env-mode record > "$O/single_nt_$k.json" 2>&1 || exit 12
  D2D_LIB_VARIANT=sflat D2D_ALLOW_ABLATION=1 timeout -k 10 300 python3 -u bench.py --legs d2denv --d2denv-env-only --steps 5 --warmup 2 --no-cpu-baseline --env-mode record > "$O/single_flat_$k.json" 2>&1 || exit 13
  D2D_NT_STORES=1 D2D_LIB_VARIANT=sflat D2D_ALLOW_ABLATION=1 timeout -k 10 300 python3 -u bench.py --legs d2denv --d2denv-env-only --steps 5 --warmup 2 --no-cpu-baseline --env-mode record > "$O/single_flatnt_$k.json" 2>&1 || exit 14
done
for f in "$O"/single_*.json; do python3 -c "
import json,sys; s=open('$f').read(); d=json.loads(s[s.index('{\"metric\"'):]); print('$f'.split('/')[-1], round(d['d2denv']['kernel_avg_us'],1), round(d['d2denv']['hbm_frac'],3))"; done
timeout -k 10 400 python3 -u bench.py --legs configs --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench_configs.json" 2> "$O/bench_configs.err"
rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
BARGS=(--legs d2denv --d2denv-env-only --steps 5 --warmup 2 --no-cpu-baseline --env-mode record)
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD \
  --kernel-include-regex single_kernel -d "$O/sq1" -o run --output-format csv -- python3 "$R/bench.py" "${BARGS[@]}" > "$O/sq1.log" 2>&1 || exit 21
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS \
  --kernel-include-regex single_kernel -d "$O/sq2" -o run --output-format csv -- python3 "$R/bench.py" "${BARGS[@]}" > "$O/sq2.log" 2>&1 || exit 22
echo done
