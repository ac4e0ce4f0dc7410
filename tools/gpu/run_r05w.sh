# round 5: GRU update with the padding-region BPTT collapsed (PADC): GRU + learner tests, xp_load update / iteration
# A/B against the PADC=0 build, c5 GRU leg at 128 / 256 agents
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05w"; mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests/test_gru_gpu.py tests/test_learner_gpu.py -m gpu -q \
  --timeout 400 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
g=d['gru']; print('$2', 'update_ms', round(g['update']['ms'], 2), 'iteration_s', round(g['d2d_iteration_s'], 4))"; }
for k in 1 2; do
  timeout -k 10 400 python3 -u bench.py --legs gru --steps 5 --warmup 2 --no-cpu-baseline > "$O/gru_new_$k.json" 2> "$O/gru_new_$k.err" || exit 11
  show "$O/gru_new_$k.json" new
  D2D_LIB_VARIANT=padc0 D2D_ALLOW_ABLATION=1 timeout -k 10 400 python3 -u bench.py --legs gru --steps 5 --warmup 2 \
    --no-cpu-baseline > "$O/gru_old_$k.json" 2> "$O/gru_old_$k.err" || exit 12
  show "$O/gru_old_$k.json" old
done
timeout -k 10 600 python3 -u bench.py --legs gru_c5 --gru-c5-agents 64,128,256 --no-cpu-baseline > "$O/gru_c5.json" 2> "$O/gru_c5.err" || exit 13
python3 -c "
import json; d=json.loads(open('$O/gru_c5.json').read().strip().splitlines()[-1])
print(json.dumps(d.get('c5_gru_summary'))[:1500])"
