# round 5: the tiles' entry row as a zeroed row of the entry sums (history_len 1 safe): GRU tests on the product lib
# (incl. history_len 1 cases), then the xp_load update / iteration vs the previous build (p1l), alternating
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05za"; mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_gru_gpu.py -m gpu -q -x \
  --timeout 400 --timeout-method thread -p no:cacheprovider > "$O/pytest_main.log" 2>&1
rc=$?; echo "pytest main rc=$rc"; tail -n 3 "$O/pytest_main.log"; [ $rc -eq 0 ] || exit $rc
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
g=d['gru']; print('$2', 'update_ms', round(g['update']['ms'], 2), 'iteration_s', round(g['d2d_iteration_s'], 4))"; }
for k in 1 2; do
  timeout -k 10 400 python3 -u bench.py --legs gru --steps 5 --warmup 2 --no-cpu-baseline > "$O/base_$k.json" 2> "$O/base_$k.err" || exit 11
  show "$O/base_$k.json" base
  for v in p1l; do
    D2D_LIB_VARIANT=$v D2D_ALLOW_ABLATION=1 timeout -k 10 400 python3 -u bench.py --legs gru --steps 5 --warmup 2 \
      --no-cpu-baseline > "$O/${v}_$k.json" 2> "$O/${v}_$k.err" || exit 12
    show "$O/${v}_$k.json" $v
  done
done
