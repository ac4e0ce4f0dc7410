# round 5: critic fwd 2 chunks/iteration, one shared return column; A/B on real rollouts; central critic tests;
# configs + train legs; the fusion bound probe
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05k"; mkdir -p "$O"
timeout -k 10 300 python3 -u tools/gpu/upd_ab.py 2048 64 10 real > "$O/upd_ab_real.json" 2>> "$O/upd_ab.err"
rc=$?; echo "upd_ab real rc=$rc"; cat "$O/upd_ab_real.json"; [ $rc -eq 0 ] || { tail -20 "$O/upd_ab.err"; exit $rc; }
timeout -k 10 400 python3 -u -m pytest tests/test_learner_gpu.py tests/test_update_gpu.py -m gpu -v -s -k "central_critic or deferred or d2d_mlp or ippo_mlp" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" "$O/pytest.log" | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u bench.py --legs train,configs --no-cpu-baseline --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
t=d['train']; print('train', t['s_per_iteration'], t['phase_ms'])
c=d['configs']; print('c2', c['c2']['d2d_iteration_s'], c['c2']['phase_ms'])
[print('c5', s['agents'], s['d2d_iteration_s'], s['phase_ms']) for s in c['c5']['sweep']]" || tail -20 "$O/bench.err"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/gpu/fusion_bound.py > "$O/fusion_bound.json" 2> "$O/fusion_bound.err"
rc=$?; echo "fusion rc=$rc"; tail -12 "$O/fusion_bound.json"; tail -3 "$O/fusion_bound.err"
exit $rc
