# round 4: policy-kernel Philox placement A/B (default = drawn before the tile MFMAs; prng0 = in the epilogue;
# psgb = early + scheduling-group hints), rollout leg at the headline slot.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04i"; mkdir -p "$O"
for v in default prng0 psgb default prng0 psgb; do
  if [ $v = default ]; then VE=""; else VE="D2D_LIB_VARIANT=$v D2D_ALLOW_ABLATION=1"; fi
  env $VE timeout -k 10 200 python3 bench.py --legs rollout --steps 5 --warmup 2 --no-cpu-baseline \
    --rollout-steps 60 > "$O/policy_$v.json" 2> "$O/policy_$v.err"
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit $rc; }
  python3 -c "
import json,sys
for l in open(sys.argv[1]).read().splitlines():
    if l.startswith('{'):
        r=json.loads(l)['rollout']; print(sys.argv[2], round(r['policy_kernel_us'],1), round(r['env_kernel_us'],1))
" "$O/policy_$v.json" $v
done
timeout -k 10 300 python3 -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_policy_gpu.py \
  tests/test_learner_gpu.py -k "sampl or philox or graph or matches_reference" > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$O/pytest.log"
exit $rc
