# round 4: GRU update accumulator-flush placement A/B (default: between 64-step chunks; gflin: in-loop conditional)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04q"; mkdir -p "$O"
for v in default gflin default gflin; do
  if [ $v = default ]; then VE=""; else VE="D2D_LIB_VARIANT=$v D2D_ALLOW_ABLATION=1"; fi
  env $VE timeout -k 10 200 python3 tools/gpu/gru_iter.py 256 > "$O/gru_iter_$v.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 "$O/gru_iter_$v.log"; exit $rc; }
  echo "$v $(grep 'GRU D2D' "$O/gru_iter_$v.log" | tail -2 | tr '\n' ' ')"
done
timeout -k 10 400 python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gru_gpu.py \
  -k "grads" > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$O/pytest.log"
exit $rc
