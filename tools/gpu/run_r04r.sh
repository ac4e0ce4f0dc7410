# round 4: GRU BPTT chunking -- the small-H gradient tests on the default build and on the in-loop-flush build
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04r"; mkdir -p "$O"
for v in default gflin; do
  if [ $v = default ]; then VE=""; else VE="D2D_LIB_VARIANT=$v D2D_ALLOW_ABLATION=1"; fi
  env $VE timeout -k 10 300 python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gru_gpu.py \
    -k "grads_match_autograd" > "$O/pytest_$v.log" 2>&1
  echo "$v rc=$? $(tail -1 "$O/pytest_$v.log")"
done
timeout -k 10 200 python3 tools/gpu/gru_iter.py 256 > "$O/gru_iter.log" 2>&1
echo "gru_iter rc=$? $(grep 'GRU D2D' "$O/gru_iter.log" | tail -1)"
