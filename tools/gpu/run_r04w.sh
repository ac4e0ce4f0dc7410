# round 4: GRU kernels without SLP vectorisation (packed f32 VALU beside MFMAs) -- A/B of the xp_load iteration
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04w"; mkdir -p "$O"
for v in default gnoslp default gnoslp; do
  if [ $v = default ]; then VE=""; else VE="D2D_LIB_VARIANT=$v D2D_ALLOW_ABLATION=1"; fi
  env $VE timeout -k 10 200 python3 tools/gpu/gru_iter.py 256 > "$O/gru_iter_$v.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 "$O/gru_iter_$v.log"; exit $rc; }
  echo "$v $(grep 'GRU D2D' "$O/gru_iter_$v.log" | tail -2 | tr '\n' ' ')"
done
