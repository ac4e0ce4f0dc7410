# round 6: every bench leg through the 2-rank self-launch on one GPU (gloo rehearsal of the driver's N > 1 runs):
# no leg may deadlock or fail at world size 2.
# usage (GPU box): bash tools/gpu/run_r06m.sh
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r06m"; mkdir -p "$O"
D2D_BENCH_BACKEND=gloo D2D_BENCH_SHARE_GPU=1 timeout -k 10 1000 python3 -u bench.py --gpus 2 --steps 20 --warmup 5 \
  > "$O/bench_2ranks.json" 2> "$O/bench_2ranks.err"
rc=$?; echo "bench rc=$rc"; tail -c 300 "$O/bench_2ranks.err"
python3 -c "
import json; s=open('$O/bench_2ranks.json').read(); d=json.loads(s[s.index('{\"metric\"'):])
print('n_gpus', d['n_gpus'], 'ranks_seen', d['ranks_seen'], d['dist_backend'], 'value', round(d['value']/1e6,1), 'M', 'legs', [k for k in ('rollout','ppo','train','configs','d2denv','gru','gru_c5') if k in d])
print('ppo phases', d['ppo']['phase_ms_per_update'])"
exit $rc
