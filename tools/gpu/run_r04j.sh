# round 4: env step with streaming (non-temporal) record stores vs default stores (D2D_NT_STORES)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04j"; mkdir -p "$O"
for nt in 0 1 0 1 0 1; do
  D2D_NT_STORES=$nt timeout -k 10 200 python3 bench.py --legs env --steps 300 --warmup 30 --no-cpu-baseline \
    > "$O/env_nt.json" 2> "$O/env_nt.err"
  rc=$?; [ $rc -eq 0 ] || { echo "env nt=$nt rc=$rc"; exit $rc; }
  python3 -c "
import json,sys
for l in open(sys.argv[1]).read().splitlines():
    if l.startswith('{'):
        d=json.loads(l); print('nt', sys.argv[2], round(d['value']/1e6,1), 'M env-steps/s', round(d['roofline']['kernel_avg_us'],2), 'us', round(d['fp32_obs']['env_steps_per_s']/1e6,1) if d.get('fp32_obs') else '')
" "$O/env_nt.json" $nt
done
