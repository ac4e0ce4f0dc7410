# round 5: env kernel A/B on one box (current comb_step build vs the pre-refactor env kernels, twice each, alternating);
# PMC of the central critic's forward kernel at 256 agents (two SQ passes)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05o"; mkdir -p "$O"
for k in 1 2; do
  timeout -k 10 200 python3 -u bench.py --legs env --no-cpu-baseline --steps 50 --warmup 10 > "$O/env_new_$k.json" 2> "$O/env_new_$k.err" || exit 11
  D2D_LIB_VARIANT=envold D2D_ALLOW_ABLATION=1 timeout -k 10 200 python3 -u bench.py --legs env --no-cpu-baseline --steps 50 --warmup 10 \
    > "$O/env_old_$k.json" 2> "$O/env_old_$k.err" || exit 12
  python3 -c "
import json
for n in ('new', 'old'):
    d = json.loads(open('$O/env_' + n + '_$k.json').read().strip().splitlines()[-1])
    print(n, $k, round(d['value'] / 1e6, 1), 'M', d['roofline']['kernel_avg_us'])"
done
cd /tmp && export TMPDIR=/tmp
D="$O/pmc_critic"; mkdir -p "$D"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$D/stats" -o run --output-format csv -- \
  python3 "$R/tools/gpu/critic_probe.py" 256 3 > "$D/stats.log" 2>&1 || exit 13
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE \
  --kernel-include-regex "critic_fwd" -d "$D/p1" -o run --output-format csv -- python3 "$R/tools/gpu/critic_probe.py" 256 3 > "$D/p1.log" 2>&1 || exit 14
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS \
  --kernel-include-regex "critic_fwd" -d "$D/p2" -o run --output-format csv -- python3 "$R/tools/gpu/critic_probe.py" 256 3 > "$D/p2.log" 2>&1 || exit 15
S=$(ls "$D"/stats/*kernel_stats.csv | head -1); P1=$(ls "$D"/p1/*counter_collection.csv | head -1); P2=$(ls "$D"/p2/*counter_collection.csv | head -1)
python3 "$R/tools/pmc_mfma.py" --stats "$S" --pmc "$P1" "$P2" --kernel "critic_fwd" --out "$O/pmc_critic_fwd.json" --commit wip \
  --workload "tools/gpu/critic_probe.py 256 3" || exit 16
python3 -c "
import json; d = json.load(open('$O/pmc_critic_fwd.json'))
for k in d['kernels']: print(k['kernel'][:60], k['avg_duration_us'], k['mfma_busy_frac'], k['valu_per_mfma'], k.get('wave_time_split'))"
