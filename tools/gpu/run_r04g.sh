# round 4: GRU long-window value case with the head relu-flip-aware reference; the configs leg (graph env rates).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r04g"; mkdir -p "$O"
timeout -k 10 400 python3 -u tools/gpu/gru_long_diag.py > "$O/gru_long_diag.log" 2>&1
rc=$?; echo "diag rc=$rc"; grep -E "^(value|sigmoid)|ambiguous" "$O/gru_long_diag.log" | cut -c1-600
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gru_gpu.py \
  -k "long_window or xp_load or large_batch" > "$O/pytest_gru.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" "$O/pytest_gru.log" | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python3 bench.py --legs configs --steps 5 --warmup 2 --no-cpu-baseline > "$O/configs.json" 2> "$O/configs.err"
rc=$?; echo "configs rc=$rc"
python3 - "$O/configs.json" <<'PY'
import json, sys
for l in open(sys.argv[1]).read().splitlines():
    if l.startswith("{"):
        d = json.loads(l)["configs"]
        c2 = d["c2"]
        print("c2", round(c2["env_steps_per_s"] / 1e6, 2), "M eager,", round(c2["env_steps_per_s_graph"] / 1e6, 2), "M graph, iter",
              round(c2["d2d_iteration_s"] * 1e3, 1), "ms")
        for s in d["c5"]["sweep"]:
            print("c5", s["agents"], round(s["env_steps_per_s"] / 1e6, 2), round(s["env_steps_per_s_graph"] / 1e6, 2),
                  round(s["d2d_iteration_s"] * 1e3, 1), "ms", {k: round(v, 2) for k, v in s["phase_ms"].items()})
PY
exit $rc
