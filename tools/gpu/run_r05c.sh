# round 5: critic on occupancy-sized grids; A/B + PMC of the update kernels
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 9
O="$R/gpurun_out/r05c"; mkdir -p "$O"
timeout -k 10 200 python3 -u tools/gpu/upd_ab.py 2048 64 > "$O/upd_ab_h64.json" 2>> "$O/upd_ab.err"
rc=$?; echo "upd_ab rc=$rc"; cat "$O/upd_ab_h64.json"; [ $rc -eq 0 ] || { tail -20 "$O/upd_ab.err"; exit $rc; }
timeout -k 10 200 python3 -u tools/gpu/upd_ab.py 65536 64 3 > "$O/upd_ab_h64_65536.json" 2>> "$O/upd_ab.err"
rc=$?; echo "upd_ab 65536 rc=$rc"; cat "$O/upd_ab_h64_65536.json"; [ $rc -eq 0 ] || { tail -20 "$O/upd_ab.err"; exit $rc; }
bash tools/gpu/pmc_upd.sh r05c wip 2048 64 > "$O/pmc.log" 2>&1
rc=$?; echo "pmc rc=$rc"; tail -8 "$O/pmc.log"
exit $rc
