# smoke() then the whole GPU parity suite, each under its own time limit; stops at the first failure.
#   gpurun --timeout 1200 -- bash tools/smoke_and_tests.sh [pytest -k expr]
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p "$R/gpurun_out"
cd "$R" && timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > "$R/gpurun_out/smoke.log" 2>&1; rc=$?
tail -3 "$R/gpurun_out/smoke.log"; [ $rc -ne 0 ] && exit $rc
bash "$R/tools/gpu_tests.sh" "${1:-}"
