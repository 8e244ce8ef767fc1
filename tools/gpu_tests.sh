#!/bin/bash
# GPU parity suite + smoke, each under its own time limit.
#   gpurun --timeout 900 -- bash tools/gpu_tests.sh [pytest -k expr]
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out"
mkdir -p "$O"
K="${1:-}"
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest "$R/tests" -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > "$O/gpu_tests.log" 2>&1
else
  timeout -k 10 900 python -u -m pytest "$R/tests" -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
fi
rc=$?
tail -5 "$O/gpu_tests.log"
exit $rc
