#!/bin/bash
# Run a subset of the GPU test suite on the box: bash tools/gpu_tests.sh <pytest args...>
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$R/gpurun_out"
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu "$@" > "$R/gpurun_out/gpu_tests_sel.log" 2>&1
rc=$?
tail -40 "$R/gpurun_out/gpu_tests_sel.log"
exit $rc
