#!/bin/bash
# Per-kernel time and HBM traffic of the RQ-VAE train step (tools/pmc_rqstep.py: 6 whole steps at the bench
# workload): one kernel-trace pass and two PMC passes (FETCH_SIZE, WRITE_SIZE), summarised per kernel per
# step by tools/rqstep_traffic.py.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/rqstep_traffic"; mkdir -p "$O"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d "$O/trace" -o t -- python3 "$R/tools/pmc_rqstep.py" 6 > "$O/trace.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$O/fetch" -o f -- python3 "$R/tools/pmc_rqstep.py" 6 > "$O/fetch.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$O/write" -o w -- python3 "$R/tools/pmc_rqstep.py" 6 > "$O/write.log" 2>&1 || exit 1
python3 "$R/tools/rqstep_traffic.py" "$O" 6 > "$O/summary.txt" && cat "$O/summary.txt"
