#!/bin/bash
# rocprofv3 kernel trace of the RQ-VAE headline step alone (bench.py without decoder / extras / PMC / CPU leg)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out"; mkdir -p "$O"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o rqonly -- python3 "$R/bench.py" --no-cpu-baseline \
  --no-pmc --no-extras --no-decoder > "$O/prof_rqonly.json" 2> "$O/prof_rqonly.err" || { tail "$O/prof_rqonly.err"; exit 1; }
cat "$O/prof_rqonly.json"
T=$(find "$O/prof" -name "rqonly_kernel_trace.csv" | head -1)
python3 "$R/tools/step_breakdown.py" "$T" 10 60 > "$O/rq_step_breakdown.txt" && head -60 "$O/rq_step_breakdown.txt"
