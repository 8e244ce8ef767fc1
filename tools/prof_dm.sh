#!/bin/bash
# rocprofv3 kernel summary of the ML-32M decoder step at B=64/GPU (bench.py --decoder-only --dm-batch 64)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out"; mkdir -p "$O"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o dm64 -- python3 "$R/bench.py" --decoder-only --dm-batch 64 \
  > "$O/prof_dm64.json" 2> "$O/prof_dm64.err" || { tail "$O/prof_dm64.err"; exit 1; }
cat "$O/prof_dm64.json"
