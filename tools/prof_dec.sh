#!/bin/bash
# rocprofv3 kernel trace of one decoder config (bench.py --decoder-only [--dm-batch N]) and its per-step
# kernel breakdown (tools/step_breakdown.py): bash tools/prof_dec.sh <tag> [dm_batch]
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out"; mkdir -p "$O"; export TMPDIR=/tmp
TAG="$1"; shift
ARGS="--decoder-only"; [ $# -gt 0 ] && ARGS="$ARGS --dm-batch $1"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_$TAG" -o dec -- python3 "$R/bench.py" $ARGS \
  > "$O/prof_$TAG.json" 2> "$O/prof_$TAG.err" || { tail "$O/prof_$TAG.err"; exit 1; }
T=$(find "$O/prof_$TAG" -name "dec_kernel_trace.csv" | head -1)
python3 "$R/tools/step_breakdown.py" "$T" 10 80 > "$O/${TAG}_step_breakdown.txt" && head -3 "$O/${TAG}_step_breakdown.txt"
