#!/bin/bash
# rocprofv3 kernel trace of the C4 per-rank decoder step (bench.py --decoder-only --dm-batch 8) and its
# per-step kernel breakdown (tools/step_breakdown.py).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out"; mkdir -p "$O"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_c4" -o c4 -- python3 "$R/bench.py" --decoder-only --dm-batch 8 \
  > "$O/prof_c4.json" 2> "$O/prof_c4.err" || { tail "$O/prof_c4.err"; exit 1; }
T=$(find "$O/prof_c4" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/step_breakdown.py" "$T" > "$O/c4_step_breakdown.txt"
head -60 "$O/c4_step_breakdown.txt"
