#!/bin/bash
# rocprofv3 kernel + HIP API trace of the drop-in trainers (tools/trainer_probe.py): when does the host
# enqueue each step's work relative to the GPU (the decoder trainer's inter-step gaps).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out"; mkdir -p "$O"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace -f csv -d "$O/trhost" -o trainer -- python3 "$R/tools/trainer_probe.py" \
  > "$O/prof_trainer_host.json" 2> "$O/prof_trainer_host.err" || { tail "$O/prof_trainer_host.err"; exit 1; }
ls -la "$O/trhost"
