#!/bin/bash
# rocprofv3 kernel trace of the drop-in trainers (tools/trainer_probe.py: train_rqvae.train, then
# train_decoder.train at the Amazon config) and the decoder trainer's GPU busy / idle per steady step
# (tools/step_gaps.py over the last AdamW-delimited steps).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out"; mkdir -p "$O"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d "$O/trprof" -o trainer -- python3 "$R/tools/trainer_probe.py" \
  > "$O/prof_trainer.json" 2> "$O/prof_trainer.err" || { tail "$O/prof_trainer.err"; exit 1; }
T=$(find "$O/trprof" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/step_gaps.py" "$T" > "$O/trainer_step_gaps.txt"
cat "$O/trainer_step_gaps.txt"; cat "$O/prof_trainer.json"
