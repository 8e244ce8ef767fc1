#!/bin/bash
# Amazon decoder step with the HIP batch-sum prologue (RQ_BATCH_SUM=1) vs torch broadcast add / repeat (0)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/bsab"; mkdir -p "$O"
for rep in 1 2 3; do for v in 0 1; do
  RQ_BATCH_SUM=$v timeout -k 10 200 python3 -u "$R/bench.py" --decoder-only --no-dm > "$O/$v.$rep.json" 2> "$O/err" \
    || { tail "$O/err"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.$rep.json')); print('batch_sum $v', $rep, d['decoder_amazon']['ms_per_step'])"
done; done
