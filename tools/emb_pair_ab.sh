#!/bin/bash
# Amazon decoder step with the paired embedding (RQ_EMB_PAIR=1) vs cat + slice (0), alternating, same box
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/embab"; mkdir -p "$O"
for rep in 1 2 3; do for v in 0 1; do
  RQ_EMB_PAIR=$v timeout -k 10 200 python3 -u "$R/bench.py" --decoder-only --no-dm > "$O/$v.$rep.json" 2> "$O/err" \
    || { tail "$O/err"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.$rep.json')); print('pair $v', $rep, d['decoder_amazon']['ms_per_step'])"
done; done
