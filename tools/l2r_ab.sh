#!/bin/bash
# l2norm + recon rows-per-wave: kernel A/B, then the RQ-VAE headline step at RQ_L2R_RPW = 1 / 2 / 4 (same box)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/l2r"; mkdir -p "$O"
timeout -k 10 120 python3 -u "$R/tools/l2r_ab.py" || exit 1
for rep in 1 2; do for v in 1 2 4; do
  RQ_L2R_RPW=$v timeout -k 10 200 python3 -u "$R/bench.py" --no-decoder --no-extras --no-cpu-baseline --no-pmc \
    > "$O/$v.$rep.json" 2> "$O/err" || { tail "$O/err"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.$rep.json')); print('rpw $v', $rep, d['ms_per_step'])"
done; done
