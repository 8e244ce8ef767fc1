#!/bin/bash
# RQ-VAE headline step A/B of library builds (build_ab/<v>.so), alternating, same box:
#   bash tools/rq_ab.sh A B
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/rqab"; mkdir -p "$O"
for rep in 1 2 3; do for v in "$@"; do
  RQVAE_HIP_LIB="$R/build_ab/$v.so" timeout -k 10 200 python3 -u "$R/bench.py" --no-decoder --no-extras --no-cpu-baseline --no-pmc \
    > "$O/$v.$rep.json" 2> "$O/err" || { tail "$O/err"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.$rep.json')); print('$v', $rep, d['ms_per_step'], d['roofline']['frac'], d['roofline']['all_gemm_launches']['ms_per_step_total'])"
done; done
