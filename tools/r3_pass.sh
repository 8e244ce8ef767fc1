#!/bin/bash
# Round-3 measurement pass: key-split forward prefetch A/B (C4 per-rank config), rocprofv3 kernel stats of
# the RQ-VAE step with the base / current library (slab-reduction unroll), then decoder profiles + bench.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out"; mkdir -p "$O"; export TMPDIR=/tmp
REPS=3 timeout -k 10 300 bash "$R/tools/lib_ab.sh" dm8 cur kvpf1 || exit 1
cd /tmp
for v in base cur; do
  RQVAE_HIP_LIB="$R/build_ab/$v.so" timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$O/profrq_$v" -o rq -- \
    python3 "$R/bench.py" --no-decoder --no-extras --no-cpu-baseline --no-pmc > "$O/profrq_$v.json" 2> "$O/profrq_$v.err" || exit 1
done
cd "$R"
bash "$R/tools/gpu_check.sh" profdm8 profdec bench
