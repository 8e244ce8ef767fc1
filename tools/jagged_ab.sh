#!/bin/bash
# jagged conversion A/B at HBM scale: bash tools/jagged_ab.sh A B C (build_ab/<v>.so), alternating twice
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p "$R/gpurun_out"
for rep in 1 2; do for v in "$@"; do
  timeout -k 10 120 python3 -u "$R/tools/jagged_probe.py" "$R/build_ab/$v.so" 2>&1 | grep '^{' || exit 1
done; done
