set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p "$R/gpurun_out"
timeout -k 10 200 python3 -u "$R/tools/gemm_epi_ab.py" 20 > "$R/gpurun_out/gemm_epi_ab.jsonl" 2>&1; rc=$?
cat "$R/gpurun_out/gemm_epi_ab.jsonl"; exit $rc
