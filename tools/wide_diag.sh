#!/bin/bash
# wide GEMM diagnostics: gemm_shape_time.py under each library variant (build_ab/<v>.so from
# tools/build_variant.sh; "default" = the in-tree library): bash tools/wide_diag.sh v1 v2 ...
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/wdiag"; mkdir -p "$O"
for v in "$@"; do
  if [ "$v" = default ]; then L="$R/rq-vae-recommender_amd/rqvae_hip/librqvae_hip.so"; else L="$R/build_ab/$v.so"; fi
  RQVAE_HIP_LIB="$L" timeout -k 10 120 python3 -u "$R/tools/gemm_shape_time.py" "$v" >> "$O/shape_time.jsonl" 2> "$O/$v.err" || { echo "$v failed"; tail -3 "$O/$v.err"; exit 1; }
  echo "$v done"
done
