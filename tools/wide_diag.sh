#!/bin/bash
# wide GEMM diagnostics: each library variant over the sweep
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/wdiag"; mkdir -p "$O"
for v in default diag1 diag2 diag3 epidirect; do
  if [ "$v" = default ]; then L="$R/rq-vae-recommender_amd/rqvae_hip/librqvae_hip.so"; else L="$R/build_ab/$v.so"; fi
  RQVAE_HIP_LIB="$L" timeout -k 10 120 python3 -u "$R/tools/gemm_wide_sweep.py" > "$O/$v.jsonl" 2> "$O/$v.err" || { echo "$v failed"; tail -3 "$O/$v.err"; exit 1; }
  echo "$v done"
done
