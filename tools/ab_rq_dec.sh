#!/bin/bash
# Same-box A/B of the in-tree library against build_ab/<variant>.so: RQ-VAE step sequence (tools/prof_rq.sh)
# and the Amazon decoder step breakdown (tools/prof_dec.sh), alternating A B A B so a slow box hits both.
#   bash tools/ab_rq_dec.sh <variant> [rounds]
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out"; mkdir -p "$O"
V="$1"; N="${2:-1}"
for i in $(seq 1 "$N"); do
  for side in new "$V"; do
    if [ "$side" = new ]; then unset RQVAE_HIP_LIB; else export RQVAE_HIP_LIB="$R/build_ab/$V.so"; fi
    rm -rf "$O/prof"
    bash "$R/tools/prof_rq.sh" > "$O/prof_rq_$side$i.out" 2>&1 || exit 1
    python3 "$R/tools/step_sequence.py" "$(find "$O/prof" -name "rqonly_kernel_trace.csv" | head -1)" > "$O/rq_seq_$side$i.txt"
    head -1 "$O/rq_step_breakdown.txt" | sed "s/^/$side$i rq: /"
    bash "$R/tools/prof_dec.sh" "amz_$side$i" > /dev/null || exit 1
    head -1 "$O/amz_${side}${i}_step_breakdown.txt" | sed "s/^/$side$i amz: /"
    rm -rf "$O/prof" "$O/prof_amz_$side$i"
  done
done
unset RQVAE_HIP_LIB
