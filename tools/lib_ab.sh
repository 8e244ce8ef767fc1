#!/bin/bash
# Cross-process A/B of library builds (RQVAE_HIP_LIB): interleaved rounds of the decoder steps (tools/attr_ab.py,
# default variant only) and the RQ-VAE bench step (tools/rq_policy_ab.py) per library.
#   bash tools/lib_ab.sh <name>=<path.so> [...]   ("default" = the in-tree library)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
for rnd in 1 2; do
  for spec in default "$@"; do
    name="${spec%%=*}"; lib="${spec#*=}"
    [ "$spec" = default ] && lib="$R/rq-vae-recommender_amd/rqvae_hip/librqvae_hip.so"
    RQVAE_HIP_LIB="$lib" AB_ROUNDS=1 timeout -k 10 300 python3 -u "$R/tools/attr_ab.py" | sed "s/^/{\"lib\": \"$name\", \"r\": $rnd, \"x\": /; s/$/}/" || exit 1
    RQVAE_HIP_LIB="$lib" timeout -k 10 300 python3 -u "$R/tools/rq_policy_ab.py" | sed "s/^/{\"lib\": \"$name\", \"r\": $rnd, \"rq\": /; s/$/}/" || exit 1
  done
done
