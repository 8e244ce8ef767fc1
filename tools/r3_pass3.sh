#!/bin/bash
# Padded per-wave partial tiles in the few-query / short attention kernels: attention parity tests,
# kernel-level probe (pad0 / pad1 libraries), decoder Amazon and C4 per-rank steps (base / pad1).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out"; mkdir -p "$O"
bash "$R/tools/gpu_check.sh" attntests || exit 1
for v in pad0 pad1; do
  RQVAE_HIP_LIB="$R/build_ab/$v.so" timeout -k 10 180 python3 -u "$R/tools/attn_probe.py" > "$O/probe_$v.jsonl" 2> "$O/probe_$v.err" || exit 1
done
grep -h amazon "$O/probe_pad0.jsonl" "$O/probe_pad1.jsonl"
REPS=3 timeout -k 10 300 bash "$R/tools/lib_ab.sh" amazon base pad1 || exit 1
REPS=2 timeout -k 10 200 bash "$R/tools/lib_ab.sh" dm8 base pad1 || exit 1
echo pass3 done
