#!/bin/bash
# GEMM parity, small-S slab reduction A/B (Amazon, C4 per-rank, RQ-VAE), per-shape GEMM plans at the C4
# config, SQ counter passes on the decoder GEMM shapes and the attention kernels.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out"; mkdir -p "$O"
bash "$R/tools/gpu_check.sh" gemmtests || exit 1
timeout -k 10 300 python -u -m pytest "$R/tests/test_train_gpu.py" -m gpu -x -q --timeout 120 --timeout-method thread -k amp > "$O/amp_test.log" 2>&1 || { tail -30 "$O/amp_test.log"; exit 1; }
tail -2 "$O/amp_test.log"
REPS=3 timeout -k 10 300 bash "$R/tools/lib_ab.sh" amazon base red16 || exit 1
REPS=3 timeout -k 10 300 bash "$R/tools/lib_ab.sh" dm8 base red16 || exit 1
REPS=2 timeout -k 10 200 bash "$R/tools/lib_ab.sh" rq base red16 || exit 1
timeout -k 10 150 python3 "$R/tools/dec_gemm_keys.py" 5 dm8 > "$O/dm8_gemm_keys.jsonl" 2> "$O/dm8_gemm_keys.err" || exit 1
bash "$R/tools/gpu_check.sh" sqdec || exit 1
timeout -k 10 500 bash "$R/tools/attn_pmc.sh" || exit 1
echo pass2 done
