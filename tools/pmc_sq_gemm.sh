#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each) over tools/pmc_gemm.py for the split-bf16 GEMM.
#   bash tools/pmc_sq_gemm.sh M N K a_kc b_kc a_split b_split tag
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/pmc_gemm_$8"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
A="$1 $2 $3 $4 $5 5 $6 $7"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES \
  --kernel-include-regex "gemm_(bf16x3|x3w)" -f csv -d "$O" -o p1 -- python3 "$R/tools/pmc_gemm.py" $A > "$O/p1.log" 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  --kernel-include-regex "gemm_(bf16x3|x3w)" -f csv -d "$O" -o p2 -- python3 "$R/tools/pmc_gemm.py" $A > "$O/p2.log" 2>&1 || exit 1
echo ok
