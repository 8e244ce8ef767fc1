#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each) over the Amazon decoder step (bench.py --decoder-only),
# kernels matching REGEX, summarised by tools/pmc_summary.py: bash tools/pmc_dec.sh <tag> [regex]
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/pmc_dec_$1"; mkdir -p "$O"
RX="${2:-attn_|gemm_}"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES \
  --kernel-include-regex "$RX" -f csv -d "$O" -o p1 -- python3 "$R/bench.py" --decoder-only --no-graph > "$O/p1.log" 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  --kernel-include-regex "$RX" -f csv -d "$O" -o p2 -- python3 "$R/bench.py" --decoder-only --no-graph > "$O/p2.log" 2>&1 || exit 1
python3 "$R/tools/pmc_summary.py" "$1" $(find "$O" -name "*counter_collection.csv") > "$O/summary.txt" && echo ok
