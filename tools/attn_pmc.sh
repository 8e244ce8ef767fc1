#!/bin/bash
# Attention kernels on the GPU box: HIP-event timing at the decoder shapes (tools/attn_probe.py),
# a rocprofv3 kernel-trace summary, and two SQ PMC passes (MFMA busy, waits, LDS conflicts).
#   gpurun --timeout 600 -- bash tools/attn_pmc.sh [lib.so]
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/attn"
mkdir -p "$O"
export TMPDIR=/tmp
run() {
  local name="$1" secs="$2"; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$secs" "$@"
  local rc=$?
  echo "[$(date +%T)] $name exit $rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run probe 180 python3 -u "$R/tools/attn_probe.py" "$@" > "$O/probe.jsonl" 2> "$O/probe.err"
cat "$O/probe.jsonl"
cd /tmp
run trace 180 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace" -o attn -- python3 "$R/tools/attn_probe.py" "$@" > "$O/trace.log" 2>&1
run pmc1 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES \
  --kernel-include-regex attn -f csv -d "$O/pmc1" -o attn -- python3 "$R/tools/attn_probe.py" "$@" > "$O/pmc1.log" 2>&1
run pmc2 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  --kernel-include-regex attn -f csv -d "$O/pmc2" -o attn -- python3 "$R/tools/attn_probe.py" "$@" > "$O/pmc2.log" 2>&1
echo done
