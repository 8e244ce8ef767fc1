#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/attnf"; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest "$R/tests/test_jagged_attention_gpu.py" -m gpu -x -v --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1; rc=$?
tail -5 "$O/tests.log"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" "$O/tests.log" | head -30; exit $rc; }
timeout -k 10 180 python3 -u "$R/tools/attn_probe.py" > "$O/probe.jsonl" 2> "$O/probe.err" || { tail "$O/probe.err"; exit 1; }
cat "$O/probe.jsonl"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace" -o attn -- python3 "$R/tools/attn_probe.py" > "$O/trace.log" 2>&1 || exit 1
echo done
