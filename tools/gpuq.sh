#!/bin/bash
# Queue helper (run from the repo root): tools/gpuq.sh <log> <gpurun args...>
# queue helper: re-submit a gpurun call while the pool reports a transient (nothing-charged) status
out="$1"; shift
for i in $(seq 1 30); do
  timeout 3000 /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  if grep -q "status=transient" "$out"; then sleep 60; continue; fi
  break
done
echo "[gpuq] attempts=$i" >> "$out"
