#!/bin/bash
# A/B of attention-kernel variants on the GPU box: per variant library build_ab/<name>.so, a
# rocprofv3 kernel-trace summary of tools/attn_probe.py (Amazon / ML-32M / C5 shapes), twice, in
# alternating order. bash tools/attn_ab.sh A B C ...
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/ab"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for rep in 1 2; do
  for v in "$@"; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$O/$v.$rep" -o p -- \
      python3 "$R/tools/attn_probe.py" "$R/build_ab/$v.so" > "$O/$v.$rep.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v failed ($rc)"; tail -5 "$O/$v.$rep.log"; exit $rc; fi
  done
done
python3 "$R/tools/ab_summary.py" "$O" "$@"
