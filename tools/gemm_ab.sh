#!/bin/bash
# A/B of split-bf16 GEMM library variants (build_ab/<name>.so) on the GPU box:
#   bash tools/gemm_ab.sh reps W0 W1 ...  -> gpurun_out/gemm_ab_<name>.jsonl (two passes, alternating)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
reps="$1"; shift
for pass in 1 2; do
  for v in "$@"; do
    RQVAE_HIP_LIB="$R/build_ab/$v.so" timeout -k 10 240 python3 -u "$R/tools/gemm_ab.py" "$reps" \
      > "$R/gpurun_out/gemm_ab_${v}_$pass.jsonl" 2>&1 || { echo "variant $v failed"; tail -5 "$R/gpurun_out/gemm_ab_${v}_$pass.jsonl"; exit 1; }
  done
done
python3 - "$R" "$@" <<'PY'
import json, sys, collections
R, vs = sys.argv[1], sys.argv[2:]
tab = collections.defaultdict(dict)
for v in vs:
    for p in (1, 2):
        for l in open(f"{R}/gpurun_out/gemm_ab_{v}_{p}.jsonl"):
            if l.startswith("{"):
                d = json.loads(l)
                k = (d["case"], d["kernel"])
                tab[k].setdefault(v, []).append(d["us"])
print("case".ljust(28), "".join(v.rjust(16) for v in vs))
for k, row in tab.items():
    print(f"{k[0]+' '+k[1]:28s}", "".join(f"{min(row.get(v,[0])):16.1f}" for v in vs))
PY
