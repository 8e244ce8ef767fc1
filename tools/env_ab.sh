#!/bin/bash
# Step A/B of runtime switches (environment settings), alternating over REPS rounds, same box and library:
#   bash tools/env_ab.sh amazon|dm8|rq "RQ_X3_REDUCE_US=4" "RQ_X3_REDUCE_US=8" ...
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; mode="$1"; shift
O="$R/gpurun_out/envab_$mode"; mkdir -p "$O"
case "$mode" in
  amazon) args="--decoder-only --no-dm" ;;
  dm8) args="--decoder-only --dm-batch 8" ;;
  rq) args="--no-decoder --no-extras --no-cpu-baseline --no-pmc" ;;
  *) echo "mode?"; exit 2 ;;
esac
i=0
for rep in $(seq 1 ${REPS:-3}); do for v in "$@"; do
  i=$((i + 1))
  env $v timeout -k 10 200 python3 -u "$R/bench.py" $args > "$O/$i.json" 2> "$O/$i.err" || { tail "$O/$i.err"; exit 1; }
  python3 - "$O/$i.json" "$mode" "$v" "$rep" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
mode = sys.argv[2]
if mode == "rq":
    ms = d["ms_per_step"]
elif mode == "amazon":
    ms = d.get("decoder_amazon", d).get("ms_per_step")
else:
    dm = d.get("decoder_ml32m", d)
    ms = (dm.get("per_gpu_batch_8") or dm).get("ms_per_step")
print(mode, sys.argv[3], sys.argv[4], ms, flush=True)
PY
done; done
