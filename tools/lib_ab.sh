#!/bin/bash
# Step A/B of library builds (build_ab/<v>.so), alternating over 3 rounds, same box:
#   bash tools/lib_ab.sh amazon|dm8|rq A B [C ...]
# amazon: decoder Amazon step; dm8: decoder ML-32M at 8 sequences (the C4 per-rank config); rq: RQ-VAE step.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; mode="$1"; shift
O="$R/gpurun_out/libab_$mode"; mkdir -p "$O"
case "$mode" in
  amazon) args="--decoder-only --no-dm" ;;
  dm8) args="--decoder-only --dm-batch 8" ;;
  rq) args="--no-decoder --no-extras --no-cpu-baseline --no-pmc" ;;
  *) echo "mode?"; exit 2 ;;
esac
for rep in $(seq 1 ${REPS:-3}); do for v in "$@"; do
  RQVAE_HIP_LIB="$R/build_ab/$v.so" timeout -k 10 200 python3 -u "$R/bench.py" $args > "$O/$v.$rep.json" 2> "$O/$v.$rep.err" \
    || { tail "$O/$v.$rep.err"; exit 1; }
  python3 - "$O/$v.$rep.json" "$mode" "$v" "$rep" <<'PY'
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
