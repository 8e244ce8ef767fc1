#!/bin/bash
# Amazon decoder step A/B of library builds (build_ab/<v>.so), alternating, same box:
#   bash tools/dec_ab.sh A B
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/decab"; mkdir -p "$O"
for rep in 1 2 3; do for v in "$@"; do
  RQVAE_HIP_LIB="$R/build_ab/$v.so" timeout -k 10 200 python3 -u "$R/bench.py" --decoder-only --no-dm \
    > "$O/$v.$rep.json" 2> "$O/err" || { tail "$O/err"; exit 1; }
  python3 - "$O/$v.$rep.json" "$v" "$rep" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
def find(o):
    if isinstance(o, dict):
        if "decoder_amazon" in o: return o["decoder_amazon"]
        for v in o.values():
            r = find(v)
            if r is not None: return r
find_d = find(d) or d
print(sys.argv[2], sys.argv[3], find_d.get("ms_per_step"))
PY
done; done
