#!/bin/bash
# decoder-step A/B of the few-query fused backward threshold (RQ_ATTN_FEWQ_MIN_K), alternating twice
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/fewq"; mkdir -p "$O"
for rep in 1 2; do for v in 33 129; do
  RQ_ATTN_FEWQ_MIN_K=$v timeout -k 10 200 python3 -u "$R/bench.py" --decoder-only > "$O/amz_$v.$rep.json" 2> "$O/err" || { tail "$O/err"; exit 1; }
  RQ_ATTN_FEWQ_MIN_K=$v timeout -k 10 200 python3 -u "$R/bench.py" --decoder-only --dm-batch 8 > "$O/dm8_$v.$rep.json" 2>> "$O/err" || { tail "$O/err"; exit 1; }
  python3 -c "
import json,sys
a=json.load(open('$O/amz_$v.$rep.json')); b=json.load(open('$O/dm8_$v.$rep.json'))
fa=lambda d: [v for k,v in d.items() if isinstance(v,dict) and 'ms_per_step' in v] or [d]
print('min_k=$v rep=$rep', 'amazon', [x.get('ms_per_step') for x in fa(a)], 'dm8', [x.get('ms_per_step') for x in fa(b)])"
done; done
