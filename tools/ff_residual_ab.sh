#!/bin/bash
# decoder tests touching the fused feed-forward residual, then decoder-step A/B (RQ_FF_RESIDUAL=1 / 0)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/ffr"; mkdir -p "$O"; cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_fused_decoder_gpu.py tests/test_direct_grad_gpu.py tests/test_jagged_attention_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
for rep in 1 2; do for v in 1 0; do
  RQ_FF_RESIDUAL=$v timeout -k 10 200 python3 -u bench.py --decoder-only > "$O/amz_$v.$rep.json" 2> "$O/err" || { tail "$O/err"; exit 1; }
  RQ_FF_RESIDUAL=$v timeout -k 10 200 python3 -u bench.py --decoder-only --dm-batch 64 > "$O/dm_$v.$rep.json" 2>> "$O/err" || { tail "$O/err"; exit 1; }
  python3 -c "
import json
a=json.load(open('$O/amz_$v.$rep.json')); b=json.load(open('$O/dm_$v.$rep.json'))
print('ff_residual=$v rep $rep amazon', list(a.values())[0]['ms_per_step'], 'dm64', list(b.values())[0]['ms_per_step'])"
done; done
