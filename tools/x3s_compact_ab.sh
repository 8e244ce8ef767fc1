#!/bin/bash
# 64-tile GEMM compact-LDS A/B: GEMM GPU tests on the tree, then per-shape x3 / x3s / auto timings and the
# decoder steps (Amazon, ML-32M B=64) for build_ab/A.so and B.so, alternating.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/x3c"; mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gemm_bf16x3_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
for v in A B; do timeout -k 10 200 python3 -u tools/x3s_ab.py "$R/build_ab/$v.so" > "$O/shapes_$v.jsonl" 2>&1 || { tail "$O/shapes_$v.jsonl"; exit 1; }; done
for rep in 1 2; do for v in A B; do
  RQVAE_HIP_LIB="$R/build_ab/$v.so" timeout -k 10 200 python3 -u bench.py --decoder-only > "$O/amz_$v.$rep.json" 2> "$O/err" || { tail "$O/err"; exit 1; }
  RQVAE_HIP_LIB="$R/build_ab/$v.so" timeout -k 10 200 python3 -u bench.py --decoder-only --dm-batch 64 > "$O/dm_$v.$rep.json" 2>> "$O/err" || { tail "$O/err"; exit 1; }
  python3 -c "
import json
a=json.load(open('$O/amz_$v.$rep.json')); b=json.load(open('$O/dm_$v.$rep.json'))
print('$v rep $rep amazon', list(a.values())[0]['ms_per_step'], 'dm64', list(b.values())[0]['ms_per_step'])"
done; done
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
A = [json.loads(l) for l in open(f"{O}/shapes_A.jsonl") if l.startswith("{")]
B = [json.loads(l) for l in open(f"{O}/shapes_B.jsonl") if l.startswith("{")]
for a, b in zip(A, B):
    print(f"{a['shape']:28s} x3s {b['x3s']:7.1f} -> {a['x3s']:7.1f}   auto {b['auto']:7.1f} ({b['auto_plan'][0]}) -> {a['auto']:7.1f} ({a['auto_plan'][0]})  x3 {a['x3']:7.1f}")
PY
