#!/bin/bash
# 64-tile GEMM: per-shape A/B (tools/x3s_ab.py), its GPU tests, then the decoder step with the
# 64-tile form on (default) and off (RQ_X3S=0).   gpurun -- bash tools/ab_x3s.sh
set -u
O=gpurun_out
timeout -k 10 200 python -u tools/x3s_ab.py > $O/x3s_ab.jsonl 2> $O/x3s_ab.err || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3s_gpu.py tests/test_gemm_splitk_epi_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/x3s_tests.log 2>&1
tail -3 $O/x3s_tests.log
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --decoder-only > $O/dec_x3s_on_$k.json 2> $O/dec_x3s_on.err || exit 1
  RQ_X3S=0 timeout -k 10 300 python -u bench.py --decoder-only > $O/dec_x3s_off_$k.json 2> $O/dec_x3s_off.err || exit 1
done
