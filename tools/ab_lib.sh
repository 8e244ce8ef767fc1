#!/bin/bash
# Same-box A/B of two builds of the C-ABI library: per-shape GEMM times (tools/x3s_ab.py) and the
# bench's decoder / RQ-VAE steps, alternating.   gpurun -- bash tools/ab_lib.sh build_ab/old.so [tag]
set -u
O=gpurun_out/ablib; mkdir -p $O
B="$1"; T="${2:-ab}"
RQVAE_HIP_LIB=$B timeout -k 10 200 python -u tools/x3s_ab.py > $O/${T}_shapes_B.jsonl 2>/dev/null || exit 1
timeout -k 10 200 python -u tools/x3s_ab.py > $O/${T}_shapes_A.jsonl 2>/dev/null || exit 1
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc --no-dm > $O/${T}_bench_A$k.json 2>/dev/null || exit 1
  RQVAE_HIP_LIB=$B timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc --no-dm > $O/${T}_bench_B$k.json 2>/dev/null || exit 1
done
echo done
