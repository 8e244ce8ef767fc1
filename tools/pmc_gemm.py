#!/usr/bin/env python3
"""Short program for rocprofv3 --pmc passes: N launches of the split-bf16 GEMM (rq_gemm_bf16x3) at
one shape / operand layout, nothing else on the GPU besides input setup. One counter group per
process, e.g.

  rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm_bf16x3 -d out -o g -f csv -- \
      python3 tools/pmc_gemm.py 65536 512 768 1 1 5 [a_split b_split]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402

from rqvae_hip import ops  # noqa: E402


def main():
    M, N, K, a_kc, b_kc = (int(v) for v in sys.argv[1:6])
    n = int(sys.argv[6]) if len(sys.argv) > 6 else 5
    a_sp = len(sys.argv) > 7 and sys.argv[7] == "1"
    b_sp = len(sys.argv) > 8 and sys.argv[8] == "1"
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn((M, K) if a_kc else (K, M), generator=g, device=dev)
    b = torch.randn((N, K) if b_kc else (K, N), generator=g, device=dev)
    a = ops.split_bf16x3(a) if a_sp else a
    b = ops.split_bf16x3(b) if b_sp else b
    for _ in range(n):
        ops.gemm_x3(a, bool(a_kc), b, bool(b_kc), M, N, K)
    torch.cuda.synchronize()
    print(f"pmc_gemm: {n} launches of rq_gemm_bf16x3 at M={M} N={N} K={K} layouts a_kc={a_kc} b_kc={b_kc}")


if __name__ == "__main__":
    main()
