#!/usr/bin/env python3
"""Per-launch-shape device times of the split-bf16 GEMMs inside the RQ-VAE train step (HIP events
via ops.TIMER), at the bench workload. Keys: gemm_bf16x3:MxNxK:<a_kc><b_kc><a_split><b_split><epi>.

  python tools/gemm_keys.py [steps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from rqvae_hip import ops  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    from data.schemas import SeqBatch
    m = bench.build_model(dev)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=0.01, fused=True)
    x = bench.make_items(65536, 768, torch.Generator(device=dev).manual_seed(0), dev)

    def step():
        opt.zero_grad(set_to_none=True)
        m(SeqBatch(None, None, None, x, None, None), gumbel_t=0.2).loss.backward()
        opt.step()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ops.TIMER.reset()
    ops.TIMER.enabled = True
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ops.TIMER.enabled = False
    tot = 0.0
    rows = []
    for k in sorted(ops.TIMER.events):
        ms, n = ops.TIMER.mean_ms(k)
        tot += ms * n / steps
        if k.startswith("gemm_bf16x3:"):
            M, N, K = (int(v) for v in k.split(":")[1].split("x"))
            rows.append(dict(key=k, us=round(ms * 1e3, 1), per_step=n // steps,
                             tflops=round(2.0 * M * N * K / (ms * 1e-3) / 1e12, 1)))
        else:
            rows.append(dict(key=k, us=round(ms * 1e3, 1), per_step=n // steps))
    for r in rows:
        print(json.dumps(r))
    print(json.dumps({"timed_ms_per_step": round(tot, 3)}))


if __name__ == "__main__":
    main()
