"""Same-process A/B of the ML-32M decoder step at 8 sequences per GPU (C4 per-rank shape) under forced query
splits of the fused attention backward (ops.ATTN_QSPLIT(n); 0 = the automatic choice), interleaved rounds
of bench.measure_decoder. One JSON line per (round, qsplit)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    import bench
    from rqvae_hip import gemm_tuning, ops
    gemm_tuning.enable()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for rnd in range(3):
        for n in (0, 2, 4, 6, 8):
            with ops.attn_policy(ops.ATTN_QSPLIT(n) if n else 0):
                r = bench.measure_decoder(dev, cfg=bench.DEC_DM, B=8, stats=False)
            print(json.dumps({"B": 8, "round": rnd, "qsplit": n, "ms_per_step": r["ms_per_step"]}), flush=True)


if __name__ == "__main__":
    main()
