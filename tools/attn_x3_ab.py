"""Same-process A/B of the ML-32M decoder steps (8 and 64 sequences per GPU) with the long-range attention
in split-bf16 (matmul 'high') vs exact fp32, interleaved rounds of bench.measure_decoder. `--bwd`: split-bf16
forwards in both arms, the fused backward's split-bf16 form (ops._ATTN_X3_BWD) on vs off; default: the
forwards (ops._ATTN_X3) on vs off. `--amazon`: the Amazon config (256 sequences) instead of ML-32M. One JSON
line per (batch, round, mode)."""
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
    attr = "_ATTN_X3_BWD" if "--bwd" in sys.argv else "_ATTN_X3"
    runs = [(bench.DEC, 256)] if "--amazon" in sys.argv else [(bench.DEC_DM, 8), (bench.DEC_DM, 64)]
    for cfg, B in runs:
        for rnd in range(3):
            for x3 in (True, False):
                setattr(ops, attr, x3)
                r = bench.measure_decoder(dev, cfg=cfg, B=B, stats=False)
                print(json.dumps({"cfg": cfg["name"], "B": B, "round": rnd, attr.lower().lstrip("_"): x3, "ms_per_step": r["ms_per_step"]}),
                      flush=True)
    setattr(ops, attr, True)


if __name__ == "__main__":
    main()
