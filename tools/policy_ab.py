"""Same-process A/B of the decoder steps under GEMM policies (ops.gemm_policy around bench.measure_decoder:
every split-bf16 GEMM of the captured steps carries the flags), interleaved rounds. One JSON line per
(config, round, policy).   python tools/policy_ab.py [policy ...]   (names of ops.GEMM_* constants)"""
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
    pols = [("default", 0)] + [(n, getattr(ops, n)) for n in sys.argv[1:]]
    for cfg, B in ((bench.DEC, None), (bench.DEC_DM, 8)):
        for rnd in range(3):
            for name, fl in pols:
                with ops.gemm_policy(fl):
                    r = bench.measure_decoder(dev, cfg=cfg, B=B, stats=False)
                print(json.dumps({"config": cfg["name"], "B": B, "round": rnd, "policy": name,
                                  "ms_per_step": r["ms_per_step"]}), flush=True)


if __name__ == "__main__":
    main()
