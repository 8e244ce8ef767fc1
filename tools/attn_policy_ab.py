"""Same-process A/B of the decoder steps under attention kernel policies (ops.attn_policy around
bench.measure_decoder: every varlen attention launch of the captured steps carries the RQ_ATTN_* flags),
interleaved rounds. python tools/attn_policy_ab.py [--b64] [policy ...] (names of ops.ATTN_* constants)."""
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
    names = [a for a in sys.argv[1:] if not a.startswith("--")]
    pols = [("default", 0)] + [(n, getattr(ops, n)) for n in names]
    batches = (8, 64) if "--b64" in sys.argv else (8,)
    for B in batches:
        for rnd in range(3):
            for name, fl in pols:
                with ops.attn_policy(fl):
                    r = bench.measure_decoder(dev, cfg=bench.DEC_DM, B=B, stats=False)
                print(json.dumps({"B": B, "round": rnd, "policy": name, "ms_per_step": r["ms_per_step"]}), flush=True)


if __name__ == "__main__":
    main()
