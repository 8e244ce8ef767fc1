"""Same-process A/B of the RQ-VAE bench step (bench.py's timed step: forward, backward, bucket sync, AdamW at
B = 65,536) under GEMM policies, interleaved rounds. One JSON line per (round, policy).

  python tools/rq_policy_ab.py GEMM_SLAB_IO [...]   (names of ops.GEMM_* constants)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    import bench
    from data.schemas import SeqBatch
    from rqvae_hip import dp, gemm_tuning, ops
    gemm_tuning.enable()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = bench.build_model(dev)
    buckets = dp.GradBuckets([list(model.decoder.parameters()) + list(model.layers.parameters()),
                              list(model.encoder.parameters())], flat_views=True)
    opt = bench.make_adamw(model.parameters(), bench.CFG["lr"], bench.CFG["wd"])
    gen = torch.Generator(device=dev).manual_seed(1000)
    pool = [bench.make_items(65536, bench.CFG["input_dim"], gen, dev) for _ in range(4)]
    it = [0]

    def step():
        xb = pool[it[0] % len(pool)]
        it[0] += 1
        buckets.zero_grad()
        out = model(SeqBatch(None, None, None, xb, None, None), gumbel_t=0.2)
        out.loss.backward()
        buckets.synchronize()
        opt.step()

    pols = [("default", 0)] + [(n, getattr(ops, n)) for n in sys.argv[1:]]
    for rnd in range(3):
        for name, fl in pols:
            with ops.gemm_policy(fl):
                for _ in range(5):
                    step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(20):
                    step()
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / 20 * 1e3
            print(json.dumps({"round": rnd, "policy": name, "ms_per_step": round(ms, 4)}), flush=True)


if __name__ == "__main__":
    main()
