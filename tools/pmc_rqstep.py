#!/usr/bin/env python3
"""Short program for rocprofv3 --pmc passes over WHOLE RQ-VAE train steps (bench workload: ML-32M dims,
B = 65,536 items per step, 'high' matmul precision, HIP AdamW): the model, its k-means-like codebooks and
the items are built on the host and copied in (copies are not kernels, so the counters see only the train
steps), then `n` steps run. bench.py divides the summed FETCH_SIZE / WRITE_SIZE of every dispatch by n:
the step's HBM traffic, for its achieved-HBM % (BASELINE metric).

  rocprofv3 --pmc FETCH_SIZE -d out -o s -f csv -- python3 tools/pmc_rqstep.py 6
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    import bench
    from data.schemas import SeqBatch
    dev = torch.device("cuda", 0)
    m = bench.build_model(torch.device("cpu")).to(dev)
    g = torch.Generator().manual_seed(1000)
    x = torch.randn(65536, bench.CFG["input_dim"], generator=g)
    x = (x / x.norm(dim=1, keepdim=True)).to(dev)
    opt = bench.make_adamw(m.parameters(), bench.CFG["lr"], bench.CFG["wd"])
    for _ in range(n):
        opt.zero_grad(set_to_none=False)
        m(SeqBatch(None, None, None, x, None, None), gumbel_t=0.2).loss.backward()
        opt.step()
    torch.cuda.synchronize()
    print(f"pmc_rqstep: {n} RQ-VAE train steps at B=65536")


if __name__ == "__main__":
    main()
