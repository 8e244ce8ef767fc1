"""Same-process A/B of the decoder steps under module-attribute switches (the model's fusion flags,
e.g. modules.model:_FUSED_PROLOGUE=False), interleaved rounds so box-to-box clock spread cancels.
One JSON line per (config, round, variant).

  python tools/attr_ab.py "modules.model:_FUSED_PROLOGUE=False" [more variants ...]
"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def _parse(spec):
    sets = []
    for item in spec.split(","):
        lhs, val = item.split("=")
        mod, attr = lhs.split(":")
        sets.append((importlib.import_module(mod), attr, eval(val)))   # literal flag values (True / False / ints)
    return sets


def main():
    import bench
    from rqvae_hip import gemm_tuning
    gemm_tuning.enable()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    variants = [("default", [])] + [(s, _parse(s)) for s in sys.argv[1:]]
    rounds = int(os.environ.get("AB_ROUNDS", "3"))
    for cfg, B in ((bench.DEC, None), (bench.DEC_DM, 8)):
        for rnd in range(rounds):
            for name, sets in variants:
                prev = [(m, a, getattr(m, a)) for m, a, _ in sets]
                for m, a, v in sets:
                    setattr(m, a, v)
                try:
                    r = bench.measure_decoder(dev, cfg=cfg, B=B, stats=False)
                finally:
                    for m, a, v in prev:
                        setattr(m, a, v)
                print(json.dumps({"config": cfg["name"], "B": B, "round": rnd, "variant": name,
                                  "ms_per_step": r["ms_per_step"]}), flush=True)


if __name__ == "__main__":
    main()
