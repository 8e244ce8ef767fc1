#!/usr/bin/env python3
"""The drop-in trainers' own timing (bench.measure_trainers: train_rqvae.train / train_decoder.train with
their LAST_RUN spans), one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

if __name__ == "__main__":
    from rqvae_hip import gemm_tuning
    gemm_tuning.enable()
    print(json.dumps(bench.measure_trainers()), flush=True)
