import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "rq-vae-recommender_amd"), ROOT, os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch
import pytest
import test_graph_gpu as t
mp = pytest.MonkeyPatch()
print("start", flush=True)
t.test_graph_replay_equals_eager(torch.device("cuda", 0), mp)
print("done", flush=True)
