"""Debug driver (GPU box): the RQ-VAE trainer at world 1 (twice) and world 2 (gloo, shared device), a
checkpoint every iteration; per-iteration, per-tensor relative differences as JSON lines."""
import glob
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_dist_trainers_gpu import _env, _port, PROBE  # noqa: E402

import torch  # noqa: E402


def run(world, out, graphs="1"):
    port = _port()
    ps = []
    for r in range(world):
        env = _env(r, world, port)
        env.update(PROBE_RQ_ONLY="1", PROBE_SAVE_EVERY="1", PROBE_RQ_ITERS="4", PROBE_GRAPHS=graphs)
        ps.append(subprocess.Popen([sys.executable, PROBE, out], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                   text=True))
    for p in ps:
        o, e = p.communicate(timeout=200)
        print(o.strip()[-400:], e.strip()[-1500:] if p.returncode else "", flush=True)


tmp = tempfile.mkdtemp()
for name, world, graphs in (("a", 1, "1"), ("b", 1, "1"), ("c", 2, "1"), ("d", 2, "0"), ("e", 1, "0")):
    run(world, f"{tmp}/{name}", graphs)
for it in range(0, 5):
    ref = f"{tmp}/a/vae/checkpoint_{it}.pt"
    if not os.path.exists(ref):
        continue
    A = torch.load(ref, map_location="cpu", weights_only=True)["model"]
    for name in "bcde":
        p = f"{tmp}/{name}/vae/checkpoint_{it}.pt"
        if not os.path.exists(p):
            print(json.dumps({"it": it, "run": name, "missing": True}))
            continue
        B = torch.load(p, map_location="cpu", weights_only=True)["model"]
        d = {k: round(float((v.double() - B[k].double()).norm() / v.double().norm().clamp_min(1e-30)), 8)
             for k, v in A.items() if torch.is_floating_point(v)}
        worst = sorted(d.items(), key=lambda kv: -kv[1])[:4]
        print(json.dumps({"it": it, "run": name, "worst": worst}), flush=True)
