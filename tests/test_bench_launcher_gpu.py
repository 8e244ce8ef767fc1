"""bench.py --gpus 2 on a one-GPU box: the parent starts two ranks through
torch.distributed.run; both share the one MI355X (RQVAE_SHARE_DEVICE=1) over gloo (RCCL refuses two ranks
on one GPU). The line must report two ranks (n_gpus, parallelism dp2, the process group's census, the
decoder's data-parallel line), and a rank that dies must make the parent exit nonzero."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--gpus", "2", "--no-extras", "--no-pmc", "--no-cpu-baseline", "--no-dm", "--steps", "3", "--warmup", "2"]


def _run(env):
    """bench.py as a child; its stderr (progress lines) streams into gpurun_out/ while it runs."""
    log_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(log_dir, exist_ok=True)
    with open(os.path.join(log_dir, "test_bench_launcher.log"), "a") as log:
        p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), *ARGS], stdout=subprocess.PIPE,
                           stderr=log, text=True, timeout=240, env=env, cwd=ROOT)
    return p


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(RQVAE_DIST_BACKEND="gloo", RQVAE_SHARE_DEVICE="1", PYTHONUNBUFFERED="1", **kw)
    return env


def test_bench_gpus_2_runs_two_ranks():
    r = _run(_env())
    assert r.returncode == 0, r.stdout[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{\"metric\"")]
    assert len(lines) == 1, r.stdout[-2000:]   # one line: rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    assert line["config"]["global_batch"] == 2 * line["config"]["per_gpu_batch"]
    c = line["rccl_ranks"]
    assert c["process_group_size"] == 2 and c["allreduce_rank_count"] == 2 and c["backend"] == "gloo"
    assert [d["device"] for d in c["devices"]] == [0, 0] and all(d["share_device"] for d in c["devices"])
    assert line["decoder_amazon"]["n_gpus"] == 2 and line["decoder_amazon"]["parallelism"] == "dp2"
    assert line["value"] > 0 and line["decoder_amazon"]["ctx_tokens_per_s"] > 0


def test_bench_gpus_2_rank_failure_is_nonzero_exit():
    r = _run(_env(RQVAE_BENCH_FAIL_RANK="1"))
    assert r.returncode != 0
    with open(os.path.join(ROOT, "gpurun_out", "test_bench_launcher.log")) as f:
        assert "RQVAE_BENCH_FAIL_RANK: rank 1" in f.read()
    assert not [l for l in r.stdout.splitlines() if l.startswith("{\"metric\"")]
