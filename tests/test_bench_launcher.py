"""bench.py --gpus N outside torchrun: the parent starts N ranks through
torch.distributed.run as child processes and returns torchrun's status. CPU checks: the launcher command,
and that N rank processes really start (each one reaches the GPU check after joining a gloo group of N and
fails there on this GPU-less host) and a rank's failure is a nonzero exit of the parent."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_launcher_cmd_is_the_driver_form():
    import bench
    cmd = bench.launcher_cmd(4, ["--gpus", "4", "--steps", "3"], 29533)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=4" in cmd and "--master-port=29533" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1"
    assert cmd[-5:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "3"]


def test_gpus_2_starts_two_ranks_and_propagates_failure():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(RQVAE_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-extras"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0
    out = r.stdout + r.stderr
    # both ranks ran main() past the process-group join: each exits at the GPU check
    assert out.count("bench.py needs an MI355X") >= 2, out[-3000:]
    assert "{\"metric\"" not in r.stdout
