"""The captured gradient exchange (rqvae_hip.graph.GraphedSteps, in-graph RCCL all-reduces) on the GPU.

A one-GPU box cannot run two RCCL ranks, so the probe uses a world-1 RCCL group with
dp.GradBuckets(force_exchange=True): the same collectives, hooks, ordering and final wait are captured
into the replayed graph as at N ranks (a one-rank all-reduce is the identity, so every replayed step's
gradients must equal an eager step's bit for bit). Multi-rank semantics of the same code path are
covered on CPU by tests/test_dp.py ('graphed', 'empty'). The probe runs as a child process under a
timeout so that a hang inside a captured collective cannot outlive the test."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("race", ["", "race", "race_forever"])
def test_in_graph_exchange_matches_eager(race):
    """race: the capture starts with an eager all-reduce in flight, a second thread polling its Work the
    way the process group's watchdog does, and host memory pinned meanwhile (the round-3 abort): the
    quiesced capture must hold the exchange. race_forever: a poller that never stops fails the capture on
    ROCm even in thread-local mode (when it lands inside the capture window) — the step must fall back to the
    post-replay exchange, same gradients."""
    args = [sys.executable, os.path.join(ROOT, "tools", "graph_exchange_probe.py"), str(_port())] + ([race] if race else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["buckets"] > 1
    assert res["in_graph_default"], "RCCL group: the exchange should be captured in the graph"
    if race:
        assert res["race_polls"] > 0
    if race == "race_forever":
        # usually the never-ending poll fails the capture (then the step exchanges after its replay), but
        # whether the poller's query lands inside the capture window is up to the GIL / scheduler: a capture
        # it missed holds the exchange. Either outcome must be consistent and give the same gradients.
        assert (not res["in_graph"] and res["capture_error"] is not None) or \
            (res["in_graph"] and res["capture_error"] is None), res
    else:
        assert res["capture_error"] is None and res["in_graph"], res["capture_error"]
    assert res["steps"][-1]["graphs"] == 1
    for s in res["steps"]:
        assert s["max_abs_grad_diff"] == 0.0, res
