"""Does hipGraphLaunch (torch.cuda.CUDAGraph.replay) return before the graph has run? Host time of
replay() vs the graph's GPU time, for graphs of N kernels only, and with memset / memcpy nodes added, and
with a second host thread enqueueing on another stream during the replay. One JSON line per case."""
import json
import threading
import time

import torch


def build(kind, n=300, size=1 << 20):
    dev = torch.device("cuda", 0)
    a = torch.randn(size, device=dev)
    b = torch.randn(size, device=dev)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()

    def body():
        for i in range(n):
            a.mul_(1.0001).add_(b)     # two kernels
            if kind == "memset" and i % 20 == 0:
                b.zero_()
            if kind == "memcpy" and i % 20 == 0:
                b.copy_(a)
    with torch.cuda.stream(side):
        body()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        body()
    return g


def measure(kind, threaded=False):
    g = build(kind)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    other = torch.cuda.Stream()
    x = torch.zeros(1 << 16, device="cuda")
    host_other = []

    def side_work():
        t = time.perf_counter()
        with torch.cuda.stream(other):
            for _ in range(20):
                x.add_(1.0)
        host_other.append(time.perf_counter() - t)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    t0 = time.perf_counter()
    th = None
    if threaded:
        th = threading.Thread(target=lambda: (time.sleep(0.0005), side_work()))
        th.start()
    g.replay()
    t1 = time.perf_counter()
    ev1.record()
    if th is not None:
        th.join()
    torch.cuda.synchronize()
    return {"kind": kind, "threaded": threaded, "replay_host_ms": round((t1 - t0) * 1e3, 3),
            "graph_gpu_ms": round(ev0.elapsed_time(ev1), 3),
            "other_thread_host_ms": round(host_other[0] * 1e3, 3) if host_other else None}


def back_to_back(n_graphs):
    """Replay graphs back to back with no host sync: host time of each launch (the previous launch of the
    same graph exec still running on the GPU)."""
    gs = [build("kernels") for _ in range(n_graphs)]
    for g in gs:
        g.replay()
    torch.cuda.synchronize()
    host = []
    for i in range(6):
        t0 = time.perf_counter()
        gs[i % n_graphs].replay()
        host.append(round((time.perf_counter() - t0) * 1e3, 3))
    torch.cuda.synchronize()
    return {"kind": "back_to_back", "graphs": n_graphs, "replay_host_ms": host}


if __name__ == "__main__":
    print(json.dumps(back_to_back(1)), flush=True)
    print(json.dumps(back_to_back(2)), flush=True)
    for kind in ("kernels", "memset", "memcpy"):
        print(json.dumps(measure(kind)), flush=True)
    print(json.dumps(measure("kernels", threaded=True)), flush=True)
