#!/usr/bin/env python3
"""What the process group's flight recorder (FR) shows about the watchdog's work list, and whether an
event poller on ANOTHER process group's collective breaks a capture (world-1 RCCL, one GPU).

  TORCH_FR_BUFFER_SIZE=64 python3 tools/fr_probe.py PORT

Prints one JSON line per phase: the FR entries (id, pg, state, retired) after an eager all-reduce, how
long until the watchdog retires it, what a captured all-reduce leaves in the FR, and whether a capture
on the default group survives a thread that keeps polling a Work of a second group."""
import json
import os
import sys
import threading
import time

import torch
import torch.distributed as dist
import torch._C._distributed_c10d as c10d


def entries():
    d = json.loads(c10d._dump_nccl_trace_json(includeCollectives=True, onlyActive=False))
    return [{k: e.get(k) for k in ("record_id", "pg_id", "collective_seq_id", "state", "retired",
                                   "time_discovered_completed_ns", "profiling_name")}
            for e in d.get("entries", [])]


def out(phase, **kw):
    print(json.dumps(dict(phase=phase, **kw), default=str), flush=True)


def main():
    port = sys.argv[1] if len(sys.argv) > 1 else "29541"
    os.environ.setdefault("TORCH_FR_BUFFER_SIZE", "64")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    pg2 = dist.new_group([0])
    x = torch.ones(1 << 20, device=dev)
    w = dist.all_reduce(x, async_op=True)
    out("eager_issued", entries=entries())
    w.wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        es = entries()
        if es and all(e["retired"] for e in es):
            break
        time.sleep(0.005)
    out("eager_retired", after_ms=round((time.perf_counter() - t0) * 1e3, 1), entries=entries())
    # a captured all-reduce: is it recorded, and does the watchdog ever retire it?
    g = torch.cuda.CUDAGraph()
    err = None
    try:
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            x.mul_(0.5)
            dist.all_reduce(x)
    except Exception as e:   # noqa: BLE001
        err = repr(e)[:300]
    out("captured", err=err, entries=entries())
    if err is None:
        g.replay()
        torch.cuda.synchronize()
        time.sleep(0.3)
        out("after_replay", entries=entries())
    # capture on the default group while a thread keeps polling a completed Work of pg2
    w2 = dist.all_reduce(torch.ones(1024, device=dev), group=pg2, async_op=True)
    w2.wait()
    torch.cuda.synchronize()
    stop, polls = threading.Event(), [0]

    def poll():
        while not stop.is_set():
            w2.is_completed()
            polls[0] += 1
    th = threading.Thread(target=poll, daemon=True)
    th.start()
    time.sleep(0.01)
    g2 = torch.cuda.CUDAGraph()
    err2 = None
    try:
        with torch.cuda.graph(g2, capture_error_mode="thread_local"):
            x.mul_(0.5)
            dist.all_reduce(x)
    except Exception as e:   # noqa: BLE001
        err2 = repr(e)[:300]
    stop.set()
    th.join()
    out("capture_with_other_group_poller", err=err2, polls=polls[0])
    # and the same with the poller on a Work of the default group (the known failure)
    w3 = dist.all_reduce(torch.ones(1024, device=dev), async_op=True)
    w3.wait()
    torch.cuda.synchronize()
    stop2, polls2 = threading.Event(), [0]

    def poll2():
        while not stop2.is_set():
            w3.is_completed()
            polls2[0] += 1
    th2 = threading.Thread(target=poll2, daemon=True)
    th2.start()
    time.sleep(0.01)
    g3 = torch.cuda.CUDAGraph()
    err3 = None
    try:
        with torch.cuda.graph(g3, capture_error_mode="thread_local"):
            x.mul_(0.5)
            dist.all_reduce(x)
    except Exception as e:   # noqa: BLE001
        err3 = repr(e)[:300]
    stop2.set()
    th2.join()
    out("capture_with_same_group_poller", err=err3, polls=polls2[0])
    torch.cuda.synchronize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
