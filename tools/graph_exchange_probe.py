"""GPU probe for the captured gradient exchange (run as a child process by
tests/test_graph_exchange_gpu.py, so a hang in a captured collective is killed by its timeout).

One process, a world-1 RCCL group, dp.GradBuckets(force_exchange=True) with several buckets: the
decoder model's forward + backward replayed from GraphedSteps with the buckets' all-reduces captured
inside the graph (in_graph_exchange). Prints one JSON line: whether the collectives were captured,
and the max |grad| difference of each replayed step against an eager step of an identical model
copy (a one-rank all-reduce is the identity, so the gradients must match bit for bit).

`race` (argv[2]): the capture starts while an eager all-reduce is in flight and another thread does
what the process group's watchdog does — polls the Work's is_completed() until it reports completion —
and pins host memory (what a trainer's feed thread does). GraphedSteps waits until the watchdog has
retired every eager collective (flight recorder) before an in-graph capture, so the exchange must be captured.
`race_forever`: the poller never stops querying the (completed) Work: on ROCm that fails the capture
even in thread-local mode ("dependency created on uncaptured work in another stream"), and
GraphedSteps must fall back to the post-replay exchange with the same gradients.
`race_pin`: pinning only (no poll)."""
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    port = sys.argv[1] if len(sys.argv) > 1 else "29533"
    mode = sys.argv[2] if len(sys.argv) > 2 else ""
    race = mode.startswith("race")
    do_poll = race and mode in ("race", "race_forever")
    do_pin = race and mode in ("race", "race_pin")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from rqvae_hip import dp as _dp
    _dp.enable_watchdog_record()   # what dp.init_from_env does: GraphedSteps checks the watchdog's list
    dist.init_process_group("nccl", device_id=dev)
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    from rqvae_hip import dp
    from rqvae_hip.graph import GraphedSteps
    from ops.jagged import copy_row_counts
    torch.manual_seed(0)
    m = EncoderDecoderRetrievalModel(embedding_dim=64, attn_dim=128, dropout=0.0, num_heads=4, n_layers=4,
                                     num_embeddings=64, sem_id_dim=4, inference_verifier_fn=None, max_pos=80).to(dev)
    m.eval()   # no dropout anywhere (the model's hard-coded Dropout(0.5) would draw different keys per step)
    ref = copy.deepcopy(m)
    buckets = dp.GradBuckets(m.parameters(), bucket_bytes=256 << 10, flat_views=True, force_exchange=True)
    gs = GraphedSteps(lambda b: m(b).loss, lambda b: 0, buckets,
                      prepare=lambda static, b: copy_row_counts(static.seq_mask, b.seq_mask))
    res = {"buckets": len(buckets.buckets), "in_graph_default": gs.in_graph, "steps": []}
    batch = synthetic_tokenized_batch(8, 20, 4, 64, 11, dev)
    import threading
    stop = threading.Event()
    polls = [0]
    poller = None
    for step in range(4):
        if race and step == 1:   # step 1 captures: an eager collective in flight + a thread polling it
            side = torch.ones(1 << 20, device=dev)
            work = dist.all_reduce(side, async_op=True) if do_poll else None
            done = [work is None]

            def poll():
                while not stop.is_set():
                    if not done[0]:   # the watchdog stops querying a Work once it has completed
                        done[0] = work.is_completed() and mode != "race_forever"
                    if do_pin:
                        torch.empty(4096).pin_memory()
                    polls[0] += 1
            poller = threading.Thread(target=poll, daemon=True)
            poller.start()
        gs(batch)
        if poller is not None and step == 1:
            stop.set()
            poller.join()
            if work is not None:
                work.wait()
        buckets.synchronize()
        for p in ref.parameters():
            p.grad = None
        ref(batch).loss.backward()
        diff = 0.0
        for (n, p), q in zip(m.named_parameters(), ref.parameters()):
            if q.grad is None:
                continue
            diff = max(diff, float((p.grad - q.grad).abs().max()))
        res["steps"].append({"graphs": len(gs.graphs), "max_abs_grad_diff": diff})
        with torch.no_grad():   # same SGD update on both copies so the next step differs
            for p, q in zip(m.parameters(), ref.parameters()):
                if q.grad is not None:
                    p.add_(p.grad, alpha=-1e-2)
                    q.add_(q.grad, alpha=-1e-2)
    torch.cuda.synchronize()
    res["in_graph"] = gs.in_graph
    res["capture_error"] = gs.capture_error
    res["race_polls"] = polls[0]
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
