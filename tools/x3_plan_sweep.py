"""Plan sweep of the split-bf16 GEMM calls of one train step: every distinct call (shape, operand forms,
epilogue, accumulation) recorded from a real step, then timed under each kernel (planner / 128-tile / 64-tile
/ wide) x split-K count S, as a hipGraph of 10 back-to-back calls whose deferred slab reductions are flushed
inside the graph (so a plan pays its own slab traffic). One JSON line per call: the planner's plan and time,
the best plan and time, and the full table.

  python tools/x3_plan_sweep.py rqvae | amazon | c4   [> sweep.jsonl]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

SPLITS = [1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64]
REPS = 10


def record(step, ops):
    recs = {}
    orig = ops._x3_setup

    def rec(a, a_kcontig, b, b_kcontig, M, N, K, epilogue=0, Z=None, p=0.0, seed=0, out=None, accumulate=False,
            defer=False, flags=None):
        key = (int(M), int(N), int(K), bool(a_kcontig), bool(b_kcontig), isinstance(a, ops.Split),
               isinstance(b, ops.Split), int(epilogue), bool(accumulate))
        r = recs.setdefault(key, {"calls": 0, "p": float(p), "defer": bool(defer)})
        r["calls"] += 1
        return orig(a, a_kcontig, b, b_kcontig, M, N, K, epilogue, Z, p, seed, out, accumulate, defer, flags)

    ops._x3_setup = rec
    try:
        step()
        torch.cuda.synchronize()
    finally:
        ops._x3_setup = orig
    return recs


def time_call(ops, fn, flags):
    with ops.gemm_policy(flags):
        fn()
        ops.flush_reductions()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(REPS):
                fn()
            ops.flush_reductions()
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1000.0 / REPS
        best = t if best is None else min(best, t)
    del g
    return best


def sweep(key, info, ops, dev):
    M, N, K, akc, bkc, asp, bsp, epi, acc = key
    gen = torch.Generator(device=dev).manual_seed(M + N + K)
    a = torch.randn((M, K) if akc else (K, M), generator=gen, device=dev)
    b = torch.randn((N, K) if bkc else (K, N), generator=gen, device=dev) * 0.05
    a = ops.split_bf16x3(a) if asp else a
    b = ops.split_bf16x3(b) if bsp else b
    Z = torch.randn(M, N, generator=gen, device=dev) if epi in (ops.EPI_SILU_BWD, ops.EPI_ADD) else None
    out = torch.zeros(M, N, device=dev) if acc else None
    p = info["p"]

    def fn():
        ops.gemm_x3(a, akc, b, bkc, M, N, K, epi, Z=Z, p=p, seed=3, out=out, accumulate=acc,
                    defer=acc and info["defer"])
    rows = []
    kernels = [("auto", 0), ("128", ops.GEMM_ONLY_128), ("64", ops.GEMM_ONLY_64)]
    if asp and bsp:
        kernels.append(("wide", ops.GEMM_FORCE_WIDE))
    seen = set()
    for kname, kf in kernels:
        for S in [0] + SPLITS:
            flags = kf | ops.gemm_split(S)
            with ops.gemm_policy(flags):
                kern, s_ = ops.gemm_x3_choice(M, N, K, asp, bsp, akc, bkc, epi)
            if (kern, s_) in seen:
                continue
            seen.add((kern, s_))
            try:
                t = time_call(ops, fn, flags)
            except Exception as e:   # noqa: BLE001 - a plan the kernel rejects
                rows.append({"kernel": kern, "S": s_, "flags": flags, "error": str(e)[:80]})
                continue
            rows.append({"kernel": kern, "S": s_, "flags": flags, "us": round(t, 2), "planner": kname == "auto" and S == 0})
    ok = [r for r in rows if "us" in r]
    base = next(r for r in ok if r["planner"])
    best = min(ok, key=lambda r: r["us"])
    return {"key": list(key), "calls": info["calls"], "planner": base, "best": best,
            "gain_us": round((base["us"] - best["us"]) * info["calls"], 2), "table": rows}


def main():
    import bench
    from rqvae_hip import dp, gemm_tuning, ops
    gemm_tuning.enable()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    which = sys.argv[1] if len(sys.argv) > 1 else "rqvae"
    if which == "rqvae":
        from data.schemas import SeqBatch
        model = bench.build_model(dev)
        buckets = dp.GradBuckets([list(model.decoder.parameters()) + list(model.layers.parameters()),
                                  list(model.encoder.parameters())], flat_views=True)
        xb = bench.make_items(65536, bench.CFG["input_dim"], torch.Generator(device=dev).manual_seed(1), dev)

        def step():
            buckets.zero_grad()
            model(SeqBatch(None, None, None, xb, None, None), gumbel_t=0.2).loss.backward()
            buckets.synchronize()
    else:
        from data.processed import synthetic_tokenized_batch
        from modules.model import EncoderDecoderRetrievalModel
        cfg, B = (bench.DEC, bench.DEC["B"]) if which == "amazon" else (bench.DEC_DM, 8)
        torch.manual_seed(3)
        model = EncoderDecoderRetrievalModel(embedding_dim=cfg["E"], attn_dim=cfg["A"], dropout=cfg["dropout"],
                                             num_heads=cfg["H"], n_layers=cfg["layers"], num_embeddings=cfg["K"],
                                             sem_id_dim=cfg["sem_id_dim"], inference_verifier_fn=None,
                                             max_pos=cfg["max_items"] * cfg["sem_id_dim"]).to(dev).train()
        buckets = dp.GradBuckets(model.parameters(), overlap=True, flat_views=True)
        batch = synthetic_tokenized_batch(B, cfg["max_items"], cfg["sem_id_dim"], cfg["K"], 50, dev)

        def step():
            buckets.zero_grad()
            model(batch).loss.backward()
            buckets.synchronize()
    step()
    recs = record(step, ops)
    total = 0.0
    for key, info in sorted(recs.items(), key=lambda kv: -kv[0][0] * kv[0][1] * kv[0][2]):
        r = sweep(key, info, ops, dev)
        total += r["gain_us"]
        print(json.dumps(r), flush=True)
    print(json.dumps({"config": which, "calls": len(recs), "total_gain_us_per_step": round(total, 1)}), flush=True)


if __name__ == "__main__":
    main()
