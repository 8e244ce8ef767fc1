#!/usr/bin/env python3
"""Benchmark: RQ-VAE training throughput on MI355X (BASELINE.json metric, configs[1]).

Workload (one "step"): a full RQ-VAE train step at the MovieLens-32M config
(configs/rqvae_ml32m.gin: input 768 -> [512, 256, 128] -> D=64, K=256 codewords, L=3 levels,
ROTATION_TRICK, beta 0.25, AdamW lr 1e-4 wd 0.01), synthetic unit-norm 768-d items resident in
HBM, per-GPU batch 65,536 items (throughput shape; the config's B=64 latency is reported
beside it): encoder MLP -> fused HIP L-level quantize -> decoder MLP -> losses -> backward
(HIP quantize VJP) -> RCCL gradient all-reduce (N>1) -> AdamW.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-cpu-baseline] [--no-extras]
                  [--no-pmc]

N>1 is launched by torch.distributed.run (one process per GPU); every rank processes its own
disjoint 65,536-item shard ("weak" scaling) and rank 0 prints ONE JSON line.

Matmul precision follows the reference: it sets torch.set_float32_matmul_precision('high') at
import (modules/rqvae.py:19), so the MLP matmuls run on the split-bf16 GEMM (rq_gemm_bf16x3);
the same step at 'highest' (exact fp32) is reported beside it (exact_fp32_highest).

The timed region carries no instrumentation; kernel statistics come from an untimed pass of 5 more
steps of the same loop with HIP events on the launching stream.
roofline: the dominant kernel — the split-bf16 GEMM at its largest-time launch shape (fp32-matmul
FLOPs 2MNK / mean device time, peak = bf16 dense MFMA / 3 products); roofline_quantize: the fused quantize forward
(rq_quantize_fwd), algorithmic FLOPs 2*K*D*L per item, peak = fp32 MFMA 157.3
TFLOP/s. traffic: HBM bytes per launch from two rocprofv3 PMC passes (FETCH_SIZE x2 +
WRITE_SIZE, child processes running the same kernel at the same shape, N=1 only) next to the
algorithmic bytes. cpu_baseline: the same train step as eager torch-CPU (oracle/rqvae_torch.py, itself
checked against the pinned numpy oracle oracle/rqvae.py in tests/test_oracle.py) on a bounded sample,
timed on this host.

decoder_amazon (configs[2]) / decoder_ml32m (configs[3], 8 and 64 sequences per GPU): decoder train
steps replayed from one hipGraph per context row bucket (eager ms beside it), context tokens/s over
all ranks, a roofline over the step's algorithmic FLOPs, attention / jagged kernel statistics from an
untimed eager pass, and the pinned torch-CPU decoder oracle (oracle/decoder.py) as its cpu_baseline.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))   # seeded input generators (cpu_baseline)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32-in MFMA = vector peak (spec)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (no sparsity)
HBM_PEAK_GBS = 8000.0

CFG = dict(input_dim=768, hidden=[512, 256, 128], D=64, K=256, L=3, lr=1e-4, wd=0.01, beta=0.25)


def make_adamw(params, lr, wd):
    """The HIP multi-tensor AdamW (one launch per step); RQVAE_TORCH_ADAMW=1 selects torch's fused AdamW
    (A/B switch for tools/gpu_check.sh)."""
    if os.environ.get("RQVAE_TORCH_ADAMW") == "1":
        return torch.optim.AdamW(params, lr=lr, weight_decay=wd, fused=True)
    from rqvae_hip import optim as hip_optim
    return hip_optim.AdamW(params, lr=lr, weight_decay=wd)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU). Without torchrun env and N > 1, bench.py starts torch.distributed.run "
                         "with N processes itself and exits with its status; under torchrun it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=65536, help="items per GPU per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--no-decoder", action="store_true", help="skip the data-parallel decoder measurement")
    ap.add_argument("--no-tunable", action="store_true", help="library GEMMs on their default heuristic")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--decoder-only", action="store_true", help="profile helper: run only the decoder extra")
    ap.add_argument("--no-graph", action="store_true", help="decoder steps eager instead of hipGraph replays")
    ap.add_argument("--no-dm", action="store_true", help="skip the ML-32M decoder lines")
    ap.add_argument("--dm-batch", type=int, default=0, help="with --decoder-only: the ML-32M config at this batch")
    return ap.parse_args()


def make_items(n, dim, gen, device):
    x = torch.randn(n, dim, generator=gen, device=device)
    return x / x.norm(dim=1, keepdim=True)


def build_model(device, seed=0):
    from modules.quantize import QuantizeForwardMode
    from modules.rqvae import RqVae
    torch.manual_seed(seed)
    m = RqVae(input_dim=CFG["input_dim"], embed_dim=CFG["D"], hidden_dims=CFG["hidden"], codebook_size=CFG["K"],
              codebook_kmeans_init=False, codebook_mode=QuantizeForwardMode.ROTATION_TRICK, n_layers=CFG["L"],
              commitment_weight=CFG["beta"], n_cat_features=0).to(device)
    # k-means-init-like codebooks: level l = K residual rows of disjoint random items
    g = torch.Generator(device=device).manual_seed(seed + 1)
    with torch.no_grad():
        res = m.encode(make_items(CFG["K"] * CFG["L"], CFG["input_dim"], g, device))
        for l, layer in enumerate(m.layers):
            cb = res[l * CFG["K"]:(l + 1) * CFG["K"]].clone()
            layer.embedding.weight.copy_(cb)
    return m


def time_region(fn, steps, warmup, sync_all):
    for _ in range(warmup):
        fn()
    sync_all()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync_all()
    return time.perf_counter() - t0


def gemm_launch_stats(timer, steps=1):
    """Split-bf16 GEMM launches recorded in the kernel-statistics pass (ops.TIMER keys
    'gemm_bf16x3:MxNxK:<a_kc><b_kc>...' and 'gemm_pair:<key1>+<key2>'): the single launch shape with the
    largest total device time, its mean launch time, fp32-matmul TFLOP/s (2MNK / time) and algorithmic
    bytes (fp32 A, B in, C out), plus the aggregate over every GEMM launch of the step (paired ones too)."""
    keys = [k for k in timer.events if k.startswith("gemm_bf16x3:")]
    pairs = [k for k in timer.events if k.startswith("gemm_pair:")]   # one launch, two problems
    if not keys:
        return None

    def mnk(k):
        return tuple(int(v) for v in k.split(":")[1].split("x"))
    tot_ms, tot_flops, best, n_launch = 0.0, 0.0, None, 0
    for k in pairs:
        ms, n = timer.mean_ms(k)
        k1, k2 = k[len("gemm_pair:"):].split("+")
        tot_ms += ms * n
        tot_flops += sum(2.0 * a * b * c for a, b, c in (mnk(k1), mnk(k2))) * n
        n_launch += n
    for k in keys:
        ms, n = timer.mean_ms(k)
        M, N, K = mnk(k)
        lay = [int(c) for c in k.split(":")[2]] + [0, 0, 0]
        tot_ms += ms * n
        tot_flops += 2.0 * M * N * K * n
        n_launch += n
        # the roofline kernel: the largest-time launch with the plain epilogue (a PMC driver can
        # replay exactly that variant: same shape, layouts and operand formats)
        if lay[4] == 0 and (best is None or ms * n > best[0]):
            best = (ms * n, ms, n, M, N, K, *lay[:4])
    _, ms, n, M, N, K, akc, bkc, asp, bsp = best
    red_ms, red_n = timer.mean_ms("reduce_partials") if "reduce_partials" in timer.events else (0.0, 0)
    return {"shape": [M, N, K, akc, bkc], "operands_split": [asp, bsp], "epilogue": "store",
            "splitk_reduction": "deferred: the weight-grad slab reductions of a step run batched in "
                                "rq_reduce_partials launches (%.1f per step, %.4f ms each), not in this launch"
                                % (red_n / steps, red_ms) if red_n else "in-launch",
            "launch_ms": round(ms, 4), "launches": n,
            "flops_per_launch": 2 * M * N * K, "algorithmic_bytes": 4 * (M * K + N * K + M * N),
            "achieved_tflops": round(2.0 * M * N * K / (ms * 1e-3) / 1e12, 2),
            "all_gemm_launches": {"launches_per_step": round(n_launch / steps, 1),
                                  "paired_launches_per_step": round(sum(timer.mean_ms(k)[1] for k in pairs) / steps, 1),
                                  "ms_per_step_total": round(tot_ms / steps, 4),
                                  "tflops": round(tot_flops / (tot_ms * 1e-3) / 1e12, 2),
                                  "note": "every split-bf16 GEMM launch of the step (single and paired: one launch, "
                                          "two problems' FLOPs), device time by HIP events over 5 steps"}}


def quantize_algorithmic_bytes(B, D, K, L):
    """Bytes one rq_quantize_fwd launch must move: x and the codebooks (+|c|^2) in; residuals and
    emb_out (L,B,D, saved for the VJP), emb_sum (B,D), ids (B,L) int64 and qloss (B,) out."""
    return 4 * B * D + 4 * L * K * (D + 1) + 4 * B * (2 * L * D + D + 1) + 8 * B * L


def pmc_traffic(timeout_s=75, regex="rq_fwd", script=("pmc_quantize.py", "5"), launches=None):
    """HBM bytes per launch of the kernels matching `regex` from two rocprofv3 --pmc passes
    (FETCH_SIZE, WRITE_SIZE: they do not fit one TCC pass) over a short driver (tools/pmc_*.py) that
    runs the same kernel at the same shape, as child processes (this process never execs). Both
    counters are in KiB; FETCH_SIZE is doubled (gfx950 tallies 128-B streaming reads at 64 B,
    MI355X_MICROARCH.md 'HBM'). With `launches`, one logical launch is several dispatches (a split-K GEMM
    and its slab reduction): the counters of every matched dispatch are summed and divided by it."""
    import csv
    import shutil
    import subprocess
    import tempfile
    if any(k.startswith("ROCPROF") for k in os.environ):
        return None, "skipped: already running under rocprofv3"
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not found"
    vals = {}
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            cmd = ["timeout", "-s", "KILL", str(timeout_s), exe, "--pmc", ctr, "--kernel-include-regex", regex,
                   "-f", "csv", "-d", d, "-o", ctr, "--", sys.executable, os.path.join(ROOT, "tools", script[0]),
                   *script[1:]]
            r = subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), capture_output=True, text=True)
            path = os.path.join(d, f"{ctr}_counter_collection.csv")
            if r.returncode != 0 or not os.path.exists(path):
                return None, f"{ctr} pass failed (exit {r.returncode}): {r.stderr[-200:]}"
            v = sorted(float(row["Counter_Value"]) for row in csv.DictReader(open(path)) if row["Counter_Name"] == ctr)
            if not v:
                return None, f"{ctr}: no {regex} dispatches recorded"
            vals[ctr] = sum(v) / launches if launches else v[len(v) // 2]
    fetch = 2.0 * vals["FETCH_SIZE"] * 1024
    write = vals["WRITE_SIZE"] * 1024
    return dict(bytes=fetch + write, fetch_bytes_x2=fetch, write_bytes=write), None


def cpu_baseline(budget_s, B=2048):
    """The RqVae train step (fwd + bwd + AdamW) as eager PyTorch on the host CPU (oracle/rqvae_torch.py,
    checked against the pinned numpy oracle in tests/test_oracle.py), same dims, on this process's
    CPU share (torch.set_num_threads), bounded sample of ~budget_s seconds."""
    from oracle import rqvae as R
    from oracle.rqvae_torch import RqVaeTorchCPU
    import gen_inputs as gi  # tests/golden (seeded synthetic inputs)
    threads = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        D, K, L, inp, hid = CFG["D"], CFG["K"], CFG["L"], CFG["input_dim"], CFG["hidden"]
        st = {f"encoder.mlp.{2 * j}.weight": w for j, w in enumerate(gi.mlp_weights([inp] + hid + [D], 5))}
        st.update({f"decoder.mlp.{2 * j}.weight": w for j, w in enumerate(gi.mlp_weights([D] + hid[::-1] + [inp], 6))})
        enc_items = gi.items(K * L, inp, 7)
        res0, _ = R.mlp_fwd(enc_items, [st[f"encoder.mlp.{2 * j}.weight"] for j in range(len(hid) + 1)], False)
        for l in range(L):
            st[f"layers.{l}.embedding.weight"] = res0[l * K:(l + 1) * K].copy()
        m = RqVaeTorchCPU(st, L, lr=CFG["lr"], weight_decay=CFG["wd"])
        x = torch.from_numpy(gi.items(B, inp, 8))
        m.train_step(x)          # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            m.train_step(x)
            n += 1
            if time.perf_counter() - t0 >= budget_s or n >= 400:
                break
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    return dict(value=round(n * B / dt, 1), unit="items/s", cores=threads, kind="port", cpu_model=cpu_model(),
                sample=f"{n} eager torch-CPU RqVae train steps (fwd+bwd+AdamW, oracle/rqvae_torch.py) at B={B}, "
                       f"ML-32M dims, {dt:.1f} s on {threads} host threads")


def _log(msg):
    """Progress to stderr (stdout carries only rank 0's JSON line)."""
    rk = os.environ.get("RANK", "0")
    print(f"[bench rank {rk} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_cmd(n, argv, port):
    """The torch.distributed.run command that starts `n` ranks of this script on one node (the driver's
    own form: --nnodes=1, 127.0.0.1 rendezvous), forwarding `argv` unchanged (it carries --gpus n)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def launch_ranks(n, argv):
    """`python bench.py --gpus N` outside torchrun: start N fresh rank processes (one per GPU) as CHILDREN
    of this process, which never touches the GPU itself (no exec: the box forbids replacing a process that
    initialised the GPU). Rank 0's JSON line reaches stdout directly; torchrun's exit status — nonzero when
    any rank dies — is returned."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC: RCCL / tensor sharing across ranks
    return subprocess.run(launcher_cmd(n, argv, _free_port()), env=env).returncode


def rank_census(device, ws):
    """What the process group really spans: its size and backend, the number of ranks one all-reduce of
    ones over it counts (RCCL's own count with the nccl backend), and each rank's device (index, PCI bus
    id), gathered on every rank. Runs once, outside the timed region."""
    props = torch.cuda.get_device_properties(device)
    mine = {"device": device.index, "pci_bus_id": getattr(props, "pci_bus_id", None),
            "name": props.name, "share_device": os.environ.get("RQVAE_SHARE_DEVICE", "0") == "1"}
    if ws == 1:
        return {"process_group_size": 1, "backend": None, "allreduce_rank_count": 1, "devices": [mine]}
    one = torch.ones(1, device=device)
    dist.all_reduce(one)
    devs = [None] * ws
    dist.all_gather_object(devs, mine)
    return {"process_group_size": dist.get_world_size(), "backend": dist.get_backend(),
            "allreduce_rank_count": int(one.item()), "devices": devs,
            "distinct_devices": len({(d["device"], d["pci_bus_id"]) for d in devs})}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    from rqvae_hip import dp, ops
    from data.schemas import SeqBatch
    rk, ws, lr = dp.init_from_env()
    if args.gpus is not None and args.gpus != ws:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {ws} rank(s) (WORLD_SIZE)")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs an MI355X (no GPU visible)")
    if os.environ.get("RQVAE_BENCH_FAIL_RANK") == str(rk):   # test hook: a rank that dies after init
        raise RuntimeError(f"RQVAE_BENCH_FAIL_RANK: rank {rk} exits on purpose")
    if not args.no_tunable:
        # library GEMMs (fwd / data-grad) dispatched to the fastest measured hipBLASLt/rocBLAS
        # solution per shape; shapes missing from the shipped table are tuned in the warmup
        from rqvae_hip import gemm_tuning
        gemm_tuning.enable()
    if args.decoder_only:   # profile helper: one decoder config (amazon, or ml32m with --dm-batch)
        cfg, b = (DEC_DM, args.dm_batch) if args.dm_batch else (DEC, None)
        print(json.dumps({f"decoder_{cfg['name']}": measure_decoder(torch.device("cuda", lr), ws, rk, cfg, B=b,
                                                                     graphs=not args.no_graph, stats=False)}),
              flush=True)
        return
    device = torch.device("cuda", lr)
    torch.cuda.set_device(device)
    census = rank_census(device, ws)
    _log(f"world {ws}: {census['allreduce_rank_count']} ranks answered the census all-reduce")
    B = args.batch

    model = build_model(device)
    # grads become ready decoder -> codebooks -> encoder: the first bucket's all-reduce overlaps the
    # encoder MLP backward
    # flat views even at N=1 (as train_rqvae.py runs it): weight grads accumulate straight into the
    # buckets (no AccumulateGrad pass) and their split-K reductions share a few deferred launches
    buckets = dp.GradBuckets([list(model.decoder.parameters()) + list(model.layers.parameters()),
                              list(model.encoder.parameters())], flat_views=True)
    buckets.broadcast_params()
    opt = make_adamw(model.parameters(), CFG["lr"], CFG["wd"])
    gen = torch.Generator(device=device).manual_seed(1000 + rk)
    pool = [make_items(B, CFG["input_dim"], gen, device) for _ in range(4)]   # resident in HBM
    it = [0]

    def step():
        xb = pool[it[0] % len(pool)]
        it[0] += 1
        buckets.zero_grad()
        out = model(SeqBatch(None, None, None, xb, None, None), gumbel_t=0.2)
        out.loss.backward()
        buckets.synchronize()
        opt.step()
        return out

    def sync_all():
        torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    sync_all()
    t0 = time.perf_counter()            # timed region: no kernel events (they are taken in a separate pass)
    for _ in range(args.steps):
        last = step()
    sync_all()
    elapsed = time.perf_counter() - t0
    _log(f"rq-vae timed: {elapsed / args.steps * 1e3:.3f} ms/step")
    if ws > 1:
        t = torch.tensor([elapsed], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    loss = float(last.loss.detach())
    del last
    # kernel statistics from an untimed pass of the same step (HIP events on the launching stream)
    ops.TIMER.reset()
    ops.TIMER.enabled = True
    for _ in range(5):
        step()
    sync_all()
    ops.TIMER.enabled = False
    q_ms, q_n = ops.TIMER.mean_ms("rq_quantize_fwd")
    gemm = gemm_launch_stats(ops.TIMER, 5)
    exact = None
    if not args.no_extras and ws == 1 and torch.get_float32_matmul_precision() != "highest":
        # the same step with exact-fp32 matmuls ('highest': library fp32 GEMMs + split-K wgrad kernel)
        prev = torch.get_float32_matmul_precision()
        torch.set_float32_matmul_precision("highest")
        try:
            dt = time_region(step, 10, 3, sync_all)
        finally:
            torch.set_float32_matmul_precision(prev)
        exact = {"ms_per_step": round(dt / 10 * 1e3, 3), "items_per_s": round(B * 10 / dt, 1)}

    # decoder-train tokens/s (BASELINE metric, second half): data parallel over the same ranks
    dec = dec_dm = None
    if not args.no_decoder:
        _log("decoder amazon")
        dec = measure_decoder(device, ws, rk, DEC, graphs=not args.no_graph,
                              cpu_seconds=0.0 if args.no_cpu_baseline else 8.0)
        if ws == 1 and not args.no_extras and not args.no_graph:
            eager = measure_decoder(device, ws, rk, DEC, steps=10, warmup=3, graphs=False, stats=False)
            dec["eager_ms_per_step"] = eager["ms_per_step"]
        if not args.no_dm:
            dec_dm = {}
            for b in (8, 64):   # the config's global 64 split over 8 ranks, and 64 per rank (throughput)
                _log(f"decoder ml32m, {b} sequences per rank")
                # warmup >= the 4 cycled batches, so every row bucket's graph is captured before timing
                dec_dm[f"per_gpu_batch_{b}"] = measure_decoder(device, ws, rk, DEC_DM, B=b, steps=10, warmup=5,
                                                               graphs=not args.no_graph, stats=(b == 64))
    extras = {}
    if not args.no_extras and rk == 0 and ws == 1:
        _log("extras")
        extras = measure_extras(model, device, pool[0])
        extras["trainers"] = measure_trainers()

    if rk != 0:
        if ws > 1:
            dist.barrier()
        return
    flops_per_item = 2 * CFG["K"] * CFG["D"] * CFG["L"]
    achieved = flops_per_item * B / (q_ms * 1e-3) / 1e12
    alg_bytes = quantize_algorithmic_bytes(B, CFG["D"], CFG["K"], CFG["L"])
    traffic, traffic_note = (None, "skipped (--no-pmc or N>1)")
    gtraffic, gtraffic_note = (None, "skipped (--no-pmc or N>1)")
    if not args.no_pmc and ws == 1 and B == 65536:
        traffic, traffic_note = pmc_traffic()
        if gemm is not None:
            M, N, K, akc, bkc = gemm["shape"]
            asp, bsp = gemm["operands_split"]
            gtraffic, gtraffic_note = pmc_traffic(   # the GEMM kernel alone (its slab reduction is deferred)
                regex="gemm_bf16x3_kernel|gemm_x3w_kernel", launches=5, script=(
                    "pmc_gemm.py", str(M), str(N), str(K), str(akc), str(bkc), "5", str(asp), str(bsp)))
    q_roof = {"kernel": "rq_quantize_fwd", "bound": "mfma", "achieved": round(achieved, 3),
              "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
              "traffic": round(traffic["bytes"]) if traffic else None, "launch_ms": round(q_ms, 4),
              "launches": q_n, "flops_per_launch": flops_per_item * B, "algorithmic_bytes": alg_bytes,
              "traffic_detail": traffic if traffic else traffic_note,
              "hbm_GBps_at_algorithmic_bytes": round(alg_bytes / (q_ms * 1e-3) / 1e9, 1)}
    roof = q_roof
    if gemm is not None:   # the split-bf16 GEMM is the dominant kernel at 'high' precision
        roof = {"kernel": "gemm_bf16x3 (rq_gemm_bf16x3_run: the step's largest-time plain-epilogue launch, M x N x K)",
                "bound": "mfma",
                "achieved": gemm["achieved_tflops"], "peak": round(BF16_MFMA_PEAK_TFLOPS / 3, 1), "unit": "TFLOP/s",
                "frac": round(gemm["achieved_tflops"] / (BF16_MFMA_PEAK_TFLOPS / 3), 4),
                "traffic": round(gtraffic["bytes"]) if gtraffic else None,
                "peak_note": "fp32-matmul FLOPs; the split runs 3 bf16 MFMA products per fp32 product, so the "
                             "ceiling is the bf16 dense MFMA peak (2.5 PFLOP/s) / 3",
                **{k: v for k, v in gemm.items() if k != "achieved_tflops"},
                "traffic_detail": gtraffic if gtraffic else gtraffic_note}
    # the whole step against its roofline (6 P_mlp + 2 K D L FLOP per item; MLP matmuls on the
    # split-bf16 ceiling, the quantize distances on fp32 MFMA) and its achieved HBM % (PMC bytes of every
    # dispatch of whole steps, tools/pmc_rqstep.py)
    ms_step = elapsed / args.steps * 1e3
    dims = [CFG["input_dim"]] + CFG["hidden"] + [CFG["D"]]
    p_mlp = 2 * sum(a * b for a, b in zip(dims[:-1], dims[1:]))   # encoder + decoder weights
    mlp_flops, q_flops = 6.0 * p_mlp * B, float(flops_per_item * B)
    step_roof = {"flops_per_item": 6 * p_mlp + flops_per_item,
                 "achieved_tflops": round((mlp_flops + q_flops) / (ms_step * 1e-3) / 1e12, 2),
                 "frac_of_gemm_peak": round((mlp_flops + q_flops) / (ms_step * 1e-3) / 1e12 / (BF16_MFMA_PEAK_TFLOPS / 3), 4),
                 "frac_of_step_roofline": round((mlp_flops / (BF16_MFMA_PEAK_TFLOPS / 3 * 1e12) +
                                                 q_flops / (FP32_MFMA_PEAK_TFLOPS * 1e12)) / (ms_step * 1e-3), 4),
                 "note": "frac_of_step_roofline = (MLP matmul FLOPs / 833 TF + quantize FLOPs / 157.3 TF) / step time"}
    if not args.no_pmc and ws == 1 and B == 65536:
        st_traffic, st_note = pmc_traffic(timeout_s=120, regex=".*", script=("pmc_rqstep.py", "6"), launches=6)
        if st_traffic:
            step_roof.update(hbm_bytes_per_step=round(st_traffic["bytes"]),
                             achieved_hbm_GBps=round(st_traffic["bytes"] / (ms_step * 1e-3) / 1e9, 1),
                             achieved_hbm_frac=round(st_traffic["bytes"] / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                             hbm_note="PMC FETCH_SIZE x2 + WRITE_SIZE summed over every dispatch of 6 whole steps / 6 "
                                      "(Infinity-Cache hits are counted as fetched), over the timed step time")
        else:
            step_roof["hbm_bytes_per_step"] = st_note
    line = {
        "metric": "decoder-train tokens/sec + RQ-VAE items/sec at 1/2/4/8 MI355X; achieved HBM %",
        "value": round(ws * B * args.steps / elapsed, 1),
        "unit": "items/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "matmul_precision": torch.get_float32_matmul_precision(),
        "matmul_precision_note": "the reference sets torch.set_float32_matmul_precision('high') at import "
                                 "(modules/rqvae.py:19, model.py:27); gfx950 has no xf32, so 'high' runs the MLP "
                                 "matmuls as split-bf16 (a = hi + lo, 3 bf16 MFMA products, fp32 accumulate; "
                                 "per-product rel. error <= ~2^-17 vs TF32's 2^-11). Quantize distances, argmin, "
                                 "losses and attention stay exact fp32. exact_fp32_highest = the same step at "
                                 "'highest'.",
        "data": "synthetic (seeded unit-norm 768-d items resident in HBM; random-init MLPs, k-means-like codebooks)",
        "config": {"workload": "RQ-VAE MovieLens-32M train step (configs[1]): 768->[512,256,128]->D64, K256, L3, "
                               "ROTATION_TRICK, AdamW", "global_batch": ws * B, "per_gpu_batch": B,
                   "parallelism": f"dp{ws}"},
        "rccl_ranks": census,
        "roofline": roof,
        "step_roofline": step_roof,
        "loss_last": round(loss, 5),
        "gemm_selection": "default heuristic" if args.no_tunable else "TunableOp (rqvae_hip.gemm_tuning)",
    }
    if roof is not q_roof:
        line["roofline_quantize"] = q_roof
    if exact is not None:
        line["exact_fp32_highest"] = exact
    if dec is not None:
        line["decoder_amazon"] = dec
    if dec_dm is not None:
        line["decoder_ml32m"] = dec_dm
    line.update(extras)
    if not args.no_cpu_baseline and ws == 1:
        line["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    print(json.dumps(line), flush=True)
    if ws > 1:
        dist.barrier()


def measure_trainers(iters=30):
    """The drop-in trainers themselves (train_rqvae.train / train_decoder.train: data pipeline, hipGraph
    step with the in-graph gradient exchange, AdamW, host loop) timed by their own LAST_RUN span — the
    per-step time a user of the reference's scripts sees, beside the bench loop's. RQ-VAE at the bench
    config (ML-32M dims, 65,536 items per step, synthetic 87,585-item corpus, k-means init); the decoder
    at the Amazon config (256 sequences, tokenizer = the RQ-VAE checkpoint just written)."""
    import contextlib
    import glob
    import io
    import tempfile
    import train_decoder
    import train_rqvae
    from data.processed import RecDataset
    from modules.quantize import QuantizeForwardMode
    out = {}
    vae = dict(vae_input_dim=CFG["input_dim"], vae_embed_dim=CFG["D"], vae_hidden_dims=CFG["hidden"],
               vae_codebook_size=CFG["K"], vae_n_cat_feats=0, vae_n_layers=CFG["L"])
    with tempfile.TemporaryDirectory() as tmp, contextlib.redirect_stdout(io.StringIO()):
        t0 = time.perf_counter()
        train_rqvae.train(iterations=iters, batch_size=65536, learning_rate=CFG["lr"], weight_decay=CFG["wd"],
                          dataset=RecDataset.ML_32M, do_eval=False, save_dir_root=tmp + "/vae/", log_every=10 ** 9,
                          vae_codebook_mode=QuantizeForwardMode.ROTATION_TRICK, commitment_weight=CFG["beta"], **vae)
        r = dict(train_rqvae.LAST_RUN)
        out["rqvae_ml32m"] = {**r, "items_per_s": round(65536 / (r["iter_ms"] * 1e-3), 1),
                              "wall_s": round(time.perf_counter() - t0, 1)}
        ckpt = sorted(glob.glob(tmp + "/vae/checkpoint_*.pt"))[-1]
        t0 = time.perf_counter()
        # the synthetic Amazon corpus at the bench step's length distribution (histories of U{3..21} items,
        # whole windows: U{2..20} context items per sequence), so the trainer's tokens/s compares with
        # decoder_amazon.ctx_tokens_per_s at matched batches
        from data import processed
        prev = processed.SYNTHETIC_HIST_LEN.get(RecDataset.AMAZON)
        processed.SYNTHETIC_HIST_LEN[RecDataset.AMAZON] = (DEC.get("min_items", 2) + 1, DEC["max_items"] + 2)
        try:
            train_decoder.train(iterations=2 * iters, batch_size=DEC["B"], learning_rate=DEC["lr"],
                                weight_decay=DEC["wd"], dataset=RecDataset.AMAZON, pretrained_rqvae_path=ckpt,
                                decoder_embed_dim=DEC["E"], dropout_p=DEC["dropout"], attn_heads=DEC["H"],
                                attn_embed_dim=DEC["A"], attn_layers=DEC["layers"], save_dir_root=tmp + "/dec/",
                                log_every=10 ** 9, train_data_subsample=False, **vae)
        finally:
            if prev is None:
                processed.SYNTHETIC_HIST_LEN.pop(RecDataset.AMAZON, None)
            else:
                processed.SYNTHETIC_HIST_LEN[RecDataset.AMAZON] = prev
        r = dict(train_decoder.LAST_RUN)
        out["decoder_amazon"] = {**{k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()},
                                 "wall_s": round(time.perf_counter() - t0, 1)}
    out["rqvae_ml32m"]["iter_ms"] = round(out["rqvae_ml32m"]["iter_ms"], 3)
    return out


def measure_extras(model, device, x):
    """Secondary rows of BASELINE C2 on rank 0 (outside the timed region)."""
    from rqvae_hip import ops
    from data.schemas import SeqBatch
    out = {}
    sync = torch.cuda.synchronize
    # quantize-only fwd+bwd (items quantized / s)
    with torch.no_grad():
        res0 = model.encode(x)
    cbs = torch.stack([l.embedding.weight.detach() for l in model.layers]).requires_grad_(True)
    r0 = res0.clone().requires_grad_(True)

    def qstep():
        emb, res, ids, ql, es = ops.rq_quantize(r0, cbs, ops.MODE_ROTATION, 0.25)
        (es.sum() + ql.sum()).backward()
    dt = time_region(qstep, 10, 3, sync)
    out["quantize_fwd_bwd_items_per_s"] = round(10 * x.shape[0] / dt, 1)
    # eval tokenization (encoder + eval quantize)
    model.eval()

    def tok():
        with torch.no_grad():
            model.get_semantic_ids(x)
    dt = time_region(tok, 10, 3, sync)
    out["eval_tokenize_items_per_s"] = round(10 * x.shape[0] / dt, 1)
    model.train()
    # config batch B=64 step latency: eager, and the whole step replayed as one hipGraph
    from rqvae_hip.graph import CapturedStep
    xs = x[:64].contiguous()
    m64 = build_model(device, seed=5)   # fresh module: no autograd state from the timed region
    opt = torch.optim.AdamW(m64.parameters(), lr=1e-4, weight_decay=0.01, foreach=True, capturable=True)

    def small():
        opt.zero_grad(set_to_none=False)
        o = m64(SeqBatch(None, None, None, xs, None, None), gumbel_t=0.2)
        o.loss.backward()
        opt.step()
        return o.loss
    dt = time_region(small, 20, 5, sync)
    out["b64_step_ms"] = round(dt / 20 * 1e3, 3)
    try:
        g = CapturedStep(small)
        dt = time_region(g, 50, 5, sync)
        out["b64_step_ms_hipgraph"] = round(dt / 50 * 1e3, 4)
        out["b64_items_per_s_hipgraph"] = round(50 * 64 / dt, 1)
    except Exception as e:  # report, never hide
        out["b64_hipgraph_error"] = repr(e)[:300]
    out["quantize_synthetic"] = measure_quantize_synthetic(device)
    out["jagged_c5"] = measure_jagged_c5(device)
    out["quantize_c5_rank"] = measure_quantize_c5_rank(device)
    out["jagged_c5_rank"] = measure_jagged_c5_rank(device)
    return out


def measure_jagged_c5(device, B=4096, max_items=256, L1=5, D=128, reps=10):
    """BASELINE configs[4] jagged half at HBM scale: B user sequences of 5 U{2..256} + 1 context rows
    (<= 1281) x D = 128 fp32 embeddings, padded -> jagged (with the reference's +1-1 rounding) and back
    (the backward's zero-filled scatter), HIP events over `reps` launches. Algorithmic bytes: gather
    2 * 4 D sum(n) (valid rows read + written), scatter 4 D (B N + sum(n))."""
    from rqvae_hip import ops
    from rqvae_hip._lib import call, ptr, stream_handle
    g = np.random.Generator(np.random.PCG64(5))
    lens = L1 * g.integers(2, max_items + 1, size=B) + 1
    N = L1 * max_items + 1
    x = torch.randn(B, N, D, device=device)
    off = ops.jagged_offsets(torch.from_numpy(lens).to(device), N)
    T = int(lens.sum())
    vals = torch.empty((T, D), device=device)
    back = torch.empty_like(x)
    st = stream_handle(device)
    gather = lambda: call("jagged_from_padded_rows", ptr(x), B, N, D, ptr(off), ptr(vals), T, 0, 1, st)  # noqa: E731
    scatter = lambda: call("jagged_to_padded", ptr(vals), ptr(off), B, N, D, ptr(back), 0, st)  # noqa: E731

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps
    tg, ts = timed(gather), timed(scatter)
    gb_g, gb_s = 2.0 * 4 * D * T / 1e9, 4.0 * D * (B * N + T) / 1e9
    res = {"shape": {"sequences": B, "max_rows": N, "D": D, "valid_rows": T}, "gather_ms": round(tg, 4),
           "scatter_ms": round(ts, 4), "gather_GBps": round(gb_g / (tg * 1e-3), 1),
           "scatter_GBps": round(gb_s / (ts * 1e-3), 1),
           "gather_hbm_frac": round(gb_g / (tg * 1e-3) / HBM_PEAK_GBS, 4),
           "scatter_hbm_frac": round(gb_s / (ts * 1e-3) / HBM_PEAK_GBS, 4)}
    del x, vals, back
    torch.cuda.empty_cache()
    return res


def _events_ms(fn):
    """fn() bracketed by HIP events on torch's current stream (the stream every op here launches on)."""
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b)


def measure_quantize_c5_rank(device, items=1_250_000, chunk=65536, D=1024, K=2048, L=4):
    """BASELINE configs[4] at its per-rank scale: 10 M items over 8 GPUs = 1.25 M items of D = 1,024 per GPU
    (5.1 GB fp32, resident before timing), streamed through the L = 4, K = 2,048 residual quantization in
    65,536-item chunks — forward alone, then forward + backward (the codebook gradient accumulating over the
    chunks, grad of the residual input per chunk), HIP events around the whole stream. FLOPs: 2 K D L per
    item, the forward's distance GEMMs."""
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(91)
    x = torch.randn(items, D, generator=g, device=device)
    x = x / x.norm(dim=1, keepdim=True)
    cbs = torch.randn(L, K, D, generator=g, device=device)
    cbs = cbs / cbs.norm(dim=2, keepdim=True) * torch.tensor([1.0, 0.5, 0.25, 0.125], device=device).view(L, 1, 1)
    cbs.requires_grad_(True)
    spans = [(a, min(items, a + chunk)) for a in range(0, items, chunk)]

    def fwd():
        with torch.no_grad():
            for a, b in spans:
                ops.rq_quantize(x[a:b], cbs, ops.MODE_ROTATION, 0.25)

    def fwd_bwd():
        for a, b in spans:
            r = x[a:b].detach().requires_grad_(True)
            emb, res, ids, ql, es = ops.rq_quantize(r, cbs, ops.MODE_ROTATION, 0.25)
            (es.sum() + ql.sum()).backward()
    ops.rq_quantize(x[:chunk], cbs.detach(), ops.MODE_ROTATION, 0.25)   # warm-up (library init, plans)
    t_f = _events_ms(fwd)
    cbs.grad = None
    t_fb = _events_ms(fwd_bwd)
    tf = 2.0 * K * D * L * items / (t_f * 1e-3) / 1e12
    out = {"shape": {"items": items, "chunk": chunk, "D": D, "K": K, "L": L}, "fwd_ms": round(t_f, 2),
           "fwd_items_per_s": round(items / (t_f * 1e-3), 1), "fwd_TFLOPs": round(tf, 2),
           "fwd_frac_fp32_mfma_peak": round(tf / FP32_MFMA_PEAK_TFLOPS, 4), "fwd_bwd_ms": round(t_fb, 2),
           "fwd_bwd_items_per_s": round(items / (t_fb * 1e-3), 1),
           "note": "1.25 M items = 10 M / 8 GPUs (BASELINE configs[4]); inputs resident in HBM before timing"}
    del x, cbs
    torch.cuda.empty_cache()
    return out


def measure_jagged_c5_rank(device, sequences=1 << 20, chunk=4096, max_items=256, L1=5, D=128):
    """BASELINE configs[4]'s jagged half at a per-rank scale: 1,048,576 user sequences (50 M over 8 GPUs is
    6.25 M; 1 M already moves ~0.7 TB) of 5 U{2..256} + 1 context rows x D = 128 fp32, streamed in chunks of
    4,096 sequences through padded -> jagged (+1-1 rounding) and back (zero-filled scatter). The length
    stream is seeded; every chunk's offsets are built before timing; one padded buffer serves every chunk
    (a byte mover: contents do not change its work). Algorithmic bytes as measure_jagged_c5."""
    from rqvae_hip import ops
    from rqvae_hip._lib import call, ptr, stream_handle
    g = np.random.Generator(np.random.PCG64(6))
    lens = L1 * g.integers(2, max_items + 1, size=sequences) + 1
    N = L1 * max_items + 1
    x = torch.randn(chunk, N, D, device=device)
    chunks = []
    for a in range(0, sequences, chunk):
        ln = lens[a:a + chunk]
        chunks.append((ops.jagged_offsets(torch.from_numpy(ln).to(device), N), int(ln.sum()), len(ln)))
    T_max = max(c[1] for c in chunks)
    vals = torch.empty((T_max, D), device=device)
    back = torch.empty_like(x)
    st = stream_handle(device)

    def gather():
        for off, T, B in chunks:
            call("jagged_from_padded_rows", ptr(x), B, N, D, ptr(off), ptr(vals), T, 0, 1, st)

    def scatter():
        for off, T, B in chunks:
            call("jagged_to_padded", ptr(vals), ptr(off), B, N, D, ptr(back), 0, st)
    off0, T0, B0 = chunks[0]
    call("jagged_from_padded_rows", ptr(x), B0, N, D, ptr(off0), ptr(vals), T0, 0, 1, st)   # warm-up
    tg, ts = _events_ms(gather), _events_ms(scatter)
    T_all = int(lens.sum())
    gb_g, gb_s = 2.0 * 4 * D * T_all / 1e9, 4.0 * D * (sequences * N + T_all) / 1e9
    out = {"shape": {"sequences": sequences, "chunk": chunk, "max_rows": N, "D": D, "valid_rows": T_all},
           "gather_ms": round(tg, 2), "scatter_ms": round(ts, 2),
           "gather_rows_per_s": round(T_all / (tg * 1e-3), 1), "sequences_per_s": round(sequences / (tg * 1e-3), 1),
           "gather_GBps": round(gb_g / (tg * 1e-3), 1), "scatter_GBps": round(gb_s / (ts * 1e-3), 1),
           "gather_hbm_frac": round(gb_g / (tg * 1e-3) / HBM_PEAK_GBS, 4),
           "scatter_hbm_frac": round(gb_s / (ts * 1e-3) / HBM_PEAK_GBS, 4)}
    del x, vals, back, chunks
    torch.cuda.empty_cache()
    return out


def measure_quantize_synthetic(device, B=16384, D=1024, K=2048, L=4):
    """BASELINE configs[4] quantize roofline shape (synthetic D=1024, K=2048, L=4) on one GPU: the
    fused forward (auto path = split distance GEMM + partial argmin) timed with HIP events."""
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(77)
    x = torch.randn(B, D, generator=g, device=device)
    x = x / x.norm(dim=1, keepdim=True)
    cbs = torch.randn(L, K, D, generator=g, device=device)
    cbs = cbs / cbs.norm(dim=2, keepdim=True) * torch.tensor([1.0, 0.5, 0.25, 0.125], device=device).view(L, 1, 1)
    for _ in range(3):
        ops.rq_quantize(x, cbs, ops.MODE_ROTATION, 0.25)
    torch.cuda.synchronize()
    ops.TIMER.reset()
    ops.TIMER.enabled = True
    for _ in range(10):
        ops.rq_quantize(x, cbs, ops.MODE_ROTATION, 0.25)
    torch.cuda.synchronize()
    ops.TIMER.enabled = False
    ms, n = ops.TIMER.mean_ms("rq_quantize_fwd")
    tf = 2.0 * K * D * L * B / (ms * 1e-3) / 1e12
    return {"shape": [B, D, K, L], "fwd_ms": round(ms, 4), "items_per_s": round(B / (ms * 1e-3), 1),
            "achieved_TFLOPs": round(tf, 2), "frac_fp32_mfma_peak": round(tf / FP32_MFMA_PEAK_TFLOPS, 4)}


# decoder configs: configs[2] (decoder_amazon.gin) and configs[3] (decoder_ml32m.gin; its lr / wd are
# train_decoder.train's defaults, its dropout the default dropout_p 0.1 — the gin's attn_dropout binds
# nothing, SURVEY A-8)
DEC = dict(name="amazon", B=256, max_items=20, E=128, A=512, H=8, layers=8, F=1024, K=256, sem_id_dim=4, dropout=0.3,
           lr=3e-4, wd=0.035)
DEC_DM = dict(name="ml32m", B=64, max_items=200, E=128, A=384, H=6, layers=8, F=1024, K=256, sem_id_dim=4,
              dropout=0.1, lr=1e-3, wd=0.01)


def decoder_flops(cfg, ctx_lens):
    """Algorithmic FLOPs of one decoder train step (step = 3 x forward) for a batch with
    context lengths `ctx_lens` (tokens incl. the user token): (dense projections / MLPs / output
    layer, attention score + value products)."""
    E, A, F, K = cfg["E"], cfg["A"], cfg["F"], cfg["K"]
    Le = Ld = cfg["layers"] // 2
    nf = cfg["sem_id_dim"] + 1                        # bos + the L+1 future sem-id tokens
    n = np.asarray(ctx_lens, np.float64)
    B = len(n)
    dense = n.sum() * (2 * E * A + Le * (8 * A * A + 4 * A * F) + Ld * 4 * A * A) + \
        B * nf * (2 * E * A + Ld * (12 * A * A + 4 * A * F) + 2 * A * K)
    attn = Le * 4 * A * (n * n).sum() + Ld * 4 * A * nf * n.sum() + Ld * 4 * A * nf * nf * B
    return 3.0 * dense, 3.0 * attn


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """Threads for the CPU baselines: the process's affinity cores, capped at the one-GPU box's CPU
    share (16; os.cpu_count() there reports the whole host)."""
    return max(1, min(16, len(os.sched_getaffinity(0))))


def decoder_cpu_baseline(cfg, budget_s, B=16, seed=60):
    """The pinned CPU restatement of the decoder train step (oracle/decoder.py: eager torch on the
    host, forward + autograd backward + torch AdamW) on a bounded subset of `B` sequences of the
    same config, same length law; context tokens / s."""
    from oracle import decoder as Dm
    from modules.model import EncoderDecoderRetrievalModel
    th = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(th)
    try:
        import gen_inputs as gi
        m = EncoderDecoderRetrievalModel(embedding_dim=cfg["E"], attn_dim=cfg["A"], dropout=cfg["dropout"],
                                         num_heads=cfg["H"], n_layers=cfg["layers"], num_embeddings=cfg["K"],
                                         sem_id_dim=cfg["sem_id_dim"], inference_verifier_fn=None,
                                         max_pos=cfg["max_items"] * cfg["sem_id_dim"])
        P = {n: torch.from_numpy(gi.named_param(n, p.shape, seed)).requires_grad_(True) for n, p in m.named_parameters()}
        del m
        opt = torch.optim.AdamW(list(P.values()), lr=cfg["lr"], weight_decay=cfg["wd"])
        from data.processed import synthetic_tokenized_batch
        b = synthetic_tokenized_batch(B, cfg["max_items"], cfg["sem_id_dim"], cfg["K"], seed, torch.device("cpu"))
        batch = dict(b._asdict())
        toks = int(b.seq_mask.sum()) + B

        def step():
            opt.zero_grad()
            loss, _, _ = Dm.decoder_forward(P, batch, cfg["K"], cfg["sem_id_dim"], cfg["H"], cfg["layers"],
                                            dropout=cfg["dropout"])
            loss.backward()
            opt.step()
        step()
        n, t0 = 0, time.perf_counter()
        while True:
            step()
            n += 1
            if time.perf_counter() - t0 >= budget_s or n >= 50:
                break
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    return dict(value=round(n * toks / dt, 1), unit="ctx_tokens/s", cores=th, kind="port", cpu_model=cpu_model(),
                sample=f"{n} oracle decoder train steps (oracle/decoder.py: torch-CPU fwd + bwd + AdamW) on {B} "
                       f"sequences ({toks} ctx tokens/step) of the {cfg['name']} config, {dt:.1f} s, {th} threads")


def measure_decoder(device, ws=1, rk=0, cfg=DEC, B=None, steps=20, warmup=5, graphs=True, stats=True,
                    cpu_seconds=0.0):
    """Decoder train steps/s and context tokens/s, data parallel over the ranks: each rank trains on
    its own synthetic tokenized batches (n_items ~ U{2..max_items}, B sequences per rank, weak
    scaling), gradients all-reduced by GradBuckets (RCCL), HIP AdamW. `graphs`: forward + backward
    replayed from one hipGraph per context row bucket (rqvae_hip.graph.GraphedSteps); else eager.
    Tokens/s = context tokens of all ranks / max time. `stats`: an untimed eager pass with kernel
    events on the jagged and attention launches (their own throughput / roofline fractions)."""
    from rqvae_hip import dp, gemm_tuning, ops
    from rqvae_hip.graph import GraphedSteps
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    from ops.jagged import copy_row_counts
    B = B or cfg["B"]
    torch.manual_seed(3)
    m = EncoderDecoderRetrievalModel(embedding_dim=cfg["E"], attn_dim=cfg["A"], dropout=cfg["dropout"],
                                     num_heads=cfg["H"], n_layers=cfg["layers"], num_embeddings=cfg["K"],
                                     sem_id_dim=cfg["sem_id_dim"], inference_verifier_fn=None,
                                     max_pos=cfg["max_items"] * cfg["sem_id_dim"]).to(device).train()
    # overlap: bucket all-reduces launched from the grad hooks as backward produces them — captured
    # inside each replayed graph with RCCL (GraphedSteps in-graph exchange), eager otherwise
    buckets = dp.GradBuckets(m.parameters(), overlap=True, flat_views=graphs)
    buckets.broadcast_params()
    opt = make_adamw(m.parameters(), cfg["lr"], cfg["wd"])
    batches = [synthetic_tokenized_batch(B, cfg["max_items"], cfg["sem_id_dim"], cfg["K"], 50 + 97 * rk + i, device)
               for i in range(4)]
    ctx_lens = [(b.seq_mask.sum(1) + 1).cpu().tolist() for b in batches]   # host copies, before timing
    ctx_tokens = [int(sum(c)) for c in ctx_lens]
    bucket = gemm_tuning.ROW_BUCKET if gemm_tuning.is_enabled() else None
    gs = GraphedSteps(lambda b: m(b).loss, lambda b: m.context_rows(b, bucket), buckets,
                      prepare=lambda static, b: copy_row_counts(static.seq_mask, b.seq_mask)) if graphs else None
    it = [0]

    def step():
        b = batches[it[0] % len(batches)]
        it[0] += 1
        if gs is not None:
            gs(b)
        else:
            buckets.zero_grad()
            m(b).loss.backward()
        buckets.synchronize()
        opt.step()

    def sync_all():
        torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()
            torch.cuda.synchronize()
    for _ in range(warmup):
        step()
    sync_all()
    it[0] = 0
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync_all()
    dt = time.perf_counter() - t0
    toks = sum(ctx_tokens[i % len(batches)] for i in range(steps))
    dense = attn = 0.0
    for i in range(steps):
        d_, a_ = decoder_flops(cfg, ctx_lens[i % len(batches)])
        dense, attn = dense + d_, attn + a_
    tot = torch.tensor([dt, float(toks), dense, attn], device=device, dtype=torch.float64)
    if ws > 1:
        mx = tot[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dt, toks, dense, attn = float(mx), float(tot[1]), float(tot[2]), float(tot[3])
    ms = dt / steps * 1e3
    fut = ws * steps * B * (cfg["sem_id_dim"] + 1)
    # roofline: dense matmuls on the split-bf16 GEMM (ceiling bf16 peak / 3), attention on fp32 MFMA
    gemm_peak, attn_peak = BF16_MFMA_PEAK_TFLOPS / 3, FP32_MFMA_PEAK_TFLOPS
    t_min = (dense / (gemm_peak * 1e12) + attn / (attn_peak * 1e12)) / ws
    out = {"config": f"decoder_{cfg['name']} (A={cfg['A']}, H={cfg['H']}, {cfg['layers']} layers, max "
                     f"{cfg['max_items']} items -> ctx <= {cfg['max_items'] * cfg['sem_id_dim'] + 1})",
           "ctx_tokens_per_s": round(toks / dt, 1), "ctx_plus_fut_tokens_per_s": round((toks + fut) / dt, 1),
           "ms_per_step": round(ms, 3), "per_gpu_batch": B, "ctx_tokens_per_step_rank": round(toks / steps / ws, 1),
           "n_gpus": ws, "parallelism": f"dp{ws}",
           "scaling": "weak", "step_mode": "hipgraph per row bucket" if graphs else "eager",
           "graphs_captured": len(gs.graphs) if gs is not None else 0,
           "grad_exchange": ("none (1 rank)" if ws == 1 else
                             ("in-graph, overlapped with backward" if gs is not None and gs.in_graph else
                              "after the replay" if gs is not None else "eager, overlapped with backward")),
           "roofline": {"bound": "mfma", "achieved": round((dense + attn) / dt / 1e12, 2),
                        "peak": round(gemm_peak, 1), "unit": "TFLOP/s",
                        "frac": round((dense + attn) / dt / 1e12 / gemm_peak, 4),
                        "frac_of_step_roofline": round(t_min / dt, 4) if dt > 0 else None,
                        "flops_per_step_per_gpu": round((dense + attn) / steps / ws),
                        "attention_flops_share": round(attn / (dense + attn), 4),
                        "note": "algorithmic FLOPs (SURVEY 8d, step = 3 x forward); peak = split-bf16 GEMM ceiling "
                                "(2.5 PF / 3); frac_of_step_roofline = (dense / 833 TF + attention / 157.3 TF) / step time "
                                "(attention priced at the fp32 MFMA peak: the short backward is exact fp32, while the "
                                "forwards and the long-range backward run split-bf16 at 'high' against the 833 TF "
                                "ceiling, so this t_min is an upper bound for those launches)"}}
    if gs is not None and gs.capture_error:
        out["graph_capture_error"] = gs.capture_error
    if stats and rk == 0:
        out["kernels"] = decoder_kernel_stats(m, buckets, batches[0], ctx_lens[0], cfg)
    if cpu_seconds > 0 and rk == 0 and ws == 1:
        out["cpu_baseline"] = decoder_cpu_baseline(cfg, cpu_seconds)
    return out


def decoder_kernel_stats(m, buckets, batch, ctx_lens, cfg, reps=3):
    """Untimed eager passes with HIP events on the attention and jagged launches of one step: device
    time per step, TFLOP/s vs the fp32 MFMA peak (attention: algorithmic 4 A n^2-type products, the
    backward counted as 2 x forward) and GB/s of the jagged conversions."""
    from rqvae_hip import ops
    n = np.asarray(ctx_lens, np.float64)
    A, nf, Le, Ld, Bn = cfg["A"], cfg["sem_id_dim"] + 1, cfg["layers"] // 2, cfg["layers"] // 2, len(ctx_lens)
    attn_fwd = Le * 4 * A * (n * n).sum() + Ld * 4 * A * nf * n.sum() + Ld * 4 * A * nf * nf * Bn
    # algorithmic HBM bytes (fp32, each operand touched once): fwd reads q, k, v and writes o; bwd reads
    # q, k, v, o, dO and writes dq, dk, dv. Encoder self-attention over the T context rows, decoder
    # self-attention over the Tf future rows, cross-attention Tf queries over T keys.
    T, Tf = n.sum(), nf * Bn
    attn_fwd_bytes = 4 * A * (Le * 4 * T + Ld * 4 * Tf + Ld * (2 * Tf + 2 * T))
    attn_bwd_bytes = 4 * A * (Le * 8 * T + Ld * 8 * Tf + Ld * (4 * Tf + 4 * T))
    # rank 0 alone runs these passes: the gradient hooks must not start an exchange its peers never join
    with buckets.suspended():
        for _ in range(2):
            buckets.zero_grad()
            m(batch).loss.backward()
        torch.cuda.synchronize()
        ops.TIMER.reset()
        ops.TIMER.only = {"jagged_", "varlen_attn", "dec_prologue"}
        ops.TIMER.enabled = True
        for _ in range(reps):
            buckets.zero_grad()
            m(batch).loss.backward()
        torch.cuda.synchronize()
        ops.TIMER.enabled = False
        ops.TIMER.only = None
        buckets.zero_grad()
    fwd_ms, nf_ = ops.TIMER.mean_ms("varlen_attn_fwd")
    bwd_ms, nb_ = ops.TIMER.mean_ms("varlen_attn_bwd")
    f_step, b_step = fwd_ms * nf_ / reps, bwd_ms * nb_ / reps
    res = {"attention": {"launches_per_step": {"fwd": nf_ // reps, "bwd": nb_ // reps},
                         "fwd_ms_per_step": round(f_step, 4), "bwd_ms_per_step": round(b_step, 4),
                         "fwd_TFLOPs": round(attn_fwd / (f_step * 1e-3) / 1e12, 2),
                         "bwd_TFLOPs": round(2 * attn_fwd / (b_step * 1e-3) / 1e12, 2),
                         "frac_fp32_peak": round(3 * attn_fwd / ((f_step + b_step) * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4),
                         "fwd_GBps": round(attn_fwd_bytes / (f_step * 1e-3) / 1e9, 1),
                         "bwd_GBps": round(attn_bwd_bytes / (b_step * 1e-3) / 1e9, 1),
                         "frac_hbm_peak": round((attn_fwd_bytes + attn_bwd_bytes) / ((f_step + b_step) * 1e-3) / 1e9
                                                / HBM_PEAK_GBS, 4),
                         "note": "algorithmic attention FLOPs per step (fwd 4 A sum_b n_q n_k over the 12 "
                                 "calls; bwd = 2 x fwd) / device time of the varlen_attn launches; GBps / "
                                 "frac_hbm_peak: algorithmic bytes (fwd q, k, v read + o written; bwd q, k, v, o, "
                                 "dO read + dq, dk, dv written, fp32, once each) over the same device time"},
           "jagged": jagged_stats(ops.TIMER, n, cfg, reps)}
    return res


def jagged_stats(timer, n, cfg, reps):
    """The decoder step's padded <-> jagged conversions. The step no longer runs the standalone
    gather: the fused prologue (rq_dec_prologue_fwd, offsets + values launches) writes the jagged context
    itself, and its backward scatters the context gradient with jagged_to_padded. Algorithmic bytes as C3 —
    gather 2 * 4 E sum(n) (valid rows read + written), scatter 4 E (B (N + 1) + sum(n)) — plus the prologue's
    own traffic (per context / future row: a sem-table row and a position / type row read, the row written,
    12 E bytes) beside it, over the HIP-event device time of those launches."""
    E, B = cfg["E"], len(n)
    T, N1 = float(n.sum()), cfg["max_items"] * cfg["sem_id_dim"] + 1
    nf = cfg["sem_id_dim"] + 1
    p_ms, p_n = timer.mean_ms("dec_prologue")
    s_ms, s_n = timer.mean_ms("jagged_to_padded")
    out = {}
    if p_n:
        g_bytes, own = 2.0 * 4 * E * T, 12.0 * E * (T + B * nf)
        out["prologue_fwd"] = {"launch_ms": round(p_ms, 4), "per_step": p_n // reps,
                               "gather_equiv_bytes": round(g_bytes), "own_bytes": round(own),
                               "gather_equiv_GBps": round(g_bytes / (p_ms * 1e-3) / 1e9, 1),
                               "own_GBps": round(own / (p_ms * 1e-3) / 1e9, 1),
                               "hbm_frac": round(own / (p_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    if s_n:
        s_bytes = 4.0 * E * (B * N1 + T)
        out["scatter_bwd"] = {"launch_ms": round(s_ms, 4), "per_step": s_n // reps, "bytes": round(s_bytes),
                              "GBps": round(s_bytes / (s_ms * 1e-3) / 1e9, 1),
                              "hbm_frac": round(s_bytes / (s_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    for k, name in (("gather_standalone", "jagged_from_padded"),):
        if timer.events.get(name):   # composition path only (prologue off): the standalone gather
            out[k] = {"GBps": round(timer.gbps(name), 1), "hbm_frac": round(timer.gbps(name) / HBM_PEAK_GBS, 4)}
    out["note"] = ("the decoder's per-step context is ~11 k rows x 128 fp32 (~6 MB): these launches are latency-bound; "
                   "the same kernels at HBM scale are bench jagged_c5 / jagged_c5_rank")
    return out


if __name__ == "__main__":
    main()
