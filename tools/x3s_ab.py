#!/usr/bin/env python3
"""A/B of the 128-tile split-bf16 GEMM vs its 64-tile form vs the planner (auto) at decoder / RQ-VAE shapes:
mean us per call (HIP events, 30 calls). python tools/x3s_ab.py"""
import sys, os, json, torch
sys.path.insert(0, "rq-vae-recommender_amd")
from rqvae_hip import ops
dev = torch.device("cuda", 0)
ops.gemm_x3w_enable(True)
# decoder 1,280-row shapes (key: MxNxK:akc bkc asp bsp)
shapes = [(1280,512,512,1,1,0,1),(1280,1536,512,1,1,0,1),(1280,1024,512,1,1,0,1),(1280,512,1024,1,0,1,1),
          (1280,512,1536,1,0,0,1),(512,512,1280,0,0,0,0),(1536,512,1280,0,0,0,0),(1024,512,1280,0,0,1,0),
          (512,1024,1280,0,0,0,1),(256,512,1280,0,0,0,0),(1280,256,512,1,1,0,1),(1280,128,512,1,0,0,1),
          (11332,512,512,1,1,0,1),(512,512,11332,0,0,0,0),(11332,1024,512,1,1,0,1),(11332,128,512,1,0,0,1),
          (512,128,11332,0,0,0,0),(65536,128,256,1,1,1,1),(128,64,65536,0,0,1,1),
          # decoder ML-32M context rows (B = 64 / GPU)
          (26880,384,1152,1,0,0,1),(26880,384,1024,1,0,0,1),(26880,1152,384,1,1,0,1),(26880,384,384,1,1,0,1),
          (1152,384,26880,0,0,0,0)]
if len(sys.argv) > 1:   # A/B: another build of the library
    from rqvae_hip import _lib
    _lib._lib = _lib.load(sys.argv[1])
def t(fn, n=30):
    """Device time per call: n calls captured in one hipGraph (host launch cost out of the picture)."""
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(gr, stream=s):
            for _ in range(n): fn()
    torch.cuda.synchronize()
    gr.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3): gr.replay()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * n) * 1e3
g = torch.Generator(device=dev).manual_seed(0)
for (M,N,K,akc,bkc,asp,bsp) in shapes:
    a = torch.randn((M,K) if akc else (K,M), generator=g, device=dev)
    b = torch.randn((N,K) if bkc else (K,N), generator=g, device=dev)
    a = ops.split_bf16x3(a) if asp else a
    b = ops.split_bf16x3(b) if bsp else b
    r = {"shape": f"{M}x{N}x{K}:{akc}{bkc}{asp}{bsp}"}
    for mode, name in ((0, "x3"), (2, "x3s"), (1, "auto")):
        ops.gemm_x3s_enable(mode)
        r[name] = round(t(lambda: ops.gemm_x3(a, bool(akc), b, bool(bkc), M, N, K)), 1)
        r[name + "_plan"] = ops.gemm_x3_choice(M, N, K, bool(asp), bool(bsp), bool(akc), bool(bkc))
    print(json.dumps(r), flush=True)
