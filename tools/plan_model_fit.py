"""Offline check of the split-bf16 GEMM planner's time model against measured plan sweeps
(tools/x3_plan_sweep.py output): re-implements x3_plan / x3w_choose (csrc/linear.hip) with adjustable
constants, lets the model pick (kernel, S) for every recorded call, and prices the pick with the measured
time of that plan (nearest measured S of the same kernel). Prints, per constant set, the step total of the
model's picks against the per-call measured optimum.

  python tools/plan_model_fit.py profiles/r05/plan_sweep/sweep_*.jsonl
"""
import itertools
import json
import math
import sys

CUS = 256


def plan_s(M, N, K, S, wide, ts=128):
    T = 256 if wide else ts
    tiles = math.ceil(M / T) * math.ceil(N / T)
    chunk = math.ceil(math.ceil(K / S) / 32) * 32
    S = max(1, math.ceil(K / chunk))
    return {"ts": T, "tiles": tiles, "S": S, "chunk": chunk}


def plan_time(p, M, N, wide, c):
    wgs = p["tiles"] * p["S"]
    small = p["ts"] == 64
    tile = p["ts"] ** 2
    rate = c["r64"] if small else c["r128"] * (c["wide"] if wide else 1.0)
    if wgs <= CUS:
        t = tile * p["chunk"] / ((rate if wide else (c["r64_1"] if small else c["r128_1"])) * 1e6)
    else:
        per_cu = 1 if wide else ((4 if wgs > 2 * CUS else 2) if small else 2)
        slots = CUS * per_cu
        rounds = wgs / slots if c["frac"] else math.ceil(wgs / slots)
        if c["frac"]:
            rounds = max(1.0, rounds)
        t = rounds * per_cu * tile * p["chunk"] / (rate * 1e6)
    if p["S"] > 1:
        t += 2 * p["S"] * M * N * 4 / c["slab"] + c["red"]
    return t


def split_cap(M, N):
    return max(64, (64 << 20) // (4 * M * N))


def plan_t(M, N, K, ts, c):
    p = plan_s(M, N, K, 1, False, ts)
    if p["tiles"] < 256 and (M * N) % 4 == 0:
        S = 512 // p["tiles"]
        S = min(S, math.ceil(K / 64), split_cap(M, N))
        if ts == 64:
            s2 = 2
            while s2 < S:
                q = plan_s(M, N, K, s2, False, ts)
                if plan_time(q, M, N, False, c) < plan_time(p, M, N, False, c):
                    p = q
                s2 *= 2
        if S > 1:
            q = plan_s(M, N, K, S, False, ts)
            if plan_time(q, M, N, False, c) < plan_time(p, M, N, False, c):
                p = q
    return p


def plan(M, N, K, c):
    p, q = plan_t(M, N, K, 128, c), plan_t(M, N, K, 64, c)
    return q if plan_time(q, M, N, False, c) < plan_time(p, M, N, False, c) else p


def wplan(M, N, K, c):
    if K % 32:
        return None
    fits = lambda R: R % 256 == 0 or R >= 2048   # noqa: E731
    if not (fits(M) and fits(N)):
        return None
    p = plan_s(M, N, K, 1, True)
    if p["tiles"] < 128 and (M * N) % 4 == 0:
        S = min(256 // p["tiles"], K // 256, split_cap(M, N))
        if S > 1:
            q = plan_s(M, N, K, S, True)
            if plan_time(q, M, N, True, c) < plan_time(p, M, N, True, c):
                p = q
    return p if p["tiles"] * p["S"] >= 64 else None


def choose(key, c):
    M, N, K, akc, bkc, asp, bsp, epi, acc = key
    p = plan(M, N, K, c)
    combo = epi == 0 or (epi == 1 and akc and bkc) or (epi == 2 and akc and not bkc) or (epi == 3 and akc and bkc)
    if asp and bsp and combo:
        w = wplan(M, N, K, c)
        if w is not None and plan_time(w, M, N, True, c) < plan_time(p, M, N, False, c):
            return "wide", w["S"]
    return ("x3s" if p["ts"] == 64 else "x3"), p["S"]


def measured(table, kern, S):
    rows = [r for r in table if r.get("kernel") == kern and "us" in r]
    if not rows:
        return None
    return min(rows, key=lambda r: (abs(r["S"] - S), r["S"]))["us"]


def main():
    recs = []
    for path in sys.argv[1:]:
        for line in open(path):
            d = json.loads(line)
            if "key" in d:
                recs.append((path.split("sweep_")[-1].split(".")[0], d))
    base = dict(r128=0.53, r128_1=0.4, r64=0.35, r64_1=0.3, wide=1.3, slab=3.0e6, red=3.0, frac=True)
    grid = {"r64": [0.35, 0.45, 0.55], "r128": [0.45, 0.53], "frac": [False, True], "red": [2.0, 4.0],
            "slab": [3.0e6, 5.0e6]}
    results = []
    for vals in itertools.product(*grid.values()):
        c = dict(base, **dict(zip(grid.keys(), vals)))
        tot, opt, per = 0.0, 0.0, {}
        for cfg, d in recs:
            kern, S = choose(tuple(d["key"]), c)
            t = measured(d["table"], kern, S)
            best = d["best"]["us"]
            t = best * 1.5 if t is None else t
            tot += t * d["calls"]
            opt += best * d["calls"]
            per[cfg] = per.get(cfg, 0.0) + (t - best) * d["calls"]
        results.append((tot - opt, {k: round(v, 1) for k, v in per.items()}, dict(zip(grid.keys(), vals))))
    results.sort(key=lambda r: r[0])
    c = dict(base)
    cur = sum(((measured(d["table"], *choose(tuple(d["key"]), c)) or 0) - d["best"]["us"]) * d["calls"] for _, d in recs)
    print(json.dumps({"current_constants_excess_us": round(cur, 1)}))
    for r in results[:8]:
        print(json.dumps({"excess_us": round(r[0], 1), "per_config": r[1], "constants": r[2]}))


if __name__ == "__main__":
    main()
