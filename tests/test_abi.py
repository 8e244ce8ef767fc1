"""C-ABI library: builds, loads, and exports every symbol include/rqvae_hip.h declares (CPU-only)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "rqvae_hip.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?(?:int|size_t|char\s*\*|const char\s*\*)\s*\**\s*(\w+)\s*\(", src, re.M)))


def test_header_declares_entry_points():
    names = _declared()
    for n in ("rq_quantize_fwd", "rq_quantize_bwd", "jagged_from_padded", "varlen_attn_fwd", "rq_last_error"):
        assert n in names


def test_library_exports_declared_symbols():
    import torch  # noqa: F401  (load order: torch's HIP runtime first)
    from rqvae_hip import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(_declared()) == set(_lib.EXPORTED_SYMBOLS)
    typed = _lib.load()
    assert typed.rq_abi_version() == 3
    # argument checks run on the host and never touch the device
    rc = typed.rq_quantize_fwd(None, 4, 48, None, None, 8, 1, 3, 0.25, None, None, None, None, None, None, 0, None)
    assert rc == -22 and b"null pointer" in typed.rq_last_error()
    assert typed.rq_quantize_bwd_workspace(1024, 64, 256, 3) > 1024 * 64 * 3 * 4
    # fused attention backward scratch: one dQ partial slab per 64-key block when sequences span several
    n = ctypes.c_int64(-1)
    assert typed.varlen_attn_bwd_ws_elems(64, 6, 64, 801, 801, 1000, -1, 0, ctypes.byref(n)) == 0 \
        and n.value == 13 * 1000 * 384 + 64
    assert typed.varlen_attn_bwd_ws_elems(4, 8, 64, 64, 64, 500, -1, 0, ctypes.byref(n)) == 0 and n.value == 0   # one block
    assert typed.varlen_attn_bwd_ws_elems(4, 8, 64, 5, 5, 500, -1, 0, ctypes.byref(n)) == 0 and n.value == 0   # short forms
    assert typed.varlen_attn_bwd_ws_elems(4, 8, 64, 5, 81, 500, -1, 0, ctypes.byref(n)) == 0 and n.value == 0  # short cross
    # the two-pass policy needs no scratch; a forced query split adds the dK / dV partials (Tk >= 0)
    assert typed.varlen_attn_bwd_ws_elems(64, 6, 64, 801, 801, 1000, -1, 2, ctypes.byref(n)) == 0 and n.value == 0
    assert typed.varlen_attn_bwd_ws_elems(8, 6, 64, 801, 801, 1000, 1000, 4 << 8, ctypes.byref(n)) == 0 \
        and n.value == 13 * 1000 * 384 + 8 + 2 * 4 * 1000 * 384
    assert typed.varlen_attn_bwd_ws_elems(4, 8, 64, 5, 801, 500, -1, 0, ctypes.byref(n)) == 0 and n.value == 13 * 500 * 512
    # forward scratch: LPT order (16-B padded) + split-key partials for few queries over > 128 keys
    assert typed.varlen_attn_fwd_ws_elems(5, 8, 64, 6, 801, 500, 0, 0, ctypes.byref(n)) == 0 and n.value == 8 + 7 * 500 * 8 * 66
    assert typed.varlen_attn_fwd_ws_elems(5, 8, 64, 6, 801, 500, 1, 0, ctypes.byref(n)) == 0 and n.value == 8   # causal
    assert typed.varlen_attn_bwd_ws_elems(4, 8, 48, 5, 5, 500, -1, 0, ctypes.byref(n)) == -22
    # + the query splits' dK / dV partials when the workgroups cannot fill the chip (ML-32M, 8 sequences:
    # 8 x 6 x 13 = 624 workgroups -> 3 splits at 256 CUs, the CPU-side default)
    assert typed.varlen_attn_bwd_ws_elems(8, 6, 64, 801, 801, 3200, 3200, 0, ctypes.byref(n)) == 0
    assert n.value == 13 * 3200 * 384 + 8 + 2 * 3 * 3200 * 384
    assert typed.varlen_attn_bwd_ws_elems(64, 6, 64, 801, 801, 1000, 1000, 0, ctypes.byref(n)) == 0
    assert n.value == 13 * 1000 * 384 + 64   # 4,992 workgroups: no split


def test_ops_refuse_cpu_tensors():
    import torch
    from rqvae_hip import ops, RqHipError
    x = torch.zeros(4, 16)
    cb = torch.zeros(1, 8, 16)
    with pytest.raises(RqHipError, match="no CPU fallback"):
        ops.rq_quantize(x, cb)


def test_library_exports_nothing_undeclared():
    """The C ABI is exactly the header: no internal helper or retired entry point is exported."""
    import shutil
    import subprocess
    from rqvae_hip import _lib
    if not os.path.exists(_lib.LIB_PATH) or shutil.which("nm") is None:
        pytest.skip("library not built or nm missing")
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if len(l.split()) == 3 and l.split()[1] == "T"}
    c_names = {n for n in exported if not n.startswith("_")}   # C++ (mangled) symbols are not the ABI
    assert c_names == set(_declared()), sorted(c_names ^ set(_declared()))



_LIB_NAMES = {"lib", "typed", "L", "_L"}   # names the repo binds the loaded CDLL to


def _abi_call_sites():
    """Every literal call into the C ABI in the repo's Python: `call("name", ...)`,
    `TIMER.around(key, call, "name", ...)` and `<lib>.name(...)` with `name` a typed entry point."""
    import ast
    from rqvae_hip import _lib
    files = [os.path.join(ROOT, "bench.py"), os.path.join(ROOT, "__graft_entry__.py")]
    for d in ("tools", "tests", "rq-vae-recommender_amd"):
        for dp, _, fns in os.walk(os.path.join(ROOT, d)):
            files += [os.path.join(dp, f) for f in fns if f.endswith(".py")]
    for path in files:
        tree = ast.parse(open(path).read(), filename=path)
        for node in ast.walk(tree):
            if not isinstance(node, ast.Call):
                continue
            f = node.func
            fname = f.id if isinstance(f, ast.Name) else f.attr if isinstance(f, ast.Attribute) else None
            name, args = None, None
            lit = [a.value if isinstance(a, ast.Constant) else None for a in node.args]
            if fname == "call" and lit and lit[0] in _lib._SIGS:
                name, args = lit[0], node.args[1:]
            elif fname == "around" and len(lit) >= 3 and lit[2] in _lib._SIGS:
                name, args = lit[2], node.args[3:]
            elif isinstance(f, ast.Attribute) and f.attr in _lib._SIGS and (
                    isinstance(f.value, ast.Call) or (isinstance(f.value, ast.Name) and f.value.id in _LIB_NAMES)):
                name, args = f.attr, node.args   # `_lib.load().name(...)`, `lib.name(...)`
            if name is None or any(isinstance(a, ast.Starred) for a in args) or node.keywords:
                continue
            yield os.path.relpath(path, ROOT), node.lineno, name, len(args), len(_lib._SIGS[name][0])


def test_abi_call_sites_match_signatures():
    """Guards tools / tests / bench against ABI drift: a call with the wrong argument count only
    fails at run time on the GPU box (round 4: tools/pmc_quantize.py passed 15 of 17 arguments)."""
    sites = list(_abi_call_sites())
    assert len(sites) > 60
    bad = [s for s in sites if s[3] != s[4]]
    assert not bad, bad
