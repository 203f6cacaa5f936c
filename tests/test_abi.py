"""CPU tests of the drop-in boundary (no GPU needed, no compute launched).

* libals_hip.so loads and exports every function declared in include/als_hip.h.
* The ctypes signature table in _lib.py covers exactly those symbols.
* Workspace-size functions and argument validation run host-side and return
  the documented error codes before touching a device.
* The product fails loudly (no CPU fallback) when no GPU is visible.
"""
import ctypes
import os
import re

import pytest
import torch

import als_mi355x
from als_mi355x import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "als_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*[a-z_0-9 ]+\**\s*\**\b(als_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_abi():
    names = declared_functions()
    for must in ["als_solve_half", "als_csr_build", "als_index_build", "als_yty", "als_predict",
                 "als_rmse_partial", "als_topk", "als_schedule_build", "als_last_error"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_functions():
        assert hasattr(raw, name), f"{name} declared in als_hip.h but not exported"
    assert sorted(_lib.SIGNATURES) == declared_functions()
    assert L.als_abi_version() == _lib.ABI_VERSION


def test_abi_version_macro_matches():
    m = re.search(r"#define ALS_ABI_VERSION (\d+)", open(HEADER).read())
    assert int(m.group(1)) == _lib.ABI_VERSION


def test_workspace_sizes_are_monotone_and_host_only():
    L = _lib.lib()
    assert L.als_csr_workspace_bytes(1000, 10) < L.als_csr_workspace_bytes(10 ** 7, 10 ** 5)
    assert L.als_index_workspace_bytes(10, 100) < L.als_index_workspace_bytes(10, 10 ** 6)
    ws = L.als_solve_workspace_bytes
    assert ws(64, 0, 1000, 10) < ws(64, 100, 1000, 10)
    assert ws(10, 100, 1000, 10) < ws(64, 100, 1000, 10)
    assert ws(64, 100, 1000, 10) < ws(128, 100, 1000, 10)
    assert ws(64, 100, 10, 10) < ws(64, 100, 10 ** 6, 10)
    assert ws(64, 100, 1000, 10) + 4 * 10 ** 6 <= ws(64, 100, 1000, 10 ** 6 + 10)  # rescue list
    assert L.als_yty_workspace_bytes(10 ** 6, 64) < L.als_yty_workspace_bytes(10 ** 6, 128)
    assert L.als_yty_workspace_bytes(10 ** 6, 64) > 0
    assert L.als_rmse_workspace_bytes(10 ** 6) > L.als_rmse_workspace_bytes(10)
    assert L.als_topk_workspace_bytes(10, 1000, 64, 10) < L.als_topk_workspace_bytes(10, 10 ** 5, 64, 10)
    assert L.als_topk_workspace_bytes(10, 1000, 32, 10) < L.als_topk_workspace_bytes(10, 1000, 128, 10)
    assert [L.als_k_pad(k) for k in (1, 16, 17, 32, 33, 64, 65, 128)] == [16, 16, 32, 32, 64, 64,
                                                                         128, 128]


def _solve_args(**over):
    a = dict(row_ptr=1, col=1, val=16, light=1, n_light=1, n_light_primal=1, heavy=1, slot=1,
             n_heavy=0, crow=1,
             cbeg=1, cend=1, n_chunks=0, slot2=0, slot0=0, Y=16, n_src=0, X=16, ld=64, k=64,
             reg=0.1, implicit=0, alpha=1.0,
             yty=0, status=1, ws=1, ws_bytes=1 << 20, phases=3, stream=0)
    a.update(over)
    return list(a.values())


@pytest.mark.parametrize("over,code", [
    (dict(k=0), -4), (dict(k=129, ld=132), -4), (dict(ld=62), -1), (dict(ld=32), -1),
    (dict(n_light=-1), -1), (dict(Y=0), -1), (dict(implicit=1), -1), (dict(reg=-1.0), -1),
    (dict(Y=18), -1), (dict(phases=0), -1), (dict(phases=64), -1), (dict(n_src=-1), -1),
    (dict(ws=8), -1), (dict(val=20), -1), (dict(n_chunks=1 << 20, ws_bytes=16), -2),
    (dict(n_light=1 << 28, n_light_primal=1 << 28, ws_bytes=1 << 20), -2),  # rescue list
    (dict(n_light_primal=2), -1), (dict(n_light_primal=-1), -1),
    (dict(n_light_primal=0, k=32, ld=32), -1),           # dual path needs k > 32
    (dict(n_light_primal=0, k=128, ld=128, reg=0.0), -1),  # ... and regParam > 0
    (dict(n_light_primal=0, k=128, ld=128, implicit=1, yty=8), -1),  # ... and explicit
    (dict(slot0=-1), -1), (dict(slot0=1 << 20, ws_bytes=16), -2)])  # two-segment slots
def test_solve_half_argument_errors(over, code):
    L = _lib.lib()
    rc = L.als_solve_half(*_solve_args(**over))
    assert rc == code
    assert L.als_last_error()  # a message is set


def test_phase_bits_match_the_header():
    from als_mi355x import engine as E
    src = open(HEADER).read()
    got = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define ALS_PHASE_(\w+) (\d+)", src)}
    assert got == {"LAUNCH1": E.PHASE_LAUNCH1, "LAUNCH2": E.PHASE_LAUNCH2, "PREP": E.PHASE_PREP,
                   "RSCALE": E.PHASE_RSCALE, "DUAL": E.PHASE_DUAL, "RESCUE": E.PHASE_RESCUE,
                   "ALL": E.PHASE_ALL}
    assert E.PHASE_ALL == sum(v for k, v in got.items() if k != "ALL")


def test_dual_limit_keeps_the_dual_system_full_rank():
    from als_mi355x import engine as E
    for k in range(1, 129):
        d = E.dual_limit(k)
        assert d <= k and d <= E.DUAL_MAX_RATINGS
        assert d == (min(96, k) if k > 64 else (32 if k > 32 else 0))


def test_topk_and_predict_argument_errors():
    L = _lib.lib()
    assert L.als_topk(1, 1, 1, 1, 64, 64, 0, 1, 1, 0, 0, 0) == -4      # top = 0
    assert L.als_topk(1, 1, 1, 1, 64, 64, 257, 1, 1, 0, 0, 0) == -4    # top > 256
    assert L.als_topk(1, 1, 1, 1, 60, 64, 10, 1, 1, 0, 0, 0) == -1     # ld < k
    # every (k <= 128, top <= 256) fits the split kernel's LDS: past argument checks,
    # a missing workspace is the error
    assert L.als_topk(1, 1, 1, 1, 128, 128, 256, 1, 1, 0, 0, 0) == -2
    assert L.als_topk(1, 1, 1, 1, 132, 129, 10, 1, 1, 0, 0, 0) == -4   # rank > 128
    assert L.als_predict(1, 1, 5, 1, 1, 1, 1, 1, 1, 10, 0, 1, 0) == -1  # k = 0
    assert L.als_csr_build(0, 0, 0, 0, 0, -1, 0, 0, 0, 0, 0, 0, 0) == -1
    assert L.als_index_build(0, 0, 0, 0, 0, 0, 0, 0, 0) == -1           # id_space 0


def test_zero_size_calls_are_noops():
    L = _lib.lib()
    assert L.als_predict(0, 0, 0, 0, 0, 0, 0, 0, 0, 4, 4, 0, 0) == 0
    assert L.als_topk(0, 0, 0, 0, 4, 4, 1, 0, 0, 0, 0, 0) == 0
    assert L.als_topk(1, 1, 1, 1, 64, 64, 10, 1, 1, 0, 0, 0) == -2      # split path needs ws
    assert L.als_topk(1, 1, 1, 1, 64, 64, 10, 1, 1, 8, 1 << 20, 0) == -1  # ws not 16-B aligned


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure mode")
def test_product_refuses_to_run_without_gpu():
    from als_mi355x.engine import ALSCore
    with pytest.raises(_lib.ALSNativeError, match="no CPU fallback"):
        ALSCore([0, 1], [0, 1], [1.0, 2.0])


def test_product_never_imports_the_oracle():
    pkg = os.path.dirname(als_mi355x.__file__)
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.sub(r'""".*?"""|#.*', "", src, flags=re.S), f


def test_library_override_needs_the_dev_flag(tmp_path):
    """ALS_HIP_LIB alone cannot swap the product library (only with ALS_HIP_DEV=1)."""
    import subprocess
    import sys
    code = ("import _pkgload; _pkgload.load(); from als_mi355x import _lib; "
            "print(_lib.LIB_PATH == _lib.PRODUCT_LIB)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base = {k: v for k, v in os.environ.items() if k not in ("ALS_HIP_LIB", "ALS_HIP_DEV")}
    for extra, want in (({"ALS_HIP_LIB": str(tmp_path / "x.so")}, "True"),
                        ({"ALS_HIP_LIB": str(tmp_path / "x.so"), "ALS_HIP_DEV": "1"}, "False")):
        p = subprocess.run([sys.executable, "-W", "ignore", "-c", code], cwd=root,
                           env=dict(base, **extra), capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-2000:]
        assert p.stdout.strip().splitlines()[-1] == want


_C_TYPES = {"int32_t": _lib.I32, "int64_t": _lib.I64, "float": _lib.F32, "size_t": _lib.SZ,
            "int": ctypes.c_int}


def _header_signatures():
    """name -> ctypes argtypes, parsed from the prototypes of include/als_hip.h
    (every pointer is a c_void_p on the Python side; `void` = no parameters)."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(als_[a-z_0-9]+)\s*\(([^)]*)\)\s*;", src):
        params = [p.strip() for p in m.group(2).split(",") if p.strip() not in ("", "void")]
        types = []
        for p in params:
            if "*" in p:
                types.append(_lib.P)
            else:
                base = p.replace("const ", "").split()[0]
                types.append(_C_TYPES[base])
        out[m.group(1)] = types
    return out


def test_header_parameter_types_match_the_binding():
    """Every prototype's parameter list (count and C type) is what _lib.SIGNATURES binds."""
    hdr = _header_signatures()
    assert sorted(hdr) == sorted(_lib.SIGNATURES)
    for name, (_, args) in _lib.SIGNATURES.items():
        assert hdr[name] == args, name


def _integration_stub():
    """Run the INTEGRATION.md section-2 ctypes stub against a recording stand-in for
    CDLL (no library is loaded) and return (recorded argtypes, the call's arg count)."""
    import ast
    import types
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 2."):]
    code = re.search(r"```python\n(.*?)```", sec, flags=re.S).group(1)

    class Rec(types.SimpleNamespace):
        def __getattr__(self, name):
            f = types.SimpleNamespace()
            setattr(self, name, f)
            return f

    rec = Rec()
    fake_ctypes = types.SimpleNamespace(**{k: getattr(ctypes, k) for k in dir(ctypes)
                                           if not k.startswith("_")})
    fake_ctypes.CDLL = lambda path: rec
    body = code.replace("import ctypes, torch", "pass")
    ns = {"ctypes": fake_ctypes, "torch": None}
    exec(compile(body, "INTEGRATION.md", "exec"), ns)
    n_call = None
    for node in ast.walk(ast.parse(body)):
        if (isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute)
                and node.func.attr == "als_solve_half"):
            n_call = len(node.args)
    return rec, n_call


def test_integration_stub_matches_the_abi():
    """The stand-alone binding a maintainer would copy from INTEGRATION.md binds the
    same argtypes as _lib.py (ABI 6: 29 for als_solve_half) and calls it with that many."""
    rec, n_call = _integration_stub()
    res, args = _lib.SIGNATURES["als_solve_half"]
    assert rec.als_solve_half.argtypes == args
    assert rec.als_solve_half.restype == res
    assert n_call == len(args) == len(_header_signatures()["als_solve_half"])
    assert rec.als_solve_workspace_bytes.argtypes == _lib.SIGNATURES["als_solve_workspace_bytes"][1]
