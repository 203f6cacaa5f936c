"""ctypes binding of libals_hip.so (the C ABI declared in include/als_hip.h).

`import torch` comes first on purpose: torch's bundled HIP runtime and
/opt/rocm's share the SONAME libamdhip64.so.7, so loading torch first makes
the library's kernels register with the same runtime instance whose streams
and allocations torch hands us.

There is no fallback: if the shared library is missing, fails to load, or no
GPU is visible, the calls below raise.  The CPU oracle under oracle/ is test
infrastructure and is never imported here.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load; see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
PRODUCT_LIB = os.path.join(_HERE, "libals_hip.so")


def _lib_path() -> str:
    """The in-tree product library.  ALS_HIP_LIB (another build of the same ABI, for
    dev A/B runs under tools/) is honoured only together with ALS_HIP_DEV=1, so a
    stray environment variable can never swap the library the product loads."""
    alt = os.environ.get("ALS_HIP_LIB")
    if alt and os.environ.get("ALS_HIP_DEV") == "1":
        return alt
    if alt:
        import warnings
        warnings.warn("ALS_HIP_LIB is ignored without ALS_HIP_DEV=1 (dev A/B builds only); "
                      f"loading {PRODUCT_LIB}")
    return PRODUCT_LIB


LIB_PATH = _lib_path()
_lib = None
_lock = threading.Lock()

P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
F32 = ctypes.c_float
SZ = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/als_hip.h exactly
SIGNATURES = {
    "als_abi_version": (ctypes.c_int, []),
    "als_last_error": (ctypes.c_char_p, []),
    "als_device_count": (ctypes.c_int, []),
    "als_index_workspace_bytes": (SZ, [I64, I32]),
    "als_index_build": (ctypes.c_int, [P, I64, I32, P, P, P, P, SZ, P]),
    "als_csr_workspace_bytes": (SZ, [I64, I32]),
    "als_csr_build": (ctypes.c_int, [P, P, P, P, P, I64, I32, P, P, P, P, SZ, P]),
    "als_schedule_workspace_bytes": (SZ, [I32]),
    "als_schedule_count": (ctypes.c_int, [P, I32, I32, P, P]),
    "als_schedule_build": (ctypes.c_int, [P, I32, I32, I32, I32, I32, P, P, P, P, P, P, P, SZ, P]),
    "als_solve_workspace_bytes": (SZ, [I32, I32, I64, I32]),
    "als_solve_half": (ctypes.c_int, [P, P, P, P, I32, I32, P, P, I32, P, P, P, I32, P, I32, P, I64,
                                      P, I32, I32, F32, ctypes.c_int, F32, P, P, P, SZ,
                                      ctypes.c_int, P]),
    "als_k_pad": (I32, [I32]),
    "als_yty_workspace_bytes": (SZ, [I64, I32]),
    "als_yty": (ctypes.c_int, [P, I64, I32, I32, P, P, SZ, P]),
    "als_predict": (ctypes.c_int, [P, P, I64, P, I32, P, I32, P, P, I32, I32, P, P]),
    "als_rmse_workspace_bytes": (SZ, [I64]),
    "als_rmse_partial": (ctypes.c_int, [P, P, P, I64, P, I32, P, I32, P, P, I32, I32, P, P, SZ,
                                        P]),
    "als_topk_workspace_bytes": (SZ, [I64, I64, I32, I32]),
    "als_topk": (ctypes.c_int, [P, I64, P, I64, I32, I32, I32, P, P, P, SZ, P]),
}

ABI_VERSION = 6


class ALSNativeError(RuntimeError):
    """A libals_hip.so call returned a non-zero status."""


def lib():
    """Load libals_hip.so once; raise if it is missing (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ALSNativeError(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
                "g.build()'` (or `make -C <pkg>/csrc`).  There is no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        v = L.als_abi_version()
        if v != ABI_VERSION:
            raise ALSNativeError(f"libals_hip.so ABI {v} != expected {ABI_VERSION}")
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().als_last_error()
        raise ALSNativeError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")


def require_gpu() -> None:
    """Raise unless a HIP device is usable (the product has no CPU path)."""
    lib()
    if not torch.cuda.is_available():
        raise ALSNativeError("als_mi355x needs a HIP GPU (torch.cuda.is_available() is False); "
                             "there is no CPU fallback")


def ptr(t) -> int:
    """Device pointer of a torch tensor (0 for None)."""
    return 0 if t is None else t.data_ptr()


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
