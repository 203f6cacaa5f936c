"""Dev A/B timing of half-sweep variants (NOT the bench): one workload, the library
named by ALS_HIP_LIB (a tools/ab/variant.py build) or the product one.
    ALS_HIP_DEV=1 ALS_HIP_LIB=tools/ab/libals_x.so python tools/ab_solve.py c1|c2|c3 [steps]
Prints one JSON line: ms per iteration and the event time of each phase launch."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import _pkgload  # noqa: E402

_pkgload.load()
from als_mi355x import datasets as D, engine as E  # noqa: E402
from als_mi355x import _lib as _L  # noqa: E402

if os.environ.get("ALS_AB_DUAL64"):  # dev A/B: the rank 33-64 dual-path limit
    E.DUAL_MAX_RATINGS_64 = int(os.environ["ALS_AB_DUAL64"])


def _lib_loaded():
    """The library actually loaded (ALS_HIP_LIB counts only with ALS_HIP_DEV=1)."""
    return _L.LIB_PATH


def parity(core, k, reg, imp, alpha, n_rows=3000):
    """One more item and user half-sweep, a row sample of each vs the C oracle (fp64
    restatement of Spark's dspr + dppsv) from identical source factors: max relative
    row error (the 1e-4 bar).  The sample takes the longest rows (heavy / chunked) and
    random ones (the dual-path short rows among them)."""
    import numpy as np
    from oracle import c_oracle as C
    worst = 0.0
    for block, Y, X in ((core.item_block, core.U, core.V), (core.user_block, core.V, core.U)):
        Y0 = Y[:, :k].cpu().numpy()
        yty = E.compute_yty(Y, Y.shape[0], k, core.ws_yty) if imp else None
        E.solve_half(block, Y, X, k, reg, imp, alpha, yty, core.status, core.ws)
        torch.cuda.synchronize()
        deg = (block.row_ptr[1:] - block.row_ptr[:-1])
        heavy = torch.topk(deg, 20).indices.cpu().numpy()
        rnd = np.random.default_rng(1).choice(block.n_rows, min(n_rows, block.n_rows), replace=False)
        rows = np.unique(np.concatenate([heavy, rnd]))
        rp = block.row_ptr.cpu().numpy()
        col = block.col.cpu().numpy()
        val = block.val.cpu().numpy()
        ptr = np.zeros(len(rows) + 1, np.int64)
        ptr[1:] = np.cumsum(rp[rows + 1] - rp[rows])
        idx = np.concatenate([np.arange(rp[r], rp[r + 1]) for r in rows])
        ref, st = C.half_sweep(ptr, col[idx], val[idx], Y0, reg, implicit=imp, alpha=alpha)
        got = X[torch.as_tensor(rows, device=X.device), :k].cpu().numpy().astype(np.float64)
        e = np.linalg.norm(got - ref, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-30)
        worst = max(worst, float(e.max()))
    core.check_status()
    return worst


def main():
    wl = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 10
    dev = torch.device("cuda", 0)
    if wl == "c3":
        u, i, r = D.big_config("big1b", device=dev)
        k, imp, alpha, warm = 128, False, 1.0, 1
        steps = min(steps, 3)
    else:
        u, i, r = D.synthetic_config("ml25m", device=dev)
        k, imp, alpha, warm = (64, False, 1.0, 3) if wl == "c1" else (128, True, 40.0, 3)
    chunk = int(sys.argv[sys.argv.index("--chunk") + 1]) if "--chunk" in sys.argv else E.DEFAULT_CHUNK
    core = E.ALSCore(u, i, r, device=dev, chunk=chunk)
    if "--dual" in sys.argv:  # a lower dual-path row-length limit (rank > 64), <= the built 96
        E.DUAL_MAX_RATINGS = int(sys.argv[sys.argv.index("--dual") + 1])
    del u, i, r
    torch.cuda.empty_cache()
    core.init_factors(k, seed=5)
    reg = 0.1
    ev = {}

    def half(block, Y, X, yty, name, rec):
        E.solve_half(block, Y, X, k, reg, imp, alpha, yty, core.status, core.ws,
                     E.PHASE_PREP | E.PHASE_RSCALE)
        for ph, tag in ((E.PHASE_LAUNCH1, "l1"), (E.PHASE_DUAL, "dual"),
                        (E.PHASE_LAUNCH2 | E.PHASE_RESCUE, "l2")):
            if rec:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
            E.solve_half(block, Y, X, k, reg, imp, alpha, yty, core.status, core.ws, ph)
            if rec:
                b.record()
                ev.setdefault(f"{name}_{tag}", []).append((a, b))

    def it(rec):
        yty = E.compute_yty(core.U, core.n_users, k, core.ws_yty) if imp else None
        half(core.item_block, core.U, core.V, yty, "item", rec)
        yty = E.compute_yty(core.V, core.n_items, k, core.ws_yty) if imp else None
        half(core.user_block, core.V, core.U, yty, "user", rec)

    for _ in range(warm):
        it(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        it(True)
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / steps
    core.check_status()
    rescued = {}
    for name, block, Y, X, n_src in (("item", core.item_block, core.U, core.V, core.n_users),
                                     ("user", core.user_block, core.V, core.U, core.n_items)):
        yty = E.compute_yty(Y, n_src, k, core.ws_yty) if imp else None
        E.solve_half(block, Y, X, k, reg, imp, alpha, yty, core.status, core.ws,
                     E.PHASE_ALL & ~E.PHASE_RESCUE)
        torch.cuda.synchronize()
        rescued[name] = int(core.ws.buf[8:12].view(torch.int32).item())  # rescue count word
        E.solve_half(block, Y, X, k, reg, imp, alpha, yty, core.status, core.ws, E.PHASE_RESCUE)
    torch.cuda.synchronize()
    out = {"wl": wl, "lib": _lib_loaded(), "chunk": chunk, "rescued": rescued,
           "dual_max": E.DUAL_MAX_RATINGS,
           "ms_per_iter": round(ms, 4)}
    if "--no-parity" not in sys.argv:
        out["max_row_err"] = parity(core, k, reg, imp, alpha)
    for key, lst in ev.items():
        out[key] = round(sum(a.elapsed_time(b) for a, b in lst) / len(lst), 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
