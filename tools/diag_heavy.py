"""Dev diagnostic (GPU box): per-row error of heavy (chunked) rows vs the C oracle on
the ML-25M shape, for several (rank, implicit, chunk) variants."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _pkgload  # noqa: E402

_pkgload.load()
from als_mi355x import datasets as D, engine as E  # noqa: E402
from oracle import c_oracle as C  # noqa: E402
from helpers import rel_row_errs  # noqa: E402

dev = "cuda:0"
u, i, r = D.synthetic_config("ml25m", device=dev)
variants = [(128, True, 2048), (64, True, 2048), (128, False, 2048), (128, True, 512),
            (16, True, 2048)]
if len(sys.argv) > 1:
    variants = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]]
for rank, imp, chunk in variants:
    core = E.ALSCore(u, i, r, device=dev, chunk=chunk)
    core.init_factors(rank, seed=5)
    U0 = core.U[:, :rank].cpu().numpy()
    core.half_sweep_items(0.1, bool(imp), 40.0)
    torch.cuda.synchronize()
    ib = core.item_block
    ptr, col, val = ib.row_ptr.cpu().numpy(), ib.col.cpu().numpy(), ib.val.cpu().numpy()
    deg = np.diff(ptr)
    heavy = np.nonzero(deg > chunk)[0]
    # oracle only on the heavy rows + a few light rows (subset CSR)
    light = np.nonzero(deg <= chunk)[0][:2000]
    rows = np.concatenate([heavy, light])
    sub_ptr = np.zeros(len(rows) + 1, np.int64)
    sub_ptr[1:] = np.cumsum(deg[rows])
    sub_col = np.concatenate([col[ptr[j]:ptr[j + 1]] for j in rows])
    sub_val = np.concatenate([val[ptr[j]:ptr[j + 1]] for j in rows])
    X, st = C.half_sweep(sub_ptr, sub_col, sub_val, U0, 0.1, implicit=bool(imp), alpha=40.0)
    if imp:  # the oracle above merged YtY of U0 over all rows: correct as U0 is whole
        pass
    e = rel_row_errs(core.V[:, :rank].cpu().numpy()[rows], X)
    eh, el = e[:len(heavy)], e[len(heavy):]
    nch = (deg[heavy] + chunk - 1) // chunk
    print(f"rank {rank} implicit {imp} chunk {chunk}: heavy rows {len(heavy)} max {eh.max():.2e} "
          f"median {np.median(eh):.2e}; light max {el.max():.2e}; status {int(core.status.item())}")
    for lo, hi in ((2, 4), (5, 10), (11, 20), (21, 100)):
        sel = (nch >= lo) & (nch <= hi)
        if sel.any():
            print(f"   chunks {lo}-{hi}: n {sel.sum()} max {eh[sel].max():.2e} med {np.median(eh[sel]):.2e}")
    worst = heavy[np.argmax(eh)]
    xg = core.V[worst, :rank].cpu().numpy()
    xr = X[np.argmax(eh)]
    print("   worst row", worst, "deg", deg[worst], "|x|", np.linalg.norm(xr), "max comp err",
          np.abs(xg - xr).max(), "argmax dim", np.argmax(np.abs(xg - xr)), flush=True)
    del core
    torch.cuda.empty_cache()
