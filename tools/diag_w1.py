"""Dev diagnostic (GPU box): which rows of the rank-128 mixed-norm case and of the
implicit rank-128 fit disagree with the oracle (ALS_K128_PATH selects the solve)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _pkgload  # noqa: E402

_pkgload.load()
from als_mi355x import engine as E  # noqa: E402
from oracle import als_oracle as O  # noqa: E402
from helpers import planted, rel_row_errs  # noqa: E402

DEV = "cuda:0"
path = os.environ.get("ALS_K128_PATH", "w1")


def show(tag, X, Xr, ptr, extra=""):
    e = rel_row_errs(X, Xr)
    deg = np.diff(ptr)
    bad = np.argsort(-e)[:6]
    print(f"[{path}] {tag}: max {e.max():.3e} median {np.median(e):.3e} n>1e-4 {int((e > 1e-4).sum())}"
          f"/{len(e)} {extra}")
    for b in bad:
        print(f"     row {b} deg {deg[b]} err {e[b]:.3e} |x| {np.linalg.norm(Xr[b]):.3e}")


# 1. mixed norms, explicit, rank 128, chunk 256
u1, i1, r1 = planted(760, 380, density=0.05, heavy_items=(3,), seed=23)
u2, i2, r2 = planted(600, 10, density=1.0, seed=24)
u = np.concatenate([u1, u2 + 760]).astype(np.int32)
i = np.concatenate([i1, i2 + 380]).astype(np.int32)
r = np.concatenate([r1, r2]).astype(np.float32)
for outlier in (1.0, 1e4):
    for chunk in (256, 4096):
        core = E.ALSCore(u, i, r, device=DEV, chunk=chunk)
        core.init_factors(128, seed=3)
        core.U[760:] *= outlier
        U0 = core.U[:, :128].cpu().numpy()
        core.half_sweep_items(0.1, False, 1.0)
        torch.cuda.synchronize()
        ib = core.item_block
        ptr = ib.row_ptr.cpu().numpy()
        Vr = O.half_sweep(ptr, ib.col.cpu().numpy(), ib.val.cpu().numpy(), U0, 0.1, False, 1.0)
        show(f"mixed x{outlier:g} chunk {chunk}", core.V[:, :128].cpu().numpy(), Vr, ptr,
             f"status {int(core.status.item())}")

# 2. implicit rank 128 fit, first iteration user side, from the oracle's V
u, i, r = planted(700, 450, density=0.05, seed=13, heavy_items=(4,), dup=20)
for chunk in (256, 4096):
    core = E.ALSCore(u, i, r, device=DEV, chunk=chunk)
    core.init_factors(128, seed=5)
    U0 = core.U[:, :128].cpu().numpy()
    ib, ub = core.item_block, core.user_block
    ip = (ib.row_ptr.cpu().numpy(), ib.col.cpu().numpy(), ib.val.cpu().numpy())
    up = (ub.row_ptr.cpu().numpy(), ub.col.cpu().numpy(), ub.val.cpu().numpy())
    Vr = O.half_sweep(*ip, U0, 0.1, True, 40.0)
    core.V[:, :128] = torch.as_tensor(Vr).to(DEV)
    core.half_sweep_users(0.1, True, 40.0)
    torch.cuda.synchronize()
    Ur = O.half_sweep(*up, Vr, 0.1, True, 40.0)
    G = O.yty(Vr)
    ev = np.linalg.eigvalsh(G)
    show(f"implicit user side chunk {chunk}", core.U[:, :128].cpu().numpy(), Ur, up[0],
         f"YtY eig [{ev.min():.3e}, {ev.max():.3e}] status {int(core.status.item())}")
    # condition numbers of a few user systems
    A, b, ne = O.normal_equations(*up, Vr, True, 40.0, rows=np.arange(5))
    for t in range(3):
        M = A[t] + G + 0.1 * ne[t] * np.eye(128)
        print("     cond(A_user", t, ") =", f"{np.linalg.cond(M):.3e}")
