"""Dev: one ALS iteration captured as a HIP graph (torch.cuda.CUDAGraph) vs eager
launches, at a bench workload: ms per iteration both ways, interleaved, and whether the
factors after the same number of iterations from the same state are bitwise equal; also
the bench's own phase-split iteration without and with its six timing events.
(Round 6, profiles/r06/graph_probe.jsonl: no gain from the graph, 1.87 vs 1.86-1.88 ms;
the events cost ~20 us per iteration; events created with hipEventDisableSystemFence
measured slower still, 1.908 ms, and were not kept.)
    python tools/graph_probe.py [c1|c2] [iters]"""
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


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c1"
    n_it = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    u, i, r = D.synthetic_config("ml25m", device=dev)
    core = E.ALSCore(u, i, r, device=dev)
    implicit = wl == "c2"
    rank, reg, alpha = (128, 0.1, 40.0) if implicit else (64, 0.1, 1.0)
    core.init_factors(rank, seed=5)
    for _ in range(3):
        core.iterate(reg, implicit, alpha)
    torch.cuda.synchronize()
    U0, V0 = core.U.clone(), core.V.clone()

    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm the capture stream (torch's recipe)
        core.iterate(reg, implicit, alpha)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        core.iterate(reg, implicit, alpha)
    torch.cuda.synchronize()

    def run_eager():
        for _ in range(n_it):
            core.iterate(reg, implicit, alpha)

    def run_graph():
        for _ in range(n_it):
            g.replay()

    import bench as B  # the bench's own iteration: solve_half split into its phases

    def run_phases():
        for _ in range(n_it):
            B._iteration(core, rank, reg, implicit, alpha)

    def run_events():
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(n_it)]
        for j in range(n_it):
            B._iteration(core, rank, reg, implicit, alpha, evs[j])

    res = {"wl": wl, "iters": n_it, "eager_ms": [], "graph_ms": [], "phases_ms": [],
           "phases_events_ms": []}
    for _ in range(3):
        for name, fn in (("eager_ms", run_eager), ("graph_ms", run_graph),
                         ("phases_ms", run_phases), ("phases_events_ms", run_events)):
            core.U.copy_(U0)
            core.V.copy_(V0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            res[name].append(round(1e3 * (time.perf_counter() - t0) / n_it, 4))
    core.U.copy_(U0)
    core.V.copy_(V0)
    run_eager()
    torch.cuda.synchronize()
    Ue, Ve = core.U.clone(), core.V.clone()
    core.U.copy_(U0)
    core.V.copy_(V0)
    run_graph()
    torch.cuda.synchronize()
    res["bitwise_equal"] = bool(torch.equal(Ue, core.U) and torch.equal(Ve, core.V))
    res["status"] = int(core.status.item())
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(n_it)]
    for j in range(n_it):
        B._iteration(core, rank, reg, implicit, alpha, evs[j])
    torch.cuda.synchronize()
    res["launch1_ms_torch_events"] = [round(sum(e[a].elapsed_time(e[a + 1]) for e in evs) / n_it, 4)
                                      for a in (0, 3)]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
