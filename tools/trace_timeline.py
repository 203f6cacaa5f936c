"""Dev tool: per-iteration kernel timeline from a rocprofv3 kernel_trace.csv.
    python tools/trace_timeline.py TRACE.csv [ANCHOR] [N]
Splits the trace at each launch whose name contains ANCHOR (default: the first
launch kernel of a half-sweep pair, 'gram_solve_kernel'), and for the last N
iterations prints every kernel with its duration and the idle gap before it, then
the per-name totals of one average iteration (busy vs gap)."""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "split_table_kernel"
    n_show = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    starts = [i for i, e in enumerate(ev) if anchor in e[2]]
    # one iteration = two half-sweeps = two anchor launches
    its = [(starts[j], starts[j + 2]) for j in range(0, len(starts) - 2, 2)]
    its = its[-max(n_show, 5):]
    tot = collections.defaultdict(float)
    gap_tot = 0.0
    span_tot = 0.0
    for n, (a, b) in enumerate(its):
        show = n >= len(its) - n_show
        t0 = ev[a][0]
        prev_end = ev[a - 1][1] if a > 0 else t0
        for s, e, name in ev[a:b]:
            gap = max(0, s - prev_end)
            gap_tot += gap
            tot[name.split("(")[0][:60]] += e - s
            if show:
                print(f"{(s - t0) / 1e3:9.1f} us  gap {gap / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f}  {name[:80]}")
            prev_end = max(prev_end, e)
        span_tot += ev[b][0] - t0
        if show:
            print(f"-- iteration span {(ev[b][0] - t0) / 1e3:.1f} us")
    k = len(its)
    print(f"\naverage over {k} iterations: span {span_tot / k / 1e3:.1f} us, gaps {gap_tot / k / 1e3:.1f} us")
    for name, t in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"{t / k / 1e3:9.1f} us  {name}")


if __name__ == "__main__":
    main()
