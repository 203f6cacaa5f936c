"""Dev: one-screen summary of a bench.py JSON line, and (optionally) the headline
roofline recomputed from a rocprofv3 kernel_stats.csv of the same command.
    python tools/bench_summary.py bench.json [kernel_stats.csv]"""
import csv
import json
import sys


def main():
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f"value {d['value']:.4g} ms/step {d['ms_per_step']:.4f} {r.get('bound')} frac {r['frac']:.4f} "
          f"launch_us {r['avg_launch_us']:.1f} limiter {r.get('limiter')} "
          f"dram_frac {r.get('counter_dram_frac')}")
    if d.get("dual"):
        print("dual", {k: round(v['event_ms'], 4) for k, v in d["dual"]["launches"].items()})
    cb = d.get("cpu_baseline") or {}
    print("cpu", cb.get("value"), "cores", cb.get("cores"), cb.get("cgroup_cpu_max"))
    print("topk10_ms", d.get("topk10_ms"), "lib", d.get("library", {}).get("sha256", "")[:16])
    for key in ("configs2", "configs3"):
        c = d.get(key) or {}
        print(key, c.get("ms_per_iter"), c.get("error", ""))
        if c.get("roofline"):
            print("   ", {k: round(v["event_ms"], 3) for k, v in c["roofline"]["launches"].items()},
                  "dual", {k: round(v["event_ms"], 3) for k, v in
                           ((c.get("dual") or {}).get("launches") or {}).items()})
    c4 = d.get("configs4") or {}
    print("configs4", c4.get("top10_ms"), c4.get("top100_ms"))
    if len(sys.argv) > 2:
        kern = r["kernel"]
        for row in csv.DictReader(open(sys.argv[2])):
            name = row.get("Name") or row.get("KERNEL_NAME") or ""
            if name.replace(" ", "").startswith("void als::" + kern.replace(" ", "")) or \
                    kern.replace(" ", "") in name.replace(" ", ""):
                avg_ns = float(row.get("AverageNs") or row.get("Average") or 0)
                calls = int(row.get("Calls") or 0)
                if r.get("bound") == "mfma":  # fp32-grade algorithmic flops vs 157.3 TF
                    fl = r["fp32_grade_view"]["algorithmic_flops_per_launch"]
                    frac = fl / (avg_ns * 1e-9) / 1e12 / 157.3
                else:
                    frac = r["algorithmic_bytes_per_launch"] / (avg_ns * 1e-9) / 1e9 / 8000.0
                print(f"rocprof {name[:60]} calls {calls} avg_us {avg_ns / 1e3:.1f} "
                      f"recomputed frac {frac:.4f} vs line {r['frac']:.4f} "
                      f"(2 launches/step = {2 * avg_ns / 1e6:.4f} ms vs ms_per_step "
                      f"{d['ms_per_step']:.4f})")


if __name__ == "__main__":
    main()
