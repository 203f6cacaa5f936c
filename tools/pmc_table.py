"""Print per-mode PMC ratios from tools/pmc_ablate.sh output: python tools/pmc_table.py gpurun_out/pmc_a2"""
import csv
import sys
from collections import defaultdict

base = sys.argv[1]
rows = defaultdict(dict)
for p in ("p1", "p2"):
    for r in csv.DictReader(open(f"{base}/{p}/run_counter_collection.csv")):
        if "ablate_kernel" not in r["Kernel_Name"]:
            continue
        key = (p, int(r["Dispatch_Id"]))
        rows[key]["mode"] = int(r["Kernel_Name"].split("<")[1].split(">")[0])
        rows[key]["grid"] = int(r["Grid_Size"])
        rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
# pair up: each (side, mode) runs 4 reps; take the last rep of each in both passes
seq = {p: [rows[k] for k in sorted(k for k in rows if k[0] == p)] for p in ("p1", "p2")}
print(f"{'side':5s} {'mode':>4s} {'VALU/w':>8s} {'LDS/w':>7s} {'SALU/w':>7s} {'MFMA/w':>7s} {'lifeK':>7s} "
      f"{'act%':>5s} {'wait%':>6s} {'wInst%':>6s} {'occ':>5s} {'mfma%':>6s} {'GHz':>5s}")
for a, b in zip(seq["p1"][3::4], seq["p2"][3::4]):  # last of 4 reps
    w = a["SQ_WAVES"]
    side = "item" if a["grid"] < 5e6 else "user"
    life = a["SQ_WAVE_CYCLES"] / w * 4
    dur_cyc = b["GRBM_GUI_ACTIVE"] / 8
    occ = a["SQ_WAVE_CYCLES"] * 4 / (dur_cyc * 1024)
    print(f"{side:5s} {a['mode']:4d} {a['SQ_INSTS_VALU'] / w:8.0f} {a['SQ_INSTS_LDS'] / w:7.0f} "
          f"{a['SQ_INSTS_SALU'] / w:7.0f} {a['SQ_INSTS_MFMA'] / w:7.0f} {life / 1000:7.1f} "
          f"{100 * b['SQ_ACTIVE_INST_ANY'] / a['SQ_WAVE_CYCLES']:5.1f} "
          f"{100 * b['SQ_WAIT_ANY'] / a['SQ_WAVE_CYCLES']:6.1f} "
          f"{100 * b['SQ_WAIT_INST_ANY'] / a['SQ_WAVE_CYCLES']:6.1f} {occ:5.2f} "
          f"{100 * b['SQ_VALU_MFMA_BUSY_CYCLES'] / (dur_cyc * 1024):6.1f} "
          f"{dur_cyc / 1e3:5.0f}")
