"""Dev: per-kernel register / occupancy / spill table of one HIP source (gfx950),
from clang's kernel-resource-usage remarks.
    python tools/regs.py path/to/file.hip [name-filter]"""
import os
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    inc = "-I" + os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "recommender-system-using-apache-spark-mllib-_amd", "csrc")
    extra = os.environ.get("REGS_FLAGS", "").split()
    p = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", inc] + extra + [
                        "-c", src, "-o", "/tmp/_regs.o", "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True)
    cur = None
    rows = []
    for line in p.stderr.splitlines():
        m = re.search(r"remark: \s*(.*?): (.*?) \[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1), m.group(2)
        if key == "Function Name":
            cur = {"name": val}
            rows.append(cur)
        elif cur is not None:
            cur[key] = val
    if p.returncode != 0:
        print(p.stderr[-3000:])
    for r in rows:
        if filt and filt not in r["name"]:
            continue
        dm = subprocess.run(["c++filt", r["name"]], capture_output=True,
                            text=True).stdout.strip()
        dm = re.sub(r"\(.*\)$", "", dm)
        print(f"{dm[:70]:70s} V{r.get('VGPRs', '?'):>4} A{r.get('AGPRs', '?'):>3} "
              f"occ {r.get('Occupancy [waves/SIMD]', '?')} vspill {r.get('VGPRs Spill', '?')} "
              f"sspill {r.get('SGPRs Spill', '?')} scratch {r.get('ScratchSize [bytes/lane]', '?')}")


if __name__ == "__main__":
    main()
