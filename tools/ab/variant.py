"""Dev A/B (NOT product code): build a patched copy of the working-tree csrc into
tools/ab/libals_<tag>.so (same ABI, loaded with ALS_HIP_DEV=1 ALS_HIP_LIB=...).
Each variant is a list of (file, old, new) text replacements applied to the copy;
an `old` that does not occur fails the build (the patch must still apply).
    python tools/ab/variant.py TAG [TAG ...]      (TAG from VARIANTS below; "base" = none)
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "..", "recommender-system-using-apache-spark-mllib-_amd", "csrc")
GS = "gram_solve.hip"

VARIANTS = {
    "base": [],
    # the round-4 rescue guards off: no split-window / rank-deficiency tests, no
    # pivot-spread test (timing only: rows that need the rescue are then wrong)
    "noguard": [
        (GS, "__device__ __forceinline__ bool window_miss(float diag_lane, float n_terms, float rmax_lane) {",
         "__device__ __forceinline__ bool window_miss(float diag_lane, float n_terms, float rmax_lane) {\n  return false;"),
        (GS, "  if (4 * n > (int64_t)k) return false;  // uniform: the trace only for very short rows",
         "  return false;"),
        (GS, "  return dmin > 0.f && rmax <= kCondMax * rmin && __ballot(!fin) == 0;",
         "  return dmin > 0.f && __ballot(!fin) == 0;"),
    ],
}


def build(tag: str) -> str:
    # at the depth of csrc, so its "../../include" resolves to the repo's include/
    src = os.path.join(HERE, "..", "..", ".ab", tag)
    shutil.rmtree(src, ignore_errors=True)
    shutil.copytree(CSRC, src)
    for f, old, new in VARIANTS[tag]:
        p = os.path.join(src, f)
        s = open(p).read()
        if old not in s:
            raise SystemExit(f"{tag}: patch does not apply to {f}: {old[:70]!r}")
        open(p, "w").write(s.replace(old, new))
    objs = []
    procs = []
    for s in ("csr_build", "gram_solve", "predict", "topk"):
        o = os.path.join(src, s + ".o")
        objs.append(o)
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-std=c++17",
                                       "--offload-arch=gfx950", "-c", os.path.join(src, s + ".hip"),
                                       "-o", o]))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit(f"{tag}: compile failed")
    lib = os.path.join(HERE, f"libals_{tag}.so")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950"] + objs
                          + ["-o", lib])
    shutil.rmtree(src)
    return lib


if __name__ == "__main__":
    for t in sys.argv[1:]:
        print("built", build(t), flush=True)
