"""The HIP kernels' gfx950 assembly has no unguarded register hazard around the inline
asm that LLVM's hazard recognizer cannot see (DPP / lane-swap reads of a register
just written by a VALU copy or a matrix-core op: tools/isa_hazards.py).  Register
allocation decides where such copies land, so this is re-checked on every build of
the sources rather than once (round 4: an AGPR copy right before a DPP fmac corrupted
rows of the explicit rank-128 kernel).  CPU only: hipcc cross-compiles."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "recommender-system-using-apache-spark-mllib-_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools"))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_no_unguarded_dpp_hazards(tmp_path):
    import isa_hazards
    procs = {}
    for src in ("gram_solve", "topk"):
        out = tmp_path / f"{src}.s"
        procs[src] = (out, subprocess.Popen(
            [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only", "-S",
             os.path.join(CSRC, f"{src}.hip"), "-o", str(out)],
            stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True))
    bad = []
    for src, (out, p) in procs.items():
        _, err = p.communicate(timeout=600)
        assert p.returncode == 0, err[-2000:]
        found = isa_hazards.scan(out.read_text().split("\n"))
        bad += [(src,) + f for f in found]
    assert not bad, bad[:10]


def test_scanner_follows_labels_and_branches():
    """The scanner's window runs through fall-through labels and conditional branches
    and seeds each branch target with the branching block's pending writes (the case a
    per-basic-block reset misses); an unconditional branch ends the fall-through path."""
    import isa_hazards
    asm = """
kern:
  v_mov_b32 v4, v1
.LBB0_1:
  v_fmac_f32_dpp v8, v4, v9 row_newbcast:1
  s_endpgm
kern2:
  v_mov_b32 v5, v1
  s_cbranch_scc1 .LBB1_2
  s_nop 7
  s_nop 7
.LBB1_2:
  v_fmac_f32_dpp v8, v5, v9 row_newbcast:1
  s_endpgm
kern3:
  v_mov_b32 v6, v1
  s_branch .LBB2_9
.LBB2_3:
  v_fmac_f32_dpp v8, v6, v9 row_newbcast:1
  s_endpgm
.LBB2_9:
  s_nop 1
  s_branch .LBB2_3
kern4:
  v_mov_b32 v7, v1
  s_nop 1
  v_fmac_f32_dpp v8, v7, v9 row_newbcast:1
  s_endpgm
""".split("\n")
    found = isa_hazards.scan(asm)
    fns = sorted({f[0] for f in found})
    # kern: through a fall-through label; kern2: the branch's target skips the nops;
    # kern3: the write reaches the read through two unconditional branches but with
    # the s_nop 1 + branch wait states on that path (>= 2): clean; kern4: guarded
    assert fns == ["kern", "kern2"], found
