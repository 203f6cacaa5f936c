"""Scan gfx950 assembly for data hazards that the compiler's hazard recognizer does not
see: the solve kernels read registers through DPP / lane-swap instructions written
inside inline asm (`v_fmac_f32_dpp row_newbcast`, `v_permlane*_swap`), and LLVM does
not parse inline asm text, so a VALU or matrix-core write the compiler places right
before such a statement (e.g. a `v_accvgpr_read` copy out of an AGPR) gets no wait
states.  One such case silently corrupted rows in round 4 (the C-layout sweep in the
explicit rank-128 kernel: 2.2e-2 row errors).

Rule checked (MI355X_MICROARCH / CDNA3 ISA hazard table, conservatively):
  * VALU write of VGPR v -> DPP or permlane read of v: >= 2 wait states between them;
  * MFMA write of v -> VALU read of v through DPP / permlane: >= 11 wait states for the
    16x16 shapes (at most 8 passes), >= 19 for 32x32 (16 passes).
Wait states = intervening instructions (1 each) + s_nop N (N + 1).  Straight-line code
only: the window restarts at labels and branches, which hold their own waits.

    python tools/isa_hazards.py file.s        (exit 1 and a listing when any is found)
"""
import re
import sys

_VGPR = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def _regs(op: str):
    out = set()
    for m in _VGPR.finditer(op):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def _split(ins: str):
    parts = ins.replace(",", " ").split()
    return parts[0], parts[1:]


def _is_dpp_read(op: str, ins: str) -> bool:
    return "row_newbcast" in ins or "permlane" in op or "_dpp" in op


def scan(lines):
    """-> [(function, writer, reader, wait_states)] of hazardous pairs."""
    found = []
    fn = None
    recent = []  # (op, dst regs, is_mfma, is_valu) of the straight-line window, newest last
    waits_since = []  # wait states elapsed after each entry of `recent`
    for raw in lines:
        line = raw.split(";")[0].rstrip()
        if not line.strip():
            continue
        if re.match(r"^[_A-Za-z.$][\w.$]*:", line):
            if not line.startswith(".L"):
                fn = line.split(":")[0]
            recent, waits_since = [], []
            continue
        ins = line.strip()
        if ins.startswith("."):
            continue
        op, args = _split(ins)
        if op.startswith("s_cbranch") or op == "s_branch" or op.startswith("s_setpc"):
            recent, waits_since = [], []
            continue
        if op == "s_nop":
            n = int(args[0], 0) + 1 if args else 1
            waits_since = [w + n for w in waits_since]
            continue
        if op.startswith("v_") and _is_dpp_read(op, ins):
            srcs = set()
            for a in args[1:]:
                srcs |= _regs(a)
            if "permlane" in op or op.startswith("v_fmac"):
                srcs |= _regs(args[0])  # tied / swapped operand is read too
            for (wop, dst, mfma, valu), w in zip(recent, waits_since):
                need = (19 if "32x32" in wop else 11) if mfma else (2 if valu else 0)
                if dst & srcs and w < need:
                    found.append((fn, wop, ins, w))
        dst = _regs(args[0]) if args and op.startswith("v_") else set()
        mfma = "mfma" in op
        valu = op.startswith("v_") and not mfma and not op.startswith(("v_readlane", "v_readfirstlane"))
        waits_since = [w + 1 for w in waits_since]
        recent.append((op, dst, mfma, valu))
        waits_since.append(0)
        if len(recent) > 24:
            recent, waits_since = recent[-24:], waits_since[-24:]
    return found


def main():
    found = scan(open(sys.argv[1]).read().split("\n"))
    for fn, w, r, n in found[:40]:
        print(f"{fn[:70]}: {w} -> {r}  ({n} wait states)")
    print(f"{len(found)} hazard(s)")
    sys.exit(1 if found else 0)


if __name__ == "__main__":
    main()
