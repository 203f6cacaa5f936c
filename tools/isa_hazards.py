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
Wait states = intervening instructions (1 each) + s_nop N (N + 1).  The window follows
the control flow: it runs on through labels (a label adds no wait states) and
conditional branches (one wait state each, fall-through path), and each label starts
from the merge (worst case) of its fall-through window and the windows of every branch
that targets it, iterated to a fixed point over back edges.  Only an unconditional
s_branch / s_setpc ends the fall-through window.

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


_LABEL = re.compile(r"^([_A-Za-z.$][\w.$]*):")
_WINDOW = 24


def _merge(a, b):
    """Worst case of two windows: every pending write of either, newest last."""
    out = sorted(set(a) | set(b), key=lambda e: -e[4])
    return out[-_WINDOW:]


def _scan_once(insns, entry, found):
    """One pass over the instructions with the label entry windows `entry` (label ->
    window); returns the windows each branch carries to its target."""
    carried = {}
    fn = None
    win = []  # (op, dst regs frozenset, is_mfma, is_valu, wait states since) newest last
    reach = True  # the current point is reached by fall-through
    for kind, a, b in insns:
        if kind == "label":
            if not a.startswith(".L"):
                fn, win = a, []
            win = _merge(win if reach else [], entry.get(a, []))
            reach = True
            continue
        op, ins, args = a, b, None
        args = _split(ins)[1]
        if op.startswith("s_cbranch") or op == "s_branch" or op.startswith("s_setpc"):
            tgt = args[0] if args else None
            if tgt is not None and tgt.startswith(".L"):
                carried[tgt] = _merge(carried.get(tgt, []), win)
            if op.startswith("s_cbranch"):
                win = [(o, d, m, v, w + 1) for (o, d, m, v, w) in win]
            else:
                win, reach = [], False
            continue
        if op == "s_nop":
            n = int(args[0], 0) + 1 if args else 1
            win = [(o, d, m, v, w + n) for (o, d, m, v, w) in win]
            continue
        if op.startswith("v_") and _is_dpp_read(op, ins):
            srcs = set()
            for x in args[1:]:
                srcs |= _regs(x)
            if "permlane" in op or op.startswith("v_fmac"):
                srcs |= _regs(args[0])  # tied / swapped operand is read too
            for (wop, dst, mfma, valu, w) in win:
                need = (19 if "32x32" in wop else 11) if mfma else (2 if valu else 0)
                if dst & srcs and w < need:
                    found.add((fn, wop, ins, w))
        dst = frozenset(_regs(args[0])) if args and op.startswith("v_") else frozenset()
        mfma = "mfma" in op
        valu = op.startswith("v_") and not mfma and not op.startswith(("v_readlane", "v_readfirstlane"))
        win = [(o, d, m, v, w + 1) for (o, d, m, v, w) in win]
        win.append((op, dst, mfma, valu, 0))
        win = win[-_WINDOW:]
    return carried


def scan(lines):
    """-> [(function, writer, reader, wait_states)] of hazardous pairs."""
    insns = []
    for raw in lines:
        line = raw.split(";")[0].rstrip()
        if not line.strip():
            continue
        m = _LABEL.match(line)
        if m:
            insns.append(("label", m.group(1), None))
            continue
        ins = line.strip()
        if ins.startswith("."):
            continue
        insns.append(("ins", _split(ins)[0], ins))
    entry = {}
    found = set()
    for _ in range(4):  # back edges: iterate the label entry windows to a fixed point
        found = set()
        carried = _scan_once(insns, entry, found)
        if carried == entry:
            break
        entry = carried
    return sorted(found, key=lambda f: (str(f[0]), f[2]))


def main():
    found = scan(open(sys.argv[1]).read().split("\n"))
    for fn, w, r, n in found[:40]:
        print(f"{fn[:70]}: {w} -> {r}  ({n} wait states)")
    print(f"{len(found)} hazard(s)")
    sys.exit(1 if found else 0)


if __name__ == "__main__":
    main()
