"""Inline-asm hazard check over gfx950 ISA (hipcc -S output): the round-4 parity break's cause.

gfx950 needs 3 wait states between a v_dot* (or MFMA) that writes a VGPR and another VALU
instruction that reads it; LLVM's hazard recognizer inserts `s_nop`s before the compiler's own
readers, but it does not treat a (non-empty) inline-asm statement as a reader, so a scheduler that
moves the asm right behind the dot (LLVM's max-ilp did, in particles.hip at 9732acd^) reads a stale
register.  This tool lists every non-empty inline-asm block of a .s file and flags each source
VGPR written by a v_dot*/v_mfma* fewer than 3 wait states earlier (counting s_nop N as N + 1, every
other instruction as 1, an empty asm block as 0; a label or branch ends the look-back).

    python tools/asm_hazards.py file.s [...]      # exit 1 if any hazard is found

DESIGN.md section 3 quotes its finding for particles.hip; the product units carry no non-empty
inline asm since round 5 (tests/test_no_inline_asm.py).
"""
import re
import sys

_REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
_WAIT = 3


def _regs(text):
    out = set()
    for m in _REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def _split(ins):
    """(mnemonic, dst regs, src regs) of one instruction line."""
    parts = ins.split(None, 1)
    op = parts[0]
    if len(parts) == 1:
        return op, set(), set()
    ops = [o.strip() for o in parts[1].split(",")]
    if op.startswith(("global_store", "buffer_store", "ds_write", "ds_add", "flat_store", "s_")):
        return op, set(), _regs(parts[1])
    return op, _regs(ops[0]), _regs(",".join(ops[1:]))


def scan(lines):
    """Yield (line number, asm text, reg, writer, wait states) for each hazard; also returns the
    number of non-empty asm blocks via the `blocks` list."""
    hist = []  # (line no, op, dst regs, wait states it counts)
    blocks, hazards = [], []
    i = 0
    while i < len(lines):
        s = lines[i].split(";")[0].strip() if not lines[i].strip().startswith(";;#ASM") else lines[i].strip()
        if s == ";;#ASMSTART":
            body = []
            j = i + 1
            while j < len(lines) and lines[j].strip() != ";;#ASMEND":
                t = lines[j].split(";")[0].strip()
                if t:
                    body.append((j + 1, t))
                j += 1
            if body:
                blocks.append((i + 1, [t for _, t in body]))
                for ln, t in body:
                    _, dst, src = _split(t)
                    for r in sorted(src):
                        ws = 0
                        for hln, hop, hdst, hw in reversed(hist):
                            if r in hdst:
                                if (hop.startswith("v_dot") or hop.startswith("v_mfma")) and ws < _WAIT:
                                    hazards.append((ln, t, r, f"{hop} (line {hln})", ws))
                                break
                            ws += hw
                            if ws >= _WAIT:
                                break
                    hist.append((ln, t.split()[0], dst, 1))
            i = j + 1
            continue
        if not s or s.startswith("."):
            i += 1
            continue
        if s.endswith(":") or s.startswith(("s_branch", "s_cbranch", "s_setpc", "s_swappc")):
            hist = []
            i += 1
            continue
        op, dst, _ = _split(s)
        w = int(s.split()[1], 0) + 1 if op == "s_nop" else 1
        hist.append((i + 1, op, dst, w))
        if len(hist) > 16:
            hist.pop(0)
        i += 1
    return blocks, hazards


def main(paths):
    bad = 0
    for p in paths:
        blocks, hazards = scan(open(p).read().splitlines())
        print(f"{p}: {len(blocks)} non-empty inline-asm blocks, {len(hazards)} hazards")
        for ln, t, r, w, ws in hazards:
            print(f"  line {ln}: `{t}` reads v{r} {ws} wait states after {w}")
        bad += len(hazards)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
