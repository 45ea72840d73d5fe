"""Per-loop instruction mix of one kernel in a hipcc -S listing (tools only).

usage: python tools/isa_loops.py file.s kernel_symbol_substring
Prints every backward-branch loop body (label .. branch back) with counts by class."""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
        return "valu-x"
    if op.startswith("v_") and "_f64" in op:
        return "valu-f64"
    if op.startswith(("v_rcp", "v_sqrt", "v_rsq", "v_exp", "v_log", "v_sin", "v_cos")):
        return "valu-trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_store", "global_store")):
        return "store"
    if op.startswith(("buffer_load", "global_load", "s_load", "s_buffer")):
        return "load"
    return "other"


def main(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym) or (sym in l and l.rstrip().endswith(":") and not l.startswith("\t")))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(body):
        m = re.match(r"^\s+(s_cbranch_\w+|s_branch)\s+(\.LBB\d+_\d+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            a = labels[m.group(2)]
            c = Counter()
            for x in body[a:i + 1]:
                x = x.strip()
                if not x or x.startswith((";", ".")) or x.endswith(":"):
                    continue
                c[classify(x.split()[0])] += 1
            print(f"loop {m.group(2)} lines {a}-{i}: total {sum(c.values())}", dict(sorted(c.items())))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
