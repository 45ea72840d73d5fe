"""Static in-order issue model of one wave's basic blocks in a hipcc -S listing (tools only).

usage: python tools/sched_model.py file.s kernel_symbol [first_label last_label]

For every basic block of the kernel (or the blocks between two labels) it replays the
instructions in program order on ONE wave: an instruction issues when the previous one has
issued (issue costs below) and when its source registers are ready (producer's issue time +
latency).  Cross-block dependencies are ignored (registers are ready at block entry), so the
figure is a per-block schedule quality estimate for comparing compiler schedules of the SAME
code, not a cycle-accurate prediction.  Costs: MI355X_MICROARCH.md's one-wave issue table
(v_fma_f32 4, transcendental 8) and tools/microbench/vdep.hip's dependent-chain latencies
(about 8-9 cycles for VALU -> VALU, about 40 more for a v_cmp feeding s_cbranch)."""
import re
import sys

ISSUE = {"valu": 4, "trans": 8, "salu": 4, "smem": 4, "vmem": 8, "lds": 4, "branch": 4, "nop": 4, "wait": 0}
LAT = {"valu": 8, "trans": 16, "salu": 2, "lds": 64, "vmem": 500, "cvt_slow": 40}
SLOW = ("v_cvt_i32_f64", "v_cvt_f64_i32", "v_cvt_u32_f64", "v_cvt_f64_u32")
TRANS = ("v_rcp", "v_sqrt", "v_rsq", "v_exp", "v_log", "v_sin", "v_cos", "v_div_fmas", "v_div_scale", "v_div_fixup")

reg_re = re.compile(r"\b([vs])\[(\d+):(\d+)\]|\b([vs])(\d+)\b|\b(vcc|exec|scc)\b")


def regs(text):
    out = []
    for m in reg_re.finditer(text):
        if m.group(1):
            out += [f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)]
        elif m.group(4):
            out.append(f"{m.group(4)}{m.group(5)}")
        else:
            out.append(m.group(6))
    return out


def kind(op):
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith(TRANS):
        return "trans"
    return "valu"


def simulate(block):
    t = 0          # next issue slot
    ready = {}     # reg -> cycle its value is usable
    lds_pending = []  # completion times of outstanding LDS ops (lgkmcnt)
    vm_pending = []
    lat_stall = 0
    for line in block:
        parts = line.split(None, 1)
        op = parts[0]
        args = parts[1] if len(parts) > 1 else ""
        k = kind(op)
        if k == "wait":
            m = re.search(r"lgkmcnt\((\d+)\)", args)
            if m:
                n = int(m.group(1))
                done = sorted(lds_pending)
                if len(done) > n:
                    t = max(t, done[len(done) - n - 1])
                lds_pending = done[len(done) - n:] if n else []
            m = re.search(r"vmcnt\((\d+)\)", args)
            if m:
                n = int(m.group(1))
                if len(vm_pending) > n:
                    t = max(t, sorted(vm_pending)[len(vm_pending) - n - 1])
            continue
        rs = regs(args)
        if k in ("vmem", "lds") and op.startswith(("buffer_store", "global_store", "ds_write")):
            dsts, srcs = [], rs
        elif k == "branch":
            dsts, srcs = [], (["vcc"] if "vcc" in op else []) + (["scc"] if "scc" in op else []) + (
                ["exec"] if "exec" in op else [])
        else:
            dsts, srcs = rs[:1], rs[1:]
            if op.startswith(("v_cmp", "s_cmp", "s_bitcmp")) and not op.endswith("_e64") and "vcc" not in rs[:1]:
                dsts = ["vcc" if op.startswith("v_cmp") else "scc"]
                srcs = rs
            if op.startswith("s_") and k == "salu" and not op.startswith(("s_cmp", "s_bitcmp")):
                dsts = rs[:1] + ["scc"]
            if "_dpp" in op or "dpp" in args or op.startswith(("v_cndmask", "v_addc", "v_subb")):
                srcs = rs[1:] + ["vcc"]
            if op.startswith("v_fmac") or op.startswith("v_mac") or "_dpp" in op:
                srcs = rs  # accumulates into / may keep its destination
        start = max([t] + [ready.get(r, 0) for r in srcs])
        lat_stall += start - t
        if k == "branch" and "vcc" in op:
            start = max(start, ready.get("vcc", 0) + LAT["cvt_slow"])
        lat = LAT["cvt_slow"] if op.startswith(SLOW) else LAT.get(k, 8)
        if k == "lds" and not op.startswith("ds_write"):
            lds_pending.append(start + LAT["lds"])
        if k == "vmem":
            vm_pending.append(start + LAT["vmem"])
        for d in dsts:
            ready[d] = start + lat
        t = start + ISSUE[k]
    return t, lat_stall


def main(path, sym, first=None, last=None):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, name = [], [], "entry"
    for l in lines[start + 1:end]:
        s = l.strip()
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            blocks.append((name, cur))
            name, cur = m.group(1), []
            continue
        if not s or s.startswith((";", ".")):
            continue
        cur.append(s.split(";")[0].strip())
    blocks.append((name, cur))
    on = first is None
    total = 0
    for name, b in blocks:
        if name == first:
            on = True
        if on and b:
            c, st = simulate(b)
            total += c
            print(f"{name:14s} insts {len(b):4d} cycles {c:6d} latency-stall {st:5d}")
        if name == last:
            break
    print("total cycles", total)


if __name__ == "__main__":
    main(*sys.argv[1:])
