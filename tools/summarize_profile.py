"""Summarise a tools/profile.sh run (gpurun_out/<tag>) into profiles/<tag>/: the rocprofv3
kernel-stats CSV, per-kernel PMC averages, and pmc_<workload>.json (per-launch HBM bytes of the
SyncTest kernel, read by bench.py's roofline.traffic).

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE are KiB from the L2's
memory-side request counters (TCC_EA0_RDREQ/WRREQ); on gfx950 FETCH_SIZE reports exactly half the
bytes of a wide streaming read, so the corrected figure doubles it.  Both are kept.

    python tools/summarize_profile.py <tag> <workload> <kernel substring> [last K dispatches] [units]

`units` (default 1): work units one launch of the kernel covers (configs 3/4: the rounds of one
fused ggrs_branch_rounds launch); pmc_<workload>.json then holds bytes and duration per unit.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc_means(path, kernel_substr, last=0):
    """Per-counter mean over the kernel's dispatches (the last `last` ones if last > 0)."""
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if kernel_substr in r["Kernel_Name"]:
            per[r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out, n = {}, {}
    for k, v in per.items():
        v.sort()
        vals = [x for _, x in (v[-last:] if last else v)]
        out[k], n[k] = sum(vals) / len(vals), len(vals)
    return out, n


def trace_mean_ns(path, kernel_substr, last=0):
    rows = [r for r in csv.DictReader(open(path)) if kernel_substr in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if last:
        rows = rows[-last:]
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    return sum(d) / len(d), len(d)


def main(tag, workload, kernel="synctest_kernel", last="0", units="1"):
    last, units = int(last), int(units)
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "trace_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(dst, "kernel_stats.csv")))}
    kname = next(n for n in stats if kernel in n)
    avg_ns, ncalls = trace_mean_ns(os.path.join(src, "trace", "trace_kernel_trace.csv"), kernel, last)
    out = {"tag": tag, "workload": workload, "kernel": kname, "calls_in_trace": int(stats[kname]["Calls"]),
           "dispatches_averaged": ncalls, "avg_duration_ns": avg_ns,
           "note": f"averages over the last {last} dispatches (the timed steps)" if last else "all dispatches"}
    for group in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_grbm"):
        p = os.path.join(src, group, "pmc_counter_collection.csv")
        if os.path.exists(p):
            means, counts = pmc_means(p, kernel, last)
            out[group] = means
    fetch_kib = out.get("pmc_fetch", {}).get("FETCH_SIZE")
    write_kib = out.get("pmc_write", {}).get("WRITE_SIZE")
    if fetch_kib is not None and write_kib is not None:
        out["hbm_bytes_per_launch_raw"] = (fetch_kib + write_kib) * 1024
        out["hbm_bytes_per_launch"] = (2 * fetch_kib + write_kib) * 1024  # gfx950 FETCH x2
    sq = out.get("pmc_sq", {})
    if sq.get("SQ_WAVES"):
        out["valu_insts_per_wave"] = sq["SQ_INSTS_VALU"] / sq["SQ_WAVES"]
    if sq.get("SQ_WAVE_CYCLES"):
        # SQ_WAVE_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* count quad-cycles (MI355X_MICROARCH.md)
        wc = sq["SQ_WAVE_CYCLES"]
        out["valu_active_frac_of_wave_cycles"] = sq.get("SQ_ACTIVE_INST_VALU", 0) / wc
        out["wait_inst_frac"] = sq.get("SQ_WAIT_INST_ANY", 0) / wc
        out["wait_any_frac"] = sq.get("SQ_WAIT_ANY", 0) / wc
        out["active_any_frac"] = sq.get("SQ_ACTIVE_INST_ANY", 0) / wc
    gr = out.get("pmc_grbm", {})
    if gr.get("GRBM_GUI_ACTIVE"):
        # effective clock ~= GRBM_GUI_ACTIVE / 8 (summed over XCDs) / kernel time
        out["effective_clock_ghz"] = gr["GRBM_GUI_ACTIVE"] / 8 / avg_ns
    if sq.get("SQ_INSTS_VALU"):
        # VALU issue fraction: wave-instructions x 2 cycles (a wave64 VALU op occupies its SIMD for
        # 2 cycles at best, MI355X_MICROARCH.md) over the chip's SIMD-cycles during the kernel
        clk = out.get("effective_clock_ghz") or 2.4
        out["valu_issue_frac"] = sq["SQ_INSTS_VALU"] * 2 / (1024 * avg_ns * clk)
        # the same per wave at the rate ONE wave sustains alone (4 cycles per VALU instruction,
        # MI355X_MICROARCH.md 'vector-instruction ISSUE cost'): the ceiling of a one-wave-per-SIMD
        # kernel is 1.0 here (0.5 on valu_issue_frac)
        if out.get("valu_insts_per_wave"):
            out["valu_wave_issue_frac"] = out["valu_insts_per_wave"] * 4 / (avg_ns * clk)
    with open(os.path.join(dst, "summary.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    if "hbm_bytes_per_launch" in out:
        with open(os.path.join(ROOT, "profiles", f"pmc_{workload}.json"), "w") as fh:
            json.dump({"tag": tag, "kernel": kname, "hbm_bytes_per_launch": out["hbm_bytes_per_launch"] / units,
                       "hbm_bytes_per_launch_raw": out["hbm_bytes_per_launch_raw"] / units,
                       "avg_duration_ns": avg_ns / units, "units_per_launch": units,
                       "valu_active_frac_of_wave_cycles": out.get("valu_active_frac_of_wave_cycles"),
                       "valu_insts_per_wave": out.get("valu_insts_per_wave"),
                       "valu_issue_frac": out.get("valu_issue_frac"),
                       "valu_wave_issue_frac": out.get("valu_wave_issue_frac"),
                       "wait_any_frac": out.get("wait_any_frac")}, fh, indent=1)
    for f in ("bench_trace.log",):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
