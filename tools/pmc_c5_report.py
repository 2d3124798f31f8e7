#!/usr/bin/env python3
"""Summarise tools/profile_c5.sh's counter passes into one JSON object per kernel.

Per kernel: mean over its dispatches (the first dropped) of every counter collected, the
kernel's mean duration from the kernel-trace pass, and derived figures:
  kernel_cycles        GRBM_GUI_ACTIVE / 8 (rocprofv3 sums GRBM over the 8 XCDs) on a dispatch of
                       0.3 ms or more, where that quotient tracks the clock; on a shorter one it
                       reads high (MI355X_MICROARCH.md, DVFS note: 3.77 GHz for a 12 us rollout
                       dispatch), so kernel_cycles is duration x 2.4 GHz, the part's top clock:
                       an upper bound on the cycles, which makes every per-cycle figure below a
                       LOWER bound there (cycle_source says which)
  clock_ghz            kernel_cycles / duration (only where GRBM sets kernel_cycles)
  valu_ipc_per_cu      SQ_INSTS_VALU / 256 CUs / kernel_cycles; a wave64 VALU op holds a SIMD
                       >= 2 cycles (MI355X_MICROARCH.md cycle table), so the issue ceiling is
                       4 SIMDs / 2 = 2.0 per CU per cycle for 32-bit ops (fp64 and transcendental
                       ops cost more)
  valu_busy            SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x kernel_cycles)  (gfx94x formula; on
                       gfx950 SQ_ACTIVE_INST_VALU reads as an instruction count, = SQ_INSTS_VALU)
  wave_cycle_split     SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_ANY, SQ_WAIT_ANY as fractions of
                       SQ_WAVE_CYCLES (disjoint, MI355X_MICROARCH.md PMC table)
  resident_waves_cu    SQ_WAVE_CYCLES x 4 (quad-cycles) / kernel_cycles / 256 CUs
  lds_conflict_frac    SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  lane_util            SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU): mean active lanes per VALU
                       instruction (1.0 = no divergence; oc_step_n, branch-free SWAR, reads 0.996)
  hbm_read/write_bytes FETCH_SIZE x 1024 x read factor (calibrated on oc_checksum_kernel's known
                       23 x 2^18 bytes of the same batch), WRITE_SIZE x 1024
usage: pmc_c5_report.py OUT_DIR   (reads OUT_DIR/p1..p5 and OUT_DIR/trace)
       pmc_c5_report.py --rederive PMC_C5.JSON   (recompute the derived figures of an earlier
                                                  report from the counters it kept)
"""
import csv
import glob
import json
import os
import sys

KERNELS = ("oc_rollout_kernel", "oc_rollout_group_kernel", "oc_bounds_kernel", "oc_likelihood_compact_kernel", "oc_likelihood_kernel", "oc_checksum_kernel",
           "oc_step_n_kernel", "oc_render_kernel")
CUS, SIMDS = 256, 1024
TOP_CLOCK_GHZ = 2.4     # MI355X peak engine clock
GRBM_MIN_NS = 300_000   # below this GRBM_GUI_ACTIVE / 8 / duration reads high
CHECKSUM_BYTES = 23 * (1 << 18)  # 3A + 2K + 3 planes x pitch, full-divider_salad 4 agents


def kernel_key(name):
    return next((k for k in KERNELS if k + "<" in name or name.startswith(k) or (" " + k) in name), None)


def counters(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = kernel_key(row["Kernel_Name"])
                if k is None:
                    continue
                did = int(row.get("Dispatch_Id", 0))
                c = out.setdefault(k, {}).setdefault(row["Counter_Name"], {})
                c[did] = c.get(did, 0.0) + float(row["Counter_Value"])
    return out


def mean_tail(byid):
    v = [byid[i] for i in sorted(byid)]
    v = v[1:] if len(v) > 1 else v
    return sum(v) / len(v)


def durations(d):
    res = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = kernel_key(row["Kernel_Name"])
                if k:
                    res.setdefault(k, []).append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return {k: sum(v[1:] or v) / len(v[1:] or v) for k, v in res.items()}


def derive(c, dur, rf):
    """Derived figures of one kernel from its mean counters `c` and mean duration `dur` (ns)."""
    g = c.get("GRBM_GUI_ACTIVE_p1") or c.get("GRBM_GUI_ACTIVE_p2")
    r = {"counters": c, "duration_ns": dur}
    cyc = None
    if g and dur and dur >= GRBM_MIN_NS:
        cyc = g / 8.0
        r["cycle_source"] = "GRBM_GUI_ACTIVE / 8 (dispatch >= 0.3 ms)"
        r["clock_ghz"] = cyc / dur
    elif dur:
        cyc = dur * TOP_CLOCK_GHZ
        r["cycle_source"] = ("duration x %.1f GHz (dispatch < 0.3 ms: GRBM_GUI_ACTIVE / 8 / duration would read %s "
                             "GHz); per-cycle figures are lower bounds" % (TOP_CLOCK_GHZ,
                                                                            "%.2f" % (g / 8.0 / dur) if g else "n/a"))
    if cyc:
        r["kernel_cycles"] = cyc
        if "SQ_INSTS_VALU" in c:
            r["valu_ipc_per_cu"] = c["SQ_INSTS_VALU"] / CUS / cyc
        if "SQ_ACTIVE_INST_VALU" in c:
            r["valu_busy"] = c["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * cyc)
        if "SQ_WAVE_CYCLES" in c:
            r["resident_waves_cu"] = c["SQ_WAVE_CYCLES"] * 4 / cyc / CUS
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        r["wave_cycle_split"] = {n: c[n] / wc for n in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")
                                 if n in c}
    if c.get("SQ_WAVES"):
        r["per_wave"] = {n: c[n] / c["SQ_WAVES"] for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                                                           "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR") if n in c}
        if wc:
            r["per_wave"]["wave_quad_cycles"] = wc / c["SQ_WAVES"]
    if c.get("SQ_LDS_IDX_ACTIVE"):
        r["lds_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"]
    if c.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in c:
        r["lane_util"] = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
    if "FETCH_SIZE" in c and rf:
        r["hbm_read_bytes"] = c["FETCH_SIZE"] * 1024 * rf
    if "WRITE_SIZE" in c:
        r["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
    return r


def main():
    if sys.argv[1] == "--rederive":
        old = json.load(open(sys.argv[2]))
        res = {"read_factor": old.get("read_factor"), "kernels": {}}
        for k, r in old["kernels"].items():
            res["kernels"][k] = derive(r["counters"], r.get("duration_ns"), old.get("read_factor"))
        print(json.dumps(res, indent=1))
        return
    out_dir = sys.argv[1]
    merged = {}
    for p in ("p1", "p2", "p3", "p4", "p5"):
        for k, cs in counters(os.path.join(out_dir, p)).items():
            for name, byid in cs.items():
                merged.setdefault(k, {})["%s" % name if name != "GRBM_GUI_ACTIVE" else "GRBM_GUI_ACTIVE_" + p] = \
                    mean_tail(byid)
    dur = durations(os.path.join(out_dir, "trace"))
    rf = None
    if "oc_checksum_kernel" in merged and merged["oc_checksum_kernel"].get("FETCH_SIZE"):
        rf = CHECKSUM_BYTES / (merged["oc_checksum_kernel"]["FETCH_SIZE"] * 1024)
    res = {"read_factor": rf, "kernels": {}}
    for k, c in merged.items():
        res["kernels"][k] = derive(c, dur.get(k), rf)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
