#!/usr/bin/env python3
"""Summarise one profiles/r05/prof.sh output directory into JSON (round 4:
profiles/r02/summarize.py plus a fourth PMC pass and the issue-rate fields).

Per kernel (name without template arguments, cold front-end launches told
apart by grid size): launches and average / total duration (kernel trace),
HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024; FETCH_SIZE
doubled per MI355X_MICROARCH.md "HBM [CDNA4]": on gfx950 it reports half the
bytes of wide coalesced streaming reads; WRITE_SIZE exact for 16-B stores),
and the SQ counters of the third pass per launch: SQ_INSTS_MFMA,
SQ_VALU_MFMA_BUSY_CYCLES (cycles), SQ_WAVE_CYCLES / SQ_WAIT_ANY / SQ_BUSY_CYCLES
(quad-cycles), SQ_INSTS_VALU, GRBM_GUI_ACTIVE (sum over the 8 XCDs).
Fourth pass: SQ_ACTIVE_INST_VALU (quad-cycles), SQ_INSTS_SALU, SQ_INSTS_LDS,
SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_LDS, SQ_LDS_BANK_CONFLICT, SQ_WAVES.
Derived: mfma_busy = MFMA busy cycles / (GRBM_GUI_ACTIVE / 8 x 256 CUs x 4
SIMDs), the fraction of SIMD cycles the MFMA pipes were busy during the
kernel; wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES; valu_busy =
SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), the fraction of
SIMD cycles with a VALU instruction in issue; clock_ghz =
GRBM_GUI_ACTIVE / 8 / kernel time (MI355X_MICROARCH.md, DVFS give-back).

usage: summarize.py DIR WORKLOAD STREAMS FRAMES WEIGHTS INPUT OUT.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def kname(full: str, grid: int = 0) -> str:
    base = full.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()
    short = base.split("<")[0]
    if short in ("proj_kernel", "recur_pipe_kernel", "recur_kernel"):
        net = {"28": "vad", "64": "kws", "72": "s2i"}
        parts = base.split("<", 2)
        tag = "gen"
        if len(parts) > 2:
            args = parts[2].split(",")
            tag = net.get(args[6].strip(), "gen") if len(args) > 6 else "gen"
        short = f"{short}[{tag}]"
    # fe_kernel<MODE, PORT> / fe_kernel2<MODE, PORT> (two frames per wave):
    # MODE 0 batch, 1 shared (cascade), 2 cold (cascade rounds)
    if short in ("fe_kernel", "fe_kernel2"):
        mode = base.split("<", 1)[1].split(">")[0].split(",")[0].strip() if "<" in base else ""
        return {"0": "fe_kernel[batch]", "1": "fe_kernel[shared]", "2": "fe_kernel[cold]"}.get(mode, short)
    return short


def counters(path_glob):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(path_glob, recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = kname(row["Kernel_Name"], int(row.get("Grid_Size") or 0))
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def main():
    d, workload, S, T, weights, inp, out = sys.argv[1:8]
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                dur[kname(row["Kernel_Name"], int(row.get("Grid_Size_X") or 0))].append(
                    (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    c = {}
    for i in (1, 2, 3, 4):
        for k, v in counters(os.path.join(d, f"p{i}", "**", "*counter_collection.csv")).items():
            c.setdefault(k, {}).update(v)
    res = {"workload": workload, "streams": int(S), "frames": int(T), "weights": weights, "input": inp,
           "source": d, "kernels": {}}
    for k in sorted(set(dur) | set(c)):
        e = {}
        if dur.get(k):
            e["launches"] = len(dur[k])
            e["avg_ms"] = sum(dur[k]) / len(dur[k])
            e["total_ms"] = sum(dur[k])
        ck = c.get(k, {})
        avg = {n: sum(v) / len(v) for n, v in ck.items() if v}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            e["fetch_bytes_per_launch_x2"] = 2 * 1024 * avg["FETCH_SIZE"]
            e["write_bytes_per_launch"] = 1024 * avg["WRITE_SIZE"]
            e["hbm_bytes_per_launch"] = e["fetch_bytes_per_launch_x2"] + e["write_bytes_per_launch"]
            tot = 2 * 1024 * sum(ck["FETCH_SIZE"]) + 1024 * sum(ck["WRITE_SIZE"])
            e["hbm_bytes_all_launches"] = tot
        for n in ("SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_INSTS_VALU",
                  "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                  "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAVES"):
            if n in avg:
                e[n] = avg[n]
        if avg.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            e["mfma_busy"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
        if avg.get("GRBM_GUI_ACTIVE") and "SQ_ACTIVE_INST_VALU" in avg:
            e["valu_busy"] = avg["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * avg["GRBM_GUI_ACTIVE"] / 8)
        if avg.get("GRBM_GUI_ACTIVE") and e.get("avg_ms"):
            e["clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / (e["avg_ms"] * 1e-3) / 1e9
        if avg.get("SQ_WAVE_CYCLES"):
            e["wait_frac"] = avg.get("SQ_WAIT_ANY", 0) / avg["SQ_WAVE_CYCLES"]
        res["kernels"][k] = e
    # steps (chunks) profiled: one shared front end (cascade) or one batch
    # front end (single net) per step; per-step HBM bytes of every kernel
    nsteps = (res["kernels"].get("fe_kernel[shared]") or res["kernels"].get("fe_kernel[batch]") or {}).get("launches", 0)
    res["steps"] = nsteps
    for e in res["kernels"].values():
        if nsteps and "hbm_bytes_all_launches" in e:
            e["hbm_bytes_per_step"] = e["hbm_bytes_all_launches"] / nsteps
        if nsteps and "SQ_INSTS_VALU" in e and e.get("launches"):
            e["valu_insts_per_step"] = e["SQ_INSTS_VALU"] * e["launches"] / nsteps
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, v in res["kernels"].items():
        if v.get("total_ms", 0) > 0.05:
            print(f"{k:28s} n={v.get('launches', 0):4d} avg={v.get('avg_ms', 0) * 1e3:8.1f}us "
                  f"tot={v.get('total_ms', 0):7.2f}ms hbm/launch={v.get('hbm_bytes_per_launch', 0) / 1e6:8.1f}MB "
                  f"mfma_busy={v.get('mfma_busy', 0):.4f} valu_busy={v.get('valu_busy', 0):.3f} wait={v.get('wait_frac', 0):.2f} "
                  f"valu/launch={v.get('SQ_INSTS_VALU', 0):.3g}")


if __name__ == "__main__":
    main()
