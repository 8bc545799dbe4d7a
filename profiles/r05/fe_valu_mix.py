#!/usr/bin/env python3
"""Issue-cost-weighted VALU mix of the shared front end's frame loop
(fe_kernel<FE_MODE_SHARED, shipped>), for roofline.valu_occupancy in bench.py
(VERDICT r4 next #6).

valu_busy counts VALU *instructions* (SQ_ACTIVE_INST_VALU: one quad-cycle
each).  Instructions do not cost the same issue time: the measured SIMD cycles
per wave64 instruction (profiles/microbench/) are ~2.8 for an add, ~4.3 for
v_mul_hi_i32, ~5.0 for v_mad_i64_i32, ~9 for a permlane swap.  This script
compiles the kernel (hipcc -S, the development probes' s_memtime markers FCLK
0..5 delimit the stages), counts the static VALU opcodes of each stage and
prices them:

  * v_add_u32 / v_mul_i32_i24 / v_mul_hi_i32 / v_mad_i64_i32: the full-chip
    issue rates of profiles/microbench/valu_rates_mi355x.json
    (cycles = 64 lanes / (lane-ops/s / (CUs x 4 SIMDs x clock)));
  * every other form: its cost relative to v_add_u32 in
    profiles/microbench/valu_rates2_mi355x.json times the add's cycles;
  * forms in neither file: the add's cost.

Writes profiles/fe_valu_mix.json: per stage the static count and weighted
cycles, and the count-weighted average cycles per VALU instruction.  bench.py
multiplies that average by the PMC's dynamic SQ_INSTS_VALU and divides by the
SIMD-cycles of the launch.

usage: python profiles/r05/fe_valu_mix.py [out.json]
"""
import json
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SYM = "_Z9fe_kernelILi1ELb0EEv6FeArgs"
STAGES = ["prefetch+window+ring store", "cFFT", "split+power", "Mel MACs", "sums+log10+norm x3"]


def costs():
    r1 = json.load(open(os.path.join(ROOT, "profiles", "microbench", "valu_rates_mi355x.json")))
    r2 = json.load(open(os.path.join(ROOT, "profiles", "microbench", "valu_rates2_mi355x.json")))
    per_simd_clk = r1["compute_units"] * 4 * r1["clock_khz"] * 1e3
    c = {op: 64.0 / (rate / per_simd_clk) for op, rate in r1["rates"].items()}
    add = c["v_add_u32"]
    for op, cyc in r2["cycles"].items():
        if op not in c:
            c[op] = add * cyc / r2["cycles"]["v_add_u32"]
    return c, add


def base_op(op):
    op = re.sub(r"_e(32|64)$", "", op)
    op = op.replace("_sdwa", "").replace("_dpp", "")
    return op


def price(op, table, add):
    b = base_op(op)
    if b in table:
        return table[b]
    if b.startswith("v_permlane"):
        return table.get("v_permlane32_swap", 3 * add)
    if re.match(r"v_cmp\w*_[iu]64", b):
        return table.get("v_cmp_gt_i64", add)
    if b in ("v_mad_u64_u32",):
        return table["v_mad_i64_i32"]
    return add


def isa():
    out = os.path.join(tempfile.mkdtemp(), "k.s")
    src = os.path.join(ROOT, "nnsp_amd", "csrc", "kernels", "nnsp_kernels.hip")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-DNNSP_PROBES=1",
                    "--cuda-device-only", "-S", src, "-o", out], check=True, capture_output=True)
    lines = open(out).read().split("\n")
    a = next(i for i, ln in enumerate(lines) if ln.startswith(SYM + ":"))
    b = next(i for i in range(a, len(lines)) if lines[i].strip().startswith("s_endpgm"))
    return lines[a:b]


def main():
    table, add = costs()
    body = isa()
    marks = [i for i, ln in enumerate(body) if "s_memtime" in ln]
    assert len(marks) == 6, marks
    stages, tot_n, tot_c = [], 0, 0.0
    for k in range(5):
        ops = Counter()
        for ln in body[marks[k]:marks[k + 1]]:
            t = ln.strip().split()
            if t and t[0].startswith("v_"):
                ops[t[0]] += 1
        # the probe's own store block (s_memtime -> global_store_dwordx2) holds 2 VALU moves
        ops["v_mov_b32_e32"] -= 2
        n = sum(ops.values())
        cyc = sum(price(op, table, add) * m for op, m in ops.items())
        stages.append({"stage": STAGES[k], "valu_static": n, "weighted_cycles": round(cyc, 1),
                       "top_ops": dict(ops.most_common(8))})
        tot_n += n
        tot_c += cyc
    out = {"kernel": "fe_kernel<FE_MODE_SHARED, shipped> frame loop (static, hipcc -S)",
           "cost_cycles_per_wave64_instruction": {k: round(v, 2) for k, v in sorted(table.items())},
           "default_cost": round(add, 2), "stages": stages, "valu_static": tot_n,
           "weighted_cycles_static": round(tot_c, 1), "avg_cycles_per_valu": round(tot_c / tot_n, 3),
           "how": "per-opcode SIMD issue cycles (profiles/microbench) x static count per stage; "
                  "avg = sum / count; valu_occupancy = SQ_INSTS_VALU x avg / (SIMDs x kernel cycles)"}
    dst = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "fe_valu_mix.json")
    json.dump(out, open(dst, "w"), indent=1)
    for s in stages:
        print(f"{s['stage']:28s} {s['valu_static']:4d} VALU  {s['weighted_cycles']:8.1f} cycles")
    print(f"total {tot_n} VALU, {tot_c:.0f} cycles, {tot_c / tot_n:.3f} cycles per VALU")


if __name__ == "__main__":
    main()
