#!/usr/bin/env python3
"""Per-stage VALU instruction counts of the shared front end's frame loop
(fe_kernel<FE_MODE_SHARED, shipped>) from hipcc -S output, split at the
development probes' s_memtime markers (FCLK 0..5 in nnsp_kernels.hip):

  FCLK0 -> FCLK1  prefetch of the next window, window products, previous frame's ring stores
  FCLK1 -> FCLK2  the 256-point q31 cFFT (4 radix-4 stages, T1/T3 permlane transposes, T2 via LDS)
  FCLK2 -> FCLK3  split (arm_split_rfft_q31) + power spectrum (spec2pspec_arm)
  FCLK3 -> FCLK4  Mel MACs (one lane segment per lane)
  FCLK4 -> FCLK5  bank sums, log10, the three nets' normalisation, ring values packed

Static counts of the straight-line code between the markers; the probes'
own blocks (memtime + store) are excluded, the prefetch's uncommon paths
(frames before the chunk, history stores) are listed apart.

usage: python fe_stage_isa.py [nnsp_kernels.hip]   (compiles it with hipcc -S)
"""
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

SYM = "_Z9fe_kernelILi1ELb0EEv6FeArgs"
STAGES = ["prefetch+window+ring store", "cFFT", "split+power", "Mel MACs", "sums+log10+norm x3"]


def isa(src):
    out = os.path.join(tempfile.mkdtemp(), "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-DNNSP_PROBES=1", "--cuda-device-only", "-S",
                    src, "-o", out], check=True, capture_output=True)
    lines = open(out).read().split("\n")
    a = next(i for i, l in enumerate(lines) if l.startswith(SYM + ":"))
    b = next(i for i in range(a, len(lines)) if lines[i].strip().startswith("s_endpgm"))
    return lines[a:b]


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "..", "nnsp_amd",
                                                             "csrc", "kernels", "nnsp_kernels.hip")
    body = isa(src)
    # the six FCLK probes are the kernel's only s_memtime (FCLK 0 sits just
    # before the rotated loop's header)
    marks = [i for i, l in enumerate(body) if "s_memtime" in l]
    assert len(marks) == 6, marks
    rows = []
    for k in range(5):
        seg = body[marks[k]:marks[k + 1]]
        c = Counter()
        for l in seg:
            t = l.strip().split()
            if not t or t[0].startswith((".", ";")):
                continue
            op = t[0]
            if op.startswith("v_"):
                c["valu"] += 1
                c[op] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
        # the probe's own store block (memtime -> global_store_dwordx2) holds 2 VALU
        c["valu"] -= 2
        rows.append((STAGES[k], c))
    tot = sum(c["valu"] for _, c in rows)
    print("| stage | VALU | LDS | main ops |")
    print("|---|---|---|---|")
    for name, c in rows:
        ops = ", ".join(f"{o.replace('_e32', '')} {n}" for o, n in c.most_common() if o.startswith("v_"))[:160]
        print(f"| {name} | {c['valu']} | {c['lds']} | {ops} |")
    print(f"| total (static, all paths) | {tot} | | |")


if __name__ == "__main__":
    main()
