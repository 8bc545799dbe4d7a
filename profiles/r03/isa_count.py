"""Static instruction mix of one kernel's hottest loop from hipcc -S output.

usage: python isa_count.py file.s SYMBOL

Finds the kernel's basic blocks, takes the largest backward-branch loop (the
frame loop) and counts the instructions in it by class (VALU, SALU, LDS,
VMEM, branch, waitcnt), each counted once per static occurrence.  Blocks on
conditional side paths (debug probes, rare edges) are counted too, so this is
an upper bound on the per-iteration mix.
"""
import re
import sys
from collections import Counter


def body(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    return lines[start:end]


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_load", "s_buffer")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    L = body(path, sym)
    labels = {}
    for i, l in enumerate(L):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, l in enumerate(L):
        m = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((i - labels[m.group(1)], labels[m.group(1)], i))
    loops.sort(reverse=True)
    # the hot loop: the largest one holding the kernel's q31 products
    hot = [lp for lp in loops if any(("v_mul_hi_i32" in l or "v_mfma" in l) for l in L[lp[1]:lp[2] + 1])]
    n, a, b = (hot or loops)[0]
    c = Counter()
    ops = Counter()
    for l in L[a:b + 1]:
        s = l.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        c[classify(op)] += 1
        ops[op] += 1
    print(f"{sym}: loop lines {a}..{b}")
    for k, v in sorted(c.items(), key=lambda x: -x[1]):
        print(f"  {k:8s} {v}")
    print("  top ops:", ", ".join(f"{o} {v}" for o, v in ops.most_common(40)))


if __name__ == "__main__":
    main()
