#!/usr/bin/env python3
"""LDS bank conflicts of recur_pipe_kernel's B-fragment reads (load_b, nnsp_nn.h): lane (sc = lane & 15,
q = lane >> 4) reads 16 int16 at row sc, k = 64 kt + 16 q, as two ds_read_b128 (dwords +0..3, +4..7).
ds_read_b128 is serviced in four groups of 16 lanes (MI355X_MICROARCH.md, LDS table); within a group, the
number of distinct 16-byte addresses on the busiest bank is the cycles that group takes.  Prints, per row
stride RS (int16), the mean cycles per group (1 = conflict-free) for kt = 0, 1 and both halves."""
GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
          list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
          list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]


def cycles(s, kt, half):
    tot = 0
    for g in GROUPS:
        banks = {}
        for lane in g:
            d = (lane & 15) * s + 32 * kt + 8 * (lane >> 4) + 4 * half
            for b in range(d, d + 4):
                banks.setdefault(b % 64, set()).add(d)
        tot += max(len(v) for v in banks.values())
    return tot / 4


if __name__ == "__main__":
    for rs in range(64, 156, 8):
        print(f"RS {rs:3d} int16:", [cycles(rs // 2, kt, h) for kt in (0, 1) for h in (0, 1)])
