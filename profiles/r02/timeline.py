#!/usr/bin/env python3
"""Print the kernel timeline of one cascade chunk from a rocprofv3 kernel trace
(profiles/r02/trace.sh): start / end (us, relative to the chunk's shared
front end), duration, kernel, workgroups, queue.  usage: timeline.py TRACE.csv [chunk]"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize import kname  # noqa: E402

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    wg = int(r.get("Workgroup_Size_X") or 1)
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kname(r["Kernel_Name"]),
                 int(r.get("Grid_Size_X") or 0) // max(wg, 1), r.get("Queue_Id") or r.get("Stream_Id")))
rows.sort()
ck = [r for r in rows if r[2] == "casc_begin_kernel"]
k = int(sys.argv[2]) if len(sys.argv) > 2 else -2
t0, t1 = ck[k][0], ck[k + 1][0] if k + 1 < len(ck) and k != -1 else rows[-1][1]
for r in rows:
    if t0 - 3000000 <= r[0] <= t1 and r[1] >= t0 - 100000:
        print(f"{(r[0] - t0) / 1000:9.1f} {(r[1] - t0) / 1000:9.1f} {(r[1] - r[0]) / 1000:8.1f}us {r[2]:26s} wg={r[3]:6d} q={r[4]}")
print(f"chunk {(t1 - t0) / 1000:.1f} us")
