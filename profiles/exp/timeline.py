"""Print one cascade chunk's kernel timeline from a rocprofv3 kernel trace and
the per-round gap accounting (development helper)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
big = [i for i, r in enumerate(rows) if r["Kernel_Name"].replace("void ", "").startswith("fe_kernel<1")
       and int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 1e6]
i0, i1 = big[-2], big[-1]
t0 = int(rows[i0]["Start_Timestamp"])
short = lambda n: n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:40]
busy_end = t0
idle = 0
for r in rows[i0:i1]:
    s = int(r["Start_Timestamp"]); e = int(r["End_Timestamp"])
    if s > busy_end: idle += s - busy_end
    busy_end = max(busy_end, e)
    if len(sys.argv) > 2:
        print(f"{(s-t0)/1e3:9.1f} {(e-t0)/1e3:9.1f} {(e-s)/1e3:7.1f} q{r['Queue_Id']:>2s} {short(r['Kernel_Name'])}")
print(f"chunk {(int(rows[i1]['Start_Timestamp'])-t0)/1e3:.1f} us, GPU idle (no kernel running) {idle/1e3:.1f} us")
