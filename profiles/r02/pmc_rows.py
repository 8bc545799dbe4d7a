"""Average the PMC counters of one kernel (name prefix) over its dispatches in a
rocprofv3 --pmc csv.  usage: pmc_rows.py counter_collection.csv 'fe_kernel<1'"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
want = sys.argv[2]
acc = collections.defaultdict(float)
disp = set()
for r in rows:
    if not r["Kernel_Name"].replace("void ", "").startswith(want):
        continue
    disp.add(r["Dispatch_Id"])
    acc[r["Counter_Name"]] += float(r["Counter_Value"])
n = max(len(disp), 1)
print(f"{want}: {len(disp)} dispatches")
for k, v in sorted(acc.items()):
    print(f"  {k:24s} {v / n:16.1f}")
