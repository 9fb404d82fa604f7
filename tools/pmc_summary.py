"""Summarise tools/pmc.sh output: mean counter value per kernel (per dispatch)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r["Kernel_Name"][28:60], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, d, c), v in per.items():
        acc[k][c].append(v)
for k, cs in sorted(acc.items()):
    print(k)
    for c, vs in sorted(cs.items()):
        print(f"   {c:34s} {sum(vs) / len(vs):16.1f}")
