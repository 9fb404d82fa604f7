"""Summarise a rocprofv3 kernel trace (GPU box): the kernels of one captured training step
(between two k_gru_fwd launches late in the run) with durations, and launch counts by name."""
import csv
import sys
from collections import Counter

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
cnt = Counter(r["Kernel_Name"][:90] for r in rows)
print("launches", len(rows))
for n, c in cnt.most_common(12):
    print(f"{c:8d}  {n}")
idx = [i for i, r in enumerate(rows) if "k_gru_fwd" in r["Kernel_Name"]]


def show(title, a, b):
    tot = 0.0
    print(f"\n{title}:")
    for r in rows[a:b]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        tot += d
        print(f"{r['Kernel_Name'][:80]:80s} {d:8.2f}")
    print("sum", round(tot, 1), "span", (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1000,
          "n", b - a)


# the headline step runs first (its timed replays are the longest run of GRU launches), the
# e2e leg (residual build + step) last
k = len(idx) // 3
show("headline step (replay %d of %d)" % (k, len(idx)), idx[k], idx[k + 1])
show("one step", idx[-4], idx[-3])
