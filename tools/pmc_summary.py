"""Per-kernel averages of rocprofv3 --pmc counter_collection.csv files."""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for path in sys.argv[1:]:
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"].replace("(anonymous namespace)::", "")[:70]
        acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for name, cnt in acc.items():
    print(name)
    for c, v in sorted(cnt.items()):
        print(f"    {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
