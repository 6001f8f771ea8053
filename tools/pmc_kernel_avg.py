"""Average of each PMC counter per kernel over its dispatches (rocprofv3
counter_collection.csv files): python tools/pmc_kernel_avg.py <csv>..."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        k = k.split("(")[0].split("::")[-1]
        c = r["Counter_Name"]
        acc[k][c] += float(r["Counter_Value"])
        disp[k][c].add(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(disp[k][c]))
for k in sorted(acc):
    vals = {c: acc[k][c] / max(len(disp[k][c]), 1) for c in acc[k]}
    print(k, " ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))
