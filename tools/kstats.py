"""Summarise a rocprofv3 kernel_stats.csv: calls, average and share per kernel.
    python tools/kstats.py <kernel_stats.csv>..."""
import csv
import re
import sys

for f in sys.argv[1:]:
    print("==", f)
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        n = re.sub(r"\(.*$", "", n.replace("(anonymous namespace)::", ""))
        n = re.sub(r"HIP_vector_type<[^>]*>", "", n)
        print(f'{n[-60:]:60s} {r["Calls"]:>6} {float(r["AverageNs"])/1e3:9.1f} us {float(r["Percentage"]):6.2f} %')
