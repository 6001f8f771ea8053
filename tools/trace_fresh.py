"""Batch by batch, the last convergence-on loop of a rocprofv3 kernel trace
(a fresh registration's: OF2D_CONV_FRESH=1 tools/time_convergence.py): for
each jacobi3_mid launch, the time to the next one and how long each Logger
kernel family of the batches in flight ran (union of intervals) inside it.
    python tools/trace_fresh.py <kernel_trace.csv>"""
import csv
import sys

FAMS = ("jacobi3_mid", "seqnorm_tables", "seqnorm_check", "seqnorm_entries", "seqnorm_walk",
        "seqnorm_decide")


def fam(name):
    for k in FAMS:
        if k in name:
            return k
    return "other"


rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam(r["Kernel_Name"]))
              for r in csv.DictReader(open(sys.argv[1])))
mids = [r for r in rows if r[2] == "jacobi3_mid"]
runs, cur = [], [mids[0]]
for a, b in zip(mids, mids[1:]):
    if b[0] - a[0] < 2_000_000:
        cur.append(b)
    else:
        runs.append(cur)
        cur = [b]
runs.append(cur)
run = runs[-1]
t_first, t_last = run[0][0], run[-1][1]
tail = max(b for a, b, f in rows if a >= t_first)
print(f"{len(runs)} loops; last: {len(run)} batches, first mid -> last kernel "
      f"{(tail - t_first) / 1e3:.1f} us")


def busy(lo, hi, f):
    iv = sorted((max(a, lo), min(b, hi)) for a, b, g in rows if g == f and b > lo and a < hi)
    tot, end = 0, lo
    for a, b in iv:
        if b <= end:
            continue
        tot += b - max(a, end)
        end = b
    return tot / 1e3


print("batch   start     dt  " + " ".join(f"{f.split('_')[-1]:>8s}" for f in FAMS))
bounds = [r[0] for r in run] + [tail]
for i in range(len(run)):
    lo, hi = bounds[i], bounds[i + 1]
    print(f"{i:5d} {(lo - t_first) / 1e3:7.1f} {(hi - lo) / 1e3:6.1f}  "
          + " ".join(f"{busy(lo, hi, f):8.1f}" for f in FAMS))
