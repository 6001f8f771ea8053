"""Where a convergence-on loop's time goes, from a rocprofv3 kernel trace
(tools/gpu.sh convprof): per batch of the exact Logger pipeline (one
jacobi3_mid launch), the interval between consecutive mid launches and how
much of it each kernel family was running (union of its launches' intervals),
plus the GPU-idle time.  Uses the longest run of consecutive mid launches.
    python tools/trace_batches.py <kernel_trace.csv>"""
import csv
import re
import sys
from collections import defaultdict


def fam(name):
    for k in ("jacobi3_mid", "jacobi3_fused", "seqnorm_headers", "seqnorm_merge", "seqnorm_tables",
              "seqnorm_walk", "seqnorm_fix", "seqnorm_entries", "seqnorm_check",
              "jacobi3_kernel", "jacobi_kernel"):
        if k in name:
            return k
    return "other"


rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam(r["Kernel_Name"]),
                 r["Queue_Id"]))
rows.sort()
mids = [r for r in rows if r[2] in ("jacobi3_mid", "jacobi3_fused")]
# the longest run of mid launches less than 2 ms apart
best, cur = [], [mids[0]]
for a, b in zip(mids, mids[1:]):
    if b[0] - a[0] < 2_000_000:
        cur.append(b)
    else:
        best = max(best, cur, key=len)
        cur = [b]
best = max(best, cur, key=len)
t0, t1 = best[0][0], best[-1][0]
nb = len(best) - 1
print(f"{nb} batches, {((t1 - t0) / nb) / 1e3:.1f} us per batch ({(t1 - t0) / nb / 3e3:.1f} us per iteration)")


def union(iv):
    iv = sorted(iv)
    tot, s, e = 0, None, None
    for a, b in iv:
        a, b = max(a, t0), min(b, t1)
        if b <= a:
            continue
        if s is None or a > e:
            if s is not None:
                tot += e - s
            s, e = a, b
        else:
            e = max(e, b)
    if s is not None:
        tot += e - s
    return tot


by = defaultdict(list)
for a, b, f, q in rows:
    by[f].append((a, b))
span = t1 - t0
for f, iv in sorted(by.items(), key=lambda kv: -union(kv[1])):
    u = union(iv)
    if u:
        n = sum(1 for a, b in iv if b > t0 and a < t1)
        print(f"  {f:16s} busy {u / nb / 1e3:7.1f} us per batch ({100 * u / span:5.1f} %), {n / nb:.2f} launches per batch")
allb = union([(a, b) for a, b, f, q in rows])
print(f"  {'any kernel':16s} busy {allb / nb / 1e3:7.1f} us per batch; idle {100 * (1 - allb / span):.1f} %")

# a few consecutive batches in the middle of the run: each launch's start and
# end relative to the first mid launch shown (us), by queue
if len(sys.argv) > 2:
    k0 = len(best) // 2
    a0 = best[k0][0]
    a1 = best[min(k0 + int(sys.argv[2]), len(best) - 1)][0]
    print(f"\ntimeline from mid launch {k0} ({a0}), us:")
    for a, b, f, q in rows:
        if b > a0 and a < a1:
            print(f"  q{q:>3} {f:16s} {(a - a0) / 1e3:8.1f} .. {(b - a0) / 1e3:8.1f}  ({(b - a) / 1e3:6.1f})")
