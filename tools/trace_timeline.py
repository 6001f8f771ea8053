"""Timeline of a few steady-state batches of a convergence-on loop from a
rocprofv3 kernel trace: every kernel's start / end (us) relative to the first
shown jacobi3_mid launch, its queue, and how long it waited after the previous
kernel of its queue ended (a launch that starts late behind a full GPU shows
up as a long wait with its queue otherwise idle).
    python tools/trace_timeline.py <kernel_trace.csv> [first_batch] [nbatches]"""
import csv
import sys


def short(name):
    for k in ("jacobi3_mid", "jacobi3_fused", "seqnorm_headers", "seqnorm_merge",
              "seqnorm_tables", "seqnorm_walk", "seqnorm_entries",
              "seqnorm_check_sums", "seqnorm_check_scan", "seqnorm_check", "seqnorm_decide",
              "seqnorm_offset", "reduce_partials", "fillBuffer", "copyBuffer",
              "jacobi3_kernel", "jacobi_kernel"):
        if k in name:
            return k
    return name.split("(")[0][-30:]


rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                 int(r["Queue_Id"])))
rows.sort()
first = int(sys.argv[2]) if len(sys.argv) > 2 else 40
nb = int(sys.argv[3]) if len(sys.argv) > 3 else 3
mids = [r for r in rows if r[2] in ("jacobi3_mid", "jacobi3_fused")]
t0 = mids[first][0]
t1 = mids[first + nb][0]
last_end = {}
for a, b, n, q in rows:
    if b < t0 - 500_000:
        last_end[q] = b
        continue
    if a > t1:
        break
    w = (a - last_end[q]) / 1e3 if q in last_end else float("nan")
    last_end[q] = b
    if b < t0:
        continue
    print(f"q{q:<3} {n:20s} {(a - t0) / 1e3:9.1f} {(b - t0) / 1e3:9.1f}  dur {(b - a) / 1e3:7.1f}"
          f"  after-prev {w:7.1f}")
