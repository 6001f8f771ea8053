"""Per-run kernel accounting of a rocprofv3 kernel trace (runs: kernel
sequences separated by > 5 ms of no launch): span, GPU-busy union, summed
kernel time, average concurrency, queues, and the eight largest kernel
families (count, total, average, grid in workgroups).
    python tools/trace_runs.py <kernel_trace.csv> [min_kernels]"""
import collections
import csv
import sys

FAM = ("jacobi3_mid", "jacobi3_kernel", "jacobi2", "jacobi_kernel", "seqnorm_tables",
       "seqnorm_walk", "seqnorm_entries", "seqnorm_check", "seqnorm_decide", "seqnorm_offset",
       "seqnorm_total", "copy_lines", "copyBuffer", "fillBuffer", "reduce_partials", "sum_ranks",
       "warp", "gradients", "accumulate", "d2f", "compose", "precheck")
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    n = next((k for k in FAM if k in n), n.split("(")[0][-25:])
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) // max(
        1, int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]))
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, int(r["Queue_Id"]), g))
rows.sort()
minimum = int(sys.argv[2]) if len(sys.argv) > 2 else 200
runs, cur = [], [rows[0]]
for r in rows[1:]:
    if r[0] - max(x[1] for x in cur[-50:]) > 5_000_000:
        runs.append(cur)
        cur = [r]
    else:
        cur.append(r)
runs.append(cur)
for ru in runs:
    if len(ru) < minimum:
        continue
    t0, t1 = ru[0][0], max(r[1] for r in ru)
    tot, s, e = 0, None, None
    for a, b in sorted((a, b) for a, b, *_ in ru):
        if s is None or a > e:
            if s is not None:
                tot += e - s
            s, e = a, b
        else:
            e = max(e, b)
    tot += e - s
    busy = sum(b - a for a, b, *_ in ru)
    c = collections.defaultdict(lambda: [0, 0, 0])
    for a, b, n, q, g in ru:
        c[n][0] += 1
        c[n][1] += b - a
        c[n][2] = g
    print(f"run: span {(t1 - t0) / 1e6:.2f} ms, {len(ru)} kernels, GPU busy {tot / 1e6:.2f} ms, "
          f"kernel time {busy / 1e6:.2f} ms, concurrency {busy / tot:.2f}, "
          f"{len(set(r[3] for r in ru))} queues")
    for n, (k, d, g) in sorted(c.items(), key=lambda x: -x[1][1])[:8]:
        print(f"   {k:6d} x {n:18s} {d / 1e6:8.2f} ms  avg {d / k / 1e3:7.1f} us  grid {g}")
