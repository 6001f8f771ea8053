"""GPU idle time inside a rocprofv3 kernel trace: the union of the kernels'
[start, end) intervals against the span from the first kernel's start to the
last one's end, and the idle gaps longer than a threshold (where the GPU
waited for the host).  Optionally only the kernels between the first and last
launch whose name contains a pattern (e.g. the Fluid loop's sweep).
    python tools/gpu_idle.py <kernel_trace.csv> [name_pattern] [gap_us]"""
import csv
import sys


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    thr = float(sys.argv[3]) if len(sys.argv) > 3 else 5.0
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(path)))
    if pat:
        idx = [i for i, r in enumerate(rows) if pat in r[2]]
        if not idx:
            sys.exit(f"no kernel matches {pat!r}")
        rows = rows[idx[0]:idx[-1] + 1]
    busy, gaps = 0, []
    cur_s, cur_e = rows[0][0], rows[0][1]
    for s, e, _ in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e) / 1e3)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = rows[-1][1] - rows[0][0]
    big = [g for g in gaps if g > thr]
    print(f"{len(rows)} kernels over {span / 1e6:.3f} ms: busy {busy / 1e6:.3f} ms, "
          f"idle {(span - busy) / 1e6:.3f} ms ({100.0 * (span - busy) / span:.2f} %); "
          f"{len(big)} gaps > {thr} us totalling {sum(big) / 1e3:.3f} ms"
          + (f", median {sorted(big)[len(big) // 2]:.1f} us" if big else ""))


if __name__ == "__main__":
    main()
