#!/usr/bin/env python3
"""HBM traffic of the HS Jacobi kernel from rocprofv3 PMC counters.

Two separate --pmc passes over `tools/hs_variants 4096 N product` (FETCH_SIZE,
then WRITE_SIZE; they do not fit one pass on gfx950).  The probe kernel in the
same binary moves a KNOWN byte count with the same access mix (16-B u and dI
loads, 8-B It loads, 16-B stores), so it calibrates the counters for this
pattern (MI355X_MICROARCH.md: FETCH_SIZE under-reports wide streaming reads
by 2x on gfx950; other widths are uncalibrated).  Writes
profiles/hs_traffic.json with the corrected bytes per launch.
usage: pmc_traffic.py [--out F] <fetch_counter_collection.csv> <write_counter_collection.csv> [n]
                      [--bench <fetch_csv> <write_csv>]
With --bench the kernel measured is the product triple kernel as bench.py
launches it (two more --pmc passes over `bench.py`), corrected with the
probe's calibration from the harness passes.
"""
import csv
import json
import os
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    args = sys.argv[1:]
    out_path = None
    bench = None
    if args and args[0] == "--out":
        out_path, args = args[1], args[2:]
    if "--bench" in args:
        i = args.index("--bench")
        bench = (args[i + 1], args[i + 2])
        args = args[:i] + args[i + 3:]
    fetch_csv, write_csv = args[0], args[1]
    n = int(args[2]) if len(args) > 2 else 4096
    P = (n + 255) // 256 * 256
    fetch = per_kernel(fetch_csv, "FETCH_SIZE")  # KB
    write = per_kernel(write_csv, "WRITE_SIZE")  # KB
    probe = [k for k in fetch if "probe_kernel" in k][0]
    jac = ([k for k in fetch if "jacobi3_kernel" in k] or [k for k in fetch if "jacobi2_kernel" in k]
           or [k for k in fetch if "jacobi_kernel" in k])[0]
    per_launch = 3 if "jacobi3_kernel" in jac else (2 if "jacobi2_kernel" in jac else 1)
    px = P * n  # the probe sweeps the pitched rows
    probe_read_true = 20.0 * px
    probe_write_true = 8.0 * px
    fcal = probe_read_true / (fetch[probe] * 1024.0)
    wcal = probe_write_true / (write[probe] * 1024.0)
    source = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on tools/hs_variants, "
              "calibrated on the probe kernel's known bytes")
    if bench:
        bf = per_kernel(bench[0], "FETCH_SIZE")
        bw = per_kernel(bench[1], "WRITE_SIZE")
        jac = [k for k in bf if "jacobi3_kernel" in k][0]
        fetch[jac], write[jac] = bf[jac], bw[jac]
        per_launch = 3
        source = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over bench.py's own "
                  "launches of the product kernel, calibrated on the probe kernel's known bytes "
                  "(tools/hs_variants passes in the same session)")
    rd = fetch[jac] * 1024.0 * fcal
    wr = write[jac] * 1024.0 * wcal
    alg = 28.0 * n * n
    out = {
        "kernel": jac,
        "grid": [n, n],
        "fetch_raw_bytes": fetch[jac] * 1024.0,
        "write_raw_bytes": write[jac] * 1024.0,
        "fetch_calibration": fcal,
        "write_calibration": wcal,
        "read_bytes_per_launch": rd,
        "write_bytes_per_launch": wr,
        "bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": alg,
        "iterations_per_launch": per_launch,
        "traffic_over_algorithmic": (rd + wr) / alg,
        "source": source,
    }
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if out_path is None:  # on the GPU box write under gpurun_out/ (merged back), copy by hand
        out_path = os.path.join(root, "profiles", "hs_traffic.json")
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
