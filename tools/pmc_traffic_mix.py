#!/usr/bin/env python3
"""HBM traffic of the HS triple kernel per launch from rocprofv3 PMC counters,
calibrated per access mix (MI355X_MICROARCH.md: FETCH_SIZE reports half the
bytes of 16-B streaming reads on gfx950; other widths are uncalibrated).

The probes of tools/hs_gi_ab (PMC mode -2) stream a KNOWN byte count with
each kernel mix over the same grid: probe_field_kernel (16-B u, 16-B dI, 8-B
It in; 16-B out: 20 + 8 B/px) and probe_image_kernel (16-B u, 8-B Iaux, 8-B
It in; 16-B out: 16 + 8 B/px).  The triple kernel of the mix it uses is
corrected with that probe's factors.
usage: pmc_traffic_mix.py --grid DIMX DIMY --pitch P --mix image|field
         --probe FETCH_CSV WRITE_CSV --kernel FETCH_CSV WRITE_CSV [--out F]
"""
import argparse
import csv
import json
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") == counter:
                acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, nargs=2, required=True)
    ap.add_argument("--pitch", type=int, required=True)
    ap.add_argument("--mix", choices=["image", "field"], required=True)
    ap.add_argument("--probe", nargs=2, required=True)
    ap.add_argument("--kernel", nargs=2, required=True)
    ap.add_argument("--out")
    a = ap.parse_args()
    dimx, dimy = a.grid
    pf, pw = per_kernel(a.probe[0], "FETCH_SIZE"), per_kernel(a.probe[1], "WRITE_SIZE")
    kf, kw = per_kernel(a.kernel[0], "FETCH_SIZE"), per_kernel(a.kernel[1], "WRITE_SIZE")
    pname = "probe_image_kernel" if a.mix == "image" else "probe_field_kernel"
    probe = [k for k in pf if pname in k][0]
    px = a.pitch * dimy  # the probes sweep the pitched rows
    rd_true, wr_true = (16.0 if a.mix == "image" else 20.0) * px, 8.0 * px
    fcal = rd_true / (pf[probe] * 1024.0)
    wcal = wr_true / (pw[probe] * 1024.0)
    jac = [k for k in kf if "jacobi3_kernel" in k][0]
    rd = kf[jac] * 1024.0 * fcal
    wr = kw[jac] * 1024.0 * wcal
    bpp = 24.0 if a.mix == "image" else 28.0
    alg = bpp * dimx * dimy
    out = {
        "kernel": jac,
        "grid": [dimx, dimy],
        "gradients": a.mix,
        "fetch_raw_bytes": kf[jac] * 1024.0,
        "write_raw_bytes": kw[jac] * 1024.0,
        "fetch_calibration": fcal,
        "write_calibration": wcal,
        "read_bytes_per_launch": rd,
        "write_bytes_per_launch": wr,
        "bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": alg,
        "iterations_per_launch": 3,
        "traffic_over_algorithmic": (rd + wr) / alg,
        "source": ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, kernel trace only) "
                   "over bench.py's own launches, calibrated on the streaming probe of the same "
                   f"access mix ({pname}, tools/hs_gi_ab PMC mode) at the same grid"),
    }
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
