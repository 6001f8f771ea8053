#!/usr/bin/env python3
"""Horn-Schunck Jacobi throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size S]

One step = one Horn-Schunck iteration of the reference loop
(ImageRegistrationOpticalFlow.cpp:123-135): OpticalFlowDiffusion::get_update +
the Logger norms over the whole grid, the per-chunk norm reduction /
convergence read-back, and — for N > 1 — the RCCL halo exchange.  Iterations
run in threes fused into one pass over HBM (hs::jacobi3_kernel: 28 B/px per
launch, three iterations per launch, bit-identical to three single steps;
chunks of 33 iterations are eleven launches, and a single step or a pair fills
the run's tail), with a three-j-line halo exchange per launch overlapped with
the interior bands.  Early exit is disabled
(fixed_iters) so that exactly K iterations run.

Workload: N = 1 is BASELINE config 2 (Horn-Schunck 4096^2 fp32).  For N > 1
every rank owns a 4096-row slab of a 4096 x (4096 N) grid (weak scaling, the
row-slab decomposition of config 5 with a real halo exchange per iteration).
Inputs are a synthetic procedural texture pair generated per slab.  For N > 1
launch with torch.distributed.run (one process per GPU); torch.distributed
(gloo) bootstraps the RCCL communicator, barriers and takes the max time.
Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpixel-iterations/sec + achieved HBM GB/s, Horn-Schunck 4096^2 @ 1/2/4/8 GPU"
BYTES_PER_PX_IT = 28  # read u 8 + dI 8 + It 4, write u 8
# the fused kernel moves those 28 B/px once per launch and advances THREE iterations
BYTES_PER_PX_LAUNCH = 28
ITERS_PER_LAUNCH = 3
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s peak (spec)
ALPHA = 0.1


def cpu_baseline(size: int, iters: int):
    """The oracle (C restatement, 1 thread, reference loop order i-outer/j-inner)
    timed on `iters` Horn-Schunck iterations of the same size-x-size workload."""
    from oracle import oracle as O
    from opticalflow2d_amd import synthetic as S
    L = O.lib()
    ref, mov = S.procedural_pair(size, 0, size)
    I = np.ascontiguousarray(mov.reshape(-1, order="F").astype(np.float32))
    Ir = np.ascontiguousarray(ref.reshape(-1, order="F").astype(np.float32))
    n = size * size
    dI = np.zeros(2 * n, np.float32)
    It = np.zeros(n, np.float32)
    L.oracle_spatial_derivative(I, size, size, dI)
    L.oracle_temporal_derivative(Ir, I, n, It)
    u = np.zeros(2 * n, np.float32)
    errs = np.zeros(iters, np.float32)
    L.oracle_set_reference_loop_order(1)
    t0 = time.perf_counter()
    L.oracle_hs_loop(u, dI, It, size, size, ALPHA, iters, 1, errs)
    dt = time.perf_counter() - t0
    L.oracle_set_reference_loop_order(0)
    return {"value": n * iters / dt / 1e6, "unit": "Mpx-it/s", "cores": 1, "kind": "port",
            "sample": f"oracle HS loop (Jacobi + Logger), {size}x{size}, {iters} iterations, "
                      f"reference loop order, {dt:.1f} s"}


def load_traffic():
    p = os.path.join(ROOT, "profiles", "hs_traffic.json")
    if os.path.exists(p):
        try:
            return json.load(open(p))
        except Exception:
            return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # the default warm-up runs past the clock transient of the first ~40 ms of
    # sustained load (profiles/r01_v14_bench_warmup.log: W=50 times the dip)
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--warmup", type=int, default=1500)
    ap.add_argument("--size", type=int, default=4096, help="dimx and rows per GPU")
    ap.add_argument("--cpu-iters", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--timing-launches", type=int, default=200)
    ap.add_argument("--rccl", action="store_true",
                    help="N = 1: run the Logger all-reduces through a one-rank RCCL communicator")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print("bench.py: --gpus > 1 must be launched with torch.distributed.run",
                  file=sys.stderr)
            sys.exit(2)

    # libof2d (and the /opt/rocm HIP runtime and RCCL it links) loads before
    # torch at every N: torch ships its own libamdhip64 / librccl under the same
    # sonames, and whichever loads first serves both
    from opticalflow2d_amd import SlabSolver, lib
    from opticalflow2d_amd import synthetic as S
    from opticalflow2d_amd.slab import halo_rows, rccl_unique_id
    lib()

    dist = None
    if world > 1 or "WORLD_SIZE" in os.environ:  # launched by torch.distributed.run
        import torch.distributed as dist  # noqa: F811
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    uid = None
    if world == 1 and args.rccl:
        uid = rccl_unique_id()  # one-rank communicator: the RCCL all-reduces run too
    elif world > 1:
        obj = [rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]

    dimx, dimy = args.size, args.size * world
    solver = SlabSolver(dimx, dimy, ALPHA, rank, world, device=local, unique_id=uid)
    lo, hi = halo_rows(dimy, rank, world)
    ref, mov = S.procedural_pair(dimx, lo, hi)
    solver.set_images(ref, mov)

    def barrier():
        if dist is not None:
            dist.barrier()
        try:  # drains every stream of the device (the solver's own stream included)
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize(local)
        except Exception:
            pass

    if args.warmup > 0:
        solver.run(args.warmup, fixed_iters=True)
    barrier()
    t0 = time.perf_counter()
    done = solver.run(args.steps, fixed_iters=True)  # returns after the stream is drained
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    gpu_ms = solver.last_run_ms()
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert done == args.steps

    # dominant kernel: average duration per launch over the timed region, from
    # the HIP events the solver records around the run on its own stream (the
    # run is triple launches except a pair / single step per run tail; the
    # per-chunk partial reductions between them are included)
    avg_us = gpu_ms * 1000.0 * ITERS_PER_LAUNCH / args.steps
    # and back-to-back launches of the kernel alone, after the run
    iso_us = solver.time_kernel(args.timing_launches)
    px_rank = dimx * (solver.row_end - solver.row_begin)
    achieved = BYTES_PER_PX_LAUNCH * px_rank / (avg_us * 1e-6) / 1e9
    traffic = load_traffic()

    result = None
    if rank == 0:
        total_px = dimx * dimy
        value = total_px * args.steps / elapsed / 1e6
        result = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "Mpx-it/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * elapsed / args.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (procedural texture pair, shift (1.5,-0.75))",
            "config": {
                "workload": "Horn-Schunck Jacobi (config 2: 4096^2 fp32 per GPU; N>1: "
                            "row slabs of a 4096 x 4096N grid with RCCL halo)",
                "grid": [dimx, dimy],
                "alpha": ALPHA,
                "iterations": args.steps,
                "fixed_iters": True,
                "parallelism": f"row-slab x{world}",
                "gpu_ms_rank0": round(gpu_ms, 3),
                # the path's own algorithmic traffic (28 B/px per fused launch) per GPU
                "hbm_GBps_from_step_time": round(BYTES_PER_PX_LAUNCH * total_px * args.steps
                                                 / ITERS_PER_LAUNCH / elapsed / 1e9 / world, 1),
                # the reference algorithm's 28 B per pixel-iteration at this rate
                "ref_bytes_GBps_equiv": round(BYTES_PER_PX_IT * total_px * args.steps
                                              / elapsed / 1e9 / world, 1),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "of2d::hs::jacobi3_kernel<0,4,true,4,4,true,1,0,1,true>",
                "iterations_per_launch": ITERS_PER_LAUNCH,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "avg_launch_us": round(avg_us, 3),
                "avg_launch_source": "HIP events around the timed run on the solver's stream "
                                     "(gpu ms x 3 / steps)",
                "isolated_launch_us": round(iso_us, 3),
                "bytes_per_launch": BYTES_PER_PX_LAUNCH * px_rank,
                "traffic": (traffic or {}).get("bytes_per_launch"),
                # the unfused reference algorithm's 28 B per pixel-iteration at the
                # kernel's per-iteration rate, as a fraction of the HBM peak
                "ref_equiv_frac": round(BYTES_PER_PX_IT * px_rank * ITERS_PER_LAUNCH
                                        / (avg_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic_source": (traffic or {}).get("source"),
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(args.size, args.cpu_iters)
        print(json.dumps(result), flush=True)
    solver.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
