"""bench.py's JSON line (the driver's contract) without a GPU: the workload
each N selects, and the record's fields and arithmetic for N = 1 (config 2)
and N > 1 (config 5, strong-scaled 16384^2 row slabs)."""
import json

import pytest

import bench

CONTRACT = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
            "roofline", "cpu_baseline", "default_semantics"}


def test_default_workloads():
    a = bench.parse_args([])
    assert a.iters_per_step == 1000  # BASELINE config 2: 1000 Jacobi iterations
    w1 = bench.workload(a, 1)
    assert (w1["dimx"], w1["dimy"], w1["scaling"]) == (4096, 4096, "strong")
    assert w1["workload"].startswith("config 2")
    for n in (2, 4, 8):
        w = bench.workload(a, n)
        assert (w["dimx"], w["dimy"], w["scaling"]) == (16384, 16384, "strong")
        assert w["workload"].startswith("config 5")
    g = bench.workload(bench.parse_args(["--grid", "16384"]), 1)
    assert (g["dimx"], g["dimy"]) == (16384, 16384) and g["workload"].startswith("config 5")
    w = bench.workload(bench.parse_args(["--weak", "--grid", "4096"]), 4)
    assert (w["dimx"], w["dimy"], w["scaling"]) == (4096, 16384, "weak")


def _record(world, dimx, dimy, rows):
    wl = bench.workload(bench.parse_args(["--grid", str(dimx)]), world)
    info = {"nranks": world, "rccl_ranks": world if world > 1 else 0, "halo_lines": 3 if world > 1 else 0,
            "split": 1 if world > 1 else 0}
    # config 2's slab keeps dI + It in the MALL (field), config 5's do not (image)
    return bench.make_record(world=world, wl=wl, steps=20, warmup=5, elapsed=0.6,
                             gpu_ms=580.0, avg_us=87.0, iso_us=85.0, px_rank=dimx * rows,
                             info=info, traffic=None, cpu=None, rows_per_rank=rows,
                             iters_per_step=1000, gradients="field" if world == 1 else "image")


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_record_schema(world):
    dimx = 4096 if world == 1 else 16384
    rows = dimx // world
    r = _record(world, dimx, dimx, rows)
    assert CONTRACT <= set(r)
    json.loads(json.dumps(r))  # serialisable
    assert r["n_gpus"] == world and r["steps"] == 20 and r["warmup"] == 5
    assert r["higher_is_better"] is True and r["vs_baseline"] is None
    assert r["unit"] == "Mpx-it/s" and r["dtype"] == "fp32"
    # a step is one 1000-iteration HS loop (config 2's niter);
    # value = whole-job pixel-iterations / max-over-ranks time
    assert r["value"] == pytest.approx(dimx * dimx * 20000 / 0.6 / 1e6, rel=1e-6)
    assert r["ms_per_step"] == pytest.approx(30.0, rel=1e-6)
    c = r["config"]
    assert c["iterations_per_step"] == 1000 and c["iterations"] == 20000
    assert c["grid"] == [dimx, dimx] and c["rows_per_rank"] == rows
    assert c["rccl_ranks"] == (world if world > 1 else 0)
    assert c["halo_bytes_per_exchange"] == (2 * 3 * dimx * 8 if world > 1 else 0)
    rf = r["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(rf)
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    # per GPU: the kernel's bytes per px of the rank's slab per launch (28:
    # u 8 + dI 8 + It 4 in, u 8 out; 24 with dI derived from Iaux 4) over the
    # launch time
    b = 28 if world == 1 else 24
    assert rf["bytes_per_px_launch"] == b
    assert rf["achieved"] == pytest.approx(b * dimx * rows / 87e-6 / 1e9, rel=1e-3)
    assert rf["frac"] == pytest.approx(rf["achieved"] / 8000.0, rel=1e-3)
    assert rf["traffic"] is None and rf["traffic_source"] is None
    assert rf["kernel"].startswith("of2d::hs::jacobi3_kernel")
    assert r["default_semantics"] is None  # measured on a GPU only, outside `value`


def test_default_semantics_flag():
    assert bench.parse_args(["--no-default-semantics"]).no_default_semantics
    assert not bench.parse_args([]).no_default_semantics


def test_traffic_only_for_its_grid_and_kernel():
    t = bench.load_traffic(4096, 4096, "field")
    assert t is not None and t["grid"] == [4096, 4096]
    assert bench.load_traffic(4096, 4096, "image") is None
    assert bench.load_traffic(16384, 8192, "field") is None
