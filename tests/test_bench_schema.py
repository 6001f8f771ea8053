"""bench.py's JSON line (the driver's contract) without a GPU: the workload
each N selects, and the record's fields and arithmetic for N = 1 (config 2)
and N > 1 (config 5, strong-scaled 16384^2 row slabs)."""
import json

import pytest

import bench

CONTRACT = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
            "roofline", "cpu_baseline"}


def test_default_workloads():
    a = bench.parse_args([])
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
    return bench.make_record(world=world, wl=wl, steps=300, warmup=50, elapsed=0.03,
                             gpu_ms=29.0, avg_us=87.0, iso_us=85.0, px_rank=dimx * rows,
                             info=info, traffic=None, cpu=None, rows_per_rank=rows)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_record_schema(world):
    dimx = 4096 if world == 1 else 16384
    rows = dimx // world
    r = _record(world, dimx, dimx, rows)
    assert CONTRACT <= set(r)
    json.loads(json.dumps(r))  # serialisable
    assert r["n_gpus"] == world and r["steps"] == 300 and r["warmup"] == 50
    assert r["higher_is_better"] is True and r["vs_baseline"] is None
    assert r["unit"] == "Mpx-it/s" and r["dtype"] == "fp32"
    # value = whole-job pixel-iterations / max-over-ranks time
    assert r["value"] == pytest.approx(dimx * dimx * 300 / 0.03 / 1e6, rel=1e-6)
    assert r["ms_per_step"] == pytest.approx(0.1, rel=1e-6)
    c = r["config"]
    assert c["grid"] == [dimx, dimx] and c["rows_per_rank"] == rows
    assert c["rccl_ranks"] == (world if world > 1 else 0)
    assert c["halo_bytes_per_exchange"] == (2 * 3 * dimx * 8 if world > 1 else 0)
    rf = r["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(rf)
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    # per GPU: 28 B per px of the rank's slab per launch over the launch time
    assert rf["achieved"] == pytest.approx(28 * dimx * rows / 87e-6 / 1e9, rel=1e-3)
    assert rf["frac"] == pytest.approx(rf["achieved"] / 8000.0, rel=1e-3)
    assert rf["traffic"] is None and rf["traffic_source"] is None


def test_traffic_only_for_its_grid():
    assert bench.load_traffic(4096, 4096) is not None
    assert bench.load_traffic(16384, 8192) is None
