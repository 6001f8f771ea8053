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
    assert c["halo_timing"] is None  # given by make_record's caller (GPU runs)


def test_halo_summary():
    """config.halo_timing for N > 1: rank 0, a middle rank, every rank."""
    per = [{"rank": r, "stall_us": 1.0 + r, "exchange_us": 10.0, "edges_us": 5.0, "sampled": 8}
           for r in range(8)]
    h = bench.halo_summary(per)
    assert h["sampled_launches_per_run"] == 8 and h["per_rank"] == per
    assert h["rank0"]["rank"] == 0 and h["rank_mid"]["rank"] == 4
    assert h["rank_mid"]["stall_us"] == 5.0
    # unsplit runs (N = 1 without --self-halo) sample nothing
    assert bench.halo_summary([{"rank": 0, "stall_us": 0.0, "exchange_us": 0.0,
                                "edges_us": 0.0, "sampled": 0}]) is None
    r = _record(2, 16384, 16384, 8192)
    rec = bench.make_record(**{**dict(world=2, wl=bench.workload(bench.parse_args([]), 2),
                                      steps=20, warmup=5, elapsed=0.6, gpu_ms=580.0,
                                      avg_us=87.0, iso_us=85.0, px_rank=16384 * 8192,
                                      info={"halo_lines": 3, "split": 1}, traffic=None,
                                      cpu=None, rows_per_rank=8192, iters_per_step=1000)},
                            halo=bench.halo_summary(per[:2]))
    assert rec["config"]["halo_timing"]["rank_mid"]["rank"] == 1
    assert r["config"]["interior_edge_split"] is True
    json.loads(json.dumps(rec))


def test_self_halo_flag():
    assert bench.parse_args(["--rccl", "--self-halo"]).self_halo


def test_default_semantics_flag():
    assert bench.parse_args(["--no-default-semantics"]).no_default_semantics
    assert not bench.parse_args([]).no_default_semantics


def test_traffic_only_for_its_grid_and_kernel():
    t = bench.load_traffic(4096, 4096, "field")
    assert t is not None and t["grid"] == [4096, 4096]
    assert bench.load_traffic(4096, 4096, "image") is None
    assert bench.load_traffic(16384, 8192, "field") is None
