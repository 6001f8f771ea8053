"""The RCCL side of the row-slab solver on ONE GPU.

RCCL refuses two ranks on one device, so the send/recv halo itself only runs in
the driver's multi-GPU bench; test_gpu_slab_local.py covers the slab code with
an in-process transport.  What one GPU can check is everything around it, in
the process layout the multi-GPU bench uses:

* ``bench.py`` launched by ``torch.distributed.run`` (gloo process group,
  libof2d loaded before torch, rank-0 unique id, max-over-ranks time, JSON
  line) with a one-rank RCCL communicator (``--rccl``);
* a one-rank communicator (``ncclCommInitRank`` + the Logger ``ncclAllReduce``
  per chunk + the divide-by-zero vote) against the communicator-free slab:
  bit-identical motion and the same iteration count, with convergence on;
* the halo's send / recv calls themselves, rehearsed by a one-rank
  communicator sending its boundary lines to itself between the interior and
  edge launches of split triples (option ``rccl_self_halo``).

Each case runs in a fresh process so the library load order is the bench's.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ONE_RANK = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from opticalflow2d_amd import SlabSolver, lib
from opticalflow2d_amd import synthetic as S
from opticalflow2d_amd.slab import rccl_unique_id
lib()
import torch.distributed  # noqa: F401  (torch after libof2d, as in bench.py)
n = 384
ref, mov = S.procedural_pair(n, 0, n)
out = []
for uid in (None, rccl_unique_id()):
    s = SlabSolver(n, n, 0.1, 0, 1, device=0, unique_id=uid)
    # a one-rank communicator keeps the reference's Logger (logger_fp64 auto)
    assert s.info()["logger_reference"] == 1, s.info()
    s.set_images(ref, mov)
    done = s.run(1000, fixed_iters=False)
    out.append((done, s.motion()))
    s.close()
(d0, m0), (d1, m1) = out
assert 1 < d0 <= 1000, d0
assert d0 == d1, (d0, d1)
assert np.array_equal(m0.view(np.uint64), m1.view(np.uint64))
print("ONE-RANK-OK", d0)
"""


SELF_HALO = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from opticalflow2d_amd import SlabSolver, lib
from opticalflow2d_amd import synthetic as S
from opticalflow2d_amd.slab import rccl_unique_id
lib()
import torch.distributed  # noqa: F401
n = 640
ref, mov = S.procedural_pair(n, 0, n)
for fixed, niter in ((True, 31), (False, 1000)):
    out = []
    for uid in (None, rccl_unique_id()):
        s = SlabSolver(n, n, 0.1, 0, 1, device=0, unique_id=uid)
        if uid is not None:
            s.set_option("rccl_self_halo", 1)
            s.set_option("split", 1)
            assert s.info()["split"] == 1, s.info()
        else:
            assert s.info()["split"] == 0, s.info()
        s.set_images(ref, mov)
        done = s.run(niter, fixed_iters=fixed)
        out.append((done, s.motion()))
        s.close()
    (d0, m0), (d1, m1) = out
    assert d0 == d1 and (fixed or 1 < d0 <= niter), (d0, d1)
    assert np.array_equal(m0.view(np.uint64), m1.view(np.uint64))
    print("SELF-HALO-OK", fixed, d0)
try:
    s = SlabSolver(64, 64, 0.1, 0, 1, device=0)
    s.set_option("rccl_self_halo", 1)
    raise SystemExit("rccl_self_halo accepted without a communicator")
except Exception as e:
    assert "one-rank RCCL communicator" in str(e), e
print("SELF-HALO-REFUSED")
"""


def test_rccl_halo_rehearsal_on_one_rank():
    """The halo's ncclGroupStart / ncclSend / ncclRecv between the interior and
    edge launches of split triples (the N-rank launch order, slab.cpp fused),
    sent by a one-rank communicator to itself: the fixed-iteration and
    convergence-on runs stay bit-identical to the communicator-free slab."""
    r = subprocess.run([sys.executable, "-c", SELF_HALO, ROOT], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.count("SELF-HALO-OK") == 2 and "SELF-HALO-REFUSED" in r.stdout


TWO_RANKS = r"""
import os, sys, time, numpy as np
sys.path.insert(0, sys.argv[1])
from opticalflow2d_amd import SlabSolver, lib
from opticalflow2d_amd import synthetic as S
from opticalflow2d_amd.slab import rccl_unique_id, halo_rows
lib()
rank, d, fixed = int(sys.argv[2]), sys.argv[3], sys.argv[4] == "1"
n, world = 512, 2
if rank == 0:
    open(os.path.join(d, "uid.tmp"), "wb").write(rccl_unique_id())
    os.rename(os.path.join(d, "uid.tmp"), os.path.join(d, "uid"))
while not os.path.exists(os.path.join(d, "uid")):
    time.sleep(0.05)
uid = open(os.path.join(d, "uid"), "rb").read()
lo, hi = halo_rows(n, rank, world)
ref, mov = S.procedural_pair(n, 0, n)  # the one grid's images, sliced
ref, mov = ref[:, lo:hi], mov[:, lo:hi]
s = SlabSolver(n, n, 0.1, rank, world, device=rank, unique_id=uid)
s.set_option("logger_fp64", 0)  # the reference's Logger chained over RCCL
assert s.info()["logger_reference"] == 1 and s.info()["rccl_ranks"] == 2, s.info()
s.set_images(ref, mov)
done = s.run(1000, fixed_iters=fixed)
np.save(os.path.join(d, f"m{rank}.npy"), s.motion())
np.save(os.path.join(d, f"e{rank}.npy"), s.errors())
open(os.path.join(d, f"it{rank}"), "w").write(str(done))
s.close()
"""


def _device_count():
    import ctypes
    from opticalflow2d_amd import lib
    c = ctypes.c_int(0)
    lib().of2d_device_count(ctypes.byref(c))
    return c.value


@pytest.mark.parametrize("fixed", [False, True])
def test_two_rccl_ranks_match_one_grid(tmp_path, fixed):
    """Two RCCL ranks on two devices (one process each): the halo send / recv
    between distinct devices and, with logger_fp64 = 0, the reference's Logger
    chained over RCCL — the break iteration, every error and the motion equal
    the one-rank grid's.  Needs two GPUs: skipped on a one-GPU box (it is here
    for the first multi-GPU box)."""
    if _device_count() < 2:
        pytest.skip("needs two GPUs")
    import numpy as np
    procs = [subprocess.Popen([sys.executable, "-c", TWO_RANKS, ROOT, str(r), str(tmp_path),
                               "1" if fixed else "0"], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, o[-2000:] + e[-4000:]
    from opticalflow2d_amd import SlabSolver
    from opticalflow2d_amd import synthetic as S
    n = 512
    ref, mov = S.procedural_pair(n, 0, n)
    one = SlabSolver(n, n, 0.1, 0, 1, device=0)
    one.set_images(ref, mov)
    done = one.run(1000, fixed_iters=fixed)
    want, werr = one.motion(), one.errors()
    one.close()
    got = np.concatenate([np.load(tmp_path / f"m{r}.npy") for r in range(2)], axis=1)
    for r in range(2):
        assert int(open(tmp_path / f"it{r}").read()) == done
        assert np.array_equal(np.load(tmp_path / f"e{r}.npy").view(np.uint32), werr.view(np.uint32))
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_one_rank_communicator_matches_plain_slab():
    r = subprocess.run([sys.executable, "-c", ONE_RANK, ROOT], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ONE-RANK-OK" in r.stdout


def test_bench_under_torch_distributed_run():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "99", "--warmup", "3",
           "--size", "1024", "--no-cpu-baseline", "--rccl", "--self-halo",
           "--timing-launches", "5"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 1 and res["steps"] == 99 and res["value"] > 0
    assert res["roofline"]["avg_launch_us"] > 0
    # the self-halo's split triples: the halo timing of the N > 1 line
    assert res["config"]["interior_edge_split"] is True
    h = res["config"]["halo_timing"]
    assert h["sampled_launches_per_run"] == 8 and h["rank0"]["rank"] == 0
    assert h["rank0"]["exchange_us"] > 0 and h["rank0"]["edges_us"] > 0
    assert h["rank0"]["stall_us"] >= 0
    # the grid is not config 2's: no convergence-on measurement
    assert res["default_semantics"] is None
