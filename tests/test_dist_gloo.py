"""The N > 1 row-slab decomposition, exercised on the CPU with the gloo backend.

Each rank takes its slab from the library's own partition function
(of2d_slab_bounds), keeps one ghost j-line above and below, exchanges its
first/last owned j-line with its neighbours before every Jacobi step, applies
the global-j border rule, and all-reduces the two Logger sums — the same
protocol opticalflow2d_amd/csrc/slab.cpp runs over RCCL.  The step itself is a
numpy float32 restatement (elementwise IEEE ops in the reference's order).
The gathered motion must equal the single-grid oracle bit for bit, and the
iteration count with convergence on must match the oracle's.
"""
import os
import socket
import tempfile

import numpy as np
import pytest

from opticalflow2d_amd import synthetic as S

F = np.float32


def hs_step(u, dI, It, alphasq, row0, dimy):
    """One OpticalFlowDiffusion::get_update on a slab.  u: (rows+2, dimx, 2) with
    ghost j-lines at 0 and -1; dI: (rows, dimx, 2); It: (rows, dimx)."""
    c = u[1:-1]
    rows, dimx = c.shape[0], c.shape[1]
    left = np.zeros_like(c)
    right = np.zeros_like(c)
    left[:, 1:] = c[:, :-1]
    right[:, :-1] = c[:, 1:]
    q = (((left + right) + u[:-2]) + u[2:]) / F(4.0)
    jg = row0 + np.arange(rows)[:, None]
    x = np.arange(dimx)[None, :]
    border = (x == 0) | (x == dimx - 1) | (jg == 0) | (jg == dimy - 1)
    q[border] = 0
    gx, gy = dI[..., 0], dI[..., 1]
    s = (It + q[..., 0] * gx) + q[..., 1] * gy
    den = (F(alphasq) + gx * gx) + gy * gy
    new = np.stack([q[..., 0] - (gx * s) / den, q[..., 1] - (gy * s) / den], axis=-1)
    d = (new - c).astype(np.float64)
    p = c.astype(np.float64)
    sd = float(np.sqrt(d[..., 0] ** 2 + d[..., 1] ** 2).sum())
    sp = float(np.sqrt(p[..., 0] ** 2 + p[..., 1] ** 2).sum())
    return new, sd, sp


def logger_error(sd, sp, npx):
    n = F(npx)
    prev = F(sp) / n
    return F(0.0) if prev == 0 else F(sd) / n / prev


def _worker(rank, world, port, dimx, dimy, niter, fixed, outdir):
    import torch
    import torch.distributed as dist
    from oracle import oracle as O
    from opticalflow2d_amd import slab_bounds

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    b, e = slab_bounds(dimy, rank, world)
    ref, mov = S.texture_pair(dimx, seed=21, ny=dimy)
    # derivatives of the full image restricted to the slab (IterativeSolver::set_derivatives)
    I = np.ascontiguousarray(mov.reshape(-1, order="F").astype(np.float32))
    Ir = np.ascontiguousarray(ref.reshape(-1, order="F").astype(np.float32))
    dI = np.zeros(2 * dimx * dimy, np.float32)
    It = np.zeros(dimx * dimy, np.float32)
    O.lib().oracle_spatial_derivative(I, dimx, dimy, dI)
    O.lib().oracle_temporal_derivative(Ir, I, dimx * dimy, It)
    dI = dI.reshape(dimy, dimx, 2)[b:e]
    It = It.reshape(dimy, dimx)[b:e]
    rows = e - b
    u = np.zeros((rows + 2, dimx, 2), np.float32)
    alpha = F(0.2)
    alphasq = alpha * alpha
    done = niter
    for k in range(niter):
        # halo: first owned line up, last owned line down (slab.cpp halo_exchange)
        reqs = []
        if rank > 0:
            reqs.append(dist.isend(torch.from_numpy(u[1].copy()), rank - 1))
            up = torch.empty((dimx, 2), dtype=torch.float32)
            reqs.append(dist.irecv(up, rank - 1))
        if rank < world - 1:
            reqs.append(dist.isend(torch.from_numpy(u[rows].copy()), rank + 1))
            dn = torch.empty((dimx, 2), dtype=torch.float32)
            reqs.append(dist.irecv(dn, rank + 1))
        for r in reqs:
            r.wait()
        if rank > 0:
            u[0] = up.numpy()
        if rank < world - 1:
            u[rows + 1] = dn.numpy()
        new, sd, sp = hs_step(u, dI, It, alphasq, b, dimy)
        u[1:-1] = new
        t = torch.tensor([sd, sp], dtype=torch.float64)
        dist.all_reduce(t)
        err = logger_error(float(t[0]), float(t[1]), dimx * dimy)
        if not fixed and err < F(0.001) and k > 1:
            done = k + 1
            break
    np.save(os.path.join(outdir, f"slab{rank}.npy"), u[1:-1])
    np.save(os.path.join(outdir, f"iters{rank}.npy"), np.array([done]))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,dimx,dimy,niter,fixed", [(2, 48, 40, 12, True),
                                                         (2, 40, 33, 600, False),
                                                         (3, 32, 29, 10, True)])
def test_row_slab_halo_protocol_matches_single_grid(oracle, world, dimx, dimy, niter, fixed):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), dimx, dimy, niter, fixed, d), nprocs=world,
                 join=True)
        slabs = [np.load(os.path.join(d, f"slab{r}.npy")) for r in range(world)]
        iters = {int(np.load(os.path.join(d, f"iters{r}.npy"))[0]) for r in range(world)}
    assert len(iters) == 1, "ranks disagreed on the break iteration"
    u = np.concatenate(slabs, axis=0)  # (dimy, dimx, 2)
    # single grid: the oracle's HS loop (ImageRegistrationOpticalFlow.cpp:123-135) on
    # the same derivatives
    L = oracle.lib()
    ref, mov = S.texture_pair(dimx, seed=21, ny=dimy)
    I = np.ascontiguousarray(mov.reshape(-1, order="F").astype(np.float32))
    Ir = np.ascontiguousarray(ref.reshape(-1, order="F").astype(np.float32))
    dI = np.zeros(2 * dimx * dimy, np.float32)
    It = np.zeros(dimx * dimy, np.float32)
    L.oracle_spatial_derivative(I, dimx, dimy, dI)
    L.oracle_temporal_derivative(Ir, I, dimx * dimy, It)
    want = np.zeros(2 * dimx * dimy, np.float32)
    errs = np.zeros(niter, np.float32)
    n = L.oracle_hs_loop(want, dI, It, dimx, dimy, 0.2, niter, int(fixed), errs)
    assert n == iters.pop()
    assert np.array_equal(u.reshape(-1), want)
