"""The N > 1 row-slab decomposition, exercised on the CPU with the gloo backend.

Each rank takes its slab from the library's own partition function
(of2d_slab_bounds) and runs the protocol opticalflow2d_amd/csrc/slab.cpp runs
over RCCL: chunks of 32 iterations run as fused launches of K = 3 (then a
pair / single tail); before each launch K ghost j-lines above and below are
exchanged (the first K / last K owned lines); step k of a launch is computed
on the owned rows plus K-k halo rows on each side (their gradients come from
image halo rows); the global-j border rule; the Logger's norms as the
reference takes them (Motion.cpp:42-49): one float running sum in linear
order, which crosses the slabs in rank order, so each rank continues the sums
it receives from the rank above and passes them on, and the last rank's sums
decide the break on every rank (slab.cpp run_exact: the walks chained by
ncclRecv / ncclSend, the sums broadcast from the last rank).  The step itself
is a numpy float32 restatement (elementwise IEEE ops in the reference's order).
The gathered motion must equal the single-grid oracle bit for bit, and the
iteration count with convergence on must match the oracle's.
"""
import math
import os
import socket
import tempfile

import numpy as np
import pytest

from opticalflow2d_amd import synthetic as S

F = np.float32


def hs_step(u, dI, It, alphasq, row0, dimy):
    """One OpticalFlowDiffusion::get_update on rows u[1:-1].  u: (rows+2, dimx, 2)
    with the neighbouring j-lines at 0 and -1; dI: (rows, dimx, 2); It: (rows,
    dimx); row0: global j of u[1].  Returns the new rows and the Logger sums
    over all of them."""
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
    # owned rows plus two halo rows each side (zero outside the image)
    dIf = dI.reshape(dimy, dimx, 2)
    Itf = It.reshape(dimy, dimx)
    rows = e - b
    H = 3  # ghost j-lines of u
    dIh = np.zeros((rows + 4, dimx, 2), np.float32)
    Ith = np.zeros((rows + 4, dimx), np.float32)
    lo, hi = max(b - 2, 0), min(e + 2, dimy)
    dIh[lo - (b - 2):hi - (b - 2)] = dIf[lo:hi]
    Ith[lo - (b - 2):hi - (b - 2)] = Itf[lo:hi]
    u = np.zeros((rows + 2 * H, dimx, 2), np.float32)  # owned rows at u[H:H+rows]
    alpha = F(0.2)
    alphasq = alpha * alpha

    def exchange(lines):
        reqs = []
        if rank > 0:
            reqs.append(dist.isend(torch.from_numpy(u[H:H + lines].copy()), rank - 1))
            up = torch.empty((lines, dimx, 2), dtype=torch.float32)
            reqs.append(dist.irecv(up, rank - 1))
        if rank < world - 1:
            reqs.append(dist.isend(torch.from_numpy(u[H + rows - lines:H + rows].copy()),
                                   rank + 1))
            dn = torch.empty((lines, dimx, 2), dtype=torch.float32)
            reqs.append(dist.irecv(dn, rank + 1))
        for r in reqs:
            r.wait()
        if rank > 0:
            u[H - lines:H] = up.numpy()
        if rank < world - 1:
            u[H + rows:H + rows + lines] = dn.numpy()

    def sums(new, old):
        """Logger::update_error's two norms: the float running sums continued
        from the rank above over this slab's rows (x fastest), passed on."""
        S = torch.zeros(2, dtype=torch.float32)
        if rank > 0:
            dist.recv(S, rank - 1)
        out = []
        for k, f in enumerate((new - old, old)):  # Field::operator-, then prev
            acc = F(S[k].item())
            for x, y in f.reshape(-1, 2).tolist():
                acc = F(float(acc) + math.sqrt(x * x + y * y))  # (float)((double)S + d)
            out.append(acc)
        S = torch.tensor(out, dtype=torch.float32)
        if rank < world - 1:
            dist.send(S, rank + 1)
        dist.broadcast(S, world - 1)
        return logger_error(S[0].item(), S[1].item(), dimx * dimy)

    def fused(K):
        """K iterations of one fused launch: states of the owned rows after each."""
        exchange(K)
        w = u[H - K:H + rows + K]  # owned rows + K neighbour lines each side
        states = []
        for k in range(1, K + 1):
            h = K - k  # halo rows computed by step k
            w, _, _ = hs_step(w, dIh[2 - h:2 + rows + h], Ith[2 - h:2 + rows + h], alphasq,
                              b - h, dimy)
            states.append(w[h:h + rows].copy())
        return states

    done = niter
    k0 = 0
    stop = False
    while k0 < niter and not stop:
        C = min(32, niter - k0)
        t = 0
        while t < C and not stop:
            K = 3 if C - t >= 3 else C - t
            prev = u[H:H + rows].copy()
            states = fused(K)
            olds = [prev] + states[:-1]
            for i in range(K):
                err = sums(states[i], olds[i])
                if not fixed and err < F(0.001) and k0 + t + i > 1:
                    u[H:H + rows] = states[i]
                    done = k0 + t + i + 1
                    stop = True
                    break
            if not stop:
                u[H:H + rows] = states[-1]
            t += K
        k0 += C
    np.save(os.path.join(outdir, f"slab{rank}.npy"), u[H:H + rows])
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
                                                         (3, 32, 29, 11, True),
                                                         (4, 24, 12, 37, True),
                                                         (3, 20, 10, 400, False)])
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
