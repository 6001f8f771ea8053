"""Cost figures of the device Logger norms (seqnorm) on real Horn-Schunck
iterates: u_k at 4096^2 from fixed-iteration registrations (with nrefine 1 the
returned motion is accumulate(0, u_k) = u_k), then of2d_motion_norms over the
Logger's pairs (u_k, u_{k-1}), u_{-1} = 0, on one workspace as in the loop.

    python tools/seqnorm_diag.py [n] [k]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opticalflow2d_amd import ImageRegistration, set_print_sink  # noqa: E402
from opticalflow2d_amd import synthetic as S  # noqa: E402
from opticalflow2d_amd.registration import motion_norms  # noqa: E402

set_print_sink(lambda s: None)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
ref, mov = S.texture_pair(n)
us = [np.zeros((n * n, 2), np.float32)]
for k in range(1, K + 1):
    with ImageRegistration((n, n), [k], 0, 0, [0.1], fixed_iters=1) as r:
        r.register(ref, mov)
        m = r.motion().astype(np.float32)
    us.append(np.stack([m[:, :, 0].reshape(-1, order="F"), m[:, :, 1].reshape(-1, order="F")], 1))
cur = np.stack(us[1:])
prev = np.stack(us[:-1])
t0 = time.perf_counter()
sums, st = motion_norms(cur, prev, (n, n))
print(f"{K} pairs at {n}^2 in {1e3 * (time.perf_counter() - t0):.1f} ms (incl. uploads)")
print("k  sum|du|  sum|u|  resolves(d,p)  raw segments(d,p)  recomputed tiles  "
      "walk us (d,p)  resolves us (d)")
for k in range(K):
    print(k, sums[k, 0], sums[k, 1], st[k, :2].tolist(), st[k, 2:4].tolist(), st[k, 4],
          (st[k, 5:7] / 100).tolist(), st[k, 7] / 100)
