"""The example scripts run end to end on the GPU: the reference demo's MEX call
sequence (test_opticalflow2d.m:42-59) for every regularisation, checked for a
smaller residual after warping than before (a registration that moved the
moving image towards the reference)."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = os.path.join(ROOT, "examples", "demo_registration.py")


@pytest.mark.gpu
@pytest.mark.parametrize("reg", [0, 1, 2, 3, 4, 5])
def test_demo_registration(gpu, reg):
    out = subprocess.run([sys.executable, DEMO, "--reg", str(reg), "--size", "64"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    m = re.search(r"mean \|Iref - Imov\| ([0-9.]+) -> mean \|Iref - Ireg\| ([0-9.]+)", out.stdout)
    assert m, out.stdout[-2000:]
    before, after = float(m.group(1)), float(m.group(2))
    assert after < before, (before, after)
