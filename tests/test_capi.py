"""The C-ABI library on the CPU: it loads, exports every entry point that
include/of2d.h declares, and its host-only logic (gateway state machine,
parameter validation, banner, slab partition) behaves like the reference.
No kernel is launched here (no GPU in the build container)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def header_functions():
    src = open(os.path.join(ROOT, "include", "of2d.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(of2d_[a-z0-9_]+)\s*\(", src))
    names.discard("of2d_print_fn")
    return sorted(names)


def test_library_exports_every_declared_symbol(of2d_lib):
    from opticalflow2d_amd import _lib
    names = header_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(of2d_lib, n), f"libof2d.so does not export {n}"
    assert set(names) == set(_lib.SIGNATURES), "ctypes table out of sync with include/of2d.h"


def test_library_is_gfx950_code_object():
    path = os.path.join(ROOT, "opticalflow2d_amd", "libof2d.so")
    blob = open(path, "rb").read()
    assert b"gfx950" in blob
    assert b"jacobi_kernel" in blob


def test_solver_options_values():
    from opticalflow2d_amd import MotionAccumulation, Regularisation, Verbose
    # src/SolverOptions.h:4-8
    assert [r.value for r in Regularisation] == [0, 1, 2, 3, 4, 5]
    assert [r.name for r in Regularisation] == ["Diffusion", "Curvature", "Elastic",
                                                "ThirionsDemons", "DiffeomorphicDemons", "Fluid"]
    assert (Verbose.Off, Verbose.On) == (0, 1)
    assert (MotionAccumulation.Composition, MotionAccumulation.Addition) == (0, 1)


def test_gateway_invalid_mode_message(of2d_lib):
    from opticalflow2d_amd import Of2dError, OpticalFlow2d
    # no singleton: register / get / warp / close are all invalid
    for args, nargout in [((np.zeros(4), np.zeros(4)), 0), ((), 1), ((np.zeros(4),), 1),
                          ((), 0), ((1, 2, 3), 0)]:
        with pytest.raises(Of2dError, match="invalid number of input and output variables"):
            OpticalFlow2d(*args, nargout=nargout)


def test_banner_and_parameter_validation(of2d_lib, oracle):
    """The init call prints the reference's banner (ImageRegistration.cpp:6-47)
    before validating nparams (:80 then set_solver) and fails with the
    reference's invalid_argument text; the singleton stays empty."""
    from opticalflow2d_amd import InvalidArgument, OpticalFlow2d, set_print_sink
    got = []
    set_print_sink(got.append)
    try:
        with pytest.raises(InvalidArgument, match="Invalid number of regularisation parameters"):
            OpticalFlow2d([16, 12], [3, 2], 1, 5, [0.25], 1, 1, 0)
        with pytest.raises(InvalidArgument, match="invalid regularisation given"):
            OpticalFlow2d([16, 12], [3], 0, 9, [0.25], 1, 1, 0)
    finally:
        set_print_sink(None)
    text = "".join(got)
    L = oracle.lib()
    L.oracle_clear_output()
    with pytest.raises(oracle.OracleError):
        oracle.Registration((16, 12), [3, 2], 1, 5, [0.25], 1, 0)
    assert text == L.oracle_captured_output().decode()
    assert text.count("%" * 71 + "\n") == 2 and "%" * 72 not in text
    assert "regularisation:\t\t\t\tFluid\n" in text
    assert "reg. param:\t\t\t\t0.25\n" in text


def test_banner_multi_params(of2d_lib, oracle):
    from opticalflow2d_amd import ImageRegistration, set_print_sink
    got = []
    set_print_sink(got.append)
    try:
        r = ImageRegistration((20, 24), [7, 5, 3], 2, 3, [1.0, 0.25, 2.0, 2.0, 5, 0], 2, 1)
        r.close()
    finally:
        set_print_sink(None)
    L = oracle.lib()
    L.oracle_clear_output()
    o = oracle.Registration((20, 24), [7, 5, 3], 2, 3, [1.0, 0.25, 2.0, 2.0, 5, 0], 2, 1)
    o.close()
    assert "".join(got) == L.oracle_captured_output().decode()


@pytest.mark.parametrize("dimy,nranks", [(4096, 1), (4096, 2), (4096, 8), (16384, 8), (1001, 7),
                                         (10, 10), (13, 4)])
def test_slab_bounds_partition(of2d_lib, dimy, nranks):
    from opticalflow2d_amd import slab_bounds
    spans = [slab_bounds(dimy, r, nranks) for r in range(nranks)]
    assert spans[0][0] == 0 and spans[-1][1] == dimy
    for (b0, e0), (b1, e1) in zip(spans, spans[1:]):
        assert e0 == b1
    sizes = [e - b for b, e in spans]
    assert max(sizes) - min(sizes) <= 1 and min(sizes) >= 1


def test_slab_bounds_rejects_bad_args(of2d_lib):
    b, e = C.c_int(), C.c_int()
    assert of2d_lib.of2d_slab_bounds(100, 4, 4, C.byref(b), C.byref(e)) != 0
    assert of2d_lib.of2d_slab_bounds(0, 0, 1, C.byref(b), C.byref(e)) != 0


def test_version(of2d_lib):
    assert b"gfx950" in of2d_lib.of2d_version()


@pytest.mark.parametrize("dims,ok", [((65536, 65520), True), ((65536, 65530), False),
                                     ((70000, 70000), False), ((100000, 1), True)])
def test_field_size_guard(of2d_lib, dims, ok):
    """Fields are indexed with unsigned 32-bit offsets in the gather kernels
    (the reference's indices are unsigned int, src/Field.tpp:13): a grid whose
    pitched field (+ 3 ghost j-lines each side) reaches 2^32 elements is
    refused at create, before any device work."""
    from opticalflow2d_amd import ImageRegistration, InvalidArgument, set_print_sink
    set_print_sink(lambda s: None)
    try:
        if ok:
            ImageRegistration(dims, [1], 0, 0, [0.1]).close()
        else:
            with pytest.raises(InvalidArgument, match="2\\^32"):
                ImageRegistration(dims, [1], 0, 0, [0.1])
    finally:
        set_print_sink(None)


def test_registration_options_host_validation(of2d_lib):
    """of2d_set_option's host-side checks (include/of2d.h): every documented
    key is accepted before first use, unknown keys and out-of-range ngpus are
    refused with invalid_argument, and nothing here touches a device."""
    from opticalflow2d_amd import ImageRegistration, InvalidArgument, set_print_sink
    set_print_sink(lambda s: None)
    try:
        r = ImageRegistration((32, 24), [3], 0, 0, [0.1])
        try:
            for k, v in [("fixed_iters", 1), ("fixed_iters", 0), ("logger_fp64", 1),
                         ("logger_fp64", 0), ("hs_gradients_from_image", -1),
                         ("hs_gradients_from_image", 1), ("slab_split", -1), ("slab_split", 0),
                         ("slab_split", 1), ("ngpus", 1), ("ngpus", 16), ("ngpus", 1),
                         ("ngpus_share", 1), ("ngpus_share", 0), ("chunk", 9), ("device", 0)]:
                r.set_option(k, v)
            for k, v in [("ngpus", 0), ("ngpus", 17), ("no_such_option", 1)]:
                with pytest.raises(InvalidArgument):
                    r.set_option(k, v)
        finally:
            r.close()
    finally:
        set_print_sink(None)
