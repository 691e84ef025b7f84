"""GPU: the device's exp is the oracle's exp (csrc/nk_exp.h compiled for gfx950 and for x86-64), bit for bit.

nk_vexp runs the same source the Bratu stencils inline; tests/test_exp.py pins that source against
mpmath on CPU, so equality here makes the device exp correctly rounded too.  Through it the Bratu
residual, exact JVP and FD operator are bit-identical to the oracle (tests/test_hip.py and the config /
slab / distributed tests compare them with array_equal).
"""
import numpy as np
import pytest

import _nkpath  # noqa: F401
import ariadne_hip as ah
from oracle import oracle as oc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = ah.Context(0)
    ah.set_default_context(c)
    yield c
    c.sync()


def dev_exp(x):
    g = ah.Grid.full(len(x))
    xd = ah.DeviceArray.from_numpy(np.ascontiguousarray(x), g)
    yd = xd.zero()
    ah.exp_(yd, xd)
    return yd.to_numpy()


def same(a, b):
    return (a == b) | (np.isnan(a) & np.isnan(b))


def test_device_exp_golden(ctx, golden_dir):
    d = np.load(f"{golden_dir}/exp_cr.npz")
    assert np.all(same(dev_exp(d["x"]), d["y"]))
    assert dev_exp(np.array([2.0]))[0] == 7.38905609893065  # test/runtests.jl:38


def test_device_exp_matches_oracle_million(ctx):
    rng = np.random.default_rng(12)
    x = np.concatenate([rng.uniform(-1.0, 3.0, 1_000_000), rng.uniform(-745.2, 709.8, 200_000),
                        rng.choice([-1.0, 1.0], 50_000) * 2.0 ** rng.uniform(-60, -3, 50_000)])
    assert np.all(same(dev_exp(x), oc.exp(x)))


def test_device_exp_torch_views(ctx):
    """exp_ on torch views of device arrays (what a user residual passes), odd offsets included."""
    import torch

    x = np.linspace(-3.0, 3.0, 1001)
    xd = ah.DeviceArray.from_numpy(x, ah.Grid.full(len(x)))
    yd = xd.zero()
    t, o = xd.torch(), yd.torch()
    with ctx.torch_stream():
        ah.exp_(o[1:], t[1:])
    ctx.sync()
    y = yd.to_numpy()
    assert y[0] == 0.0
    np.testing.assert_array_equal(y[1:], oc.exp(x[1:]))
    del torch
