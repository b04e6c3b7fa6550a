"""numpy.logaddexp(0, eta) as the likelihood kernels evaluate it (csrc/softplus.h).

The logistic family (cfg 5: y eta - logaddexp(0, eta), the model of the reference's
plug-in logLikelihoodFunction, posteriorSampling.py:61-102) replaced the library's
exp + log1p (181 VALU instructions on gfx950) by a range-reduced exp and log1p (~50).
Host and device run the same IEEE operations, so:
  * CPU: the host form (nmc_debug_softplus, on_device = 0) is within 2.5 ulp of a 50-digit
    mpmath reference over the whole range (measured: max 2.23, mean 0.35 ulp; numpy's own
    logaddexp: max 1.37, mean 0.28) and reproduces numpy's special values;
  * GPU: the device kernel returns the host's bits exactly.
"""

import numpy
import pytest


def _inputs():
    r = numpy.random.RandomState(11)
    parts = [r.normal(0, 1, 4000), r.normal(0, 8, 4000), r.uniform(-40, 40, 4000),
             r.uniform(-760, 760, 2000), numpy.linspace(-2, 2, 4001),
             numpy.array([0.0, -0.0, 1e-300, -1e-300, 5e-324, 0.34657359, -0.34657359,
                          0.8813735870195429, -0.8813735870195429, 36.7, -36.7, 709.7,
                          -709.7, 745.2, -745.2, 746.0, -746.0, 1e308, -1e308])]
    return numpy.ascontiguousarray(numpy.concatenate(parts))


def _softplus(lib, x, on_device):
    from nestmc._lib import check, dptr
    out = numpy.empty_like(x)
    check(lib.nmc_debug_softplus(dptr(x), len(x), dptr(out), on_device))
    return out


def test_softplus_host_accuracy_and_special_values():
    import mpmath
    from nestmc import _lib
    lib = _lib.load()
    x = _inputs()
    got = _softplus(lib, x, 0)
    mpmath.mp.dps = 50
    worst = 0.0
    for xi, gi in zip(x, got):
        want = mpmath.log1p(mpmath.exp(mpmath.mpf(float(xi))))
        w = float(want)
        ulp = numpy.spacing(abs(w)) if w != 0 else 5e-324
        err = abs(float(mpmath.mpf(float(gi)) - want)) / ulp
        worst = max(worst, err)
        assert err <= 2.5, (xi, gi, w, err)
    assert worst <= 2.5
    # numpy's own values: within 2 ulp, and the special cases exactly
    ref = numpy.logaddexp(0.0, x)
    assert numpy.allclose(got, ref, rtol=1e-15, atol=1e-307)   # (subnormal results: absolute)
    sp = numpy.array([0.0, numpy.inf, -numpy.inf, numpy.nan, 1000.0, -1000.0])
    gs = _softplus(lib, sp, 0)
    assert gs[0] == numpy.log(2.0) and gs[1] == numpy.inf and gs[2] == 0.0
    assert numpy.isnan(gs[3]) and gs[4] == 1000.0 and gs[5] == 0.0


@pytest.mark.gpu
def test_softplus_device_bits_equal_host(gpu_lib):
    x = numpy.concatenate([_inputs(), [numpy.inf, -numpy.inf, numpy.nan]])
    host = _softplus(gpu_lib, x, 0)
    dev = _softplus(gpu_lib, x, 1)
    assert numpy.array_equal(host.view(numpy.uint64)[:-1], dev.view(numpy.uint64)[:-1])
    assert numpy.isnan(dev[-1])
