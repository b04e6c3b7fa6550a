"""scipy frozen priors -> device prior families (csrc/special.h nmc_prior_logpdf).

The reference evaluates ``prior.logpdf(value)`` on scipy frozen distributions
(posteriorSampling.py:293-294) for none/complete pooling.  The device implements
the families below with scipy's formulas; gammaln(shape) and log(scale) are
computed here with scipy/numpy so those terms are bit-identical.
"""

import numpy
import scipy.special

from . import _lib

_SHAPED = {"gamma", "lognorm", "invgamma"}


def encode(dist):
    """Return (family id, params[8]) for a scipy frozen distribution."""
    name = getattr(getattr(dist, "dist", None), "name", None)
    if name not in _lib.PRIOR:
        raise ValueError("prior %r is not supported on the GPU (supported: %s)"
                         % (name, ", ".join(sorted(_lib.PRIOR))))
    shapes, loc, scale = dist.dist._parse_args(*dist.args, **dist.kwds)
    shape = float(shapes[0]) if name in _SHAPED else 0.0
    if name in _SHAPED and len(shapes) != 1:
        raise ValueError("unexpected shape parameters for %s" % name)
    loc = float(loc)
    scale = float(scale)
    with numpy.errstate(all="ignore"):
        lga = float(scipy.special.gammaln(shape)) if name in ("gamma", "invgamma") else 0.0
        ls = float(numpy.log(scale))
    return _lib.PRIOR[name], [loc, scale, shape, lga, ls, 0.0, 0.0, 0.0]


def encode_all(priors):
    fam = numpy.zeros(len(priors), dtype=numpy.int32)
    prm = numpy.zeros((len(priors), 8), dtype=numpy.float64)
    for i, d in enumerate(priors):
        fam[i], prm[i] = encode(d)
    return fam, prm
