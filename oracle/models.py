"""User log-likelihood callbacks for the oracle -- TEST INFRASTRUCTURE.

Reference convention (posteriorSampling.py:61-102): parameter[P][n] -> ll[n],
written like example/regression.py:53-67.
"""

import functools

import numpy
import scipy.stats


def _ll_regression2(parameter, x, y):
    yHat = numpy.array(parameter[0]) + numpy.array(parameter[1]) * x
    return scipy.stats.norm(loc=y, scale=1.0).logpdf(yHat)


def linreg_callback(x, y):
    """cfg 3 model: y ~ N(b0 + b1 x, 1)."""
    return functools.partial(_ll_regression2, x=x, y=y)
