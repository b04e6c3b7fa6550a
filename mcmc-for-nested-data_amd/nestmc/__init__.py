"""nestmc: MI355X-native engine for the MCMC inner loop of MCMC-for-Nested-Data.

The public entry point mirrors the reference's posteriorSampling.samplePosterior
(drop-in module next to this package).  The sample files it writes are
byte-identical to the reference's, so the reference's
sampleDiagnosis.diagnoseSamples reads them unchanged.
"""

from .data import example_distribution, example_regression, linreg, logistic  # noqa: F401
from .families import GaussianMean, LinearRegression, Logistic, is_family  # noqa: F401

__version__ = "0.1.0"
