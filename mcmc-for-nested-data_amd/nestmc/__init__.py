"""nestmc: MI355X-native engine for the MCMC inner loop of MCMC-for-Nested-Data.

Public entry points mirror the reference (posteriorSampling.samplePosterior,
sampleDiagnosis.diagnoseSamples; see the drop-in modules next to this package).
"""

from .data import example_distribution, example_regression, linreg, logistic  # noqa: F401
from .families import GaussianMean, LinearRegression, Logistic, is_family  # noqa: F401

__version__ = "0.1.0"
