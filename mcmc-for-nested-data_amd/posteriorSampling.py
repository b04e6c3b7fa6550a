"""Drop-in module: ``from posteriorSampling import samplePosterior``.

Same name, signature, defaults and output files as the reference module
(posteriorSampling.py:28-35 in tkngch/MCMC-for-Nested-Data); the MCMC loop runs on
MI355X through libnestmc (see nestmc.sampler).  The likelihood argument must be a
device family from ``nestmc`` (LinearRegression, GaussianMean, Logistic), which is
also callable with the reference's parameter[P][n] -> ll[n] convention.
"""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from nestmc.families import GaussianMean, LinearRegression, Logistic  # noqa: E402,F401
from nestmc.sampler import sample_posterior  # noqa: E402


def samplePosterior(nChains, nIter, nSamples,
                    parameterName, nGroups, nResponsesPerGroup,
                    pooling, logLikelihoodFunction,
                    outputDirectory,
                    saveLogLikelihood=True,
                    priorDistribution=None,
                    startWithMLE=False, startingPointValueRange=None,
                    nProcesses=1, displayProgress=True, loggingLevel="info", **gpu_options):
    """Sample the posterior of a nested model; samples go to outputDirectory/sample/.

    Arguments mirror the reference (posteriorSampling.py:28-145).  Keyword-only
    GPU options: seed, devices, rng, chains, return_samples (nestmc.sampler).
    Returns None like the reference unless return_samples=True.
    """
    return sample_posterior(nChains, nIter, nSamples, parameterName, nGroups,
                            nResponsesPerGroup, pooling, logLikelihoodFunction,
                            outputDirectory, saveLogLikelihood=saveLogLikelihood,
                            priorDistribution=priorDistribution, startWithMLE=startWithMLE,
                            startingPointValueRange=startingPointValueRange,
                            nProcesses=nProcesses, displayProgress=displayProgress,
                            loggingLevel=loggingLevel, **gpu_options)
