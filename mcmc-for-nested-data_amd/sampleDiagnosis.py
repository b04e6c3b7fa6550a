"""Drop-in module: ``from sampleDiagnosis import diagnoseSamples``.

Same name, signature, defaults, output files and stdout as the reference module
(sampleDiagnosis.py:11-85 in tkngch/MCMC-for-Nested-Data); the variogram behind the
effective sample size runs on MI355X through libnestmc (nestmc.diagnosis).
"""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from nestmc.diagnosis import Diagnostic, Summary, diagnose_samples  # noqa: E402,F401
from nestmc.diagnosis import hpd_interval as computeHpdInterval  # noqa: E402,F401


def diagnoseSamples(outputDirectory, assessConvergence=True, printSummary=True, nFigures=10):
    """Diagnose the samples under outputDirectory/sample/ (reference :11-44): convergence
    assessment CSVs under outputDirectory/diagnostic/, sample/summary.csv, and up to
    nFigures trace / pairwise plots under outputDirectory/figure/."""
    return diagnose_samples(outputDirectory, assessConvergence=assessConvergence,
                            printSummary=printSummary, nFigures=nFigures)
