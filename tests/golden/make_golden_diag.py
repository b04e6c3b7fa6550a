#!/usr/bin/env python
"""Capture the reference's diagnoseSamples outputs (sampleDiagnosis.py:11-85) for the
golden sample directories (tests/golden/csv/<case>/sample.<c>.csv, themselves written
by the reference's samplePosterior, and the synthetic AR(1) directories this script
writes to tests/golden/diag_inputs/) -> tests/golden/diag/<case>/:

  diagnosticAssessment.csv, diagnosticAssessmentHyperOnly.csv,
  diagnosticAssessmentIndividual.csv (as the case's pooling produces them),
  summary.csv, stdout.txt (what diagnoseSamples printed)
  or error.txt: the exception the reference raised (odd row counts cannot be halved,
  sampleDiagnosis.py:153-155)

Run in the build container (the reference is importable here, never on the GPU box):
    MPLBACKEND=Agg python tests/golden/make_golden_diag.py
"""

import contextlib
import io
import os
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _write_synthetic(root):
    """Synthetic sample directories in the reference's sample.<c>.csv format (header
    index,chain,<columns>; values %f): AR(1) chains with even row counts, one mixing and
    one sticky (autocorrelation near 1: the effective-n search runs to T = n - 1)."""
    import numpy
    cases = {"ar_partial": dict(chains=4, rows=300, names=("a", "b"), groups=4, partial=True,
                                phi=0.6, seed=1),
             "ar_none_sticky": dict(chains=3, rows=240, names=("a", "b"), groups=3,
                                    partial=False, phi=0.995, seed=2)}
    for case, c in cases.items():
        r = numpy.random.RandomState(c["seed"])
        cols = []
        for p in c["names"]:
            if c["partial"]:
                cols += [p + "_mu", p + "_sigma2"]
            cols += ["%s[%03d]" % (p, g) for g in range(c["groups"])]
        d = os.path.join(root, case)
        os.makedirs(d, exist_ok=True)
        for ch in range(c["chains"]):
            x = numpy.zeros((c["rows"], len(cols)))
            level = r.normal(size=len(cols)) * 0.3
            v = r.normal(size=len(cols))
            for i in range(c["rows"]):
                v = c["phi"] * v + r.normal(size=len(cols)) * numpy.sqrt(1 - c["phi"] ** 2)
                x[i] = level + v
            for j, name in enumerate(cols):
                if name.endswith("_sigma2"):
                    x[:, j] = numpy.abs(x[:, j]) + 0.1
            with open(os.path.join(d, "sample.%d.csv" % ch), "w") as f:
                f.write("index,chain," + ",".join(cols) + "\n")
                for i in range(c["rows"]):
                    f.write("%d,%d," % (1000 + i, ch) + ",".join("%f" % v for v in x[i]) + "\n")


def main():
    sys.path.insert(0, REF)
    import sampleDiagnosis as sd   # the reference module (read-only import)
    out_root = os.path.join(HERE, "diag")
    _write_synthetic(os.path.join(HERE, "diag_inputs"))
    sources = [(case, os.path.join(HERE, "csv", case))
               for case in sorted(os.listdir(os.path.join(HERE, "csv")))]
    sources += [(case, os.path.join(HERE, "diag_inputs", case))
                for case in sorted(os.listdir(os.path.join(HERE, "diag_inputs")))]
    for case, src in sources:
        tmp = tempfile.mkdtemp(prefix="nmc_diag_")
        try:
            shutil.copytree(src, os.path.join(tmp, "sample"))
            buf = io.StringIO()
            dst = os.path.join(out_root, case)
            os.makedirs(dst, exist_ok=True)
            try:
                with contextlib.redirect_stdout(buf):
                    sd.diagnoseSamples(tmp, assessConvergence=True, printSummary=True,
                                       nFigures=0)
            except Exception as e:   # the reference's own failure (odd row counts, :153-155)
                with open(os.path.join(dst, "error.txt"), "w") as f:
                    f.write("%s: %s\n" % (type(e).__name__, e))
                print(case, "error", type(e).__name__, e)
                continue
            for name in sorted(os.listdir(os.path.join(tmp, "diagnostic"))):
                shutil.copy(os.path.join(tmp, "diagnostic", name), os.path.join(dst, name))
            shutil.copy(os.path.join(tmp, "sample", "summary.csv"), os.path.join(dst, "summary.csv"))
            with open(os.path.join(dst, "stdout.txt"), "w") as f:
                f.write(buf.getvalue())
            print(case, sorted(os.listdir(dst)))
        finally:
            shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
