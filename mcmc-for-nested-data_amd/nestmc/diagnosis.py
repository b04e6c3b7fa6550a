"""Convergence diagnostics over the sample files: the reference's diagnoseSamples
(sampleDiagnosis.py:11-85) with its column loops vectorised and the variogram -- its
O(m n^2) per-column cost, :189-208 -- on the GPU (csrc/diag.hip, nmc_variogram).

Same inputs (sample/sample*.csv in glob order), same statistics in the same numpy
evaluation order (between/within-sequence variances :158-187, rhat :216-224, effective
n :232-255, median and 95 % HDI :419-427, the group summaries :430-491), same files and
stdout.  The variogram sums in the reference's order with correctly rounded squares
(the reference's numpy ``** 2`` goes through libm pow): values agree to a few ulp and
the printed ``%.3f`` / ``%.4f`` fields agree.  Like the reference, sample files with an
odd number of rows cannot be halved and raise ValueError.
"""

import glob
import os

import numpy
import pandas

from . import _lib

ASSESS_DTYPE = [("parameter", "S40"), ("rhat", float), ("converged", bool),
                ("effective n", float), ("enough n", bool), ("median", float),
                ("HDI lower", float), ("HDI upper", float)]


def _read(fn):
    # the C parser with correctly rounded conversions: the same doubles as the
    # reference's engine="python" (Python float())
    return pandas.read_csv(fn, float_precision="round_trip")


def hpd_interval(samples, hdi_p=95):
    """computeHpdInterval (:766-776)."""
    s = numpy.sort(numpy.asarray(samples, dtype=numpy.float64))
    n = len(s)
    gap = max(1, min(n - 1, round(n * (hdi_p / 100.))))
    width = s[gap:n] - s[0:n - gap]
    k = int(numpy.argmax(width == width.min()))
    return s[k], s[k + gap]


def variogram(x, device=0):
    """x [K][m][n] -> V [K][n] on the GPU (nmc_variogram)."""
    x = numpy.ascontiguousarray(x, dtype=numpy.float64)
    K, m, n = x.shape
    out = numpy.empty((K, n))
    lib = _lib.load()
    _lib.check(lib.nmc_variogram(int(device), _lib.dptr(x), K, m, n, _lib.dptr(out)))
    return out


class Diagnostic:
    """rhat, effective n, median and HDI of every column (sampleDiagnosis.Diagnostic)."""

    def __init__(self, sampleDirectory, device=0):
        files = glob.glob(sampleDirectory + "/sample*.csv")
        self._device = device
        self.partiallyPooled = False
        self.completelyPooled = True
        keys, blocks = None, []
        for i, fn in enumerate(files):
            d = _read(fn)
            if i == 0:
                rows = d.shape[0]
                half = rows // 2
                keys = [k for k in d.columns if k not in ("chain", "index")]
                self.partiallyPooled = any("_" in k for k in keys)
                self.completelyPooled = not any("01]" in k for k in keys)
            v = d[keys].to_numpy(dtype=numpy.float64).T   # [K, rows of this file]
            # every file is cut at the FIRST file's row count, [0:half] and [half:rows]
            # (:136-155): a longer later file is truncated; a shorter one, or an odd first
            # count, fails where the reference's assignment fails
            first, second = v[:, :half], v[:, half:rows]
            for part in (first, second):
                if part.shape[1] != half:
                    raise ValueError("could not broadcast input array from shape (%d,) into "
                                     "shape (%d,)" % (part.shape[1], half))
            blocks += [first, second]
        self._keys = keys or []
        self._m = len(blocks)
        self._n = blocks[0].shape[1] if blocks else 0
        # [K][m][n]: column k's m half-chains, in the reference's (file, half) order
        self._x = numpy.ascontiguousarray(numpy.stack(blocks, 1)) if blocks else None
        self._assessment = None
        self._summary = None

    def _assess(self):
        if self._assessment is not None:
            return
        x, m, n = self._x, self._m, self._n
        B = n * numpy.var(numpy.mean(x, axis=2), axis=1, ddof=1)
        W = numpy.mean(numpy.var(x, axis=2, ddof=1), axis=1)
        vhat = W * (n - 1) / n + B / n
        rhat = numpy.sqrt(vhat / W)
        rho = 1. - variogram(x, self._device) / (2. * vhat[:, None])
        neff = numpy.empty(len(self._keys))
        for k in range(len(self._keys)):
            r = rho[k]
            # the first even lag whose next two autocorrelations sum below zero (:241-251)
            hit = numpy.nonzero((r[1:n - 1] + r[2:n] < 0) & (numpy.arange(n - 2) % 2 == 0))[0]
            T = int(hit[0]) if hit.size else n - 1
            neff[k] = (m * n) / (1 + 2 * numpy.sum(r[0:T + 1]))
        rows = []
        for k, key in enumerate(self._keys):
            flat = x[k].reshape(-1)
            lo, hi = hpd_interval(flat, 95)
            rows.append((key.encode(), rhat[k], rhat[k] < 1.1, neff[k], neff[k] > m * 10,
                         numpy.median(flat), lo, hi))
        a = numpy.array(rows, dtype=ASSESS_DTYPE)
        self._assessment = numpy.sort(a, order="parameter")

    @property
    def assessment(self):
        self._assess()
        return self._assessment

    def _summarise(self):
        if self._summary is not None:
            return
        self._assess()
        a = self._assessment
        names = sorted(set(p.decode("ascii").split("[")[0] for p in a["parameter"] if b"[" in p))
        out = []
        for name in names:
            sel = numpy.array([b"[" in p and p.decode("ascii").split("[")[0] == name
                               for p in a["parameter"]])
            rh = a["rhat"][sel]
            out.append((name, min(rh), numpy.median(rh), max(rh),
                        numpy.mean(a["converged"][sel])))
        self._summary = numpy.array(out, dtype=[("parameter", "S40"), ("rhat min", float),
                                                ("rhat median", float), ("rhat max", float),
                                                ("proportion converged", float)])

    def print(self, csvfile, individualSummary, hyperOnly):
        """Diagnostic.print (:331-379): same checks, headings and CSV text."""
        if individualSummary and self.completelyPooled:
            raise ValueError("MCMC was completely pooled. There is no individual summary.")
        if hyperOnly and not self.partiallyPooled:
            raise ValueError("MCMC was not partially pooled. There is no hyper-parameter.")
        if individualSummary and hyperOnly:
            raise ValueError("Choose individualSummary or hyperOnly. Not both.")
        if csvfile is None:
            print("MCMC convergence diagnostic for hyper-parameters." if hyperOnly else
                  "Summary of MCMC convergence diagnostic." if individualSummary else
                  "MCMC convergence diagnostic.")
        if not individualSummary:
            self._assess()
            a = self._assessment
            out = ",".join(a.dtype.names) + "\n"
            for r in a:
                if hyperOnly and b"_" not in r[0]:
                    continue
                out += "'%s',%.3f,%s,%.3f,%s,%.3f,%.3f,%.3f\n" % (
                    r[0].decode("ascii"), r[1], r[2], r[3], r[4], r[5], r[6], r[7])
        else:
            self._summarise()
            out = ",".join(self._summary.dtype.names) + "\n"
            for r in self._summary:
                out += "'%s',%.3f,%.3f,%.3f,%.3f\n" % (r[0].decode("ascii"), r[1], r[2], r[3],
                                                       r[4])
        if csvfile is None:
            _stdout_csv(out)
        else:
            with open(csvfile, "w") as h:
                h.write(out)


class Summary:
    """Group means / medians of each parameter per recorded row (sampleDiagnosis.Summary,
    :430-491), vectorised over rows."""

    def __init__(self, sampleDirectory):
        files = glob.glob(sampleDirectory + "/sample*.csv")
        means, medians, names = {}, {}, []
        for i, fn in enumerate(files):
            d = _read(fn)
            if i == 0:
                names = list(numpy.unique([c.split("[")[0] for c in d.columns if "[" in c]))
                for k in names:
                    means[k], medians[k] = [], []
            per = {}
            for k in names:   # columns "containing <name>[" (:466-467), row by row
                v = numpy.ascontiguousarray(   # rows contiguous: numpy's pairwise row sums
                    d[[c for c in d.columns if (k + "[") in c]].to_numpy(dtype=numpy.float64))
                per[k] = (numpy.mean(v, axis=1), numpy.median(v, axis=1))
            for j in range(d.shape[0]):
                for k in names:
                    means[k].append(per[k][0][j])
                    medians[k].append(per[k][1][j])
        text = "stats,parameter,mean,median,HDI lower,HDI upper\n"
        for tag, dd in (("groupMean", means), ("groupMedian", medians)):
            for k in sorted(dd):
                v = numpy.array(dd[k])
                lo, hi = hpd_interval(v, 95.)
                text += "%s,%s,%.4f,%.4f,%.4f,%.4f\n" % (tag, k, numpy.mean(v), numpy.median(v),
                                                         lo, hi)
        self._summary = text

    def print(self, csvfile):
        if csvfile is None:
            print("Summary of individual parameters.")
            _stdout_csv(self._summary)
        else:
            with open(csvfile, "w") as h:
                h.write(self._summary)


def _stdout_csv(content):
    print("\t" + content.replace(",", ", ").replace("\n", "\n\t"))


def figures(outputDirectory, sampleDirectory, nFigures):
    """Trace and pairwise plots per group suffix and the per-chain log-likelihood trace
    (the reference's Figure, :494-759, as plain matplotlib on the Agg backend)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    files = glob.glob(sampleDirectory + "/sample*.csv")
    if not files:
        return
    data = [_read(fn) for fn in files]
    keys = [k for k in data[0].columns if k not in ("chain", "index")]
    suffixes = sorted(set("[" + k.split("[")[1] for k in keys if "[" in k))
    if any("_" in k for k in keys):
        suffixes = ["_"] + suffixes
    tdir = os.path.join(outputDirectory, "figure", "traceplot")
    bdir = os.path.join(outputDirectory, "figure", "bivariate")
    os.makedirs(tdir, exist_ok=True)
    os.makedirs(bdir, exist_ok=True)
    lls = sorted(glob.glob(sampleDirectory + "/logLikelihood*.csv"))
    if lls and sum(os.path.getsize(f) for f in lls):
        fig = plt.figure(figsize=(12, 3))
        for i, f in enumerate(lls):
            plt.plot(pandas.read_csv(f, header=None).sum(axis=1).to_numpy(), label=i)
        plt.xlabel("Iteration")
        plt.ylabel("Log Likelihood")
        plt.legend(title="Chain")
        fig.savefig(os.path.join(outputDirectory, "figure", "logLikelihood.png"))
        plt.close(fig)
    for suffix in suffixes[:nFigures]:
        sel = sorted(k for k in keys if suffix in k)
        fig, ax = plt.subplots(len(sel), 2, figsize=(12, 2 * len(sel)), squeeze=False)
        for i, k in enumerate(sel):
            for d in data:
                ax[i, 0].hist(d[k].to_numpy(), bins=max(1, len(d) // 10), density=True,
                              histtype="stepfilled", alpha=0.5)
                ax[i, 1].plot(d[k].to_numpy())
            ax[i, 0].set_title(k.replace("_", " "))
            ax[i, 1].set_title(k.replace("_", " "))
        fig.tight_layout()
        fig.savefig(os.path.join(tdir, "traceplot%s.png" % suffix))
        plt.close(fig)
        if len(sel) > 1:
            fig, ax = plt.subplots(len(sel), len(sel), figsize=(2 * len(sel), 2 * len(sel)),
                                   squeeze=False)
            for i, ky in enumerate(sel):
                for j, kx in enumerate(sel):
                    if i == j:
                        ax[i, j].set_axis_off()
                        ax[i, j].text(0.5, 0.5, kx.replace("_", " "), ha="center", va="center",
                                      transform=ax[i, j].transAxes)
                        continue
                    for d in data:
                        ax[i, j].scatter(d[kx].to_numpy(), d[ky].to_numpy(), s=5, alpha=0.1)
            fig.tight_layout()
            fig.savefig(os.path.join(bdir, "bivariate%s.png" % suffix))
            plt.close(fig)


def diagnose_samples(outputDirectory, assessConvergence=True, printSummary=True, nFigures=10,
                     device=0):
    """diagnoseSamples (sampleDiagnosis.py:11-85): same files, same stdout."""
    sampleDirectory = outputDirectory + "/sample/"
    diagnosticDirectory = outputDirectory + "/diagnostic/"
    os.makedirs(diagnosticDirectory, exist_ok=True)
    if assessConvergence:
        print("- Convergence Diagnostic -")
        diagnostic = Diagnostic(sampleDirectory, device=device)
        diagnostic.print(diagnosticDirectory + "/diagnosticAssessment.csv", False, False)
        if diagnostic.completelyPooled:
            diagnostic.print(None, False, False)
        if diagnostic.partiallyPooled:
            diagnostic.print(diagnosticDirectory + "/diagnosticAssessmentHyperOnly.csv", False, True)
            diagnostic.print(None, False, True)
        if not diagnostic.completelyPooled:
            diagnostic.print(diagnosticDirectory + "/diagnosticAssessmentIndividual.csv", True,
                             False)
            diagnostic.print(None, True, False)
    if printSummary:
        summary = Summary(sampleDirectory)
        summary.print(sampleDirectory + "/summary.csv")
        summary.print(None)
    if nFigures > 0:
        figures(outputDirectory, sampleDirectory, nFigures)
