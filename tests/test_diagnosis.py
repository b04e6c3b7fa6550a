"""diagnoseSamples: the reference's convergence diagnostics over sample
files (sampleDiagnosis.py:11-85), pinned to the reference's own outputs on the golden
sample directories (tests/golden/diag, tests/golden/make_golden_diag.py).

CPU: the oracle restatement (oracle/diagnosis.py) reproduces the reference's files
byte for byte; the product's vectorised host statistics (nestmc.diagnosis) do too when
fed the oracle's variogram.  GPU: the product end to end (the variogram kernel
nmc_variogram) writes the reference's files and stdout; the kernel's V_t agree with the
reference's Python sums to 1e-12 relative at 24 columns x 16 half-chains x 300 lags.
"""

import contextlib
import io
import os
import shutil

import numpy
import pytest

from oracle import diagnosis as od

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "diag")


def _source(case):
    for root in ("csv", "diag_inputs"):
        p = os.path.join(HERE, "golden", root, case)
        if os.path.isdir(p):
            return p
    raise KeyError(case)


CASES = sorted(c for c in os.listdir(GOLD)
               if not os.path.exists(os.path.join(GOLD, c, "error.txt")))
ERROR_CASES = sorted(c for c in os.listdir(GOLD)
                     if os.path.exists(os.path.join(GOLD, c, "error.txt")))
SMALL = [c for c in CASES if c != "regression_complete"]   # the oracle's O(m n^2) loop


def _gold(case, name):
    return open(os.path.join(GOLD, case, name)).read()


@pytest.mark.parametrize("case", SMALL)
def test_oracle_matches_reference_files(case):
    src = _source(case)
    a, partial, complete = od.assess(src)
    assert od.assessment_text(a, False) == _gold(case, "diagnosticAssessment.csv")
    if partial:
        assert od.assessment_text(a, True) == _gold(case, "diagnosticAssessmentHyperOnly.csv")
    if not complete:
        assert od.individual_text(a) == _gold(case, "diagnosticAssessmentIndividual.csv")
    assert od.summary_text(src) == _gold(case, "summary.csv")


def _run_product(case, tmp_path, monkeypatch=None):
    from nestmc import diagnosis
    if monkeypatch is not None:   # host-only check: the oracle's variogram stands in
        monkeypatch.setattr(diagnosis, "variogram", lambda x, device=0: numpy.array(
            [[od.variogram(x[k], t) for t in range(x.shape[2])] for k in range(x.shape[0])]))
    out = str(tmp_path / case)
    shutil.copytree(_source(case), os.path.join(out, "sample"))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        diagnosis.diagnose_samples(out, True, True, 0)
    return out, buf.getvalue()


def _check_files(case, out, stdout):
    for name in sorted(os.listdir(os.path.join(GOLD, case))):
        if name == "stdout.txt":
            assert stdout == _gold(case, name), case
        elif name == "summary.csv":
            assert open(os.path.join(out, "sample", name)).read() == _gold(case, name), case
        else:
            assert open(os.path.join(out, "diagnostic", name)).read() == _gold(case, name), \
                (case, name)


@pytest.mark.parametrize("case", SMALL)
def test_product_host_statistics_match_reference(case, tmp_path, monkeypatch):
    out, stdout = _run_product(case, tmp_path, monkeypatch)
    _check_files(case, out, stdout)


@pytest.mark.parametrize("case", ERROR_CASES[:2])
def test_odd_row_count_raises_like_reference(case, tmp_path, monkeypatch):
    want = _gold(case, "error.txt").split(":")[0]
    with pytest.raises(ValueError if want == "ValueError" else Exception):
        _run_product(case, tmp_path, monkeypatch)


@pytest.mark.parametrize("case", SMALL[:2])
def test_longer_later_files_cut_like_reference(case, tmp_path, monkeypatch):
    """The convergence diagnostic cuts every file at the FIRST file's row count
    (sampleDiagnosis.py:136-155): an extra row appended to every later file leaves the
    diagnostic files unchanged (the sample Summary, :382-491, reads every row, so the
    summary and stdout are not compared here)."""
    import glob
    from nestmc import diagnosis
    monkeypatch.setattr(diagnosis, "variogram", lambda x, device=0: numpy.array(
        [[od.variogram(x[k], t) for t in range(x.shape[2])] for k in range(x.shape[0])]))
    out = str(tmp_path / case)
    shutil.copytree(_source(case), os.path.join(out, "sample"))
    files = glob.glob(os.path.join(out, "sample") + "/sample*.csv")
    assert len(files) >= 2
    for fn in files[1:]:
        last = open(fn).read().splitlines()[-1]
        with open(fn, "a") as f:
            f.write(last + "\n")
    with contextlib.redirect_stdout(io.StringIO()):
        diagnosis.diagnose_samples(out, True, True, 0)
    names = [n for n in sorted(os.listdir(os.path.join(GOLD, case)))
             if n not in ("stdout.txt", "summary.csv")]
    assert names
    for name in names:
        assert open(os.path.join(out, "diagnostic", name)).read() == _gold(case, name), name


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_gpu_diagnose_samples_matches_reference(gpu_lib, case, tmp_path):
    out, stdout = _run_product(case, tmp_path)
    _check_files(case, out, stdout)


@pytest.mark.gpu
def test_gpu_variogram_matches_reference_sums(gpu_lib):
    from nestmc import diagnosis
    r = numpy.random.RandomState(3)
    x = numpy.cumsum(r.normal(size=(24, 16, 300)), axis=2) * 0.1 + r.normal(size=(24, 16, 1))
    got = diagnosis.variogram(x)
    for k in (0, 7, 23):
        want = numpy.array([od.variogram(x[k], t) for t in range(300)])
        assert numpy.allclose(got[k], want, rtol=1e-12, atol=0)


@pytest.mark.gpu
def test_gpu_sample_then_diagnose(gpu_lib, tmp_path):
    """The drop-in pair end to end: samplePosterior (GPU) writes the sample files,
    diagnoseSamples (GPU variogram) reads them; its files equal the oracle
    restatement's on the same files."""
    import posteriorSampling
    import sampleDiagnosis
    from gpu_cases import synthetic
    fam, sizes, _, _, _ = synthetic("linreg_partial", 4, 5, 40)
    out = str(tmp_path / "run")
    posteriorSampling.samplePosterior(4, 400, 200, ("b0", "b1"), 5, 40, "partial", fam, out,
                                      saveLogLikelihood=False,
                                      startingPointValueRange={"b0": [-1, 1], "b1": [0, 3]},
                                      displayProgress=False)
    with contextlib.redirect_stdout(io.StringIO()):
        sampleDiagnosis.diagnoseSamples(out, nFigures=0)
    src = os.path.join(out, "sample")
    a, partial, complete = od.assess(src)
    got = open(os.path.join(out, "diagnostic", "diagnosticAssessment.csv")).read()
    assert got == od.assessment_text(a, False)
    assert open(os.path.join(out, "diagnostic", "diagnosticAssessmentIndividual.csv")).read() \
        == od.individual_text(a)
    assert open(os.path.join(src, "summary.csv")).read() == od.summary_text(src)
