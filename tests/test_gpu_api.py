"""The drop-in API end to end on the GPU: sample_posterior (the rebuild's
samplePosterior, posteriorSampling.py:28-35) run with the reference's own variates
(replayed) must write sample.<chain>.csv files byte-identical to the ones the
reference wrote for the same inputs (tests/golden/csv, captured by
tests/golden/make_golden.py) -- host init (RandomState(chain) order), the device
loop, the schedule/recorder and the "%f" CSV writer together.
"""

import filecmp
import os

import pytest

from golden_cases import CASES, Case
from gpu_cases import family_for
from nestmc.sampler import sample_posterior

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", CASES)
def test_sample_posterior_writes_reference_csvs(gpu_lib, name, tmp_path):
    c = Case(name)
    a = c.arr
    out = str(tmp_path) + "/"
    sample_posterior(c.n_chains, c.n_iter, c.n_samples, c.names, c.n_groups, c.n_per_group,
                     c.pooling, family_for(c), out, saveLogLikelihood=False,
                     priorDistribution=c.priors, startWithMLE=c.mle,
                     startingPointValueRange=c.ranges, displayProgress=False,
                     rng="replay", replay={k: a[k] for k in ("z", "u", "hz", "hu")})
    for ch in range(c.n_chains):
        mine = os.path.join(out, "sample", "sample.%i.csv" % ch)
        assert filecmp.cmp(mine, c.csv_path(ch), shallow=False), (name, ch)


def test_save_loglikelihood_matches_reference(gpu_lib, tmp_path):
    """saveLogLikelihood=True (the reference's default, posteriorSampling.py:28-35):
    logLikelihood.<chain>.csv rows (:890-891, :907-909, :656-659) must be the
    reference's bytes -- sha256 of the whole 1000-row file captured by
    tests/golden/make_golden.py, plus its first and last rows."""
    import hashlib
    c = Case("regression_complete")
    a = c.arr
    m = c.meta
    out = str(tmp_path) + "/"
    sample_posterior(c.n_chains, c.n_iter, c.n_samples, c.names, c.n_groups, c.n_per_group,
                     c.pooling, family_for(c), out, saveLogLikelihood=True,
                     priorDistribution=c.priors, startWithMLE=c.mle,
                     startingPointValueRange=c.ranges, displayProgress=False,
                     rng="replay", replay={k: a[k] for k in ("z", "u", "hz", "hu")})
    raw = open(os.path.join(out, "sample", "logLikelihood.0.csv"), "rb").read()
    lines = raw.decode().splitlines()
    assert len(lines) == m["ll0_rows"]
    assert lines[0] == m["ll0_first"]
    assert lines[-1] == m["ll0_last"]
    assert hashlib.sha256(raw).hexdigest() == m["ll0_sha256"]
    assert filecmp.cmp(os.path.join(out, "sample", "sample.0.csv"), c.csv_path(0), shallow=False)


@pytest.mark.parametrize("name", ["linreg_partial", "regression_none"])
def test_progress_steps_resident_byte_identical(gpu_lib, name, tmp_path, monkeypatch):
    """displayProgress=True drives the loop in ten calls (posteriorSampling.py:872-891 with
    its progress prints), which share one resident step launch (nmc_set_resident): the
    sample files are byte for byte those of the one-call run on the Philox stream."""
    from nestmc.engine import Engine
    if name not in CASES:
        pytest.skip("no such golden case")
    c = Case(name)
    stats = []
    close = Engine.close

    def close_and_record(self):
        if getattr(self, "h", None):
            stats.append(self.resident_stats())
        close(self)

    monkeypatch.setattr(Engine, "close", close_and_record)
    outs = []
    for progress in (False, True):
        out = str(tmp_path / ("p%d" % progress)) + "/"
        sample_posterior(c.n_chains, c.n_iter, c.n_samples, c.names, c.n_groups, c.n_per_group,
                         c.pooling, family_for(c), out, saveLogLikelihood=False,
                         priorDistribution=c.priors, startWithMLE=c.mle,
                         startingPointValueRange=c.ranges, displayProgress=progress, seed=5)
        outs.append(out)
    assert stats[0]["launches"] == 0, stats
    assert stats[-1]["enabled"] and stats[-1]["calls"] >= 1, stats
    for ch in range(c.n_chains):
        a, b = (os.path.join(o, "sample", "sample.%i.csv" % ch) for o in outs)
        assert filecmp.cmp(a, b, shallow=False), (name, ch)
