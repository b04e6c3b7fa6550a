"""GPU: the product's multi-engine path -- samplePosterior sharding chains over several
engines (the rebuild's replacement of the reference's process fan-out,
posteriorSampling.py:182-201) -- run for real on one device.

* devices=[0, 0]: two engines on the same GPU, each holding a contiguous block of the
  chains (nestmc.parallel.shard), initialised and driven by the same host flow as one
  engine per GPU; the CSVs (samples and per-observation log-likelihoods) must be byte-
  identical to devices=[0];
* chains=: two calls holding the two halves of the chains (what two ranks of a job
  launched by torchrun do) write, between them, the files of the one-call run byte for
  byte;
* on a golden case with the reference's own variates replayed, devices=[0, 0] still
  writes the reference's bytes.
"""

import filecmp
import os

import numpy
import pytest

from golden_cases import Case
from gpu_cases import family_for, synthetic
from nestmc.sampler import sample_posterior

pytestmark = pytest.mark.gpu


def _files(d):
    return sorted(f for f in os.listdir(os.path.join(d, "sample")))


def _same_tree(a, b, names):
    for fn in names:
        pa, pb = os.path.join(a, "sample", fn), os.path.join(b, "sample", fn)
        assert filecmp.cmp(pa, pb, shallow=False), fn


@pytest.mark.parametrize("kind", ["linreg_partial", "regression3_none"])
def test_devices_and_chain_halves_byte_identical(gpu_lib, tmp_path, kind):
    C, G, N = 70, 6, 40
    fam, sizes, priors, pooling, names = synthetic(kind, C, G, N)
    ranges = {n: [-0.5, 0.5] for n in names if n != "sigma"}
    if "sigma" in names:
        ranges["sigma"] = [0.5, 1.5]
    kw = dict(saveLogLikelihood=True, priorDistribution=priors,
              startingPointValueRange=ranges, displayProgress=False, seed=17)
    one, two = str(tmp_path / "one"), str(tmp_path / "two")
    sample_posterior(C, 60, 20, names, G, N, pooling, fam, one, devices=[0], **kw)
    sample_posterior(C, 60, 20, names, G, N, pooling, fam, two, devices=[0, 0], **kw)
    files = _files(one)
    assert sum(f.startswith("sample.") for f in files) == C
    assert sum(f.startswith("logLikelihood.") for f in files) == C
    assert _files(two) == files
    _same_tree(one, two, files)
    # two "ranks": halves of the chains, each in its own call and output directory
    h0, h1 = str(tmp_path / "h0"), str(tmp_path / "h1")
    sample_posterior(C, 60, 20, names, G, N, pooling, fam, h0, chains=range(0, 33), **kw)
    sample_posterior(C, 60, 20, names, G, N, pooling, fam, h1, chains=range(33, C), **kw)
    for c in range(C):
        h = h0 if c < 33 else h1
        for fn in ("sample.%d.csv" % c, "logLikelihood.%d.csv" % c):
            assert filecmp.cmp(os.path.join(one, "sample", fn), os.path.join(h, "sample", fn),
                               shallow=False), fn
    # the returned arrays of a two-engine run are the one-engine arrays
    r1 = sample_posterior(C, 60, 20, names, G, N, pooling, fam, None, devices=[0],
                          write_files=False, return_samples=True,
                          **dict(kw, saveLogLikelihood=False))
    r2 = sample_posterior(C, 60, 20, names, G, N, pooling, fam, None, devices=[0, 0],
                          write_files=False, return_samples=True,
                          **dict(kw, saveLogLikelihood=False))
    assert numpy.array_equal(r1["rows"], r2["rows"], equal_nan=True)
    assert numpy.array_equal(r1["accepted"], r2["accepted"])


@pytest.mark.parametrize("name", ["linreg_partial", "regression_none"])
def test_devices_replay_writes_reference_csvs(gpu_lib, tmp_path, name):
    c = Case(name)
    a = c.arr
    out = str(tmp_path) + "/"
    sample_posterior(c.n_chains, c.n_iter, c.n_samples, c.names, c.n_groups, c.n_per_group,
                     c.pooling, family_for(c), out, saveLogLikelihood=False,
                     priorDistribution=c.priors, startWithMLE=c.mle,
                     startingPointValueRange=c.ranges, displayProgress=False,
                     devices=[0] * c.n_chains,
                     rng="replay", replay={k: a[k] for k in ("z", "u", "hz", "hu")})
    for ch in range(c.n_chains):
        mine = os.path.join(out, "sample", "sample.%i.csv" % ch)
        assert filecmp.cmp(mine, c.csv_path(ch), shallow=False), (name, ch)
