"""Loader for the golden fixtures captured from the reference (tests/golden/*.npz)."""

import functools
import json
import os

import numpy
import scipy.stats

from callbacks import ll_distribution, ll_logistic, ll_regression2, ll_regression3

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CASES = ["regression_complete", "regression_none", "regression3_partial",
         "linreg_partial", "linreg_ragged_partial", "distribution_none",
         "distribution_partial", "logistic_partial"]


class Case:
    def __init__(self, name):
        self.name = name
        z = numpy.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.arr = {k: z[k] for k in z.files if k != "meta"}
        self.meta = json.loads(str(z["meta"]))
        m = self.meta
        self.names = tuple(m["param_names"])
        self.n_chains = m["n_chains"]
        self.n_iter = m["n_iter"]
        self.n_samples = m["n_samples"]
        self.n_groups = m["n_groups"]
        self.n_per_group = m["n_per_group"]
        self.pooling = m["pooling"]
        self.mle = m["mle"]
        self.ranges = m["ranges"]
        self.priors = None
        a = self.arr
        if name.startswith("regression"):
            self.ll = functools.partial(ll_regression3, X=a["X"], y=a["y"])
            self.priors = [scipy.stats.norm(loc=0, scale=10),
                           scipy.stats.norm(loc=100, scale=10), scipy.stats.gamma(10)]
            if name == "regression3_partial":
                self.priors = None
        elif name.startswith("linreg"):
            self.ll = functools.partial(ll_regression2, x=a["x"], y=a["y"])
        elif name.startswith("distribution"):
            sizes = [self.n_per_group] * self.n_groups
            self.ll = functools.partial(ll_distribution, mu=a["mu"], sd=a["sd"], sizes=sizes)
            self.priors = [scipy.stats.norm(loc=0, scale=1) for _ in self.names]
        elif name.startswith("logistic"):
            self.ll = functools.partial(ll_logistic, X=a["X"], y=a["y"])
        else:
            raise KeyError(name)

    @property
    def sizes(self):
        n = self.n_per_group
        if isinstance(n, int):
            n = [n] * self.n_groups
        if self.pooling == "complete":
            n = [int(sum(n))]
        return list(n)

    def csv_path(self, chain):
        return os.path.join(GOLDEN, "csv", self.name, "sample.%i.csv" % chain)
