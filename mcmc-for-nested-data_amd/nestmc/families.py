"""Likelihood families: the device-side replacement for the user callback.

The reference takes an arbitrary Python ``logLikelihoodFunction(parameter)``
(posteriorSampling.py:61-102) and calls it once per parameter step over every
observation.  On the GPU the likelihood must be a known device functor
(csrc/families.h), so a family object carries

* the observations as a dense fp64 table in the reference's row order, and the
  constants of the model -- what the kernels stream; and
* a numpy ``__call__`` in the reference convention ``f(parameter[P][n]) -> ll[n]``
  written with the same numpy/scipy operations as the reference's examples, so the
  same object can be handed to the reference sampler, and the host-side chain
  initialisation (start-point search, Nelder-Mead MLE, posteriorSampling.py:1060-1141)
  evaluates exactly what the reference would.

Families: ``LinearRegression`` (example/regression.py:53-67, and the cfg 3/4 model
with known noise sd), ``GaussianMean`` (example/distribution.py:18-24),
``Logistic`` (cfg 5), and ``DeviceLikelihood``: any per-observation log-likelihood
written as a HIP device function, compiled for gfx950 at run time (csrc/user.hip).
"""

import numpy
import scipy.stats


class Family:
    family = None          # key of _lib.FAMILY

    n_params = 0
    n_fields = 0

    def obs(self):
        raise NotImplementedError

    def consts(self):
        raise NotImplementedError

    def bytes_per_obs(self):
        return 8 * self.n_fields

    def family_id(self):
        """The C-ABI ll_family code of this family (nmc_create)."""
        from . import _lib
        return _lib.FAMILY[self.family]

    def __call__(self, parameter):
        raise NotImplementedError


def _split_intercept(X):
    X = numpy.asarray(X, dtype=numpy.float64)
    if X.ndim == 1:
        X = X[:, None]
    intercept = X.shape[1] > 0 and bool(numpy.all(X[:, 0] == 1.0))
    stored = X[:, 1:] if intercept else X
    return X, stored, intercept


class LinearRegression(Family):
    """y ~ Normal(X beta, sigma): ``norm(loc=y, scale=sigma).logpdf(X beta)`` per row.

    ``X`` is the full design matrix in the reference's form (example/regression.py:24-27
    stores the ones column explicitly); a leading all-ones column is not streamed --
    the kernel adds the intercept instead.  Parameters, in order: one coefficient per
    column of X, then sigma unless ``sigma`` (a fixed noise sd) is given.
    """

    family = "linreg"

    def __init__(self, X, y, sigma=None):
        self.X, stored, self.intercept = _split_intercept(X)
        self.y = numpy.asarray(y, dtype=numpy.float64).reshape(-1)
        if self.X.shape[0] != self.y.shape[0]:
            raise ValueError("X and y must have the same number of rows")
        self.sigma = None if sigma is None else float(sigma)
        if self.sigma is not None and not self.sigma > 0:
            raise ValueError("sigma must be > 0")
        self._obs = numpy.ascontiguousarray(numpy.hstack([stored, self.y[:, None]]))
        self.n_fields = self._obs.shape[1]
        self.n_params = self.X.shape[1] + (1 if self.sigma is None else 0)

    @classmethod
    def simple(cls, x, y, sigma=None):
        """y = b0 + b1 x (+ noise); parameters (b0, b1[, sigma])."""
        x = numpy.asarray(x, dtype=numpy.float64).reshape(-1)
        return cls(numpy.vstack([numpy.ones_like(x), x]).T, y, sigma=sigma)

    def obs(self):
        return self._obs

    def consts(self):
        k = self.n_fields - 1
        if self.sigma is None:
            return [float(k), float(self.intercept), 0.0, 0.0]
        return [float(k), float(self.intercept), self.sigma, float(numpy.log(self.sigma))]

    def __call__(self, parameter):
        K = self.X.shape[1]
        betaHat = numpy.vstack([parameter[j] for j in range(K)]).T
        yHat = numpy.sum(self.X * betaHat, axis=1)
        noise = numpy.array(parameter[K]) if self.sigma is None else self.sigma
        return scipy.stats.norm(loc=self.y, scale=noise).logpdf(yHat)


class GaussianMean(Family):
    """Per response: sum_j norm(means[:, j], sd[j]).logpdf(theta_j) (example/distribution.py).

    ``means`` is (n_obs, P): the mean each response carries for parameter j (the
    example's mu_jg repeated over the group's responses).
    """

    family = "gauss_mean"

    def __init__(self, means, sd):
        self.means = numpy.ascontiguousarray(numpy.asarray(means, dtype=numpy.float64))
        if self.means.ndim != 2:
            raise ValueError("means must be (n_obs, n_params)")
        self.sd = numpy.asarray(sd, dtype=numpy.float64).reshape(-1)
        if self.sd.shape[0] != self.means.shape[1]:
            raise ValueError("one sd per parameter")
        self.n_fields = self.means.shape[1]
        self.n_params = self.n_fields

    @classmethod
    def from_groups(cls, mu, sd, sizes):
        """mu[P][G] group means (example/distribution.py:30-34), sizes[G]."""
        mu = numpy.asarray(mu, dtype=numpy.float64)
        g = numpy.repeat(numpy.arange(mu.shape[1]), sizes)
        return cls(mu[:, g].T, sd)

    def obs(self):
        return self.means

    def consts(self):
        return list(self.sd) + list(numpy.log(self.sd))

    def __call__(self, parameter):
        out = 0
        for j in range(self.n_params):
            out = out + scipy.stats.norm(loc=self.means[:, j], scale=self.sd[j]).logpdf(
                numpy.asarray(parameter[j], dtype=numpy.float64))
        return out


class Logistic(Family):
    """Bernoulli-logit: eta = X theta, ll = y eta - logaddexp(0, eta) (cfg 5).

    A leading all-ones column of X is the intercept (not streamed).  Parameters:
    one coefficient per column of X.
    """

    family = "logistic"

    def __init__(self, X, y):
        self.X, stored, self.intercept = _split_intercept(X)
        self.y = numpy.asarray(y, dtype=numpy.float64).reshape(-1)
        if self.X.shape[0] != self.y.shape[0]:
            raise ValueError("X and y must have the same number of rows")
        self._obs = numpy.ascontiguousarray(numpy.hstack([stored, self.y[:, None]]))
        self.n_fields = self._obs.shape[1]
        self.n_params = self.X.shape[1]

    def obs(self):
        return self._obs

    def consts(self):
        return [float(self.n_fields - 1), float(self.intercept), 0.0, 0.0]

    def __call__(self, parameter):
        theta = numpy.vstack(parameter).T
        eta = numpy.sum(self.X * theta, axis=1)
        return self.y * eta - numpy.logaddexp(0.0, eta)


_USER_IDS = {}   # (source, n_fields, n_params) -> registered family id (per process)


class DeviceLikelihood(Family):
    """A user log-likelihood as device code: the GPU form of the reference's arbitrary
    ``logLikelihoodFunction`` (posteriorSampling.py:61-102).

    ``source`` defines one observation's log-likelihood::

        __device__ double nmc_user_loglik(const double* theta,  // [n_params]
                                          const double* row,    // [n_fields]
                                          const double* k)      // consts
        { ... }

    ``obs`` is the (n_obs, n_fields) table of observations in the reference's response
    order (``row`` is one of its rows) and ``consts`` the model's constants.  The source
    is compiled with hiprtc for gfx950 the first time an engine uses it (csrc/user.hip,
    the library's own flags: IEEE fp64, no contraction), then cached for the process.
    The kernels sum the per-row values in the same fixed order as the built-in families.

    ``host_function(parameter[P][n]) -> ll[n]`` (optional) is the same model in the
    reference's calling convention; the host needs it only for ``startWithMLE`` (the
    Nelder-Mead objective, :1102-1141) -- every other evaluation runs on the device.
    """

    family = "user"

    def __init__(self, obs, source, n_params, consts=(), host_function=None):
        obs = numpy.asarray(obs, dtype=numpy.float64)
        if obs.ndim == 1:
            obs = obs[:, None]
        if obs.ndim != 2:
            raise ValueError("obs must be (n_obs, n_fields)")
        self._obs = numpy.ascontiguousarray(obs)
        self.n_fields = self._obs.shape[1]
        self.n_params = int(n_params)
        if not 1 <= self.n_params <= 16:
            raise ValueError("1 <= n_params <= 16")
        if "nmc_user_loglik" not in source:
            raise ValueError("source must define __device__ double nmc_user_loglik(...)")
        self.source = source
        self._consts = [float(v) for v in consts]
        self.host_function = host_function

    def family_id(self):
        import ctypes
        import os
        from . import _lib
        key = (self.source, self.n_fields, self.n_params)
        if key not in _USER_IDS:
            lib = _lib.load()
            inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                               "csrc")
            fid = ctypes.c_int(-1)
            _lib.check(lib.nmc_user_family_compile(self.source.encode(), self.n_fields,
                                                   self.n_params, inc.encode(),
                                                   ctypes.byref(fid)))
            _USER_IDS[key] = fid.value
        return _USER_IDS[key]

    def obs(self):
        return self._obs

    def consts(self):
        return list(self._consts)

    def __call__(self, parameter):
        if self.host_function is None:
            raise TypeError("DeviceLikelihood: no host_function given; host-side evaluation "
                            "(startWithMLE's Nelder-Mead objective) needs the model in the "
                            "reference's calling convention")
        return self.host_function(parameter)


def is_family(obj):
    return isinstance(obj, Family)
