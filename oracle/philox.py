"""Philox4x32-10 counter-based RNG in numpy -- TEST INFRASTRUCTURE (oracle).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package.  It restates the device stream spec of
``mcmc-for-nested-data_amd/csrc/philox.h`` so that the numpy oracle and the HIP
kernels draw the same variates (see DESIGN.md "Random streams").

Philox4x32-10 (Salmon et al., SC'11): 10 rounds of
    (hi0, lo0) = mulhilo(0xD2511F53, c0); (hi1, lo1) = mulhilo(0xCD9E8D57, c2)
    c = (hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0);  k += (0x9E3779B9, 0xBB67AE85)
Stream layout used by the sampler (replaces the numpy legacy MT19937 draws of
posteriorSampling.py:306, :362, :487, :498):
    key     = (global chain id, seed)
    counter = (iteration, group, parameter, purpose)
    purpose 0: proposal normal  -- Box-Muller on the block's two uniforms
    purpose 1: accept uniform   -- first uniform of the block
    purpose 2: hyper mean normal (group 0)
    purpose 3: hyper gamma boost uniform (shape < 1)
    purpose 16+2k / 17+2k: hyper gamma Marsaglia-Tsang attempt k (normal / uniform)
A block's two 53-bit uniforms are ((x1<<32|x0) >> 11) * 2^-53 and
((x3<<32|x2) >> 11) * 2^-53, both in [0, 1).
"""

import numpy

M0 = numpy.uint64(0xD2511F53)
M1 = numpy.uint64(0xCD9E8D57)
W0 = numpy.uint64(0x9E3779B9)
W1 = numpy.uint64(0xBB67AE85)
MASK = numpy.uint64(0xFFFFFFFF)
TWO_PI = 6.283185307179586
INV53 = 1.0 / 9007199254740992.0

PURPOSE_PROPOSAL = 0
PURPOSE_ACCEPT = 1
PURPOSE_HYPER_NORMAL = 2
PURPOSE_GAMMA_BOOST = 3
PURPOSE_GAMMA_BASE = 16
GAMMA_MAX_ATTEMPTS = 64


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10; all inputs broadcast, values < 2**32."""
    c0, c1, c2, c3, k0, k1 = numpy.broadcast_arrays(
        *[numpy.asarray(v, dtype=numpy.uint64) & MASK for v in (c0, c1, c2, c3, k0, k1)])
    c0 = c0.copy(); c1 = c1.copy(); c2 = c2.copy(); c3 = c3.copy()
    k0 = k0.copy(); k1 = k1.copy()
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> numpy.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> numpy.uint64(32), p1 & MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0), lo1, (hi0 ^ c3 ^ k1), lo0
        k0 = (k0 + W0) & MASK
        k1 = (k1 + W1) & MASK
    return c0, c1, c2, c3


def uniforms(it, group, param, purpose, chain, seed):
    """The block's two [0,1) doubles for the given counter/key (broadcast)."""
    x0, x1, x2, x3 = philox4x32_10(it, group, param, purpose, chain, seed)
    a = ((x1 << numpy.uint64(32)) | x0) >> numpy.uint64(11)
    b = ((x3 << numpy.uint64(32)) | x2) >> numpy.uint64(11)
    return a.astype(numpy.float64) * INV53, b.astype(numpy.float64) * INV53


def cos2pi(u):
    """cos(2 pi u), u in [0, 1), with the argument reduced exactly in u (every difference is
    exact, Sterbenz) to t in [0, 1/8] before numpy's sin / cos of 2 pi t: within ~1 ulp of the
    exact value everywhere, where cos(fl(2 pi u)) is off by up to ~3000 ulp near the zeros.
    The same function as csrc/rng.h nmc_cos2pi (which evaluates the last step with its own
    polynomials; the two agree to a few ulp)."""
    u = numpy.asarray(u, dtype=numpy.float64)
    v = numpy.where(u > 0.5, 1.0 - u, u)
    neg = v > 0.25
    w = numpy.where(neg, 0.5 - v, v)
    sn = w > 0.125
    t = numpy.where(sn, 0.25 - w, w)
    r = numpy.where(sn, numpy.sin(TWO_PI * t), numpy.cos(TWO_PI * t))
    return numpy.where(neg, -r, r)


def box_muller(ua, ub):
    """z = sqrt(-2 log(1 - ua)) cos(2 pi ub); 1 - ua is in (0, 1]."""
    return numpy.sqrt(-2.0 * numpy.log(1.0 - ua)) * cos2pi(ub)


def normal(it, group, param, purpose, chain, seed):
    ua, ub = uniforms(it, group, param, purpose, chain, seed)
    return box_muller(ua, ub)


def gamma_mt(a, it, param, chain, seed):
    """Gamma(a, 1) by Marsaglia-Tsang on the hyper gamma purposes (vector over chains).

    Restates ``nmc_gamma_mt`` of csrc/rng.h step by step (same squeeze test, same
    attempt counters) so oracle and device accept on the same attempt.
    """
    chain = numpy.asarray(chain)
    out = numpy.full(chain.shape, numpy.nan)
    boost = a < 1.0
    aa = a + 1.0 if boost else a
    d = aa - 1.0 / 3.0
    c = 1.0 / numpy.sqrt(9.0 * d)
    todo = numpy.ones(chain.shape, bool)
    for k in range(GAMMA_MAX_ATTEMPTS):
        z = normal(it, 0, param, PURPOSE_GAMMA_BASE + 2 * k, chain, seed)
        u, _ = uniforms(it, 0, param, PURPOSE_GAMMA_BASE + 2 * k + 1, chain, seed)
        v = 1.0 + c * z
        ok = v > 0.0
        v3 = v * v * v
        with numpy.errstate(divide="ignore", invalid="ignore"):
            z2 = z * z
            acc = ok & ((u < 1.0 - 0.0331 * (z2 * z2)) |
                        (numpy.log(u) < 0.5 * z2 + d * (1.0 - v3 + numpy.log(v3))))
        take = todo & acc
        out[take] = (d * v3)[take]
        todo &= ~acc
        if not todo.any():
            break
    out[todo] = d          # never reached in practice (P < 1e-100)
    if boost:
        ub, _ = uniforms(it, 0, param, PURPOSE_GAMMA_BOOST, chain, seed)
        out = out * numpy.exp(numpy.log(1.0 - ub) / a)
    return out
