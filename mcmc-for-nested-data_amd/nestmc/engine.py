"""Engine: one libnestmc context = one GPU's shard of chains.

Python-facing arrays are chain-major ([C, P, G], [C, G], [C, P]) like the oracle;
the device keeps chain-fastest SoA ([P][G][C]) so each wavefront's 64 lanes (64
chains) touch consecutive addresses.  Conversions happen only at the boundary
(state upload, sample download), never inside the iteration loop.
"""

import ctypes

import numpy

from . import _lib
from . import priors as _priors
from ._lib import as_f64, check, dptr

# step-kernel modes reported by nmc_launch_config (kernels.h NMC_MODE_*)
MODE_NAMES = {0: "NMC_MODE_NOPOOL", 1: "NMC_MODE_LAUNCH", 2: "NMC_MODE_SYNC",
              3: "NMC_MODE_SYNC_LDS", 4: "NMC_MODE_SYNC_REG", 5: "NMC_MODE_SYNC_OWN",
              6: "NMC_MODE_HALF"}


class Engine:
    def __init__(self, family, sizes, n_chains, pooling, priors=None, *, seed=0,
                 chain_base=0, device=0, rng="philox"):
        lib = _lib.load()
        self.lib = lib
        self.family = family
        self.sizes = numpy.asarray(sizes, dtype=numpy.int64)
        self.off = numpy.ascontiguousarray(numpy.concatenate([[0], numpy.cumsum(self.sizes)]),
                                           dtype=numpy.int64)
        self.G = len(self.sizes)
        self.C = int(n_chains)
        self.P = int(family.n_params)
        self.pooling = pooling
        self.chain_base = int(chain_base)
        self.device = int(device)
        obs = as_f64(family.obs())
        if obs.shape[0] != self.off[-1]:
            raise ValueError("family has %d observations, groups sum to %d"
                             % (obs.shape[0], self.off[-1]))
        consts = as_f64(family.consts())
        if pooling == "partial":
            pfam, pprm = None, None
        else:
            if priors is None or len(priors) != self.P:
                raise ValueError("Invalid prior")
            pfam, pprm = _priors.encode_all(priors)
        h = ctypes.c_void_p()
        check(lib.nmc_create(
            ctypes.byref(h), self.device, self.C, self.chain_base, self.G, self.P,
            _lib.POOLING[pooling], family.family_id(), dptr(consts), len(consts),
            self.off.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), dptr(obs),
            obs.shape[0], obs.shape[1],
            None if pfam is None else pfam.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
            None if pprm is None else dptr(pprm), ctypes.c_uint32(seed & 0xFFFFFFFF),
            _lib.RNG[rng]))
        self.h = h
        self._keep = (obs, consts, pfam, pprm)
        self.n_rows = 0
        self.cols = 0

    # -- lifecycle -----------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.nmc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- layout helpers -----------------------------------------------------
    @staticmethod
    def _pgc(a):          # [C, P, G] -> [P][G][C]
        return numpy.ascontiguousarray(numpy.transpose(numpy.asarray(a, float), (1, 2, 0)))

    @staticmethod
    def _gc(a):           # [C, G] -> [G][C]
        return numpy.ascontiguousarray(numpy.asarray(a, float).T)

    # -- state ----------------------------------------------------------------
    def set_state(self, value, log_prior, ll, mu=None, s2=None, scale=None):
        v = self._pgc(value)
        lp = self._pgc(log_prior)
        L = self._gc(ll)
        m = None if mu is None else self._gc(mu)        # [C, P] -> [P][C]
        s = None if s2 is None else self._gc(s2)
        sc = None if scale is None else self._pgc(scale)
        check(self.lib.nmc_set_state(self.h, dptr(v), dptr(lp), dptr(L), dptr(m), dptr(s),
                                     dptr(sc)))

    def get_state(self):
        C, P, G = self.C, self.P, self.G
        v = numpy.empty((P, G, C)); lp = numpy.empty((P, G, C)); L = numpy.empty((G, C))
        m = numpy.empty((P, C)); s = numpy.empty((P, C)); sc = numpy.empty((P, G, C))
        check(self.lib.nmc_get_state(self.h, dptr(v), dptr(lp), dptr(L), dptr(m), dptr(s),
                                     dptr(sc)))
        tr = lambda a: numpy.ascontiguousarray(numpy.transpose(a, (2, 0, 1)))   # noqa: E731
        return dict(value=tr(v), log_prior=tr(lp), ll=L.T.copy(), mu=m.T.copy(),
                    s2=s.T.copy(), scale=tr(sc))

    def set_replay(self, z, u, hz, hu):
        """z, u: [C, iter, P, G]; hz, hu: [C, iter, P] -> device [iter][P][G][C]."""
        zz = numpy.ascontiguousarray(numpy.transpose(z, (1, 2, 3, 0)), dtype=float)
        uu = numpy.ascontiguousarray(numpy.transpose(u, (1, 2, 3, 0)), dtype=float)
        hzz = numpy.ascontiguousarray(numpy.transpose(hz, (1, 2, 0)), dtype=float)
        huu = numpy.ascontiguousarray(numpy.transpose(hu, (1, 2, 0)), dtype=float)
        check(self.lib.nmc_set_replay(self.h, dptr(zz), dptr(uu), dptr(hzz), dptr(huu),
                                      zz.shape[0]))

    # -- schedule / run -------------------------------------------------------
    def set_schedule(self, n_iter, burn, thin, tune_interval=100):
        check(self.lib.nmc_set_schedule(self.h, n_iter, burn, thin, tune_interval))
        r, c = ctypes.c_int(), ctypes.c_int()
        check(self.lib.nmc_n_rows(self.h, ctypes.byref(r), ctypes.byref(c)))
        self.n_rows, self.cols = r.value, c.value

    def set_trace(self, enable=True):
        check(self.lib.nmc_set_trace(self.h, 1 if enable else 0))

    def run(self, iter_begin, iter_end):
        check(self.lib.nmc_run(self.h, iter_begin, iter_end))

    def synchronize(self):
        check(self.lib.nmc_synchronize(self.h))

    def prefill(self, i0, i1):
        """Draw the variates of iterations [i0, i1) now, beside whatever runs, for a later
        run() starting at i0 (nmc_prefill; run() guesses its next call by itself)."""
        check(self.lib.nmc_prefill(self.h, int(i0), int(i1)))

    def prefill_stats(self):
        """{"issued": iterations drawn by prefills, "used": iterations run() took from one}."""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        check(self.lib.nmc_prefill_stats(self.h, ctypes.byref(a), ctypes.byref(b)))
        return {"issued": a.value, "used": b.value}

    def set_resident(self, on=True):
        """One step launch for consecutive run() calls (nmc_set_resident): a call continuing
        the last is handed to the running launch.  Results are bit-identical either way."""
        check(self.lib.nmc_set_resident(self.h, 1 if on else 0))

    def resident_stats(self):
        """{"enabled", "active", "launches", "calls", "last_refusal"} (nmc_resident_stats)."""
        e, a, w = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        n, c = ctypes.c_int64(), ctypes.c_int64()
        check(self.lib.nmc_resident_stats(self.h, ctypes.byref(e), ctypes.byref(a),
                                          ctypes.byref(n), ctypes.byref(c), ctypes.byref(w)))
        return {"enabled": bool(e.value), "active": bool(a.value), "launches": n.value,
                "calls": c.value, "last_refusal": w.value}

    # -- results --------------------------------------------------------------
    def samples_raw(self, row_begin=0, n_rows=None):
        """[rows][cols][C] exactly as stored on the device."""
        if n_rows is None:
            n_rows = self.n_rows - row_begin
        out = numpy.empty((n_rows, self.cols, self.C))
        check(self.lib.nmc_get_samples(self.h, row_begin, n_rows, dptr(out)))
        return out

    def samples(self):
        """[C, rows, cols] chain-major (the oracle's row layout)."""
        return numpy.ascontiguousarray(numpy.transpose(self.samples_raw(), (2, 0, 1)))

    def accept_counts(self):
        out = numpy.empty((self.P, self.G, self.C), dtype=numpy.int64)
        check(self.lib.nmc_get_accept_counts(self.h, out.ctypes.data_as(
            ctypes.POINTER(ctypes.c_int64))))
        return numpy.transpose(out, (2, 0, 1))

    def trace(self, n_iter):
        n = n_iter * self.P * self.G * self.C
        acc = numpy.empty(n, dtype=numpy.uint8)
        llp = numpy.empty(n)
        check(self.lib.nmc_get_trace(self.h, acc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                     dptr(llp)))
        sh = (n_iter, self.P, self.G, self.C)
        # -> [C, iter, P, G]
        return (numpy.transpose(acc.reshape(sh), (3, 0, 1, 2)),
                numpy.transpose(llp.reshape(sh), (3, 0, 1, 2)))

    def eval_group_ll(self, theta):
        """theta [C, P, G] -> group log-likelihoods [C, G] on the device."""
        th = self._pgc(theta)
        out = numpy.empty((self.G, self.C))
        check(self.lib.nmc_eval_group_ll(self.h, dptr(th), dptr(out)))
        return out.T.copy()

    def obs_ll_rows(self, row_begin=0, n_rows=None):
        """Per-observation LL at recorded rows of the sample store: [C, rows, n_obs]."""
        if n_rows is None:
            n_rows = self.n_rows - row_begin
        out = numpy.empty((self.C, n_rows, int(self.off[-1])))
        check(self.lib.nmc_obs_ll_rows(self.h, row_begin, n_rows, dptr(out)))
        return out

    def write_ll_csvs(self, sample_dir, chain_ids, threads=8):
        """logLikelihood.<id>.csv for every local chain and recorded row (streamed)."""
        ids = numpy.ascontiguousarray(chain_ids, dtype=numpy.int32)
        if len(ids) != self.C:
            raise ValueError("need one file id per local chain")
        d = sample_dir if sample_dir.endswith("/") else sample_dir + "/"
        check(self.lib.nmc_write_ll_csvs(self.h, d.encode(),
                                         ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                         int(threads)))

    def eval_obs_ll(self):
        """Per-observation LL at the current state: [C, n_obs]."""
        out = numpy.empty((self.C, int(self.off[-1])))
        check(self.lib.nmc_eval_obs_ll(self.h, dptr(out)))
        return out

    # -- timing ---------------------------------------------------------------
    def event_record(self, slot):
        check(self.lib.nmc_event_record(self.h, slot))

    def event_elapsed_ms(self, a, b):
        ms = ctypes.c_float()
        check(self.lib.nmc_event_elapsed(self.h, a, b, ctypes.byref(ms)))
        return ms.value

    def set_launch_iters(self, n):
        """Cap the iterations one persistent launch covers (0: the variate chunk)."""
        check(self.lib.nmc_set_launch_iters(self.h, int(n)))

    def set_kernel_timing(self, enable):
        check(self.lib.nmc_set_kernel_timing(self.h, 1 if enable else 0))

    def kernel_timing(self):
        sm, hm = ctypes.c_double(), ctypes.c_double()
        sn, si, hn = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(self.lib.nmc_get_kernel_timing(self.h, ctypes.byref(sm), ctypes.byref(sn),
                                             ctypes.byref(si), ctypes.byref(hm),
                                             ctypes.byref(hn)))
        return dict(step_ms=sm.value, step_launches=sn.value, step_iters=si.value,
                    hyper_ms=hm.value, hyper_launches=hn.value)

    def gibbs_fallbacks(self):
        """(launch, chain block) pairs whose Gibbs tasks the step kernel updated itself
        because the separate Gibbs kernel did not run beside it (nmc_gibbs_fallbacks)."""
        n = ctypes.c_int64()
        check(self.lib.nmc_gibbs_fallbacks(self.h, ctypes.byref(n)))
        return n.value

    def launch_config(self):
        w, cb, pe, cl, md = (ctypes.c_int() for _ in range(5))
        check(self.lib.nmc_launch_config(self.h, ctypes.byref(w), ctypes.byref(cb),
                                         ctypes.byref(pe), ctypes.byref(cl), ctypes.byref(md)))
        sm, sb = ctypes.c_int(), ctypes.c_int()
        check(self.lib.nmc_split_config(self.h, ctypes.byref(sm), ctypes.byref(sb)))
        buf = ctypes.create_string_buffer(160)
        check(self.lib.nmc_kernel_name(self.h, buf, len(buf)))
        zin = ctypes.c_int()
        check(self.lib.nmc_variate_source(self.h, ctypes.byref(zin)))
        return dict(waves_per_group=w.value, chain_blocks=cb.value, persistent=bool(pe.value),
                    chains_per_block=cl.value, mode=MODE_NAMES.get(md.value, str(md.value)),
                    split_members=sm.value, chain_blocks_per_launch=sb.value,
                    kernel=buf.value.decode(), zin=zin.value)
