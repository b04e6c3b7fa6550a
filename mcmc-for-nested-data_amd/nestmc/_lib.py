"""ctypes binding of libnestmc.so (include/nestmc.h).

The library is built in-tree (``make -C mcmc-for-nested-data_amd/csrc``, or
``__graft_entry__.build()``).  There is no fallback: if the library or a GPU is
missing, sampling raises -- the product never silently runs on the CPU.
"""

import ctypes
import os

import numpy

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NESTMC_LIB") or os.path.join(_HERE, "libnestmc.so")

POOLING = {"complete": 0, "none": 1, "partial": 2}
FAMILY = {"linreg": 0, "gauss_mean": 1, "logistic": 2}
PRIOR = {"norm": 0, "gamma": 1, "uniform": 2, "expon": 3, "halfnorm": 4, "cauchy": 5,
         "laplace": 6, "lognorm": 7, "invgamma": 8}
RNG = {"philox": 0, "replay": 1}

_c_int_p = ctypes.POINTER(ctypes.c_int)
_c_double_p = ctypes.POINTER(ctypes.c_double)
_c_int64_p = ctypes.POINTER(ctypes.c_int64)
_c_int32_p = ctypes.POINTER(ctypes.c_int32)
_c_uint8_p = ctypes.POINTER(ctypes.c_uint8)
_c_uint32_p = ctypes.POINTER(ctypes.c_uint32)
_vp = ctypes.c_void_p

# name -> (restype, argtypes); every symbol include/nestmc.h declares
SIGNATURES = {
    "nmc_last_error": (ctypes.c_char_p, []),
    "nmc_version": (ctypes.c_char_p, []),
    "nmc_device_count": (ctypes.c_int, [_c_int_p]),
    "nmc_create": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  _c_double_p, ctypes.c_int, _c_int64_p, _c_double_p,
                                  ctypes.c_int64, ctypes.c_int, _c_int_p, _c_double_p,
                                  ctypes.c_uint32, ctypes.c_int]),
    "nmc_destroy": (ctypes.c_int, [_vp]),
    "nmc_set_state": (ctypes.c_int, [_vp, _c_double_p, _c_double_p, _c_double_p, _c_double_p,
                                     _c_double_p, _c_double_p]),
    "nmc_get_state": (ctypes.c_int, [_vp, _c_double_p, _c_double_p, _c_double_p, _c_double_p,
                                     _c_double_p, _c_double_p]),
    "nmc_set_replay": (ctypes.c_int, [_vp, _c_double_p, _c_double_p, _c_double_p, _c_double_p,
                                      ctypes.c_int]),
    "nmc_set_schedule": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int]),
    "nmc_n_rows": (ctypes.c_int, [_vp, _c_int_p, _c_int_p]),
    "nmc_set_trace": (ctypes.c_int, [_vp, ctypes.c_int]),
    "nmc_get_trace": (ctypes.c_int, [_vp, _c_uint8_p, _c_double_p]),
    "nmc_run": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int]),
    "nmc_synchronize": (ctypes.c_int, [_vp]),
    "nmc_prefill": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int]),
    "nmc_prefill_stats": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int64),
                                         ctypes.POINTER(ctypes.c_int64)]),
    "nmc_set_resident": (ctypes.c_int, [_vp, ctypes.c_int]),
    "nmc_resident_stats": (ctypes.c_int, [_vp, _c_int_p, _c_int_p, _c_int64_p, _c_int64_p,
                                          _c_int_p]),
    "nmc_get_samples": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _c_double_p]),
    "nmc_get_accept_counts": (ctypes.c_int, [_vp, _c_int64_p]),
    "nmc_eval_group_ll": (ctypes.c_int, [_vp, _c_double_p, _c_double_p]),
    "nmc_eval_obs_ll": (ctypes.c_int, [_vp, _c_double_p]),
    "nmc_obs_ll_rows": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _c_double_p]),
    "nmc_write_ll_csvs": (ctypes.c_int, [_vp, ctypes.c_char_p, _c_int32_p, ctypes.c_int]),
    "nmc_event_record": (ctypes.c_int, [_vp, ctypes.c_int]),
    "nmc_event_elapsed": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_float)]),
    "nmc_set_kernel_timing": (ctypes.c_int, [_vp, ctypes.c_int]),
    "nmc_set_launch_iters": (ctypes.c_int, [_vp, ctypes.c_int]),
    "nmc_get_kernel_timing": (ctypes.c_int, [_vp, _c_double_p, _c_int64_p, _c_int64_p,
                                             _c_double_p, _c_int64_p]),
    "nmc_kernel_name": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_int]),
    "nmc_split_config": (ctypes.c_int, [_vp, _c_int_p, _c_int_p]),
    "nmc_variate_source": (ctypes.c_int, [_vp, _c_int_p]),
    "nmc_gibbs_fallbacks": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int64)]),
    "nmc_variogram": (ctypes.c_int, [ctypes.c_int, _c_double_p, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, _c_double_p]),
    "nmc_user_family_compile": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_char_p, _c_int_p]),
    "nmc_user_family_shape": (ctypes.c_int, [ctypes.c_int, _c_int_p, _c_int_p]),
    "nmc_launch_config": (ctypes.c_int, [_vp, _c_int_p, _c_int_p, _c_int_p, _c_int_p,
                                              _c_int_p]),
    "nmc_write_sample_csv": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p,
                                            _c_double_p, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, _c_int32_p, ctypes.c_int,
                                            ctypes.c_int]),
    "nmc_write_ll_csv": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, _c_double_p,
                                        ctypes.c_int64, ctypes.c_int]),
    "nmc_comm_unique_id": (ctypes.c_int, [ctypes.POINTER(ctypes.c_ubyte)]),
    "nmc_comm_init": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_ubyte),
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "nmc_comm_destroy": (ctypes.c_int, [_vp]),
    "nmc_comm_size": (ctypes.c_int, [_vp, _c_int_p, _c_int_p]),
    "nmc_gather_samples": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _c_double_p, ctypes.c_int64]),
    "nmc_debug_prior_logpdf": (ctypes.c_int, [ctypes.c_int, _c_double_p, _c_double_p,
                                              ctypes.c_int, _c_double_p]),
    "nmc_debug_igamci": (ctypes.c_int, [_c_double_p, _c_double_p, _c_double_p, ctypes.c_int,
                                        _c_double_p]),
    "nmc_debug_rng": (ctypes.c_int, [_c_uint32_p, ctypes.c_int, ctypes.c_uint32,
                                     ctypes.c_double, _c_double_p]),
    "nmc_debug_stamps": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]),
    "nmc_debug_softplus": (ctypes.c_int, [_c_double_p, ctypes.c_int, _c_double_p,
                                          ctypes.c_int]),
}

_lib = None


class NestmcError(RuntimeError):
    pass


def load():
    """Load libnestmc.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NestmcError(
            "libnestmc.so not found at %s: build it with `make -C "
            "mcmc-for-nested-data_amd/csrc` (or __graft_entry__.build())" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def check(rc):
    if rc != 0:
        raise NestmcError(load().nmc_last_error().decode())


def device_count():
    n = ctypes.c_int(0)
    check(load().nmc_device_count(ctypes.byref(n)))
    return n.value


def dptr(a):
    """double* of a C-contiguous float64 array (or None)."""
    if a is None:
        return None
    assert a.dtype == numpy.float64 and a.flags["C_CONTIGUOUS"], (a.dtype, a.flags)
    return a.ctypes.data_as(_c_double_p)


def as_f64(a):
    return numpy.ascontiguousarray(a, dtype=numpy.float64)


def version():
    return load().nmc_version().decode()
