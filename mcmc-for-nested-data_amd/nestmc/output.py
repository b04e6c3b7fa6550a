"""Output files and logs with the reference's names and formats.

* outputDirectory/sample/sample.<chain>.csv   header "index,chain,<names>" then
  "%i,%i,%f,..." rows (Sampler._printHeader/_printSample, posteriorSampling.py:898-905)
* outputDirectory/sample/logLikelihood.<chain>.csv   "%f,..." per recorded row (:907-909)
* outputDirectory/log/samplePosterior.log, log/mcmc.chainNN.log (:155-160, :1054-1056)
Formatting runs in the C library (nmc_write_*_csv), one host thread per chain file.
"""

import ctypes
import datetime
import logging
import os
import shutil
from concurrent.futures import ThreadPoolExecutor

import numpy

from . import _lib
from ._lib import check, dptr

_LEVELS = {"debug": logging.DEBUG, "info": logging.INFO, "warning": logging.WARNING,
           "error": logging.ERROR}


def prepare_directories(output_directory):
    """samplePosterior :149-156 -- wipes the directory like the reference."""
    if os.path.exists(output_directory):
        shutil.rmtree(output_directory)
    sample_dir = output_directory + "/sample/"
    log_dir = output_directory + "/log/"
    os.makedirs(sample_dir, exist_ok=True)
    os.makedirs(log_dir, exist_ok=True)
    return sample_dir, log_dir


def get_logger(log_file, name, level):
    """_getLogger (:1161-1182): file handler, same format; unknown level -> ValueError."""
    if level not in _LEVELS:
        raise ValueError("loggingLevel must be one of %s" % sorted(_LEVELS))
    logger = logging.getLogger(name)
    logger.setLevel(_LEVELS[level])
    for h in list(logger.handlers):       # do not accumulate handlers across calls
        if isinstance(h, logging.FileHandler) and h.baseFilename == os.path.abspath(log_file):
            logger.removeHandler(h)
    handler = logging.FileHandler(log_file)
    handler.setLevel(_LEVELS[level])
    handler.setFormatter(logging.Formatter("%(asctime)s - %(name)s - %(levelname)s\n%(message)s\n"))
    logger.addHandler(handler)
    return logger


def close_logger(logger):
    for h in list(logger.handlers):
        if isinstance(h, logging.FileHandler):
            h.close()
            logger.removeHandler(h)


def print_progress(msg):
    now = datetime.datetime.now().strftime("%Y/%m/%d %H:%M:%S")
    print(now + "\t" + msg)


def header_names(names, n_groups, partial):
    """StepMethod.header / PartialPooling.header (:640-646, :771-778)."""
    h = []
    for n in names:
        if partial:
            h += ["%s_mu" % n, "%s_sigma2" % n]
        h += ["%s[%.3i]" % (n, g) for g in range(n_groups)]
    return h


def write_sample_csvs(sample_dir, samples_raw, local_chains, global_ids, header, row_index,
                      append=False, threads=8):
    """samples_raw: [rows][cols][C_local]; writes sample.<global id>.csv per chain."""
    lib = _lib.load()
    raw = numpy.ascontiguousarray(samples_raw, dtype=numpy.float64)
    rows, cols, C = raw.shape
    idx = numpy.ascontiguousarray(row_index, dtype=numpy.int32)
    hdr = ("index,chain," + ",".join(header)).encode() if header is not None else None

    def one(k):
        c, gid = local_chains[k], global_ids[k]
        path = os.path.join(sample_dir, "sample.%i.csv" % gid).encode()
        check(lib.nmc_write_sample_csv(path, 1 if append else 0, hdr, dptr(raw), C, c, cols,
                                       idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                       rows, gid))

    n = len(local_chains)
    if threads > 1 and n > 1:
        with ThreadPoolExecutor(max_workers=threads) as ex:
            list(ex.map(one, range(n)))
    else:
        for k in range(n):
            one(k)


def append_ll_rows(sample_dir, ll_rows, global_ids):
    """ll_rows: [C_local][rows][n_obs] -> logLikelihood.<gid>.csv (append)."""
    lib = _lib.load()
    for k, gid in enumerate(global_ids):
        a = numpy.ascontiguousarray(ll_rows[k], dtype=numpy.float64)
        path = os.path.join(sample_dir, "logLikelihood.%i.csv" % gid).encode()
        check(lib.nmc_write_ll_csv(path, 1, dptr(a), a.shape[1], a.shape[0]))
