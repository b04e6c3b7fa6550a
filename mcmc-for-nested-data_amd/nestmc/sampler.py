"""samplePosterior on the GPU: the reference's API and files, the device's loop.

Control flow of posteriorSampling.samplePosterior (:28-216) with the per-chain
Python hot loop (MCMC/Sampler/StepMethod, :790-1158) replaced by libnestmc:

  validate + prepare directories/logs        (:147-168, :1018-1043)
  shard chains over GPUs (contiguous blocks of global chain ids)      nestmc.parallel
  init of every chain, RandomState(c), LLs batched on its GPU
                                             (:1060-1141, :725-758)   nestmc.init
  device loop: nmc_run over all iterations   (:862-896)               nestmc.engine
  device sample store -> sample.<c>.csv      (:898-936)               nestmc.output
  optional per-observation LL rows           (:890-891, :907-909)

The product path never falls back to the CPU: a likelihood that is not a device
family (nestmc.families) or a missing GPU/library raises.
"""

import datetime
import os
from concurrent.futures import ThreadPoolExecutor

import numpy

from . import _lib
from . import output
from .engine import Engine
from .families import is_family
from .init import init_chains
from .parallel import shard


def schedule(n_iter, n_samples):
    """MCMC.__init__ burn/thin (posteriorSampling.py:1018-1027)."""
    if n_iter < n_samples:
        print("nIter (%i) cannot be less than nSamples (%i)." % (n_iter, n_samples))
        raise Exception()
    burn = n_iter // 2 if n_iter // 2 > n_samples else n_iter - n_samples
    thin = int(numpy.ceil((n_iter - burn) / n_samples))
    return burn, thin


def record_iterations(n_iter, burn, thin):
    return [i for i in range(n_iter) if i % thin == 0 and i >= burn]


def _sizes(n_groups, n_responses, pooling):
    if isinstance(n_responses, (int, numpy.integer)):
        sizes = [int(n_responses)] * n_groups
    else:
        sizes = [int(v) for v in n_responses]       # list or tuple (the reference: list only)
        if len(sizes) != n_groups:
            raise ValueError("nResponsesPerGroup needs one entry per group")
    if pooling == "complete":
        sizes = [int(sum(sizes))]                  # CompletePooling: one group (:667-671)
    return sizes


def sample_posterior(nChains, nIter, nSamples, parameterName, nGroups, nResponsesPerGroup,
                     pooling, logLikelihoodFunction, outputDirectory, saveLogLikelihood=True,
                     priorDistribution=None, startWithMLE=False, startingPointValueRange=None,
                     nProcesses=1, displayProgress=True, loggingLevel="info", *,
                     seed=0, devices=None, rng="philox", chains=None, return_samples=False,
                     write_files=True, replay=None, process_per_device=False, _rank=None):
    """Drop-in for posteriorSampling.samplePosterior (same positional/keyword API).

    Extra keyword-only options (all optional):
      seed       Philox seed (key = (global chain id, seed)); default 0
      devices    GPU ids to shard chains over (default: [0]); chains are split in
                 contiguous blocks so chain c always draws the same stream
      process_per_device  one process per GPU instead of one engine per GPU in this
                 process: this process starts len(devices) ranks (nestmc.ranks) before it
                 makes any HIP call; rank r runs its contiguous block of chains on
                 devices[r], and after the loop ONE RCCL gather brings every rank's sample
                 store to rank 0, which writes every sample file (the reference's process
                 fan-out, posteriorSampling.py:182-201, at the GPU level); the files are
                 byte-identical to the one-process path's
      rng        "philox" (default) or "replay" (test use)
      replay     rng="replay": dict of captured variates z, u [C, iter, P, G] and
                 hz, hu [C, iter, P] (chain axis = position in ``chains``)
      chains     run only these global chain ids (multi-process sharding)
      return_samples  also return {"rows": [C][rows][cols], "row_index", "header"}
    nProcesses sizes the host threads used for chain initialisation and CSV writing.
    """
    start_time = datetime.datetime.now()
    if not is_family(logLikelihoodFunction):
        raise TypeError(
            "logLikelihoodFunction must be a nestmc device family: a built-in one "
            "(nestmc.LinearRegression, GaussianMean, Logistic) or "
            "nestmc.DeviceLikelihood(obs_rows, source, n_params, consts=...) wrapping a "
            "per-observation '__device__ double nmc_user_loglik(theta, row, k)' that is "
            "compiled for the GPU at run time. A plain Python callable -- e.g. the "
            "reference examples' functools.partial(computeLogLikelihood, data=data) "
            "(example/regression.py:53-67, 91) -- cannot run on the GPU, and this sampler "
            "has no CPU fallback by design; pass the callable as "
            "DeviceLikelihood(..., host_function=callable) to keep it for host-side checks "
            "(INTEGRATION.md, 'Porting a likelihood callable').")
    if pooling not in ("partial", "none", "complete"):
        raise Exception("Invalid pooling: ", pooling)
    names = tuple(parameterName)
    if len(names) != logLikelihoodFunction.n_params:
        raise ValueError("parameterName has %d names, the likelihood family has %d parameters"
                         % (len(names), logLikelihoodFunction.n_params))
    if nProcesses is None or nProcesses <= 0:
        nProcesses = os.cpu_count() or 1
    threads = max(1, min(int(nProcesses), 64))
    if _rank is not None:
        # a rank of process_per_device: the parent prepared the directories and logs the run
        hg, world, rank = _rank
        displayProgress = displayProgress and rank == 0
        sample_dir = outputDirectory + "/sample/" if write_files else None
        log_dir = outputDirectory + "/log/" if write_files else None
        logger = None
    elif write_files:
        sample_dir, log_dir = output.prepare_directories(outputDirectory)
        logger = output.get_logger(log_dir + "samplePosterior.log", "samplePosterior",
                                   loggingLevel)
    else:
        sample_dir = log_dir = None
        logger = None
    msg = "MCMC sampling.\n\tpooling: %s.\n\tnChains: %i, nIterPerChain: %i, " \
          "nSamplesPerChain: %i." % (pooling, nChains, nIter, nSamples)
    if logger:
        logger.info(msg)
    if displayProgress:
        print(msg)

    burn, thin = schedule(nIter, nSamples)
    sizes = _sizes(nGroups, nResponsesPerGroup, pooling)
    G = len(sizes)
    priors = None
    if pooling in ("none", "complete"):
        if priorDistribution is None or len(priorDistribution) != len(names):
            raise ValueError("Invalid prior")
        priors = list(priorDistribution)
    elif priorDistribution is not None and logger:
        logger.info("Partial pooling ignores prior distribution.")
    # partial pooling still draws start values from the priors when given
    # (MCMC._findStartingPoint :1076-1077); the sampler itself ignores them (:713-715)
    start_priors = list(priorDistribution) if priorDistribution is not None else None
    if pooling == "partial" and G < 2:
        raise ValueError("partial pooling needs at least two groups (the invgamma update of "
                         "posteriorSampling.py:494-498 has shape (G-1)/2)")

    chain_ids = list(range(nChains)) if chains is None else [int(c) for c in chains]
    if (rng == "replay") != (replay is not None):
        raise ValueError("rng='replay' needs replay= variates (and only then)")
    devices = [0] if devices is None else list(devices)
    if process_per_device and _rank is None:
        # one process per GPU, started before this process makes any HIP call
        if chains is not None or replay is not None:
            raise ValueError("process_per_device runs all nChains chains on the Philox "
                             "stream (no chains= / replay=)")
        from . import ranks
        kw = dict(nChains=nChains, nIter=nIter, nSamples=nSamples, parameterName=names,
                  nGroups=nGroups, nResponsesPerGroup=nResponsesPerGroup, pooling=pooling,
                  logLikelihoodFunction=logLikelihoodFunction, outputDirectory=outputDirectory,
                  saveLogLikelihood=saveLogLikelihood, priorDistribution=priorDistribution,
                  startWithMLE=startWithMLE, startingPointValueRange=startingPointValueRange,
                  nProcesses=max(1, threads // len(devices)), displayProgress=displayProgress,
                  loggingLevel=loggingLevel, seed=seed, rng=rng,
                  return_samples=return_samples, write_files=write_files)
        res = ranks.run_per_device(kw, devices)
        _finish_log(logger, [], start_time, displayProgress)
        return res
    if _lib.device_count() < 1:
        raise _lib.NestmcError("no HIP device visible: the sampler runs on MI355X only")
    rank_info = None
    if _rank is not None:
        # this rank's padded contiguous shard (equal store sizes for the RCCL gather; chains
        # with ids >= nChains are padding, run and dropped) on its own device
        from .parallel import padded_shard
        s0, per, real = padded_shard(nChains, world, rank)
        chain_ids = list(range(s0, s0 + per))
        rank_info = dict(hg=hg, world=world, rank=rank, device=devices[rank], n_total=nChains)
        devices = [devices[rank]]
    partial = pooling == "partial"

    # ---- chain logs; initialisation (reference RNG order, RandomState(chain)) ----
    if displayProgress:
        output.print_progress("Initialising %d chains." % len(chain_ids))
    chain_logs = []
    if log_dir:
        for c in chain_ids:
            if c >= nChains:        # (a rank's padding chains)
                continue
            lg = output.get_logger(log_dir + "/mcmc.chain%.2i.log" % c, "mcmc.chain%.2i" % c,
                                   loggingLevel)
            lg.info("chain %i. Started looking for a reasonable starting state." % c)
            chain_logs.append(lg)
    # ---- shard contiguous blocks of chains over the devices; every device
    #      initialises its own chains, their likelihoods evaluated in batches on it --
    def make_engine(r, dev):
        s0, cnt = shard(len(chain_ids), len(devices), r)
        if cnt == 0:
            return None
        ids = chain_ids[s0:s0 + cnt]
        if ids != list(range(ids[0], ids[0] + cnt)):
            raise ValueError("chains must be contiguous global ids per device")
        eng = Engine(logLikelihoodFunction, sizes, cnt, pooling, priors, seed=seed,
                     chain_base=ids[0], device=dev, rng=rng)
        try:
            sl = slice(s0, s0 + cnt)
            st = init_chains(logLikelihoodFunction, sizes, names, ids, pooling, start_priors,
                             startingPointValueRange, startWithMLE,
                             threads=max(1, threads // len(devices)),
                             group_ll=eng.eval_group_ll)
            eng.set_state(st["value"], st["log_prior"], st["ll"], st["mu"], st["s2"])
            if replay is not None:
                eng.set_replay(*(numpy.asarray(replay[k])[sl] for k in ("z", "u", "hz", "hu")))
            eng.set_schedule(nIter, burn, thin, 100)
        except BaseException:
            eng.close()
            raise
        return (eng, s0, ids)

    # one host thread per engine: each initialises its chains (reference RNG order) with
    # their likelihoods batched on its own device, concurrently with the others
    if len(devices) > 1:
        with ThreadPoolExecutor(max_workers=len(devices)) as ex:
            futs = [ex.submit(make_engine, r, dev) for r, dev in enumerate(devices)]
        made, err = [], None
        for f in futs:                 # (every worker has finished: the pool has shut down)
            try:
                made.append(f.result())
            except BaseException as e:   # one device failed: release the others' engines
                err = err or e
        if err is not None:
            for m in made:
                if m is not None:
                    m[0].close()
            raise err
    else:
        made = [make_engine(0, devices[0])]
    engines = [e for e in made if e is not None]
    try:
        return _sample_loop(engines, nIter, burn, thin, names, G, partial, saveLogLikelihood,
                            write_files, sample_dir, threads, displayProgress, return_samples,
                            logger, chain_logs, start_time, rank_info)
    finally:
        for eng, _, _ in engines:
            eng.close()


def _finish_log(logger, chain_logs, start_time, displayProgress):
    elapsed = datetime.datetime.now() - start_time
    msg = "Finished. The elapsed time in total is %s." \
        % datetime.timedelta(seconds=int(elapsed.total_seconds()))
    for lg in chain_logs:
        lg.info("100% complete.")
        output.close_logger(lg)
    if logger:
        logger.info(msg)
        output.close_logger(logger)
    if displayProgress:
        print("")
        output.print_progress(msg)


def _gather_rank(engines, rank_info):
    """process_per_device: ONE ncclGather of every rank's sample store to rank 0 (RCCL over
    xGMI), the padding chains dropped -> rank 0: [rows][cols][nChains], others: None; the
    accepted counts travel over the host group (rank 0: [nChains, P, G])."""
    from . import parallel
    eng = engines[0][0]
    hg, world, rank, n = (rank_info[k] for k in ("hg", "world", "rank", "n_total"))
    comm = parallel.rccl_comm(hg, world, rank, rank_info["device"])
    try:
        full = parallel.gather_samples(eng, comm, root=0)
    finally:
        parallel.rccl_destroy(comm)
    reals = [parallel.padded_shard(n, world, r)[2] for r in range(world)]
    acc = hg.gather(numpy.ascontiguousarray(eng.accept_counts()).tobytes())
    if rank != 0:
        return None, None
    raw = parallel.assemble(full, reals)
    P, G = eng.P, eng.G
    accs = [numpy.frombuffer(a, dtype=numpy.int64).reshape(-1, P, G)[:reals[r]]
            for r, a in enumerate(acc)]
    return raw, numpy.concatenate(accs, axis=0)


def _sample_loop(engines, nIter, burn, thin, names, G, partial, saveLogLikelihood, write_files,
                 sample_dir, threads, displayProgress, return_samples, logger, chain_logs,
                 start_time, rank_info=None):
    """The device loop, the per-observation LL rows and the sample files of
    sample_posterior (the caller closes the engines whatever happens here).  rank_info: a
    rank of process_per_device -- this rank writes its chains' logLikelihood files, rank 0
    every sample file after the gather."""
    # ---- the device loop ----------------------------------------------------
    rec = record_iterations(nIter, burn, thin)
    if displayProgress:
        output.print_progress("Sampling started. 0% complete.")
    t_loop = datetime.datetime.now()
    steps = 10 if displayProgress and nIter >= 10 else 1
    bounds = [round(nIter * k / steps) for k in range(steps + 1)]
    # the progress steps' calls continue one another: each engine's calls share one resident
    # step launch (nmc_set_resident; bit-identical) when the engine has its device to itself
    devs = [eng.device for eng, _, _ in engines]
    if steps > 1 and len(set(devs)) == len(devs):
        for eng, _, _ in engines:
            eng.set_resident(True)
    for k in range(steps):
        for eng, _, _ in engines:
            eng.run(bounds[k], bounds[k + 1])
        if displayProgress and steps > 1:
            for eng, _, _ in engines:
                eng.synchronize()
            output.print_progress("%i%% complete." % (100 * (k + 1) // steps))
    for eng, _, _ in engines:
        eng.synchronize()
    loop_seconds = (datetime.datetime.now() - t_loop).total_seconds()
    n_total = None if rank_info is None else rank_info["n_total"]
    if saveLogLikelihood and write_files:
        # every recorded row's per-observation LL (:890-891, :907-909 at the values of
        # :656-659), re-evaluated on the device from the sample store and streamed out
        # (a rank's padding chains: file id -1, no file)
        for eng, _, ids in engines:
            fids = ids if n_total is None else [c if c < n_total else -1 for c in ids]
            eng.write_ll_csvs(sample_dir, fids, threads=threads)

    # ---- samples -> files ----------------------------------------------------
    header = output.header_names(names, G, partial)
    hdr = header if burn < nIter else None
    rows_all = []
    if rank_info is not None:
        raw, accept = _gather_rank(engines, rank_info)
        if raw is not None:
            if write_files:
                ids = list(range(n_total))
                output.write_sample_csvs(sample_dir, raw, ids, ids, hdr, rec, threads=threads)
            rows_all.append(numpy.transpose(raw, (2, 0, 1)))
        accept = [accept] if accept is not None else []
    else:
        for eng, s0, ids in engines:
            raw = eng.samples_raw()                     # [rows][cols][C_local]
            if write_files:
                output.write_sample_csvs(sample_dir, raw, list(range(len(ids))), ids, hdr, rec,
                                         threads=threads)
            if return_samples:
                rows_all.append(numpy.transpose(raw, (2, 0, 1)))
        accept = [eng.accept_counts() for eng, _, _ in engines] if return_samples else None

    # (a rank: the parent prints and logs the end of the run)
    _finish_log(logger, chain_logs, start_time, displayProgress and rank_info is None)
    if rank_info is not None and rank_info["rank"] != 0:
        return None
    if return_samples:
        return {"rows": numpy.concatenate(rows_all, axis=0), "row_index": rec,
                "header": header, "burn": burn, "thin": thin,
                "accepted": numpy.concatenate(accept, axis=0),
                "loop_seconds": loop_seconds}
    return None
