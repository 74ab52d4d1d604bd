"""CPU baseline of bench.py -- TEST / MEASUREMENT INFRASTRUCTURE ONLY.

Times the oracle's get_TOAs step (guess + fit_portrait_full + post-fit,
pptoas.py:383-530 restated in ppfit_oracle.fit_subint_pptoas) on the host
cores, one process per core with one BLAS/OpenMP thread each (BASELINE.md
"How it runs").  Workers are spawned (never forked: the bench process owns a
GPU context) and regenerate their subints from the bench's Philox seeds
before their clock starts, so only fitting is timed.
"""
import os
import time

import numpy as np


def fit_subint(port, w, flags, log10_tau, tau_guess, alpha_guess):
    from oracle import ppfit_oracle as O
    nchan = port.shape[0]
    errs = O.get_noise_PS(port, chans=True)
    return O.fit_subint_pptoas(port, w.model, w.freqs, np.ones(nchan), errs, np.ones(nchan),
                               w.P, w.DM0, flags, log10_tau=log10_tau, tau_guess=tau_guess,
                               alpha_guess=alpha_guess)


def _worker(job):
    os.environ["OMP_NUM_THREADS"] = "1"
    from threadpoolctl import threadpool_limits
    from pulseportraiture_amd import synth
    (subs, nchan, nbin, seed, tau, gm, flags, log10_tau, tau_guess, alpha_guess, barrier) = job
    ports = [synth.workload_data_host(synth.make_workload(1, nchan, nbin, seed=seed, sub0=i,
                                                          tau=tau, gm=gm))[0] for i in subs]
    w = synth.make_workload(1, nchan, nbin, seed=seed, tau=tau, gm=gm)
    with threadpool_limits(limits=1):
        fit_subint(ports[0], w, flags, log10_tau, tau_guess, alpha_guess)  # warm caches, untimed
        barrier.wait()  # every core starts fitting together
        t0 = time.time()
        for p in ports:
            fit_subint(p, w, flags, log10_tau, tau_guess, alpha_guess)
        t1 = time.time()
    return t0, t1, len(ports)


def all_cores(procs, per_proc, nchan, nbin, seed, tau, gm, flags, log10_tau, tau_guess,
              alpha_guess, first_sub=0):
    """TOAs/s of `procs` single-threaded processes fitting per_proc subints each:
    all subints / (last finish - first start), wall clock across processes."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        bar = mgr.Barrier(procs)
        jobs = [(list(range(first_sub + p * per_proc, first_sub + (p + 1) * per_proc)), nchan,
                 nbin, seed, tau, gm, list(flags), log10_tau, tau_guess, alpha_guess, bar)
                for p in range(procs)]
        with ctx.Pool(procs) as pool:
            res = pool.map(_worker, jobs)
    t0 = min(r[0] for r in res)
    t1 = max(r[1] for r in res)
    n = sum(r[2] for r in res)
    return n / (t1 - t0), n, t1 - t0
