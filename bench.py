#!/usr/bin/env python3
"""Headline benchmark: wideband TOAs/s for a phase+DM fit, 64 chan x 2048 bin, fp64.

One step = the whole hot path over one batch of synthetic subints already
resident in HBM: per-channel rfft + noise + cross-spectrum (k_data_xspec),
the get_TOAs initial guess (k_guess: dedispersed average, brute force Ns=100,
Nelder-Mead), Taylor moments of the cross-spectrum (k_moments) and the
trust-ncg fit on them (k_fit_taylor) -- or, for scattering fits, the split
exact sweeps (k_scat_sweep / k_scat_step) -- and the post-fit (k_post:
zero-covariance frequency, phi at nu_out, Woodbury covariance, snr, chi2),
then the per-TOA results copied to the host.  Steps run back to back the way
a production loop does: step k + 1 is queued before step k's results are
read (their D2H on a side stream behind step k's kernels), so a step's host
side overlaps the next step's fits.  Data: synthetic portraits from
example.gmodel with injected phi/DM and sigma=1.5 Philox noise, generated on
the device before timing.

N>1: launched by torch.distributed.run, one rank per GPU; each rank fits its
own nsub subints (weak scaling, no collective on the fit path).  value =
all ranks' TOAs / max-over-ranks time.

Beside value (N = 1, default config): the legs a caller actually gets --
``get_toas`` (GetTOAs.get_TOAs end to end on a registered 10k-subint archive,
TOA records and .tim text included; device-resident and host-resident input),
``ppalign`` (align_archives at config 5, 4096 archives x 256 x 2048,
niter 3) and ``generic_nbin`` (the fit of 2000 subints x 64 channels at
nbin 2000, not a power of two, beside the same batch at 2048).  Also
reported: the roofline of the dominant kernel (HIP-event timed on the stream
it runs on) and the CPU baseline (the oracle restatement,
one process per available host core) on a bounded sample of the same
workload, with the oracle/reference time ratio measured in the build
container per config (tests/golden/timing_r3.json).
"""
import argparse
import json
import math
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (nsub per GPU, nchan, nbin, fit_flags, tau_inj, log10_tau, gm_inj, description)
    "headline": (10000, 64, 2048, [1, 1, 0, 0, 0], 0.0, False, 0.0,
                 "config 2: 10000 subints x 64 chan x 2048 bin, phase+DM fit, fp64"),
    "scattering": (1000, 512, 1024, [1, 1, 0, 1, 1], 2e-3, True, 0.0,
                   "config 3: 1000 subints x 512 chan x 1024 bin, phase+DM+tau+alpha (log10 tau)"),
    "gm": (2000, 128, 2048, [1, 1, 1, 0, 0], 0.0, False, 0.0,
           "config 4 slice: 128 chan x 2048 bin, phase+DM+GM (per-GPU shard batch)"),
    "gm_shard": (125000, 128, 2048, [1, 1, 1, 0, 0], 0.0, False, 0.0,
                 "config 4 per-GPU shard: 125000 subints x 128 chan x 2048 bin, phase+DM+GM, "
                 "generated on the device chunk by chunk inside the timed region"),
    "gm_shard_host": (125000, 128, 2048, [1, 1, 1, 0, 0], 0.0, False, 0.0,
                      "config 4 per-GPU shard from host memory: 125000 subints x 128 chan x "
                      "2048 bin, phase+DM+GM; int16 samples (PSRFITS DATA) + DAT_SCL / "
                      "DAT_OFFS in pinned host memory, copied over PCIe, unpacked on the "
                      "device (ppf_unpack_subints) and fitted, chunk by chunk"),
    "get_toas": (10000, 64, 2048, [1, 1, 0, 0, 0], 0.0, False, 0.0,
                 "GetTOAs.get_TOAs end to end: registered 10000 x 64 x 2048 archive, "
                 "TOA records + .tim text"),
    "ppalign": (4096, 256, 2048, [1, 1, 0, 0, 0], 0.0, False, 0.0,
                "config 5: align_archives, 4096 archives x 256 chan x 2048 bin, niter 3"),
}
TIMING_KEY = {"headline": "headline", "get_toas": "headline", "gm": "gm", "gm_shard": "gm",
              "gm_shard_host": "gm",
              "scattering": "scattering", "ppalign": "ppalign"}

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6  # AMD MI355X spec, fp64 vector = fp64 matrix (not in the guide's table)
# HBM bytes per launch per kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
# passes over this same bench (tools/profile_r03.sh + tools/pmc_summary.py)
PMC_TRAFFIC = {c: os.path.join(ROOT, "profiles", "%s_pmc_traffic_%s.json" % (r, c))
               for c, r in (("headline", "r06"), ("scattering", "r06"), ("gm", "r06"),
                            ("ppalign", "r06"))}
KERNEL_SYMBOL = {"solve": "k_scat_sweep", "data_xspec": "k_data_xspec<10>",
                 "rot_accum": "k_rot_accum_w",
                 "post": "k_post<false>", "guess": "k_guess_w", "moments": "k_moments<4, false>",
                 "fit_taylor": "k_fit_taylor<true, false>"}
# ppalign with the data-spectrum cache (ppalign.SPEC_CACHE): the rotate-and-sum
# and the fit read the cached spectra
KERNEL_SYMBOL_PPALIGN = dict(KERNEL_SYMBOL, rot_accum="k_rot_accum_spec",
                             fit_taylor="k_fit_taylor<true, true>", guess="k_guess")
# align_archives calls in one `bench.py --config ppalign` run (warm-up, two
# timed, one with kernel timing): PMC bytes per call = all launches / this
PPALIGN_CALLS = 4
# fp64 operations of one scattering cell evaluation as cells_scat forms them
# (ppfit_fit.hip: phasor step 6, W 6, B 13, f 8, g1 9, three conjugate
# products 18, ten accumulations 30; the hardware reciprocal not counted)
SCAT_FLOPS_PER_CELL = 90.0


def pmc_traffic(kernel, nsub, config, per_step=False, per_call=False):
    """Counter-measured HBM bytes per subint x nsub for this config, else None.
    per_step: all the kernel's launches of the PMC run (one step, bench
    --steps 1 --warmup 0) scaled to nsub, for kernels launched many times a
    step.  per_call (ppalign): all launches / PPALIGN_CALLS, scaled."""
    f = PMC_TRAFFIC.get(config)
    if f is None or not os.path.exists(f):
        return None
    rec = json.load(open(f))
    sym = (KERNEL_SYMBOL_PPALIGN if config == "ppalign" else KERNEL_SYMBOL).get(kernel, "")
    k = rec["kernels"].get(sym)
    if k is None:
        return None
    if per_call:
        return k["bytes_all_launches"] / PPALIGN_CALLS * nsub / rec["nsub"]
    if per_step:
        return k["bytes_all_launches"] * nsub / rec["nsub"] if "bytes_all_launches" in k else None
    return k["bytes_per_subint"] * nsub


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="headline", choices=sorted(CONFIGS))
    ap.add_argument("--nsub", type=int, default=None, help="subints per GPU (override)")
    ap.add_argument("--seed", type=int, default=20240917)
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="subints the 1-core oracle fits (default per config; 0: skip)")
    ap.add_argument("--cpu-procs", type=int, default=None,
                    help="processes of the all-core CPU baseline (default: every core of "
                         "os.sched_getaffinity within the cgroup CPU quota)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU work per process of the all-core leg (s)")
    ap.add_argument("--no-timing", action="store_true", help="skip per-kernel HIP events")
    ap.add_argument("--no-legs", action="store_true",
                    help="headline only: skip the get_toas / ppalign legs")
    ap.add_argument("--shard-chunk", type=int, default=None,
                    help="gm_shard: subints generated and fitted per chunk (default 25000); "
                         "gm_shard_host: subints copied, unpacked and fitted per chunk "
                         "(default 16384: 8 GiB of int16 samples)")
    ap.add_argument("--ppalign-narch", type=int, default=4096)
    ap.add_argument("--ppalign-niter", type=int, default=3)
    ap.add_argument("--no-spec-cache", action="store_true",
                    help="--config ppalign: align without the data-spectrum cache (A/B)")
    ap.add_argument("--host-stream", type=int, default=None,
                    help="also time host-resident (pinned) input streamed over PCIe in chunks "
                         "of this many subints (default: on for config gm; 0: off)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="libppfit launch-schedule option (ppf_set_option, _lib.OPTIONS); "
                         "no option changes a result")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: every rank runs the timing and "
                         "reduction code around a no-op step over gloo (tests only; the line "
                         "says so and is not a measurement)")
    return ap.parse_args()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """--gpus N > 1 outside a torch.distributed launch: start N ranks of this
    same command through torch.distributed.run (one process per GPU, rank i
    on device LOCAL_RANK = i) as a child process -- before anything here has
    touched the GPU -- and return its exit code.  Rank 0 prints the line."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % args.gpus, "--master-addr=127.0.0.1",
           "--master-port=%d" % free_port(), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def dist_times(elapsed, world, device=None):
    """(max over ranks, every rank's time) of one timed region."""
    if world == 1:
        return elapsed, [elapsed]
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    every = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(every, t)
    every = [float(x.item()) for x in every]
    return max(every), every


def main_dry_run(args):
    """--dry-run: the rank / barrier / max-over-ranks / JSON-line path of a
    multi-rank run without a device (gloo on the CPU), each step a no-op."""
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo")
    nsub = args.nsub or CONFIGS[args.config][0]
    for _ in range(args.warmup):
        pass
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001)
    if world > 1:
        dist.barrier()
    elapsed, every = dist_times(time.perf_counter() - t0, world)
    pids = [None] * world
    if world > 1:
        dist.all_gather_object(pids, (rank, os.getpid()))
    else:
        pids = [(0, os.getpid())]
    if rank == 0:
        print(json.dumps({"metric": "dry run (launcher check, no device)", "value": None,
                          "unit": "TOAs/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
                          "rank_ms_per_step": [t / args.steps * 1e3 for t in every],
                          "higher_is_better": True, "scaling": "weak", "data": "none (dry run)",
                          "config": {"workload": args.config, "nsub_per_gpu": nsub,
                                     "parallelism": "subint-sharded dp%d" % world},
                          "rank_pids": pids}))
    if world > 1:
        dist.destroy_process_group()


def host_cores():
    """(cores to use, affinity count, cgroup quota in cores or None)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(p)
    except (OSError, ValueError):
        pass
    n = aff if quota is None else max(1, min(aff, int(math.floor(quota))))
    return n, aff, quota


def timing_ratio(config):
    f = os.path.join(ROOT, "tests", "golden", "timing_r3.json")
    if not os.path.exists(f):
        return None
    rec = json.load(open(f)).get(TIMING_KEY.get(config, config))
    return None if rec is None else rec["ratio_oracle_over_reference"]


def synth_inputs(eng, config, nsub, seed, sub0):
    """Synthetic subints of a config on the device + the fit arguments."""
    import torch
    from pulseportraiture_amd import synth, pplib
    _, nchan, nbin, flags, tau, log10_tau, gm, _ = CONFIGS[config]
    dev = eng.device
    w = synth.make_workload(nsub, nchan, nbin, seed=seed, sub0=sub0, tau=tau, gm=gm)
    data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
    nu_fit = pplib.guess_fit_freq(w.freqs)  # SNR weights = 1
    tau_g = 0.0
    init_row = [0.0, w.DM0, 0.0, 0.0, 0.0]
    if flags[3]:
        # pptoas scattering guess: tau at nu_fit from the injected reference value
        tau_g = tau * (nu_fit / w.nu_ref) ** w.alpha
        init_row[3] = np.log10(tau_g) if log10_tau else tau_g
        init_row[4] = w.alpha
    kw = dict(model=torch.as_tensor(w.model, device=dev),
              freqs=torch.as_tensor(w.freqs, device=dev),
              P=torch.full((nsub,), w.P, dtype=torch.float64, device=dev),
              init=torch.tensor([init_row] * nsub, dtype=torch.float64, device=dev),
              nu=torch.full((nsub, 3), nu_fit, dtype=torch.float64, device=dev),
              gtau=torch.full((nsub,), tau_g, dtype=torch.float64, device=dev)
              if flags[3] else None)
    return w, data, kw, tau_g


# ---------------------------------------------------------------------------
# legs beside value: get_TOAs end to end, align_archives at config 5
# ---------------------------------------------------------------------------
def leg_get_toas(eng, w, data, reps=3, host=False):
    """GetTOAs(...).get_TOAs() + write_TOAs(gt.TOA_list, outfile=...) (the
    reference's own use, examples/example.py:140) on a registered archive
    holding the bench's own subints (device tensor, or host numpy for the
    PCIe-inclusive variant)."""
    import torch
    from pulseportraiture_amd import archive, pplib, pptoas, synth
    from pulseportraiture_amd.mjd import MJD
    nsub = data.shape[0]
    sub = data.cpu().numpy()[:, None] if host else data[:, None]
    name = "bench_get_toas_host" if host else "bench_get_toas"
    archive.register_archive(name, dict(
        subints=sub, freqs=w.freqs, Ps=np.full(nsub, w.P), DM=w.DM0, telescope="GBT",
        telescope_code="gb", backend="bench", frontend="synth",
        epochs=[MJD(57000, int(30 * k), 0.0) for k in range(nsub)]))
    times = []
    gt = None
    tim = os.path.join(tempfile.gettempdir(), "bench_get_toas_%d.tim" % os.getpid())
    for r in range(reps + 1):  # the first call is the warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gt = pptoas.GetTOAs([name], synth.EXAMPLE_GMODEL, quiet=True)
        gt.get_TOAs(quiet=True)
        pplib.write_TOAs(gt.TOA_list, SNR_cutoff=0.0, outfile=tim, append=False)  # example.py:140
        t1 = time.perf_counter()
        if r:
            times.append(t1 - t0)
    archive.unregister_archive(name)
    with open(tim) as f:
        nlines = sum(1 for _ in f)
    os.unlink(tim)
    t = float(np.median(times))
    out = {"value": round(nsub / t, 1), "unit": "TOAs/s", "ms_per_call": round(t * 1e3, 2),
           "calls": reps, "tim_lines": nlines,
           "input": "host numpy, streamed through pinned buffers (PCIe-inclusive)" if host
           else "device tensor (HBM-resident)"}
    return out, gt


def leg_generic_nbin(eng, seed, nsub=2000, nchan=64, nbin=2000, reps=3):
    """The fit at an nbin that is not a power of two (ppfit_generic.hip: the
    row rfft as a GEMM on the fp64 matrix cores), beside the same batch at
    the next power of two.  Synthetic: the template rotated per subint
    (ppf_rotate_rows) plus Gaussian noise."""
    import torch
    from pulseportraiture_amd import synth
    out = {"nsub": nsub, "nchan": nchan}
    for nb in (nbin, 1 << (nbin - 1).bit_length()):
        w = synth.make_workload(1, nchan, nb, seed=seed + nb)
        g = torch.Generator(device="cuda").manual_seed(seed)
        ph = torch.rand(nsub, 1, generator=g, device="cuda", dtype=torch.float64) * 0.2 - 0.1
        model = torch.as_tensor(w.model, device="cuda")
        data = eng.rotate_rows(model.expand(nsub, nchan, nb).reshape(-1, nb).contiguous(),
                               ph.expand(nsub, nchan).reshape(-1)).reshape(nsub, nchan, nb)
        data += 1.5 * torch.randn(data.shape, generator=g, device="cuda", dtype=torch.float64)
        nu = float(np.mean(w.freqs))
        args = (data, w.model, w.freqs, w.P, [0.0, w.DM0, 0, 0, 0], [1, 1, 0, 0, 0])
        eng.fit_batch(*args, nu_fit=[nu] * 3, guess=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            res = eng.fit_batch(*args, nu_fit=[nu] * 3, guess=True)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
        ok = int((res["status"] >= 0).sum().item())
        key = "nbin_%d" % nb
        out[key] = {"ms_per_batch": round(t * 1e3, 3), "value": round(nsub / t, 1),
                    "unit": "TOAs/s", "fits_with_status": ok}
        del data
    return out


def leg_ppalign(eng, narch, niter, seed):
    """align_archives over narch registered single-subint archives of config
    5's shape (views of one device tensor), niter iterations."""
    import torch
    from pulseportraiture_amd import archive, ppalign, synth
    _, nchan, nbin, _, _, _, _, _ = CONFIGS["ppalign"]
    w = synth.make_workload(narch, nchan, nbin, seed=seed + 555)
    data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
    torch.cuda.synchronize()
    # registered together (one metadata stack over views of one device tensor)
    names = ["bench_pa_%d" % i for i in range(narch)]
    archive.register_archives(names, [dict(subints=data[i:i + 1, None], freqs=w.freqs, Ps=[w.P],
                                           epochs=[(57000 + i, 0, 0.0)], DM=w.DM0)
                                      for i in range(narch)])
    # the initial guess: the template itself, already dedispersed (dmc = 1)
    archive.register_archive("bench_pa_guess", dict(subints=w.model[None, None], freqs=w.freqs,
                                                    Ps=[w.P], epochs=[(57000, 0, 0.0)],
                                                    DM=w.DM0, dmc=1))
    # warm-up: the same call (device workspace and the caching allocator
    # reach their steady-state sizes outside the timed calls)
    ppalign.align_archives(names, "bench_pa_guess", fit_dm=True, niter=niter, quiet=True)
    calls = []
    for _ in range(2):  # the reported time is the faster of two timed calls
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        port = ppalign.align_archives(names, "bench_pa_guess", fit_dm=True, niter=niter,
                                      quiet=True)
        torch.cuda.synchronize()
        calls.append(time.perf_counter() - t0)
    t = min(calls)
    # the same call again with a synchronisation at every phase boundary and
    # HIP events around every kernel launch (diagnostic split of the time
    # above, and the roofline's kernel times; not the timed call)
    phases = {}
    eng.set_timing(True)
    eng.reset_kernel_times()
    ppalign.align_archives(names, "bench_pa_guess", fit_dm=True, niter=niter, quiet=True,
                           timings=phases)
    ktimes = {k: eng.kernel_time(k) for k in ("data_xspec", "rot_accum", "guess", "fit_taylor",
                                              "post", "noise", "irfft")}
    eng.set_timing(False)
    for nm in names + ["bench_pa_guess"]:
        archive.unregister_archive(nm)
    del data
    return {"value": round(narch * niter / t, 1), "unit": "archive-iterations/s",
            "s_per_call": round(t, 3), "s_per_call_each": [round(c, 3) for c in calls],
            "narch": narch, "niter": niter,
            "ms_per_iteration": round(t / niter * 1e3, 2),
            "data_gb": round(narch * nchan * nbin * 8 / 1e9, 2),
            "template_finite": bool(np.isfinite(port).all()),
            "phase_s": {k: round(v, 4) for k, v in phases.items() if k != "start"},
            "kernel_ms_per_iteration": {k: round(v[0] / niter, 4) for k, v in ktimes.items()},
            "kernel_launches": {k: v[1] for k, v in ktimes.items()},
            "_ktimes": ktimes,
            "workload": "config 5: %d archives x 1 subint x %d chan x %d bin, fit_dm, niter %d; "
                        "archives registered once beforehand (register_archives); opening "
                        "them and the unit stack inside the timed call"
                        % (narch, nchan, nbin, niter)}


# ---------------------------------------------------------------------------
# CPU baseline: the oracle on the host cores
# ---------------------------------------------------------------------------
def cpu_baseline(args, config, data, w, flags, log10_tau, tau_g, host, S):
    from oracle import cpu_baseline as CB
    from threadpoolctl import threadpool_limits
    _, nchan, nbin, _, tau, _, gm, _ = CONFIGS[config]
    dh = data[:S].cpu().numpy()
    refs = []
    ag = w.alpha if flags[3] else 0.0
    with threadpool_limits(limits=1):  # one core: pin BLAS/OpenMP pools
        t0 = time.perf_counter()
        for i in range(S):
            refs.append(CB.fit_subint(dh[i], w, flags, log10_tau, tau_g, ag))
        tcpu = time.perf_counter() - t0
    single = {"value": round(S / tcpu, 3), "unit": "TOAs/s", "cores": 1,
              "sample": "%d of the bench's own subints in %.1f s" % (S, tcpu)}
    cores, aff, quota = host_cores()
    procs = args.cpu_procs or cores
    per = max(1, int(math.ceil(args.cpu_seconds * S / tcpu)))
    rate, n_all, t_all = CB.all_cores(procs, per, nchan, nbin, args.seed, tau, gm, flags,
                                      log10_tau, tau_g, ag, first_sub=S)
    ratio = timing_ratio(config)
    cpu = {"value": round(rate, 3), "unit": "TOAs/s", "cores": procs, "kind": "port",
           "sample": "%d subints of this workload (%s, get_TOAs guess + fit + post-fit incl. "
                     "noise estimate): %d single-threaded processes x %d subints (>= %.0f s of "
                     "work each), %.1f s wall; numpy/scipy oracle"
                     % (n_all, config, procs, per, args.cpu_seconds, t_all),
           "host_cores": {"affinity": aff, "cgroup_quota": quota, "used": procs},
           "single_core": single,
           "oracle_over_reference_time": None if ratio is None else round(ratio, 3),
           "oracle_over_reference_source": "tests/golden/timing_r3.json (build container, "
                                           "same subints, 1 thread, config %s)"
                                           % TIMING_KEY[config],
           "reference_equivalent_value": None if ratio is None else round(rate * ratio, 3)}

    def gap(i, j):
        e = refs[i].param_errs[j]
        return abs(host["params"][i, j] - refs[i].params[j]) / e if e > 0 else 0.0
    fitted = [j for j in range(5) if flags[j]]
    parity = {"sample": S, "tolerance": "1e-3 sigma (north_star)",
              "status_match": bool(all(host["status"][i] == refs[i].return_code
                                       for i in range(S))),
              "max_over_sigma": {["phi", "DM", "GM", "tau", "alpha"][j]:
                                 float(max(gap(i, j) for i in range(S))) for j in fitted}}
    return cpu, parity


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.dry_run:
        return main_dry_run(args)
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    from pulseportraiture_amd.engine import Engine
    import pulseportraiture_amd.engine as E
    config = args.config
    nsub0, nchan, nbin, flags, tau, log10_tau, gm, desc = CONFIGS[config]
    nsub = args.nsub or nsub0
    fit_config = "headline" if config == "get_toas" else config
    if args.cpu_sample is None:
        args.cpu_sample = {"headline": 150, "gm": 60, "scattering": 4, "get_toas": 0,
                           "ppalign": 0, "gm_shard": 16, "gm_shard_host": 16}[config]
    eng = Engine(local if world > 1 else 0)
    E._engines[eng.device.index] = eng  # the drivers' get_engine() uses this context
    for o in args.opt:
        k, v = o.split("=")
        eng.set_option(k, int(v))

    if config == "ppalign":
        return main_ppalign(args, eng, rank, world)
    if config == "gm_shard":
        return main_gm_shard(args, eng, rank, world)
    if config == "gm_shard_host":
        return main_gm_shard_host(args, eng, rank, world)

    # ---- synthetic inputs, resident in HBM before timing ----
    w, data, kw, tau_g = synth_inputs(eng, fit_config, nsub, args.seed, rank * nsub)
    torch.cuda.synchronize()
    small = ["params", "param_errs", "nu_out", "red_chi2", "snr", "status", "nfev"]
    from pulseportraiture_amd.engine import results_to_host_async
    side = torch.cuda.Stream(eng.device)

    def submit():
        out = eng.fit_batch(data, kw["model"], kw["freqs"], kw["P"], kw["init"], flags,
                            nu_fit=kw["nu"], log10_tau=log10_tau, guess=True, guess_Ns=100,
                            guess_tau=kw["gtau"])
        # the per-TOA results on their way to the host: one D2H of the packed
        # span that holds them (plus nfev / status) on a side stream, behind
        # this call's kernels only
        return out, results_to_host_async(out, small, eng.stream, side)

    def step():
        out, pend = submit()
        return out, pend.wait()

    if config == "get_toas":
        return main_get_toas(args, eng, rank, world, w, data, step, desc)

    for _ in range(args.warmup):
        out, host = step()
    torch.cuda.synchronize()
    if not args.no_timing:
        eng.set_timing(True)
        eng.reset_kernel_times()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # steps back to back: step k + 1 is queued before step k's results are
    # read, so the host side of a step (fit_batch's set-up, the wait for the
    # results) runs while the device fits the next batch
    prev = None
    for _ in range(args.steps):
        cur = submit()
        if prev is not None:
            prev[1].wait()
        prev = cur
    out, host = prev[0], prev[1].wait()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t1 = time.perf_counter()
    elapsed, rank_times = dist_times(t1 - t0, world, eng.device)
    ms_step = elapsed / args.steps * 1e3
    toas = nsub * world * args.steps
    value = toas / elapsed

    ktimes = {}
    if not args.no_timing:
        for name in ["data_xspec", "guess", "moments", "fit_taylor", "solve", "post", "model_fft"]:
            ktimes[name] = eng.kernel_time(name)
        eng.set_timing(False)
    status, nfev = host["status"], host["nfev"]

    # ---- PCIe-inclusive rate (config gm): the same subints from pinned host
    # memory, copies overlapped with the fits; reported beside value ----
    hs = args.host_stream if args.host_stream is not None else (
        max(1, nsub // 8) if config == "gm" else 0)
    stream = None
    if hs and rank == 0:
        pin = torch.empty(tuple(data.shape), dtype=torch.float64, pin_memory=True)
        pin.copy_(data)

        def sstep():
            o = eng.fit_batch_streamed(pin, kw["model"], kw["freqs"], kw["P"], kw["init"], flags,
                                       chunk=hs, nu_fit=kw["nu"], log10_tau=log10_tau,
                                       guess=True, guess_Ns=100, guess_tau=kw["gtau"])
            return {k: o[k].to("cpu") for k in small}
        sstep()
        torch.cuda.synchronize()
        ts0 = time.perf_counter()
        hs_host = sstep()
        torch.cuda.synchronize()
        ts = time.perf_counter() - ts0
        stream = {"value": round(nsub / ts, 2), "unit": "TOAs/s", "chunk_subints": hs,
                  "ms_per_step": round(ts * 1e3, 3),
                  "input_gb": round(data.numel() * 8 / 1e9, 3),
                  "pcie_gbs": round(data.numel() * 8 / ts / 1e9, 1),
                  "same_results": bool(all(np.array_equal(np.nan_to_num(hs_host[k].numpy()),
                                                          np.nan_to_num(host[k]))
                                           for k in small)),
                  "note": "host-resident pinned input, H2D on a second stream overlapped with "
                          "the fits (double buffer); not `value`"}
        del pin

    legs = None
    if rank == 0 and world == 1 and config == "headline" and not args.no_legs:
        legs = {}
        g, gt = leg_get_toas(eng, w, data, reps=5)
        g["max_dphi_over_sigma_vs_fit_batch"] = float(np.max(
            np.abs(np.asarray(gt.phis[0]) - host["params"][:, 0]) / host["param_errs"][:, 0]))
        legs["get_toas"] = g
        legs["get_toas_host"], _ = leg_get_toas(eng, w, data, reps=1, host=True)
        legs["generic_nbin"] = leg_generic_nbin(eng, args.seed)
        legs["ppalign"] = leg_ppalign(eng, args.ppalign_narch, args.ppalign_niter, args.seed)
        from pulseportraiture_amd import ppalign as _ppa
        legs["ppalign"]["roofline"] = ppalign_roofline(
            legs["ppalign"].pop("_ktimes"), args.ppalign_narch, args.ppalign_niter,
            _ppa.SPEC_CACHE)

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    roof, others = roofline(args, config, nsub, nchan, nbin, flags, tau, ktimes, nfev)

    # ---- CPU baseline: the oracle's get_TOAs step on the host cores ----
    cpu = parity = None
    S = min(args.cpu_sample, nsub) if args.cpu_sample > 0 and world == 1 else 0
    if S:
        cpu, parity = cpu_baseline(args, config, data, w, flags, log10_tau, tau_g, host, S)

    line = {
        "metric": "TOAs/sec (phase+DM fit, 64ch×2048bin fp64) at 1/2/4/8 MI355X"
        if config == "headline" else "TOAs/sec (%s)" % config,
        "value": round(value, 2), "unit": "TOAs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
        "rank_ms_per_step": [round(t / args.steps * 1e3, 3) for t in rank_times],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (example.gmodel template, injected phi/DM, sigma=1.5 Philox "
                "noise; generated on device)",
        "config": {"workload": desc, "nsub_per_gpu": nsub, "nchan": nchan, "nbin": nbin,
                   "fit_flags": flags, "guess_Ns": 100,
                   "parallelism": "subint-sharded dp%d" % world},
        "status_counts": {str(k): int(v) for k, v in zip(*np.unique(status, return_counts=True))},
        "mean_nfev": float(np.mean(nfev)),
        "roofline": roof, "cpu_baseline": cpu, "parity_sample": parity,
        "host_stream": stream, "legs": legs,
        "gpu_over_cpu": None if not cpu else round(value / cpu["value"], 1),
    }
    print(json.dumps(line))
    if world > 1:
        torch.distributed.destroy_process_group()


def roofline(args, config, nsub, nchan, nbin, flags, tau, ktimes, nfev):
    """Dominant kernel against its bound: HBM for the streaming passes, the
    fp64 VALU peak for the scattering sweeps (config 3)."""
    nharm = nbin // 2 + 1
    if not ktimes:
        return None, None
    dom = max(ktimes, key=lambda k: ktimes[k][0])
    ms, n = ktimes[dom]
    avg_s = ms / 1e3 / max(n, 1)
    lps = max(n / args.steps, 1.0)
    if dom == "solve":
        # the split scattering solve is a chain of k_scat_sweep / k_scat_step
        # launches per step: every objective pass evaluates nchan x nharm cells
        cells = float(np.sum(nfev)) * nchan * nharm
        t = ms / 1e3 / args.steps
        flops = cells * SCAT_FLOPS_PER_CELL
        tf = flops / t / 1e12
        # each evaluation streams the subint's X row (16 B per cell from HBM;
        # the |M|^2 table, 8 B per cell, is one template shared by every
        # subint and stays in L2): both the fp64 and the HBM rate are given,
        # and `bound` is the one the solve is closer to
        xb = cells * 16.0
        gbs = xb / t / 1e9
        fp = {"achieved": round(tf, 2), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
              "frac": round(tf / FP64_PEAK_TFLOPS, 4), "algorithmic_flops_per_step": flops,
              "flops_model": "sum(nfev) x nchan x nharm cell evaluations x %.0f fp64 flops "
                             "(cells_scat)" % SCAT_FLOPS_PER_CELL}
        hb = {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_step": xb,
              "bytes_model": "sum(nfev) x nchan x nharm cells x 16 B of X"}
        hbm_first = hb["frac"] >= fp["frac"]
        main_, other = (hb, fp) if hbm_first else (fp, hb)
        roof = {"kernel": "solve (k_scat_sweep + k_scat_step chain, per step)",
                "bound": "hbm" if hbm_first else "fp64", **main_,
                "traffic": pmc_traffic(dom, nsub, config, per_step=True),
                "traffic_unit": "HBM bytes per step (all k_scat_sweep launches of the PMC run "
                                "/ its steps)",
                "avg_launch_ms": round(t * 1e3, 4),
                "secondary_bound": dict(bound="fp64" if hbm_first else "hbm", **other)}
    else:
        if dom == "data_xspec":
            b = nsub * (8.0 * nchan * nbin + 16.0 * nchan * nharm)
            what = "k_data_xspec: 8 B/sample read + 16 B/cell X written"
        elif dom == "moments":
            b = nsub * 16.0 * nchan * nharm
            what = "k_moments: 16 B/cell X read once (32 Taylor moments per channel written)"
        elif dom == "post":
            b = nsub * nchan * nharm * 16.0
            what = "k_post: one with-scales pass over X"
        else:
            b = nsub * nharm * 16.0 * 2
            what = "k_guess: R and mean-template spectra"
        b /= lps  # the chunk may run as several pieces (ppf_set_pipeline)
        achieved = b / avg_s / 1e9
        traffic = pmc_traffic(dom, nsub, config)
        if traffic:
            traffic /= lps
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_unit": "bytes/launch",
                "avg_launch_ms": round(avg_s * 1e3, 4), "algorithmic_bytes_per_launch": b,
                "bytes_model": what}
    src = PMC_TRAFFIC.get(config)
    roof["traffic_source"] = os.path.relpath(src, ROOT) if (src and roof["traffic"]) else None
    roof["kernel_ms_per_step"] = {k: round(v[0] / args.steps, 4) for k, v in ktimes.items()}
    roof["kernel_launches_per_step"] = {k: round(v[1] / args.steps, 2) for k, v in ktimes.items()}
    others = {}
    taylor = not flags[3] and tau == 0.0

    def avg_ms(k):  # per step's worth of subints (all pieces of the chunk)
        m, c = ktimes[k]
        return m / max(c, 1) * max(c / args.steps, 1.0)
    # the first moment pass: its own k_moments launch, or inside
    # k_fit_taylor<true> (default; that kernel then also runs the solver)
    mk = "moments" if ktimes.get("moments", (0, 0))[1] else "fit_taylor"
    if taylor and ktimes.get(mk, (0, 0))[1]:
        t = avg_ms(mk) / 1e3
        # T = V (32 x nharm powers v^m) . W (nharm x 2 nchan), fp64 MFMA
        fl = nsub * 2.0 * 32 * nharm * 2 * nchan
        tf = fl / t / 1e12
        others[mk] = {"bound": "mfma-f64", "achieved_tflops": round(tf, 2),
                             "peak_tflops": FP64_PEAK_TFLOPS,
                             "frac": round(tf / FP64_PEAK_TFLOPS, 4),
                             "hbm_gbs": round(nsub * 16.0 * nchan * nharm / t / 1e9, 1),
                             "hbm_frac": round(nsub * 16.0 * nchan * nharm / t / 1e9 /
                                               HBM_PEAK_GBS, 4),
                             "avg_launch_ms": round(avg_ms(mk), 4),
                             "work": "moment pass: 16 B/cell X read, 32 x nharm x 2 nchan "
                                     "fp64 MACs per subint" +
                                     (" (+ trust-ncg iterations)" if mk == "fit_taylor" else "")}
    if ktimes.get("data_xspec", (0, 0))[1] and roof["kernel"] != "data_xspec":
        t = avg_ms("data_xspec") / 1e3
        b = nsub * (8.0 * nchan * nbin + 16.0 * nchan * nharm)
        others["data_xspec"] = {"bound": "hbm", "achieved_gbs": round(b / t / 1e9, 1),
                                "frac": round(b / t / 1e9 / HBM_PEAK_GBS, 4),
                                "avg_launch_ms": round(t * 1e3, 4)}
    roof["other_kernels"] = others
    if roof["frac"] is not None and roof["frac"] > 1.0:  # the timed kernel cannot have done it
        roof["frac"] = roof["achieved"] = None
        roof["invalid"] = "above peak"
    return roof, others

def _oracle_fit(job):
    """One oracle fit (bench parity samples; spawned worker)."""
    os.environ["OMP_NUM_THREADS"] = "1"
    from threadpoolctl import threadpool_limits
    from oracle import cpu_baseline as CB
    from pulseportraiture_amd import synth
    port, nchan, nbin, seed, flags = job
    w = synth.make_workload(1, nchan, nbin, seed=seed)
    with threadpool_limits(limits=1):
        r = CB.fit_subint(port, w, flags, False, 0.0, 0.0)
    return np.asarray(r.params, dtype=float), np.asarray(r.param_errs, dtype=float), \
        int(r.return_code)


def main_gm_shard(args, eng, rank, world):
    """--config gm_shard: one GPU's whole shard of BASELINE config 4
    (1M subints x 128 x 2048 over 8 GPUs = 125,000 per GPU, 262 GB of
    input -- more than HBM), fitted phase+DM+GM in chunks.  Inside the timed
    region each chunk is generated on the device (k_synth: template, injected
    phi / DM, Philox noise -- what reading the archives would put in HBM),
    fitted, and its per-TOA results copied to pinned host memory.  Chunk
    i + 1 is generated into the other of two buffers on a second queue (its
    own libppfit context) while chunk i is fitted -- the way a reader would
    fill the next chunk during the fits; HIP events time each side.  Beside
    it, the same run times the 2,000-subint slice (--config gm's step) to
    compare per-TOA rates, and samples subints across the shard against the
    oracle."""
    import torch
    from pulseportraiture_amd import synth, pplib
    nsub0, nchan, nbin, flags, _, _, _, desc = CONFIGS["gm_shard"]
    N = args.nsub or nsub0
    C = min(args.shard_chunk or 25000, N)
    base = rank * N
    dev = eng.device
    w0 = synth.make_workload(1, nchan, nbin, seed=args.seed)
    nu_fit = pplib.guess_fit_freq(w0.freqs)
    model = torch.as_tensor(w0.model, device=dev)
    freqs = torch.as_tensor(w0.freqs, device=dev)
    starts = list(range(0, N, C))
    # chunk metadata (injected phases per channel) on the host before timing
    phases = [torch.as_tensor(synth.make_workload(min(C, N - s0), nchan, nbin, seed=args.seed,
                                                  sub0=base + s0).phase, device=dev)
              for s0 in starts]
    bufs = [torch.empty((C, nchan, nbin), dtype=torch.float64, device=dev)
            for _ in range(2 if len(starts) > 1 else 1)]
    buf = bufs[0]
    from pulseportraiture_amd.engine import Engine
    gstream = torch.cuda.Stream(dev)
    geng = Engine(dev.index)  # the generator's own context, on its own queue
    geng.bind_stream(gstream)
    P = torch.full((C,), w0.P, dtype=torch.float64, device=dev)
    init = torch.tensor([[0.0, w0.DM0, 0.0, 0.0, 0.0]] * C, dtype=torch.float64, device=dev)
    nu = torch.full((C, 3), nu_fit, dtype=torch.float64, device=dev)
    small = ["params", "param_errs", "status", "nfev"]
    host = {k: torch.empty((N,) + ((5,) if k.startswith("param") else ()),
                           dtype=torch.float64 if k.startswith("param") else torch.int32,
                           pin_memory=True) for k in small}
    rng = np.random.default_rng(args.seed + rank)
    S = max(0, args.cpu_sample) if world == 1 else 0
    samp = np.sort(rng.choice(N, size=min(S, N), replace=False)) if S else np.zeros(0, int)
    pport = torch.empty((max(len(samp), 1), nchan, nbin), dtype=torch.float64, pin_memory=True)
    stream = eng.stream
    ev = []

    def run(record):
        nb = len(bufs)
        gen = [None] * len(starts)   # (start, end) events of each chunk's generation
        done = [None] * len(starts)  # each chunk's fit (and sample copies) finished

        def generate(ci):
            s0 = starts[ci]
            n = min(C, N - s0)
            if ci >= nb:  # the buffer's previous chunk fitted
                gstream.wait_event(done[ci - nb])
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(gstream)
            geng.synth(w0.template, phases[ci], w0.sigma, args.seed, sub0=base + s0,
                       out=bufs[ci % nb][:n])
            b.record(gstream)
            gen[ci] = (a, b)

        generate(0)
        for ci, s0 in enumerate(starts):
            n = min(C, N - s0)
            b = bufs[ci % nb]
            if ci + 1 < len(starts):
                generate(ci + 1)
            stream.wait_event(gen[ci][1])
            e1, e2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e1.record(stream)
            out = eng.fit_batch(b[:n], model, freqs, P[:n], init[:n], flags, nu_fit=nu[:n],
                                guess=True, guess_Ns=100)
            e2.record(stream)
            with torch.cuda.stream(stream):
                for k in small:
                    host[k][s0:s0 + n].copy_(out[k], non_blocking=True)
                if record:
                    for j in np.flatnonzero((samp >= s0) & (samp < s0 + n)):
                        pport[j].copy_(b[int(samp[j]) - s0], non_blocking=True)
            d = torch.cuda.Event()
            d.record(stream)
            done[ci] = d
            if record:
                ev.append((gen[ci][0], gen[ci][1], e1, e2))
        torch.cuda.synchronize()

    # warm-up: one chunk (workspace and allocator at steady size)
    geng.synth(w0.template, phases[0], w0.sigma, args.seed, sub0=base, out=buf[:min(C, N)])
    torch.cuda.synchronize()
    eng.fit_batch(buf[:min(C, N)], model, freqs, P[:min(C, N)], init[:min(C, N)], flags,
                  nu_fit=nu[:min(C, N)], guess=True, guess_Ns=100)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(True)
    if world > 1:
        torch.distributed.barrier()
    t1 = time.perf_counter()
    elapsed, rank_times = dist_times(t1 - t0, world, dev)
    gen_ms = sum(a.elapsed_time(b) for a, b, _, _ in ev)
    fit_ms = sum(c.elapsed_time(d) for _, _, c, d in ev)
    status = host["status"].numpy()
    nfev = host["nfev"].numpy()
    # the 2,000-subint slice (--config gm's step) in the same process
    wS, dS, kwS, _ = synth_inputs(eng, "gm", 2000, args.seed, base)
    torch.cuda.synchronize()

    def sstep():
        return eng.fit_batch(dS, kwS["model"], kwS["freqs"], kwS["P"], kwS["init"], flags,
                             nu_fit=kwS["nu"], guess=True, guess_Ns=100)
    for _ in range(2):
        sstep()
    torch.cuda.synchronize()
    ts0 = time.perf_counter()
    for _ in range(10):
        sstep()
    torch.cuda.synchronize()
    slice_ms = (time.perf_counter() - ts0) / 10 * 1e3
    del dS, bufs, buf
    geng.close()
    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    parity = None
    if len(samp):
        import multiprocessing as mp
        jobs = [(pport[j].numpy().copy(), nchan, nbin, args.seed, flags) for j in range(len(samp))]
        # the sample's ports were generated with sub0 = their global index:
        # the oracle refits exactly those samples (CB.fit_subint: get_TOAs' guess + fit)
        with mp.get_context("spawn").Pool(min(16, len(jobs))) as pool:
            refs = pool.map(_oracle_fit, jobs)
        hp, he = host["params"].numpy(), host["param_errs"].numpy()
        gaps = {nm: float(max(abs(hp[i, j] - r[0][j]) / r[1][j] for i, r in zip(samp, refs)))
                for j, nm in enumerate(["phi", "DM", "GM"])}
        parity = {"sample": len(samp), "subints": [int(i) for i in samp],
                  "tolerance": "1e-3 sigma (north_star)", "max_over_sigma": gaps,
                  "status_match": bool(all(status[i] == r[2] for i, r in zip(samp, refs)))}
    per_toa_us = elapsed / N * 1e6
    line = {
        "metric": "TOAs/sec (config 4 per-GPU shard, phase+DM+GM, 128ch x 2048bin fp64)",
        "value": round(N * world / elapsed, 2), "unit": "TOAs/s", "n_gpus": world, "steps": 1,
        "warmup": 1, "ms_per_step": round(elapsed * 1e3, 3),
        "rank_ms_per_step": [round(t * 1e3, 3) for t in rank_times],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic, generated on device chunk by chunk inside the timed region",
        "config": {"workload": desc, "nsub_per_gpu": N, "chunk_subints": C, "chunks": len(starts),
                   "nchan": nchan, "nbin": nbin, "fit_flags": flags, "guess_Ns": 100,
                   "input_gb_per_gpu": round(N * nchan * nbin * 8 / 1e9, 1),
                   "parallelism": "subint-sharded dp%d" % world},
        "generate_ms": round(gen_ms, 2), "fit_ms": round(fit_ms, 2),
        "overlap": "chunk i + 1 generated on a second queue while chunk i is fitted "
                   "(two buffers); generate_ms / fit_ms are each side's own event time",
        "fit_only_value": round(N / (fit_ms / 1e3), 2),
        "per_toa_us": round(per_toa_us, 4), "fit_only_per_toa_us": round(fit_ms * 1e3 / N, 4),
        "slice_2000": {"ms_per_step": round(slice_ms, 3),
                       "per_toa_us": round(slice_ms * 1e3 / 2000, 4),
                       "value": round(2000 / slice_ms * 1e3, 2)},
        "fit_only_over_slice_per_toa": round(fit_ms / N / (slice_ms / 2000), 4),
        "status_counts": {str(k): int(v) for k, v in zip(*np.unique(status, return_counts=True))},
        "mean_nfev": float(np.mean(nfev)), "parity_sample": parity,
    }
    print(json.dumps(line))
    if world > 1:
        torch.distributed.destroy_process_group()


def main_gm_shard_host(args, eng, rank, world):
    """--config gm_shard_host: config 4's per-GPU shard (125,000 x 128 x
    2048) as a PSRFITS reader hands it over: the samples as int16 (PSRFITS
    DATA) with per-(subint, channel) DAT_SCL / DAT_OFFS, resident in pinned
    host memory (pptoas.py:246,343 reads every archive of the shard; the
    native reader returns DATA undecoded, psrfits.py).  Inside the timed
    region, chunk by chunk: the int16 samples and scales cross PCIe on a copy
    queue (two device buffers: chunk i + 1 copies while chunk i is unpacked
    and fitted), ppf_unpack_subints forms DATA * DAT_SCL + DAT_OFFS on the
    device, fit_batch fits phase+DM+GM with get_TOAs' guess, the per-TOA
    results go to pinned host memory.  Before timing the "archive" is made
    on the device (k_synth, as --config gm_shard) and quantised to int16.
    Reported beside the rate: the PCIe GB/s of the copies, each side's own
    event time, and a parity sample (the oracle refits the dequantised
    samples the device fitted)."""
    import torch
    from pulseportraiture_amd import synth, pplib
    nsub0, nchan, nbin, flags, _, _, _, desc = CONFIGS["gm_shard_host"]
    N = args.nsub or nsub0
    C = min(args.shard_chunk or 16384, N)
    base = rank * N
    dev = eng.device
    w0 = synth.make_workload(1, nchan, nbin, seed=args.seed)
    nu_fit = pplib.guess_fit_freq(w0.freqs)
    model = torch.as_tensor(w0.model, device=dev)
    freqs = torch.as_tensor(w0.freqs, device=dev)
    starts = list(range(0, N, C))
    f64 = dict(dtype=torch.float64, device=dev)
    # 1. the archive in host memory (before timing): each chunk generated on
    # the device, quantised to int16 with DAT_SCL / DAT_OFFS per profile as
    # PSRFITS stores it, copied to pinned host memory
    gbuf = torch.empty((C, nchan, nbin), **f64)
    hraw, t_prep = [], time.perf_counter()
    hscl = torch.empty((N, 1, nchan), dtype=torch.float64, pin_memory=True)
    hoff = torch.empty((N, 1, nchan), dtype=torch.float64, pin_memory=True)
    for ci, s0 in enumerate(starts):
        n = min(C, N - s0)
        ph = torch.as_tensor(synth.make_workload(n, nchan, nbin, seed=args.seed,
                                                 sub0=base + s0).phase, device=dev)
        x = gbuf[:n]
        eng.synth(w0.template, ph, w0.sigma, args.seed, sub0=base + s0, out=x)
        mn, mx = x.amin(-1), x.amax(-1)
        scl = (mx - mn) / 65534.0
        scl = torch.where(scl > 0, scl, torch.ones_like(scl))
        off = 0.5 * (mx + mn)
        q = x.sub_(off[..., None]).div_(scl[..., None]).round_().clamp_(-32767, 32767) \
            .to(torch.int16)
        h = torch.empty((n, 1, nchan, nbin), dtype=torch.int16, pin_memory=True)
        h.view(n, nchan, nbin).copy_(q)
        hscl[s0:s0 + n, 0].copy_(scl)
        hoff[s0:s0 + n, 0].copy_(off)
        hraw.append(h)
        del q
        print("gm_shard_host: archive chunk %d/%d in host memory (%.0f s)" % (
            ci + 1, len(starts), time.perf_counter() - t_prep), file=sys.stderr, flush=True)
    del gbuf
    torch.cuda.synchronize()
    # 2. device buffers: two int16 chunks (+ scales), one unpacked chunk
    nb = 2 if len(starts) > 1 else 1
    draw = [torch.empty((C, 1, nchan, nbin), dtype=torch.int16, device=dev) for _ in range(nb)]
    dscl = [torch.empty((C, 1, nchan), **f64) for _ in range(nb)]
    doff = [torch.empty((C, 1, nchan), **f64) for _ in range(nb)]
    fbuf = torch.empty((C, 1, nchan, nbin), **f64)
    P = torch.full((C,), w0.P, **f64)
    init = torch.tensor([[0.0, w0.DM0, 0.0, 0.0, 0.0]] * C, **f64)
    nu = torch.full((C, 3), nu_fit, **f64)
    small = ["params", "param_errs", "status", "nfev"]
    host = {k: torch.empty((N,) + ((5,) if k.startswith("param") else ()),
                           dtype=torch.float64 if k.startswith("param") else torch.int32,
                           pin_memory=True) for k in small}
    rng = np.random.default_rng(args.seed + rank)
    S = max(0, args.cpu_sample) if world == 1 else 0
    samp = np.sort(rng.choice(N, size=min(S, N), replace=False)) if S else np.zeros(0, int)
    pport = torch.empty((max(len(samp), 1), nchan, nbin), dtype=torch.float64, pin_memory=True)
    stream = eng.stream
    cstream = torch.cuda.Stream(dev)
    ev = []

    def run(record):
        copied = [None] * len(starts)  # (start, end) events of each chunk's copy
        freed = [None] * len(starts)   # each chunk's unpack done: its raw buffer is free

        def copy(ci):
            s0 = starts[ci]
            n = min(C, N - s0)
            b = ci % nb
            if ci >= nb:
                cstream.wait_event(freed[ci - nb])
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(cstream):
                a.record(cstream)
                draw[b][:n].copy_(hraw[ci], non_blocking=True)
                dscl[b][:n].copy_(hscl[s0:s0 + n], non_blocking=True)
                doff[b][:n].copy_(hoff[s0:s0 + n], non_blocking=True)
                e.record(cstream)
            copied[ci] = (a, e)

        copy(0)
        for ci, s0 in enumerate(starts):
            n = min(C, N - s0)
            b = ci % nb
            stream.wait_event(copied[ci][1])
            u0, u1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            u0.record(stream)
            eng.unpack_subints(draw[b][:n], dscl[b][:n], doff[b][:n], 0, out=fbuf[:n])
            u1.record(stream)
            freed[ci] = u1
            if ci + 1 < len(starts):
                copy(ci + 1)
            out = eng.fit_batch(fbuf[:n, 0], model, freqs, P[:n], init[:n], flags,
                                nu_fit=nu[:n], guess=True, guess_Ns=100)
            e2.record(stream)
            with torch.cuda.stream(stream):
                for k in small:
                    host[k][s0:s0 + n].copy_(out[k], non_blocking=True)
                if record:
                    for j in np.flatnonzero((samp >= s0) & (samp < s0 + n)):
                        pport[j].copy_(fbuf[int(samp[j]) - s0, 0], non_blocking=True)
            if record:
                ev.append((copied[ci][0], copied[ci][1], u0, u1, e2))
        torch.cuda.synchronize()

    # warm-up: one chunk's copy, unpack and fit (workspace, allocator, kernels)
    n0 = min(C, N)
    draw[0][:n0].copy_(hraw[0])
    dscl[0][:n0].copy_(hscl[:n0])
    doff[0][:n0].copy_(hoff[:n0])
    eng.unpack_subints(draw[0][:n0], dscl[0][:n0], doff[0][:n0], 0, out=fbuf[:n0])
    eng.fit_batch(fbuf[:n0, 0], model, freqs, P[:n0], init[:n0], flags, nu_fit=nu[:n0],
                  guess=True, guess_Ns=100)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(True)
    if world > 1:
        torch.distributed.barrier()
    t1 = time.perf_counter()
    elapsed, rank_times = dist_times(t1 - t0, world, dev)
    copy_ms = sum(a.elapsed_time(b) for a, b, _, _, _ in ev)
    unpack_ms = sum(c.elapsed_time(d) for _, _, c, d, _ in ev)
    fit_ms = sum(d.elapsed_time(e) for _, _, _, d, e in ev)
    raw_bytes = N * nchan * nbin * 2 + 2 * N * nchan * 8
    status = host["status"].numpy()
    nfev = host["nfev"].numpy()
    del draw, fbuf, hraw
    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    parity = None
    if len(samp):
        import multiprocessing as mp
        jobs = [(pport[j].numpy().copy(), nchan, nbin, args.seed, flags) for j in range(len(samp))]
        with mp.get_context("spawn").Pool(min(16, len(jobs))) as pool:
            refs = pool.map(_oracle_fit, jobs)
        hp = host["params"].numpy()
        gaps = {nm: float(max(abs(hp[i, j] - r[0][j]) / r[1][j] for i, r in zip(samp, refs)))
                for j, nm in enumerate(["phi", "DM", "GM"])}
        parity = {"sample": len(samp), "subints": [int(i) for i in samp],
                  "tolerance": "1e-3 sigma (north_star)", "max_over_sigma": gaps,
                  "status_match": bool(all(status[i] == r[2] for i, r in zip(samp, refs))),
                  "oracle_input": "the dequantised samples the device fitted"}
    line = {
        "metric": "TOAs/sec (config 4 per-GPU shard from host memory, phase+DM+GM, "
                  "128ch x 2048bin fp64)",
        "value": round(N * world / elapsed, 2), "unit": "TOAs/s", "n_gpus": world, "steps": 1,
        "warmup": 1, "ms_per_step": round(elapsed * 1e3, 3),
        "rank_ms_per_step": [round(t * 1e3, 3) for t in rank_times],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic int16 PSRFITS-style samples (DATA, DAT_SCL, DAT_OFFS) resident in "
                "pinned host memory; PCIe copies inside the timed region",
        "config": {"workload": desc, "nsub_per_gpu": N, "chunk_subints": C, "chunks": len(starts),
                   "nchan": nchan, "nbin": nbin, "fit_flags": flags, "guess_Ns": 100,
                   "host_input_gb_per_gpu": round(raw_bytes / 1e9, 2),
                   "parallelism": "subint-sharded dp%d" % world},
        "pcie_h2d_gbs": round(raw_bytes / (copy_ms / 1e3) / 1e9, 2),
        "pcie_bound_value": round(N / (copy_ms / 1e3), 2),
        "copy_ms": round(copy_ms, 2), "unpack_ms": round(unpack_ms, 2), "fit_ms": round(fit_ms, 2),
        "overlap": "chunk i + 1 copied on a second queue while chunk i is unpacked and fitted "
                   "(two device buffers); copy_ms / unpack_ms / fit_ms are each side's own "
                   "event time",
        "fit_only_value": round(N / (fit_ms / 1e3), 2),
        "per_toa_us": round(elapsed / N * 1e6, 4),
        "status_counts": {str(k): int(v) for k, v in zip(*np.unique(status, return_counts=True))},
        "mean_nfev": float(np.mean(nfev)), "parity_sample": parity,
    }
    print(json.dumps(line))
    if world > 1:
        torch.distributed.destroy_process_group()


def main_get_toas(args, eng, rank, world, w, data, step, desc):
    """--config get_toas: value = GetTOAs.get_TOAs TOAs/s on a registered
    archive of the bench's subints (device-resident), .tim text included."""
    import torch
    if world > 1:
        raise SystemExit("--config get_toas runs on one GPU (get_TOAs shards itself when "
                         "torch.distributed is initialised; see tests)")
    steps = max(1, args.steps)
    g, gt = leg_get_toas(eng, w, data, reps=steps)
    out, host = step()
    same = float(np.max(np.abs(np.asarray(gt.phis[0]) - host["params"][:, 0]) /
                        host["param_errs"][:, 0]))
    gh, _ = leg_get_toas(eng, w, data, reps=1, host=True)
    nsub = data.shape[0]
    line = {"metric": "TOAs/sec (GetTOAs.get_TOAs end to end, 64ch×2048bin phase+DM fp64)",
            "value": g["value"], "unit": "TOAs/s", "n_gpus": 1, "steps": steps, "warmup": 1,
            "ms_per_step": g["ms_per_call"], "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (example.gmodel template, injected phi/DM, sigma=1.5 Philox "
                    "noise; generated on device)",
            "config": {"workload": desc, "nsub_per_gpu": nsub, "nchan": 64, "nbin": 2048,
                       "fit_flags": [1, 1, 0, 0, 0], "guess_Ns": 100, "parallelism": "dp1"},
            "tim_lines": g["tim_lines"], "max_dphi_over_sigma_vs_fit_batch": same,
            "host_resident": gh, "roofline": None, "cpu_baseline": None}
    print(json.dumps(line))


def ppalign_roofline(kt, narch, niter, cache):
    """Roofline of one align_archives call at config 5's shape from its
    per-kernel HIP-event times kt ({kernel: (ms, launches)}): the dominant
    kernel's achieved HBM rate on its algorithmic bytes, the PMC traffic of
    the same kernel (profiles/, per call), the others beside it."""
    nchan, nbin = 256, 2048
    nharm = nbin // 2 + 1
    # algorithmic bytes of one align_archives call, per kernel.  With the
    # data-spectrum cache the data pass runs in the first iteration only
    # (reads every sample, writes the spectra D), the moment passes read D
    # (the template rows are L2 / MALL resident) and the rotate-and-sum reads
    # D; without it every iteration transforms the data twice.
    cell = 16.0 * nchan * nharm
    if cache:
        model = {"data_xspec": (narch * (8.0 * nchan * nbin + cell),
                                "k_data_xspec, first iteration: 8 B/sample read + 16 B/cell D "
                                "written"),
                 "rot_accum": (niter * narch * cell,
                               "k_rot_accum_spec: 16 B/cell D read per iteration (rotate-and-"
                               "sum, ppalign.py:202-208)"),
                 "fit_taylor": (niter * narch * cell,
                                "k_fit_taylor<true, DSP>: 16 B/cell D read per iteration "
                                "(moment pass)")}
    else:
        model = {"data_xspec": (niter * narch * (8.0 * nchan * nbin + cell),
                                "k_data_xspec: 8 B/sample read + 16 B/cell X written per "
                                "iteration"),
                 "rot_accum": (niter * narch * 8.0 * nchan * nbin,
                               "k_rot_accum_w: 8 B/sample read per iteration (rotate-and-sum, "
                               "ppalign.py:202-208)"),
                 "fit_taylor": (niter * narch * cell,
                                "k_fit_taylor<true>: 16 B/cell X read per iteration (moment "
                                "pass)")}
    kernels = {}
    for k, (b, what) in model.items():
        ms, n = kt[k]
        if not n:
            continue
        # achieved = the call's algorithmic bytes over the kernel's time in
        # the call (rot_accum's timed launches also count its small partial-
        # sum reduction; data_xspec's later-iteration launches under the
        # cache visit the non-Taylor subints only, none here)
        tr = pmc_traffic(k, narch, "ppalign", per_call=True) if cache else None
        secs = ms / 1e3
        kernels[k] = {"bound": "hbm", "achieved": round(b / secs / 1e9, 1), "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": round(b / secs / 1e9 / HBM_PEAK_GBS, 4),
                      "traffic": tr, "algorithmic_bytes_per_call": b,
                      "ms_per_call": round(ms, 4), "launches_per_call": n,
                      "avg_launch_ms": round(ms / n, 4), "bytes_model": what}
    dom = max(kernels, key=lambda k: kernels[k]["ms_per_call"]) if kernels else None
    roof = None
    if dom:
        roof = dict(kernel=dom, **kernels[dom])
        roof["traffic_unit"] = "HBM bytes per align_archives call (PMC run, all launches / calls)"
        src = PMC_TRAFFIC["ppalign"]
        roof["traffic_source"] = os.path.relpath(src, ROOT) if roof["traffic"] else None
        roof["other_kernels"] = {k: v for k, v in kernels.items() if k != dom}
    return roof


def main_ppalign(args, eng, rank, world):
    """--config ppalign: value = archive-iterations/s of align_archives at
    config 5 (4096 x 256 x 2048, niter 3)."""
    if world > 1:
        raise SystemExit("--config ppalign runs on one GPU here; align_archives shards its "
                         "units and all-reduces when torch.distributed is initialised")
    from pulseportraiture_amd import ppalign
    narch = args.nsub or args.ppalign_narch
    if args.no_spec_cache:
        ppalign.SPEC_CACHE = False
    cache = ppalign.SPEC_CACHE
    r = leg_ppalign(eng, narch, args.ppalign_niter, args.seed)
    kt = r.pop("_ktimes")
    r["spec_cache"] = cache
    roof = ppalign_roofline(kt, narch, args.ppalign_niter, cache)
    line = {"metric": "archive-iterations/sec (ppalign.align_archives, 256ch×2048bin fp64)",
            "value": r["value"], "unit": r["unit"], "n_gpus": 1, "steps": 1, "warmup": 1,
            "ms_per_step": round(r["s_per_call"] * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (example.gmodel template, injected phi/DM, sigma=1.5 Philox "
                    "noise; generated on device)",
            "config": {"workload": r["workload"], "narch": narch, "nchan": 256, "nbin": 2048,
                       "niter": args.ppalign_niter, "parallelism": "dp1"},
            "detail": r, "roofline": roof, "cpu_baseline": None}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
