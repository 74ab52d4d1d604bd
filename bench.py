#!/usr/bin/env python3
"""Headline benchmark: wideband TOAs/s for a phase+DM fit, 64 chan x 2048 bin, fp64.

One step = the whole hot path over one batch of synthetic subints already
resident in HBM: per-channel rfft + noise + cross-spectrum (k_data_xspec),
the get_TOAs initial guess (k_guess: dedispersed average, brute force Ns=100,
Nelder-Mead), Taylor moments of the cross-spectrum (k_moments) and the
trust-ncg fit on them (k_fit_taylor) -- or, for scattering fits, the exact
sweeps of k_solve -- and the post-fit (k_post: zero-covariance frequency,
phi at nu_out, Woodbury covariance, snr, chi2), then the per-TOA results
copied to the host.  Data: synthetic portraits from example.gmodel with
injected phi/DM and sigma=1.5 Philox noise, generated on the device before
timing.

N>1: launched by torch.distributed.run, one rank per GPU; each rank fits its
own nsub subints (weak scaling, no collective on the fit path).  value =
all ranks' TOAs / max-over-ranks time.

Also reported: roofline of the dominant kernel (HIP-event timed on the
stream it runs on) and the CPU baseline (the oracle restatement, 1 core) on a
bounded sample of the same subints, plus the sample's parity vs the oracle.
"""
import argparse
import json
import os
import sys
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
}

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6  # AMD MI355X spec, fp64 vector = fp64 matrix (not in the guide's table)
# HBM bytes per subint per kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
# passes over this same bench (tools/profile_r1.sh + tools/pmc_summary.py).
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r02_pmc_traffic.json")
KERNEL_SYMBOL = {"solve": "k_solve<false>", "data_xspec": "k_data_xspec<10>",
                 "post": "k_post<false>", "guess": "k_guess_w", "moments": "k_moments<4>",
                 "fit_taylor": "k_fit_taylor"}


def pmc_traffic(kernel, nsub, nbin, nchan, config):
    """Counter-measured HBM bytes per launch for the headline config, else None."""
    if config != "headline" or nbin != 2048 or nchan != 64 or not os.path.exists(PMC_TRAFFIC):
        return None
    rec = json.load(open(PMC_TRAFFIC))
    k = rec["kernels"].get(KERNEL_SYMBOL.get(kernel, ""))
    if k is None:
        return None
    return k["bytes_per_subint"] * nsub


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="headline", choices=sorted(CONFIGS))
    ap.add_argument("--nsub", type=int, default=None, help="subints per GPU (override)")
    ap.add_argument("--seed", type=int, default=20240917)
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="subints the 1-core oracle fits (default per config; 0: skip)")
    ap.add_argument("--cpu-procs", type=int, default=16,
                    help="processes (one per core) of the all-core CPU baseline")
    ap.add_argument("--cpu-seconds", type=float, default=24.0,
                    help="approximate CPU work (core-seconds, summed over the processes) "
                         "of the all-core leg")
    ap.add_argument("--no-timing", action="store_true", help="skip per-kernel HIP events")
    ap.add_argument("--host-stream", type=int, default=None,
                    help="also time host-resident (pinned) input streamed over PCIe in chunks "
                         "of this many subints (default: on for config gm; 0: off)")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    from pulseportraiture_amd import synth, pplib
    from pulseportraiture_amd.engine import Engine
    nsub0, nchan, nbin, flags, tau, log10_tau, gm, desc = CONFIGS[args.config]
    nsub = args.nsub or nsub0
    if args.cpu_sample is None:
        args.cpu_sample = {"headline": 150, "gm": 40, "scattering": 3}[args.config]
    eng = Engine(local if world > 1 else 0)
    dev = eng.device

    # ---- synthetic inputs, resident in HBM before timing ----
    w = synth.make_workload(nsub, nchan, nbin, seed=args.seed, sub0=rank * nsub, tau=tau,
                            gm=gm)
    data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
    model = torch.as_tensor(w.model, device=dev)
    freqs = torch.as_tensor(w.freqs, device=dev)
    P = torch.full((nsub,), w.P, dtype=torch.float64, device=dev)
    nu_fit = pplib.guess_fit_freq(w.freqs)  # SNR weights = 1
    nu = torch.full((nsub, 3), nu_fit, dtype=torch.float64, device=dev)
    tau_g = 0.0
    init_row = [0.0, w.DM0, 0.0, 0.0, 0.0]
    if flags[3]:
        # pptoas scattering guess: tau at nu_fit from the injected reference value
        tau_g = tau * (nu_fit / w.nu_ref) ** w.alpha
        init_row[3] = np.log10(tau_g) if log10_tau else tau_g
        init_row[4] = w.alpha
    init = torch.tensor([init_row] * nsub, dtype=torch.float64, device=dev)
    gtau = torch.full((nsub,), tau_g, dtype=torch.float64, device=dev) if flags[3] else None
    torch.cuda.synchronize()

    small = ["params", "param_errs", "nu_out", "red_chi2", "snr", "status", "nfev"]

    # per-TOA results come back to pinned host buffers, all copies queued on
    # the stream behind the fit and waited for once (the step's end)
    pinned = {}

    def step():
        out = eng.fit_batch(data, model, freqs, P, init, flags, nu_fit=nu, log10_tau=log10_tau,
                            guess=True, guess_Ns=100, guess_tau=gtau)
        for k in small:
            if k not in pinned:
                pinned[k] = torch.empty(out[k].shape, dtype=out[k].dtype, pin_memory=True)
            pinned[k].copy_(out[k], non_blocking=True)
        torch.cuda.current_stream().synchronize()
        return out, pinned

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
    for _ in range(args.steps):
        out, host = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_step = elapsed / args.steps * 1e3
    toas = nsub * world * args.steps
    value = toas / elapsed

    ktimes = {}
    if not args.no_timing:
        for name in ["data_xspec", "guess", "moments", "fit_taylor", "solve", "post", "model_fft"]:
            ms, n = eng.kernel_time(name)
            ktimes[name] = (ms, n)
        eng.set_timing(False)
    status = host["status"].numpy()
    nfev = host["nfev"].numpy()

    # ---- PCIe-inclusive rate: the same subints from pinned host memory,
    # copies overlapped with the fits (Engine.fit_batch_streamed); reported
    # beside value, never as value ----
    hs = args.host_stream if args.host_stream is not None else (
        max(1, nsub // 8) if args.config == "gm" else 0)
    stream = None
    if hs and rank == 0:
        if not args.no_timing:
            eng.set_timing(False)
        pinned = torch.empty(tuple(data.shape), dtype=torch.float64, pin_memory=True)
        pinned.copy_(data)

        def sstep():
            o = eng.fit_batch_streamed(pinned, model, freqs, P, init, flags, chunk=hs, nu_fit=nu,
                                       log10_tau=log10_tau, guess=True, guess_Ns=100,
                                       guess_tau=gtau)
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
                                                          np.nan_to_num(host[k].numpy()))
                                           for k in small)),
                  "note": "host-resident pinned input, H2D on a second stream overlapped with "
                          "the fits (double buffer); not `value`"}
        del pinned

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    # ---- roofline of the dominant kernel (HBM-bound passes over X) ----
    NHP = ((nbin // 2 + 1) + 7) // 8 * 8
    nharm = nbin // 2 + 1
    roof = None
    if ktimes:
        dom = max(ktimes, key=lambda k: ktimes[k][0])
        ms, n = ktimes[dom]
        avg_s = ms / 1e3 / max(n, 1)
        if dom == "solve":
            # algorithmic bytes: every objective pass streams the subint's
            # cross-spectrum once, 16 B per cell; passes = nfev.
            # The split scattering solve is a chain of k_scat_sweep /
            # k_scat_step launches per step: rate over the solve's time per step
            bytes_launch = float(np.sum(nfev)) * nchan * nharm * 16.0
            avg_s = ms / 1e3 / args.steps
            what = ("solve (k_scat_sweep + k_scat_step chain, per step): nfev passes x nchan x "
                    "nharm x 16 B of X per subint")
        elif dom == "data_xspec":
            bytes_launch = nsub * (8.0 * nchan * nbin + 16.0 * nchan * nharm)
            what = "k_data_xspec: 8 B/sample read + 16 B/cell X written"
        elif dom == "moments":
            bytes_launch = nsub * 16.0 * nchan * nharm
            what = "k_moments: 16 B/cell X read once (32 Taylor moments per channel written)"
        elif dom == "post":
            bytes_launch = nsub * nchan * nharm * 16.0
            what = "k_post: one with-scales pass over X"
        else:
            bytes_launch = nsub * nharm * 16.0 * 2
            what = "k_guess: R and mean-template spectra"
        lps = max(n / args.steps, 1.0) if dom != "solve" else 1.0
        bytes_launch /= lps  # the chunk may run as several pieces (ppf_set_pipeline)
        achieved = bytes_launch / avg_s / 1e9
        traffic = pmc_traffic(dom, nsub, nbin, nchan, args.config)
        if traffic:
            traffic /= lps
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_unit": "bytes/launch",
                "traffic_source": os.path.relpath(PMC_TRAFFIC, ROOT) if traffic else None,
                "avg_launch_ms": round(avg_s * 1e3, 4),
                "algorithmic_bytes_per_launch": bytes_launch, "bytes_model": what,
                "kernel_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in ktimes.items()},
                "kernel_launches_per_step": {k: round(v[1] / args.steps, 2) for k, v in ktimes.items()}}

    # ---- the next-largest kernels against their own bounds (only kernels
    # that did this config's work: each subint runs in exactly one solver
    # variant, the others exit at once) ----
    others = {}
    taylor = not flags[3] and tau == 0.0
    if ktimes:
        def avg_ms(k):  # per step's worth of subints (all pieces of the chunk)
            ms, n = ktimes[k]
            return ms / max(n, 1) * max(n / args.steps, 1.0)
        if taylor and ktimes.get("moments", (0, 0))[1]:
            t = avg_ms("moments") / 1e3
            # T = V (32 x nharm powers v^m) . W (nharm x 2 nchan), fp64 MFMA
            fl = nsub * 2.0 * 32 * nharm * 2 * nchan
            tf = fl / t / 1e12
            if tf <= FP64_PEAK_TFLOPS:
                others["moments"] = {"bound": "mfma-f64", "achieved_tflops": round(tf, 2),
                                     "peak_tflops": FP64_PEAK_TFLOPS,
                                     "frac": round(tf / FP64_PEAK_TFLOPS, 4),
                                     "hbm_gbs": round(nsub * 16.0 * nchan * nharm / t / 1e9, 1),
                                     "avg_launch_ms": round(avg_ms("moments"), 4)}
        if ktimes.get("data_xspec", (0, 0))[1] and roof and roof["kernel"] != "data_xspec":
            t = avg_ms("data_xspec") / 1e3
            b = nsub * (8.0 * nchan * nbin + 16.0 * nchan * nharm)
            others["data_xspec"] = {"bound": "hbm", "achieved_gbs": round(b / t / 1e9, 1),
                                    "frac": round(b / t / 1e9 / HBM_PEAK_GBS, 4)}
    if roof is not None:
        roof["other_kernels"] = others
        if roof["frac"] > 1.0:  # the timed kernel cannot have done this work
            roof["frac"] = roof["achieved"] = None
            roof["bytes_model"] += " (INVALID: above peak)"

    # ---- CPU baseline: the oracle's get_TOAs step on host cores ----
    cpu = None
    parity = None
    S = min(args.cpu_sample, nsub) if args.cpu_sample > 0 else 0
    if S:
        from oracle import cpu_baseline as CB
        from threadpoolctl import threadpool_limits
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
        procs = min(args.cpu_procs, os.cpu_count() or 1)
        per = max(1, int(round(args.cpu_seconds * S / tcpu / procs)))
        rate, n_all, t_all = CB.all_cores(procs, per, nchan, nbin, args.seed, tau, gm, flags,
                                          log10_tau, tau_g, ag, first_sub=S)
        ratio_file = os.path.join(ROOT, "tests", "golden", "timing_r2.json")
        ref_ratio = json.load(open(ratio_file)) if os.path.exists(ratio_file) else None
        cpu = {"value": round(rate, 3), "unit": "TOAs/s", "cores": procs, "kind": "port",
               "sample": "%d subints of this workload (%s, get_TOAs guess + fit + post-fit "
                         "incl. noise estimate), %d single-threaded processes x %d subints, "
                         "%.1f s wall; numpy/scipy oracle" % (n_all, args.config, procs, per,
                                                              t_all),
               "single_core": single,
               "oracle_over_reference_time": None if ref_ratio is None else
               round(ref_ratio["ratio_oracle_over_reference"], 3),
               "oracle_over_reference_source": "tests/golden/timing_r2.json (build container, "
                                               "64x2048 phase+DM, 1 thread)"}
        def gap(i, j):
            e = refs[i].param_errs[j]
            return abs(host["params"].numpy()[i, j] - refs[i].params[j]) / e if e > 0 else 0.0
        fitted = [j for j in range(5) if flags[j]]
        parity = {"sample": S, "tolerance": "1e-3 sigma (north_star)",
                  "status_match": bool(all(status[i] == refs[i].return_code for i in range(S))),
                  "max_over_sigma": {["phi", "DM", "GM", "tau", "alpha"][j]:
                                     float(max(gap(i, j) for i in range(S))) for j in fitted}}

    line = {
        "metric": "TOAs/sec (phase+DM fit, 64ch×2048bin fp64) at 1/2/4/8 MI355X"
        if args.config == "headline" else "TOAs/sec (%s)" % args.config,
        "value": round(value, 2), "unit": "TOAs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (example.gmodel template, injected phi/DM, sigma=1.5 Philox "
                "noise; generated on device)",
        "config": {"workload": desc, "nsub_per_gpu": nsub, "nchan": nchan, "nbin": nbin,
                   "fit_flags": flags, "guess_Ns": 100, "parallelism": "subint-sharded dp%d" % world},
        "status_counts": {str(k): int(v) for k, v in zip(*np.unique(status, return_counts=True))},
        "mean_nfev": float(np.mean(nfev)),
        "roofline": roof, "cpu_baseline": cpu, "parity_sample": parity,
        "host_stream": stream,
        "gpu_over_cpu": None if not cpu else round(value / cpu["value"], 1),
    }
    print(json.dumps(line))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
