#!/usr/bin/env python3
"""Timing of the split scattering solve on config 3's batch (bench.py's
synthetic subints): `eval` runs one sweep per subint (PPF_SOLVE_EVAL: f, g, H
at init), `fit` the whole trust-ncg solve.  Prints the solve kernels' HIP-
event time per call and the mean nfev.  Run it over PPF_LIB variants
(tools/build_variant.py -DPPF_PROBE_SCAT=N) to split a sweep into its parts.

usage: scat_probe.py [eval|fit] [nsub] [reps]      (GPU)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from pulseportraiture_amd.engine import Engine
    mode = sys.argv[1] if len(sys.argv) > 1 else "eval"
    nsub = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    eng = Engine(0)
    w, data, kw, _ = bench.synth_inputs(eng, "scattering", nsub, 20240917, 0)
    flags = bench.CONFIGS["scattering"][3]

    def run():
        return eng.fit_batch(data, kw["model"], kw["freqs"], kw["P"], kw["init"], flags,
                             nu_fit=kw["nu"], log10_tau=True, guess=True, guess_Ns=100,
                             guess_tau=kw["gtau"], eval_only=(mode == "eval"))
    out = run()
    torch.cuda.synchronize()
    eng.set_timing(True)
    eng.reset_kernel_times()
    for _ in range(reps):
        out = run()
    torch.cuda.synchronize()
    ms, n = eng.kernel_time("solve")
    eng.set_timing(False)
    nfev = out["nfev"].double().mean().item()
    print(json.dumps(dict(lib=os.environ.get("PPF_LIB", "default"), mode=mode, nsub=nsub,
                          solve_ms_per_call=ms / reps, launches_per_call=n / reps,
                          mean_nfev=nfev, status0=int(out["status"][0]))), flush=True)


if __name__ == "__main__":
    main()
