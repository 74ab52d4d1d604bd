"""Config-3 GetTOAs (3 subints 512 x 1024, scattering) against the reference
fixture, printing params / nu_out / nfev: for A/B of solver variants."""
import json
import os
import shutil
import sys
import tempfile

import numpy as np

sys.path.insert(0, ".")
from tests.conftest import GOLDEN  # noqa: E402
from tests.test_gpu_configs import register_synth_archive  # noqa: E402
from pulseportraiture_amd import pptoas, synth  # noqa: E402

meta = json.load(open(os.path.join(GOLDEN, "configs_r2.json")))["cfg3"]
z = np.load(os.path.join(GOLDEN, "configs_r2.npz"))
register_synth_archive("cfg3.fits", meta["nsub"], meta["nchan"], meta["nbin"], meta["seed"],
                       meta["tau"], meta["gm"])
d = tempfile.mkdtemp()
shutil.copy(synth.EXAMPLE_GMODEL, os.path.join(d, "example.gmodel"))
os.chdir(d)
gt = pptoas.GetTOAs(["cfg3.fits"], "example.gmodel", quiet=True)
gt.get_TOAs(quiet=True, **meta["kwargs"])
np.set_printoptions(precision=10)
for attr in ["phi", "DM", "tau", "alpha"]:
    got, ref, err = np.asarray(getattr(gt, attr + "s")[0]), z["cfg3_" + attr + "s"], z["cfg3_" + attr + "_errs"]
    print(attr, "dev", got, "ref", ref, "d/sigma", (got - ref) / np.where(err > 0, err, 1))
print("nu_refs dev", np.array(gt.nu_refs[0], float)[:, 0], "ref", z["cfg3_nu_refs"][:, 0])
print("nfev dev", list(gt.nfevals[0]), "ref", list(z["cfg3_nfevals"].astype(int)), "rcs", list(gt.rcs[0]))
