"""Constants shared by the golden fixtures (examples/example.par:4,8)."""
P0 = 1.0 / 345.67890123456789
DM0 = 34.56789


def zap_perturb(subints):
    """The deterministic defects make_golden_r2.gen_zap adds to the Philox
    portraits of zapA.fits (3 x 32 x 512, seed 7007): an RFI spike train, a
    noisier channel, a dead one."""
    import numpy as np
    s = subints.copy()
    s[1, 0, 5, ::37] += 9.0
    rng = np.random.default_rng(77)
    s[0, 0, 9] += rng.normal(0.0, 3.0, s.shape[-1])
    s[2, 0, 20] *= 0.02
    return s
