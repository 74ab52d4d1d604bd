"""Host-streamed fitting (Engine.fit_batch_streamed): chunks copied host ->
device on a second stream while the previous chunk is fitted must give
exactly the results of one fit_batch over the device-resident batch (every
subint's fit is independent, one workgroup each)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd.engine import get_engine
    return get_engine(0)


def test_streamed_equals_resident(gpu):
    from pulseportraiture_amd import pplib, synth
    nsub, nchan, nbin = 37, 16, 256
    w = synth.make_workload(nsub, nchan, nbin, seed=4242)
    host = torch.from_numpy(synth.workload_data_host(w)).pin_memory()
    rng = np.random.default_rng(3)
    mask = (rng.random((nsub, nchan)) > 0.1).astype(np.uint8)
    mask[:, 0] = 1
    nu = np.full((nsub, 3), pplib.guess_fit_freq(w.freqs))
    init = np.tile([0.0, w.DM0, 0.0, 0.0, 0.0], (nsub, 1))
    P = np.full(nsub, w.P)
    kw = dict(nu_fit=nu, chan_mask=mask, guess=True, guess_Ns=100)
    ref = gpu.fit_batch(host.to(gpu.device), w.model, w.freqs, P, init, [1, 1, 0, 0, 0], **kw)
    got = gpu.fit_batch_streamed(host, w.model, w.freqs, P, init, [1, 1, 0, 0, 0], chunk=8, **kw)
    torch.cuda.synchronize()
    for k, v in ref.items():
        if not isinstance(v, torch.Tensor):
            continue
        assert torch.equal(torch.nan_to_num(v), torch.nan_to_num(got[k])), k
