"""Product modules on the GPU against the reference-generated fixtures that pin them one by one
(tests/golden/make_golden.py: gen_sincnet, gen_mamba, gen_fusion run the reference's own classes of
src/models/DualStreamSEMamba.py with seeded weights):

  sincnet_encoder.npz  SincNetEncoder.forward (:238-270) output and every parameter gradient;
                       radhip.sinc.SincNetEncoder = HIP SincConv+|.|+maxpool, NHWC epilogues.
  pn_bimamba.npz       PN_BiMambas_Encoder.forward (:467-486), shared-weight flip Mamba, output, input
                       gradient and parameter gradients; the product fuses both directions in one launch.
  fusion.npz           DualStreamFusion.forward (:580-637) in BOTH time-alignment branches: nearest
                       (ratio 20/3 > 4) and linear (20/10 <= 4).

fp32 throughout (no autocast): tolerances are fp32 reassociation (1e-4 relative) except where noted."""
import numpy as np
import pytest
import torch

from seeded import seeded_fill_

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _check_grads(module, g, rtol, atol_scale, min_checked):
    n = 0
    for k, p in module.named_parameters():
        got = None if p.grad is None else p.grad.detach().double().cpu().numpy()
        if f"grad:{k}" in g:
            ref = g[f"grad:{k}"].astype(np.float64)
            assert got is not None, k
            np.testing.assert_allclose(got, ref, rtol=rtol, atol=atol_scale * np.abs(ref).max() + 1e-9, err_msg=k)
            n += 1
        elif f"gradsum:{k}" in g:
            assert got is not None, k
            s = g[f"gradsum:{k}"]
            np.testing.assert_allclose([got.sum(), (got * got).sum()], s, rtol=rtol * 10,
                                       atol=atol_scale * np.sqrt(abs(s[1])) + 1e-9, err_msg=k)
            head = g[f"gradhead:{k}"].astype(np.float64)
            np.testing.assert_allclose(got.reshape(-1)[:64], head, rtol=rtol,
                                       atol=atol_scale * np.abs(head).max() + 1e-9, err_msg=k)
            n += 1
    assert n >= min_checked, n


def test_sincnet_encoder_matches_reference_fixture(golden):
    from radhip.sinc import SincNetEncoder
    g = golden("sincnet_encoder.npz")
    enc = SincNetEncoder(sinc_channels=70)
    seeded_fill_(enc, seed=11)
    enc = enc.to(DEV).eval()
    x = torch.from_numpy(g["x"]).to(DEV)
    out = enc(x, freq_aug=False)
    np.testing.assert_allclose(out.detach().cpu().numpy(), g["out"], rtol=1e-4,
                               atol=1e-4 * np.abs(g["out"]).max())
    (out * torch.from_numpy(g["r"]).to(DEV)).sum().backward()
    _check_grads(enc, g, rtol=2e-3, atol_scale=1e-3, min_checked=40)


def test_pn_bimamba_matches_reference_fixture(golden):
    import models.DualStreamSEMamba as DS
    g = golden("pn_bimamba.npz")
    enc = DS.PN_BiMambas_Encoder(d_model=16, n_state=16)
    seeded_fill_(enc, seed=22)
    enc = enc.to(DEV)
    x = torch.from_numpy(g["x"]).to(DEV).requires_grad_(True)
    y = enc(x)
    np.testing.assert_allclose(y.detach().cpu().numpy(), g["y"], rtol=1e-4, atol=1e-5)
    (y * torch.from_numpy(g["r"]).to(DEV)).sum().backward()
    np.testing.assert_allclose(x.grad.cpu().numpy(), g["dx"], rtol=1e-4, atol=1e-5)
    _check_grads(enc, g, rtol=1e-3, atol_scale=1e-4, min_checked=15)


@pytest.mark.parametrize("branch", ["near", "lin"])
def test_fusion_both_alignment_branches_match_reference_fixture(golden, branch):
    import models.DualStreamSEMamba as DS
    g = golden("fusion.npz")
    fu = DS.DualStreamFusion(wavlm_dim=32, sinc_dim=8, out_dim=16, reduction=4)
    seeded_fill_(fu, seed=31)
    fu = fu.to(DEV).eval()
    with torch.no_grad():
        out = fu(torch.from_numpy(g["fw"]).to(DEV), torch.from_numpy(g[f"fs_{branch}"]).to(DEV))
    np.testing.assert_allclose(out.cpu().numpy(), g[f"out_{branch}"], rtol=1e-5, atol=1e-5)
