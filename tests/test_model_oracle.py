"""Oracle model and the product's host-side pieces against the reference's golden vectors (CPU)."""
import numpy as np
import pytest
import torch

from seeded import seeded_fill_


def test_oracle_model_matches_reference(golden):
    from oracle.model import OracleModel, tiny_wavlm_config
    g = golden("model_tiny.npz")
    torch.manual_seed(0)
    m = OracleModel(tiny_wavlm_config(g["wavlm_config"]), emb_size=144, num_encoders=2)
    filled = seeded_fill_(m, seed=41)
    assert len(filled) > 300
    m.eval()
    feats, logits = m(torch.from_numpy(g["x"]))
    np.testing.assert_allclose(logits.detach().numpy(), g["logits"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(feats.detach().numpy(), g["feats"], rtol=1e-4, atol=1e-5)
    (logits[:, 1].sum() - logits[:, 0].sum()).backward()
    checked = 0
    for k, p in m.named_parameters():
        if f"grad:{k}" in g:
            np.testing.assert_allclose(p.grad.numpy(), g[f"grad:{k}"], rtol=2e-3, atol=1e-6, err_msg=k)
            checked += 1
        elif f"gradsum:{k}" in g:
            gg = p.grad.numpy().astype(np.float64)
            np.testing.assert_allclose([gg.sum(), (gg * gg).sum()], g[f"gradsum:{k}"], rtol=5e-3, atol=1e-7,
                                       err_msg=k)
            checked += 1
    assert checked >= 7


def test_product_state_dict_keys_match_reference_layout(golden):
    """The product Model's state_dict keys == the oracle's (== the reference's) for the same config."""
    import models.DualStreamSEMamba as DS
    from oracle.model import OracleModel, tiny_wavlm_config
    g = golden("model_tiny.npz")
    cfg = tiny_wavlm_config(g["wavlm_config"])

    class Args:
        emb_size, num_encoders, d_state, sinc_channels, wavlm_freeze_layers = 144, 2, 16, 70, -1
        wavlm_config = dict(cfg)
    with torch.device("meta"):
        prod = DS.Model(Args(), device="cpu")
        ora = OracleModel(cfg, emb_size=144, num_encoders=2)
    pk = {k: tuple(v.shape) for k, v in prod.state_dict().items()}
    ok = {k: tuple(v.shape) for k, v in ora.state_dict().items()}
    assert pk == ok


def test_product_sinc_bank_bit_exact(golden):
    from radhip.sinc import sinc_bank
    np.testing.assert_array_equal(sinc_bank(70, 129, 16000).numpy(), golden("sinc_conv.npz")["band_pass"])
