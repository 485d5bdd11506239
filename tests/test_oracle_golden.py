"""The oracle (CPU restatement) against golden vectors produced by the reference itself
(tests/golden/make_golden.py). CPU only."""
import hashlib
import os
import random

import numpy as np
import pytest
import torch

from conftest import REFERENCE, reference_present
from seeded import seeded_fill_

from oracle import data as odata
from oracle import evaluation as oeval
from oracle import mamba as omamba
from oracle import rawboost as orb
from oracle import sinc as osinc


def test_sinc_filterbank_exact(golden):
    g = golden("sinc_conv.npz")
    bank = osinc.sinc_filterbank(70, 128, 16000).numpy()
    assert bank.shape == (70, 129)
    np.testing.assert_array_equal(bank, g["band_pass"])


def test_sincconv_and_pool(golden):
    g = golden("sinc_conv.npz")
    x = g["x"][:, 0]
    bank = g["band_pass"]
    conv = np.einsum("btk,ck->bct", np.lib.stride_tricks.sliding_window_view(x.astype(np.float64), 129, axis=1),
                     bank.astype(np.float64))
    np.testing.assert_allclose(conv, g["conv"], rtol=1e-4, atol=1e-6)
    pooled = osinc.sincconv_absmaxpool(x, bank, int(g["mask_lo"]), int(g["mask_hi"]))
    np.testing.assert_allclose(pooled, g["pooled_masked"], rtol=1e-4, atol=1e-6)


def test_band_mask_draw_matches_reference(golden):
    g = golden("sinc_conv.npz")
    np.random.seed(7)
    random.seed(7)
    lo, hi = osinc.draw_band_mask(70)
    assert (lo, hi) == (int(g["mask_lo"]), int(g["mask_hi"]))


def _check_grads(module, g, rtol=2e-4, atol=1e-6):
    n = 0
    for k, p in module.named_parameters():
        if f"grad:{k}" in g:
            np.testing.assert_allclose(p.grad.numpy(), g[f"grad:{k}"], rtol=rtol, atol=atol, err_msg=k)
            n += 1
        elif f"gradsum:{k}" in g:
            gg = p.grad.numpy().astype(np.float64)
            np.testing.assert_allclose([gg.sum(), (gg * gg).sum()], g[f"gradsum:{k}"], rtol=1e-3, atol=1e-6,
                                       err_msg=k)
            np.testing.assert_allclose(gg.reshape(-1)[:64], g[f"gradhead:{k}"], rtol=rtol, atol=atol, err_msg=k)
            n += 1
    return n


def test_mamba_block(golden):
    g = golden("mamba_block.npz")
    m = omamba.MambaRef(16, 16)
    seeded_fill_(m, seed=21)
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    y = m(x)
    np.testing.assert_allclose(y.detach().numpy(), g["y"], rtol=1e-5, atol=1e-6)
    (y * torch.from_numpy(g["r"])).sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), g["dx"], rtol=1e-4, atol=1e-6)
    assert _check_grads(m, g) == 9


def test_pn_bimamba(golden):
    g = golden("pn_bimamba.npz")
    enc = omamba.PNBiMambaRef(16, 16)
    seeded_fill_(enc, seed=22)
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    y = enc(x)
    np.testing.assert_allclose(y.detach().numpy(), g["y"], rtol=1e-5, atol=1e-6)
    (y * torch.from_numpy(g["r"])).sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), g["dx"], rtol=1e-4, atol=1e-6)
    assert _check_grads(enc, g) >= 13


@pytest.mark.parametrize("key", ["a1_s3", "a1_s4", "a2_s3", "a2_s4", "a3_s3", "a3_s4", "a4_s3", "a4_s4",
                                 "mix_s5", "mix_s6", "mix_s7", "mix_s8"])
def test_rawboost_bit_exact(golden, key):
    g = golden("rawboost.npz")
    seed = int(key.split("_s")[1])
    algos = [1, 2, 3, 4] if key.startswith("mix") else [int(key[1])]
    np.random.seed(seed)
    out = orb.process(g["x"].copy(), algos)
    np.testing.assert_array_equal(out, g[key])


def test_protocol_lists(golden):
    g = golden("protocol.json")
    lab, lst = odata.gen_spoof_list(g["lines_train"], is_train=True)
    assert lst == g["train"]["list"] and lab == g["train"]["labels"]
    lab, lst = odata.gen_spoof_list(g["lines_train"])
    assert lst == g["dev"]["list"] and lab == g["dev"]["labels"]
    assert odata.gen_spoof_list(g["lines_train"], is_eval=True) == g["eval"]
    assert odata.gen_spoof_list(g["lines_2021"], is_eval=True, is_2021=True) == g["df2021"]


@pytest.mark.parametrize("n", [1000, 64599, 64600, 70000])
def test_pad_index_maps(golden, n):
    g = golden("pad.npz")
    x = np.arange(n, dtype=np.float64)
    idx = odata.pad(x).astype(np.int64)
    assert hashlib.sha256(idx.tobytes()).digest() == bytes(g[f"pad_{n}_sha"])
    if n != 64600:
        np.random.seed(n)
        idx = odata.pad_random(x).astype(np.int64)
        assert hashlib.sha256(idx.tobytes()).digest() == bytes(g[f"padr_{n}_sha"])
    else:
        with pytest.raises(ValueError):
            odata.pad_random(x)


def test_eer_subsample(golden):
    g = golden("eval_golden.json")
    for name in ["B01", "B02"]:
        s = g[name]["subsample"]
        eer, thr = oeval.compute_eer(s["bona"], s["spoof"])
        assert eer == s["eer"] and thr == s["thr"]
        assert oeval.compute_eer_minflip(s["bona"], s["spoof"]) == pytest.approx(s["minflip_pct"], abs=1e-12)


@pytest.mark.skipif(not reference_present(), reason="reference score files only in the build container")
def test_eer_b01_b02_known_answers(golden):
    g = golden("eval_golden.json")
    for name, expect_pct in [("B01", 9.572028), ("B02", 8.089825)]:
        path = os.path.join(REFERENCE, f"tDCF_python_v2/scores/{name}_LA_primary_eval.txt")
        bona, spoof = [], []
        for ln in open(path):
            p = ln.split()
            (bona if p[4] == "bonafide" else spoof).append(float(p[5]))
        eer, _ = oeval.compute_eer(bona, spoof)
        assert eer == g[name]["eer"]
        assert round(eer * 100, 6) == expect_pct


def test_tdcf_synthetic(golden):
    g = golden("eval_golden.json")["tdcf"]
    cm = [ln.split() for ln in g["cm_lines"]]
    asv = [ln.split() for ln in g["asv_lines"]]
    bona = [float(p[3]) for p in cm if p[2] == "bonafide"]
    spoof = [float(p[3]) for p in cm if p[2] == "spoof"]
    tar = [float(p[2]) for p in asv if p[1] == "target"]
    non = [float(p[2]) for p in asv if p[1] == "nontarget"]
    sp = [float(p[2]) for p in asv if p[1] == "spoof"]
    assert oeval.compute_eer(bona, spoof)[0] * 100 == pytest.approx(g["eer_cm_pct"], abs=1e-12)
    assert oeval.min_tdcf(bona, spoof, tar, non, sp) == pytest.approx(g["min_tdcf"], rel=1e-12)
