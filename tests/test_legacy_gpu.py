"""Legacy AASIST / RawNet2 plugins on the GPU (BASELINE configs 1-2).

  * rdx_sincconv_abspool1d_fwd (RawNet2's SincConv + |.| + MaxPool1d(3)) against an fp64 conv;
  * the product plugins with seeded weights, fp32, against the reference modules' outputs, gradients
    and BatchNorm running statistics (tests/golden/legacy_*.npz from make_golden.gen_legacy), in eval
    mode and in train mode with every Dropout at p = 0;
  * the CLI end to end on RawNet2_baseline.conf (config 1: 256 train utterances, batch 32) and on
    AASIST.conf (config 2, a small subset): train one epoch, dev/eval scoring, then --eval of the saved
    weights equal to a direct forward."""
import json

import numpy as np
import pytest
import torch

from flac_writer import encode
from seeded import seeded_array, seeded_fill_

pytestmark = pytest.mark.gpu
DEV = "cuda"
LEGACY = [("AASIST", "AASIST.conf"), ("RawNet2Spoof", "RawNet2_baseline.conf")]


@pytest.mark.parametrize("C,K,L,B", [(20, 1025, 9000, 2), (7, 129, 3001, 3), (1, 65, 1000, 1), (70, 129, 5000, 2)])
def test_sincconv_abspool1d_matches_fp64_conv(C, K, L, B):
    from radhip.ops import sincconv_abspool1d
    from models.RawNet2Spoof import sinc_bank_rawnet
    w = sinc_bank_rawnet(C, K)
    x = torch.from_numpy(seeded_array(f"sp1d{C}{K}", (B, L), scale=0.3)).float()
    ref = torch.nn.functional.conv1d(x.double().unsqueeze(1), w.double().unsqueeze(1))
    ref = torch.nn.functional.max_pool1d(ref.abs(), 3).float().numpy()
    got = sincconv_abspool1d(x.to(DEV), w.to(DEV)).cpu().numpy()
    assert got.shape == ref.shape == (B, C, (L - K + 1) // 3)
    np.testing.assert_allclose(got, ref, rtol=2e-5, atol=2e-6 * np.abs(ref).max())


def _product(arch, conf, mode):
    from radhip.build import get_model, load_config
    m = get_model(load_config(conf)["model_config"], "cpu")
    seeded_fill_(m, seed=41)
    m = m.to(DEV)
    if mode == "train":
        for d in m.modules():
            if isinstance(d, torch.nn.Dropout):
                d.p = 0.0
        m.train()
    else:
        m.eval()
        if hasattr(m, "gru"):
            m.gru.train()   # MIOpen's RNN backward needs training mode; a dropout-free GRU computes the same
    return m


def _rel_l2(got, ref, floor):
    return float(np.linalg.norm(got - ref)) / (float(np.linalg.norm(ref)) + floor * np.sqrt(ref.size))


def _close_grads(m, g, mode, tol=None, tol_bn=0.15):
    """Per-tensor relative L2 error against the float64 reference gradients.

    fp32 on either device is the limit here, not the kernels: the block-0 weight gradients reduce over
    B x 24 x 21490 terms (an fp32 CPU run of the reference itself is 0.5 % off float64), and the affine
    gradients of a batch-statistics BatchNorm are sums over every position of nearly cancelling terms
    (first_bn.bias: 7.5 % for the fp32 CPU reference), hence tol_bn for those in train mode; other
    tensors behind a chain of batch-statistics BatchNorms reach 2.8 % in an fp32 CPU run (RawNet2
    fc_attention3 in train mode), hence 5 % in train mode and 1 % in eval mode (worst fp32 CPU: 0.6 %). A bias
    feeding a batch-statistics BatchNorm has an exactly-zero true gradient (float64: ~1e-13); there the
    fp32 value is the rounding residue of a sum over B x T nearly cancelling terms (MIOpen's conv bias
    gradient: up to 4e-3 of the largest gradient for RawNet2 block 2), bounded by 1e-2 of it."""
    tol = tol if tol is not None else (1e-2 if mode == "eval" else 5e-2)
    floor = 1e-5 * max(np.abs(g[k]).max() for k in list(g) if k.startswith(f"{mode}:grad:"))
    n = 0
    for k, p in m.named_parameters():
        got = None if p.grad is None else p.grad.detach().double().cpu().numpy()
        is_bn = any(q.startswith("bn") or q.endswith("_bn") for q in k.split(".")[:-1])
        t = tol_bn if mode == "train" and is_bn else tol
        if f"{mode}:grad:{k}" in g:
            ref = g[f"{mode}:grad:{k}"].astype(np.float64)
            assert got is not None, k
            if np.abs(ref).max() < 1e-4 * floor:        # exactly-zero true gradient (float64 holds ~1e-13)
                assert np.abs(got).max() < 1e3 * floor, (k, np.abs(got).max())
            else:
                assert _rel_l2(got, ref, floor) < t, (k, _rel_l2(got, ref, floor))
            n += 1
        elif f"{mode}:gradsum:{k}" in g:
            assert got is not None, k
            s = g[f"{mode}:gradsum:{k}"]
            # the plain sum cancels (its scale is the L2 norm): judged against the norm, the sum of squares
            # relatively
            assert abs(got.sum() - s[0]) < 5 * t * np.sqrt(abs(s[1])) + floor, (k, got.sum(), s[0])
            np.testing.assert_allclose((got * got).sum(), s[1], rtol=2 * t, err_msg=k)
            head = g[f"{mode}:gradhead:{k}"].astype(np.float64)
            assert _rel_l2(got.reshape(-1)[:64], head, floor) < t, k
            n += 1
        else:
            assert got is None or not np.any(got), f"{k}: gradient the reference does not have"
    return n


@pytest.mark.parametrize("mode", ["eval", "train"])
@pytest.mark.parametrize("arch,conf", LEGACY)
def test_legacy_model_matches_reference_fixture(golden, arch, conf, mode):
    g = golden(f"legacy_{arch}.npz")
    m = _product(arch, conf, mode)
    x = torch.from_numpy(seeded_array(f"{arch}.x", (2, 64600), scale=0.1).astype(np.float32)).to(DEV)
    hid, out = m(x, Freq_aug=False)
    np.testing.assert_allclose(hid.detach().cpu().numpy(), g[f"{mode}:hidden"], rtol=1e-3,
                               atol=1e-4 * np.abs(g[f"{mode}:hidden"]).max())
    np.testing.assert_allclose(out.detach().cpu().numpy(), g[f"{mode}:out"], rtol=1e-3,
                               atol=1e-4 * np.abs(g[f"{mode}:out"]).max())
    rh = torch.from_numpy(g[f"{mode}:rh"]).to(DEV)
    ro = torch.from_numpy(g[f"{mode}:ro"]).to(DEV)
    ((hid * rh).sum() + (out * ro).sum()).backward()
    n = _close_grads(m, g, mode)
    assert n >= (100 if arch == "AASIST" else 50), n
    if mode == "train":
        sd = m.state_dict()
        stats = [k for k in list(g) if k.startswith("stat:")]
        assert stats
        for k in stats:
            np.testing.assert_allclose(sd[k[5:]].cpu().numpy(), g[k], rtol=1e-4, atol=1e-6, err_msg=k)


def test_rawnet2_frontend_is_the_hip_kernel(monkeypatch):
    """The RawNet2 front end runs rdx_sincconv_abspool1d_fwd (no torch conv on the way)."""
    import radhip.ops as ops
    import models.RawNet2Spoof as R
    calls = []
    real = ops.sincconv_abspool1d
    monkeypatch.setattr(R, "sincconv_abspool1d", lambda *a, **k: calls.append(1) or real(*a, **k))
    m = _product("RawNet2Spoof", "RawNet2_baseline.conf", "eval")
    with torch.no_grad():
        m(torch.zeros(1, 64600, device=DEV))
    assert calls == [1]


# ------------------------------------------------------------------------------- CLI --------
def _write(path, n, seed):
    rng = np.random.default_rng(seed)
    x = np.clip(np.round(3000 * rng.standard_normal(n)), -32768, 32767).astype(np.int64)
    path.write_bytes(encode(x, plan=lambda f, c, b: {"kind": "verbatim"}))


def _database(root, golden, n_train):
    proto = root / "ASVspoof2019_LA_cm_protocols"
    proto.mkdir(parents=True)
    attacks = [f"A{i:02d}" for i in range(7, 20)]
    rows = {"train": [("LA_T_%07d" % i, "-" if i % 5 == 0 else "A0%d" % (1 + i % 6),
                       "bonafide" if i % 5 == 0 else "spoof") for i in range(n_train)],
            "dev": [("LA_D_%07d" % i, "-" if i % 2 == 0 else "A02", "bonafide" if i % 2 == 0 else "spoof")
                    for i in range(6)],
            "eval": [("LA_E_%07d" % i, "-", "bonafide") for i in range(2)]
            + [("LA_E_%07d" % (i + 2), a, "spoof") for i, a in enumerate(attacks)]}
    names = {"train": "train.trn", "dev": "dev.trl", "eval": "eval.trl"}
    lens = [16000, 24000, 9000, 30000]
    for split, rs in rows.items():
        d = root / f"ASVspoof2019_LA_{split}" / "flac"
        d.mkdir(parents=True)
        lines = []
        for i, (utt, att, key) in enumerate(rs):
            _write(d / f"{utt}.flac", lens[i % len(lens)], seed=sum(map(ord, utt)))
            lines.append(f"LA_00{i % 100:02d} {utt} - {att} {key}")
        (proto / f"ASVspoof2019.LA.cm.{names[split]}.txt").write_text("\n".join(lines) + "\n")
    asv = root / "ASVspoof2019_LA_asv_scores"
    asv.mkdir()
    (asv / "ASVspoof2019.LA.asv.eval.gi.trl.scores.txt").write_text(
        "\n".join(golden("eval_golden.json")["tdcf"]["asv_lines"]) + "\n")
    return rows


@pytest.mark.parametrize("conf,n_train,batch", [("RawNet2_baseline.conf", 256, None), ("AASIST.conf", 48, None)])
def test_cli_legacy_config_train_eval(tmp_path, golden, conf, n_train, batch):
    import main as cli
    from radhip import audio
    from radhip.build import get_model, load_config, load_weights
    from radhip.data import pad
    db = tmp_path / "LA"
    rows = _database(db, golden, n_train)
    cfg = load_config(conf)
    cfg.update(database_path=str(db), num_epochs=1, eval_output="eval_scores.txt")
    if batch:
        cfg["batch_size"] = batch
    stem = conf.split(".")[0]
    p = tmp_path / conf
    p.write_text(json.dumps(cfg, indent=2))
    out = tmp_path / "exp"
    cli.main(cli.parse_args(["--config", str(p), "--output_dir", str(out), "--seed", "1234"]))
    tag = out / f"LA_{stem}_ep1_bs{cfg['batch_size']}"
    for f in ("config.conf", "metric_log.txt", "eval_scores.txt", "t-DCF_EER.txt", "metrics/dev_score.txt",
              "weights/swa.pth", "weights/checkpoint_epoch_000.pth"):
        assert (tag / f).exists(), f
    lines = (tag / "eval_scores.txt").read_text().splitlines()
    assert [ln.split()[0] for ln in lines] == [u for u, _, _ in rows["eval"]]
    assert np.isfinite([float(ln.split()[3]) for ln in lines]).all()
    w = tag / "weights" / "swa.pth"
    cli.main(cli.parse_args(["--config", str(p), "--output_dir", str(out), "--eval", "--eval_model_weights",
                             str(w), "--comment", "ev"]))
    got = np.array([float(ln.split()[3]) for ln in (out / f"LA_{stem}_ep1_bs{cfg['batch_size']}_ev" /
                                                    "eval_scores.txt").read_text().splitlines()])
    m = get_model(cfg["model_config"], DEV)
    load_weights(m, w, DEV, strict=True)
    m.eval()
    paths = [db / "ASVspoof2019_LA_eval" / "flac" / f"{u}.flac" for u, _, _ in rows["eval"]]
    x = np.stack([pad(audio.read(q)[0]) for q in paths]).astype(np.float32)
    with torch.no_grad():
        _, o = m(torch.from_numpy(x).to(DEV))
    np.testing.assert_allclose(got, o[:, 1].float().cpu().numpy(), rtol=1e-4, atol=1e-5)
