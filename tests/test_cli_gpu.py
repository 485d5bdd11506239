"""End-to-end CLI (main.py) on the GPU: a tiny ASVspoof-shaped database of FLAC files, one Phase-6
training epoch through the HIP path (native decode -> GPU RawBoost/codec/pad/mixup -> graphed FGM
micro-steps -> AdamW/EMA), the reference's output layout, then --eval with the saved weights and a
2021-DF eval with the codec breakdown. Scores written by the CLI must equal a direct fp32 forward of
the same weights on the reference's numpy `pad` of each file. A run resumed from the full training
state (--save_train_state / --resume) must end where the uninterrupted run ends."""
import json
import os
import shutil

import numpy as np
import pytest
import torch

from flac_writer import encode

pytestmark = pytest.mark.gpu
ATTACKS = [f"A{i:02d}" for i in range(7, 20)]


def _write_utt(path, n, seed):
    rng = np.random.default_rng(seed)
    x = np.clip(np.round(3000 * rng.standard_normal(n)), -32768, 32767).astype(np.int64)
    path.write_bytes(encode(x, plan=lambda f, c, b: {"kind": "verbatim"}))


def _database(root, golden):
    proto = root / "ASVspoof2019_LA_cm_protocols"
    proto.mkdir(parents=True)
    lens = [64000, 70000, 30000, 66000, 20000, 64000]
    rows = {"train": [("LA_T_%07d" % i, "-" if i % 3 == 0 else "A01", "bonafide" if i % 3 == 0 else "spoof")
                      for i in range(6)],
            "dev": [("LA_D_%07d" % i, "-" if i % 2 == 0 else "A02", "bonafide" if i % 2 == 0 else "spoof")
                    for i in range(4)],
            "eval": [("LA_E_%07d" % i, "-", "bonafide") for i in range(2)]
            + [("LA_E_%07d" % (i + 2), a, "spoof") for i, a in enumerate(ATTACKS)]}
    names = {"train": "train.trn", "dev": "dev.trl", "eval": "eval.trl"}
    for split, rs in rows.items():
        d = root / f"ASVspoof2019_LA_{split}" / "flac"
        d.mkdir(parents=True)
        lines = []
        for i, (utt, att, key) in enumerate(rs):
            _write_utt(d / f"{utt}.flac", lens[i % len(lens)], seed=sum(map(ord, utt)))
            lines.append(f"LA_00{i:02d} {utt} - {att} {key}")
        (proto / f"ASVspoof2019.LA.cm.{names[split]}.txt").write_text("\n".join(lines) + "\n")
    asv = root / "ASVspoof2019_LA_asv_scores"
    asv.mkdir()
    (asv / "ASVspoof2019.LA.asv.eval.gi.trl.scores.txt").write_text("\n".join(golden("eval_golden.json")["tdcf"]["asv_lines"]) + "\n")
    return rows


def _config(tmp_path, golden, db):
    import main as cli  # noqa: F401  (puts the package on sys.path)
    from radhip.build import load_config
    cfg = load_config("Phase6_Proposed.conf")
    g = golden("model_tiny.npz")
    cfg["database_path"] = str(db)
    cfg["num_epochs"] = 1
    cfg["batch_size"] = 2
    cfg["eval_output"] = "eval_scores.txt"
    cfg["auto_eval_2021_df"] = False
    cfg["test_config"] = {"batch_size": 4, "num_workers": 0}
    cfg["training_config"]["accumulation_steps"] = 2
    cfg["model_config"]["num_encoders"] = 2
    cfg["model_config"]["wavlm_config"] = json.loads(str(g["wavlm_config"]))
    p = tmp_path / "Tiny.conf"
    p.write_text(json.dumps(cfg, indent=2))
    return p, cfg


def _direct_scores(cfg, weights, paths):
    from radhip import audio
    from radhip.build import apply_lora_to_wavlm, get_model, load_weights
    from radhip.data import pad
    m = apply_lora_to_wavlm(get_model(cfg["model_config"], "cuda"), cfg["training_config"])
    load_weights(m, weights, "cuda", strict=True)
    m.eval()
    x = np.stack([pad(audio.read(p)[0]) for p in paths]).astype(np.float32)
    with torch.no_grad():
        _, out = m(torch.from_numpy(x).cuda())
    return out[:, 1].float().cpu().numpy()


def test_cli_train_eval_and_2021(tmp_path, golden):
    import main as cli
    db = tmp_path / "LA"
    rows = _database(db, golden)
    conf, cfg = _config(tmp_path, golden, db)
    out = tmp_path / "exp"
    cli.main(cli.parse_args(["--config", str(conf), "--output_dir", str(out), "--seed", "1234"]))
    tag = out / "LA_Tiny_ep1_bs2"
    for f in ("config.conf", "metric_log.txt", "eval_scores.txt", "t-DCF_EER.txt", "metrics/dev_score.txt",
              "weights/best.pth", "weights/swa.pth",
              "weights/checkpoint_epoch_000.pth"):
        assert (tag / f).exists(), f
    assert len(list((tag / "weights").glob("epoch_0_*.pth"))) == 1
    assert "EER:" in (tag / "metric_log.txt").read_text()
    lines = (tag / "eval_scores.txt").read_text().splitlines()
    assert [ln.split()[0] for ln in lines] == [u for u, _, _ in rows["eval"]]
    assert [ln.split()[1:3] for ln in lines] == [[a, k] for _, a, k in rows["eval"]]
    scores = np.array([float(ln.split()[3]) for ln in lines])
    assert np.isfinite(scores).all()

    # --eval with the saved weights: the score file equals a direct fp32 forward of those weights
    w = tag / "weights" / "best.pth"
    cli.main(cli.parse_args(["--config", str(conf), "--output_dir", str(out), "--eval", "--eval_model_weights",
                             str(w), "--comment", "ev"]))
    ev = out / "LA_Tiny_ep1_bs2_ev"
    lines = (ev / "eval_scores.txt").read_text().splitlines()
    got = np.array([float(ln.split()[3]) for ln in lines])
    paths = [db / "ASVspoof2019_LA_eval" / "flac" / f"{u}.flac" for u, _, _ in rows["eval"]]
    ref = _direct_scores(cfg, w, paths)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)
    assert (ev / "t-DCF_EER.txt").exists() and (ev / "loaded_model_t-DCF_EER.txt").exists()

    # 2021 DF eval: "utt score" lines in protocol order + min-flip EER with the codec breakdown
    df = tmp_path / "DF"
    (df / "flac").mkdir(parents=True)
    trl, meta = [], []
    for i, (codec, key) in enumerate([("mp3m4a", "bonafide"), ("low_mp3", "spoof"), ("high_m4a", "spoof"),
                                      ("nocodec", "bonafide"), ("low_mp3", "bonafide"), ("high_m4a", "spoof")]):
        utt = "DF_E_%07d" % i
        shutil.copy(paths[i], df / "flac" / f"{utt}.flac")
        trl.append(f"LA_00{i:02d} {utt} {codec} asvspoof A{7 + i:02d} {key} notrim eval")
        meta.append(trl[-1])
    (df / "ASVspoof2021.DF.cm.eval.trl.txt").write_text("\n".join(trl) + "\n")
    (tmp_path / "meta.txt").write_text("\n".join(meta) + "\n")
    cfg21 = dict(cfg, database_path=str(df), is_eval_2021=True, key_file=str(tmp_path / "meta.txt"))
    conf21 = tmp_path / "Tiny21.conf"
    conf21.write_text(json.dumps(cfg21))
    cli.main(cli.parse_args(["--config", str(conf21), "--output_dir", str(out), "--eval", "--eval_model_weights",
                             str(w)]))
    t21 = out / "LA_Tiny21_ep1_bs2"
    lines = (t21 / "eval_scores.txt").read_text().splitlines()
    assert [ln.split()[0] for ln in lines] == ["DF_E_%07d" % i for i in range(6)]
    np.testing.assert_allclose([float(ln.split()[1]) for ln in lines], ref[:6], rtol=1e-4, atol=1e-5)
    rep = (t21 / "t-DCF_EER_2021DF.txt").read_text()
    assert "EER" in rep and "low_mp3" in rep
    os.environ.pop("WORLD_SIZE", None)


@pytest.mark.parametrize("amp", ["bf16", "fp16"])
def test_cli_full_resume_equals_continuous(tmp_path, golden, amp):
    """Two epochs in one run vs one epoch, then --resume from train_state_epoch_000.pt in a new run: the
    second epoch's weights, EMA/SWA files and dev scores agree (up to the GPU's atomic-accumulation
    order, far below any training step's effect). fp16 (the default: GradScaler state resumed too): a weight whose
    gradient is ~0 moves by ~lr * sign(g) either way, and fp16 rounding flips such signs more often than bf16's
    fixed-order paths do, so there the bound is on the whole model (5 % of its movement) with a loose per-tensor
    check; a lost optimizer / scaler / RNG state moves it by as much as the epoch itself."""
    import main as cli
    db = tmp_path / "LA"
    _database(db, golden)
    conf, cfg = _config(tmp_path, golden, db)
    cfg["num_epochs"] = 2
    conf.write_text(json.dumps(cfg, indent=2))
    out = tmp_path / "exp"
    cli.main(cli.parse_args(["--config", str(conf), "--output_dir", str(out), "--save_train_state",
                             "--comment", "cont", "--amp", amp]))
    cont = out / "LA_Tiny_ep2_bs2_cont"
    state0 = cont / "weights" / "train_state_epoch_000.pt"
    assert state0.exists() and (cont / "weights" / "train_state_epoch_001.pt").exists()
    cli.main(cli.parse_args(["--config", str(conf), "--output_dir", str(out), "--resume", str(state0),
                             "--comment", "res", "--amp", amp]))
    res = out / "LA_Tiny_ep2_bs2_res"
    # Tensor-wise L2 distance, judged against how far the second epoch moved each tensor: the runs are not
    # bitwise reproducible (fp32 atomics in the LoRA and scan gradient kernels; AdamW's first steps move a
    # weight by ~lr * sign(g), so an element whose gradient is ~0 can move either way), while a lost
    # optimizer / scheduler / RNG state would put the resumed epoch's update elsewhere entirely.
    w0 = torch.load(state0, weights_only=True, map_location="cpu")["model"]
    per = 0.05 if amp == "bf16" else 0.75
    for f in ("checkpoint_epoch_001.pth", "swa.pth", "best.pth"):
        a = torch.load(cont / "weights" / f, weights_only=True, map_location="cpu")
        b = torch.load(res / "weights" / f, weights_only=True, map_location="cpu")
        assert a.keys() == b.keys()
        d2 = m2 = 0.0
        for k in a:
            x, y = a[k].double(), b[k].double()
            moved = float((x - w0[k].double()).norm()) if k in w0 else float(x.norm())
            d = float((x - y).norm())
            # attention_pool.bias is one scalar added to every score of a softmax over time: its gradient is zero
            # up to rounding, so AdamW moves it by lr * sign(noise) either way (whole-model check below only)
            if k != "attention_pool.bias":
                assert d <= per * moved + 1e-4 * float(x.norm()) + 1e-12, (f, k, d, moved)
            if k in w0 and a[k].is_floating_point():
                d2, m2 = d2 + d * d, m2 + moved * moved
        assert d2 <= 0.05 ** 2 * m2 + 1e-24, (f, d2 ** 0.5, m2 ** 0.5)
    sa = [float(ln.split()[3]) for ln in (cont / "metrics" / "dev_score.txt").read_text().splitlines()]
    sb = [float(ln.split()[3]) for ln in (res / "metrics" / "dev_score.txt").read_text().splitlines()]
    np.testing.assert_allclose(sb, sa, rtol=1e-3 if amp == "bf16" else 1e-2, atol=1e-4 if amp == "bf16" else 1e-3)
    os.environ.pop("WORLD_SIZE", None)
