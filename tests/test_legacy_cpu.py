"""Legacy AASIST / RawNet2 plugin path on the CPU (no GPU): host plumbing of BASELINE configs 1-2.

  * the plugin loader takes the reference's legacy signature Model(d_args) (models/AASIST.py:470,
    models/RawNet2Spoof.py:170) and the Phase-5/6 Model(args, device) one (src/main.py:799-812);
  * the product plugins have the reference's state_dict keys, shapes and parameter count
    (tests/golden/legacy_*.npz, written by make_golden.py from the reference modules), so reference
    checkpoints load strictly;
  * the legacy confs (no scheduler_config) build the optimizer / scheduler (eta_min = lr_min);
  * config 1's data plumbing: a 256-utterance protocol, genSpoof_list, the shuffled micro-batch order
    and the native FLAC batch decode, on the host.
Compute parity of the two models (HIP front ends, fp32) is in tests/test_legacy_gpu.py."""
import json

import numpy as np
import pytest
import torch

from flac_writer import encode

LEGACY = [("AASIST", "AASIST.conf"), ("RawNet2Spoof", "RawNet2_baseline.conf")]


@pytest.mark.parametrize("arch,conf", LEGACY)
def test_legacy_plugin_state_dict_matches_reference(golden, arch, conf):
    import main  # noqa: F401
    from radhip.build import get_model, legacy_plugin, load_config
    from importlib import import_module
    g = golden(f"legacy_{arch}.npz")
    mc = load_config(conf)["model_config"]
    assert mc["architecture"] == arch
    assert legacy_plugin(import_module(f"models.{arch}").Model)
    before = json.dumps(mc)
    m = get_model(mc, "cpu")
    assert json.dumps(mc) == before            # the reference mutates filts; the product does not
    sd = m.state_dict()
    assert list(sd.keys()) == [str(k) for k in g["keys"]]
    assert [json.dumps(list(v.shape)) for v in sd.values()] == [str(s) for s in g["shapes"]]
    assert sum(p.numel() for p in m.parameters()) == int(g["n_params"])


def test_phase6_plugin_keeps_args_device_signature():
    import main  # noqa: F401
    from importlib import import_module
    from radhip.build import legacy_plugin
    assert not legacy_plugin(import_module("models.DualStreamSEMamba").Model)


def test_aasist_l_conf_builds():
    import main  # noqa: F401
    from radhip.build import get_model, load_config
    m = get_model(load_config("AASIST-L.conf")["model_config"], "cpu")
    assert sum(p.numel() for p in m.parameters()) == 85306      # AASIST-L's published size


@pytest.mark.parametrize("conf", ["AASIST.conf", "RawNet2_baseline.conf"])
def test_legacy_conf_optimizer_and_schedule(conf):
    import main  # noqa: F401
    from radhip.build import get_model, load_config
    from radhip.train import Trainer
    cfg = load_config(conf)
    assert "scheduler_config" not in cfg["optim_config"] and "training_config" not in cfg
    m = get_model(cfg["model_config"], "cpu")
    tr = Trainer(m, cfg, "cpu", total_steps=100, amp_dtype=torch.float32)
    c = tr.sched._schedulers[1]
    assert c.eta_min == cfg["optim_config"]["lr_min"]
    assert tr.accum == 1 and tr.fgm is None and tr.ema is None and not tr.use_mixup
    # every trainable tensor sits in the base_lr group (no wavlm_stream in the legacy models)
    assert len(tr.opt.param_groups[0]["params"]) == 0
    assert sum(p.numel() for p in tr.opt.param_groups[1]["params"]) == sum(p.numel() for p in m.parameters())
    # warm-up starts at warmup_init_factor * base_lr, as the reference's LinearLR
    assert tr.opt.param_groups[1]["lr"] == pytest.approx(0.1 * cfg["optim_config"]["base_lr"])


def test_config1_data_plumbing_256_utterances(tmp_path):
    """BASELINE config 1's data side on the host: a 256-utterance LA train protocol, labels and order
    (genSpoof_list), the shuffled drop_last micro-batches of batch_size 32, and the native decode of one
    micro-batch equal to the written samples."""
    import main  # noqa: F401
    from radhip import audio
    from radhip.build import load_config
    from radhip.data import TrainFeeder, genSpoof_list
    from radhip.train import Augmenter
    cfg = load_config("RawNet2_baseline.conf")
    root = tmp_path / "LA"
    flac = root / "ASVspoof2019_LA_train" / "flac"
    flac.mkdir(parents=True)
    proto = root / "ASVspoof2019_LA_cm_protocols"
    proto.mkdir()
    lines, samples = [], {}
    for i in range(256):
        utt = "LA_T_%07d" % i
        bona = i % 10 == 0
        lines.append(f"LA_{i % 20:04d} {utt} - {'-' if bona else 'A0%d' % (1 + i % 6)} {'bonafide' if bona else 'spoof'}")
        if i < 32:   # only what the decode check reads is written
            rng = np.random.default_rng(i)
            x = np.clip(np.round(2000 * rng.standard_normal(4000 + 97 * i)), -32768, 32767).astype(np.int64)
            (flac / f"{utt}.flac").write_bytes(encode(x, plan=lambda f, c, b: {"kind": "verbatim"}))
            samples[utt] = x
    trn = proto / "ASVspoof2019.LA.cm.train.trn.txt"
    trn.write_text("\n".join(lines) + "\n")
    main_paths = main.protocol_paths(cfg, "LA", root)
    assert main_paths[0] == trn
    labels, keys = genSpoof_list(trn, is_train=True, is_eval=False)
    assert len(keys) == 256 and sum(labels.values()) == 26
    B = int(cfg["batch_size"])
    feeder = TrainFeeder(keys, labels, root / "ASVspoof2019_LA_train", B, Augmenter("cpu"), seed=1234, threads=4)
    assert len(feeder) == 256 // B
    batches = list(feeder.epoch())
    assert sorted(k for b in batches for k in b) == sorted(keys)
    written = sorted(samples)
    flat, offs, lens, y = feeder.load(written, "cpu")
    for j, utt in enumerate(written):
        got = flat[offs[j]:offs[j] + lens[j]].numpy()
        np.testing.assert_array_equal(got, samples[utt].astype(np.float32) / 32768.0)
        assert int(y[j]) == labels[utt]
    assert audio.probe(flac / f"{written[0]}.flac")[0] == len(samples[written[0]])
