"""Generate the golden vectors under tests/golden/ by running the REFERENCE itself.

Runs only in the build container (needs /root/reference, read-only). It imports the reference's own
modules with sys.modules stubs for packages absent from the image — the same mocking pattern as the
reference's utils/check_model.py:7-23 — mapping `mamba_ssm.modules.mamba_simple.Mamba` to the
reference-owned pure-torch MambaBlock (src/models/modules/mamba_block.py). Outputs are small .npz /
.json data files (inputs + expected outputs); no reference source is copied.

    python tests/golden/make_golden.py [--ref /root/reference]
"""
import argparse
import hashlib
import io
import json
import tempfile
import os
import random
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from seeded import dirty_audio, seeded_array, seeded_fill_  # noqa: E402


def install_stubs(ref_src):
    import transformers  # noqa: F401  (must be imported before the torchaudio stub)
    sys.path.insert(0, ref_src)
    mb = {}
    exec(compile(open(os.path.join(ref_src, "models/modules/mamba_block.py")).read(),
                 "mamba_block.py", "exec"), mb)
    for name in ["mamba_ssm", "mamba_ssm.modules", "mamba_ssm.modules.mamba_simple"]:
        sys.modules[name] = types.ModuleType(name)
    sys.modules["mamba_ssm.modules.mamba_simple"].Mamba = mb["MambaBlock"]
    import importlib.machinery
    for name in ["torchaudio", "torchaudio.transforms", "soundfile", "torchcontrib", "torchcontrib.optim",
                 "torch.utils.tensorboard"]:
        sys.modules[name] = types.ModuleType(name)
        sys.modules[name].__spec__ = importlib.machinery.ModuleSpec(name, None)
    sys.modules["torchaudio"].transforms = sys.modules["torchaudio.transforms"]

    class _Stub:
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, k):
            return lambda *a, **kw: None

    sys.modules["torchcontrib.optim"].SWA = _Stub
    sys.modules["torch.utils.tensorboard"].SummaryWriter = _Stub
    return mb["MambaBlock"]


def npz(path, **arrays):
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print("wrote", os.path.relpath(path, HERE), f"{os.path.getsize(path) / 1024:.1f} KB")


def grads_of(module, full_max=4096):
    """Full gradients for small tensors; (sum, sum of squares, first 64 values) for large ones."""
    out = {}
    for k, p in module.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.detach().numpy().astype(np.float64)
        if g.size <= full_max:
            out[f"grad:{k}"] = g.astype(np.float32)
        else:
            out[f"gradsum:{k}"] = np.array([g.sum(), (g * g).sum()])
            out[f"gradhead:{k}"] = g.reshape(-1)[:64].astype(np.float32)
    return out


# ------------------------------------------------------------------------------------------------
def gen_sinc(DS):
    conv = DS.CONV(out_channels=70, kernel_size=128, in_channels=1)
    x = seeded_array("sinc.x", (1, 1, 1500), scale=0.1).astype(np.float32)
    xt = torch.from_numpy(x)
    out_plain = conv(xt, mask=False).numpy()
    np.random.seed(7)
    random.seed(7)
    out_mask = conv(xt, mask=True).numpy()
    np.random.seed(7)
    random.seed(7)
    A = int(np.random.uniform(0, 20))
    A0 = random.randint(0, 70 - A)
    # pooled front end exactly as SincNetEncoder.forward:250-253
    pooled = torch.nn.functional.max_pool2d(torch.abs(torch.from_numpy(out_mask)).unsqueeze(1), (3, 3)).numpy()
    npz(os.path.join(HERE, "sinc_conv.npz"), band_pass=conv.band_pass.numpy(), x=x, conv=out_plain,
        mask_lo=A0, mask_hi=A0 + A, pooled_masked=pooled[:, 0])


def gen_sincnet(DS):
    enc = DS.SincNetEncoder(sinc_channels=70)
    seeded_fill_(enc, seed=11)
    enc.eval()
    x = seeded_array("sincnet.x", (2, 8000), scale=0.1).astype(np.float32)
    xt = torch.from_numpy(x)
    out = enc(xt, freq_aug=False)
    r = seeded_array("sincnet.r", tuple(out.shape)).astype(np.float32)
    (out * torch.from_numpy(r)).sum().backward()
    g = grads_of(enc)
    npz(os.path.join(HERE, "sincnet_encoder.npz"), x=x, out=out.detach().numpy(), r=r, **g)


def gen_mamba(MambaBlock, DS):
    torch.manual_seed(0)
    m = MambaBlock(16, d_state=16)
    seeded_fill_(m, seed=21)
    x = seeded_array("mamba.x", (2, 23, 16)).astype(np.float32)
    xt = torch.from_numpy(x).requires_grad_(True)
    y = m(xt)
    r = seeded_array("mamba.r", tuple(y.shape)).astype(np.float32)
    (y * torch.from_numpy(r)).sum().backward()
    npz(os.path.join(HERE, "mamba_block.npz"), x=x, y=y.detach().numpy(), r=r, dx=xt.grad.numpy(), **grads_of(m))
    # Pre-Norm Bi-Mamba layer (shared-weight flip)
    enc = DS.PN_BiMambas_Encoder(d_model=16, n_state=16)
    seeded_fill_(enc, seed=22)
    x = seeded_array("pnbimamba.x", (2, 19, 16)).astype(np.float32)
    xt = torch.from_numpy(x).requires_grad_(True)
    y = enc(xt)
    r = seeded_array("pnbimamba.r", tuple(y.shape)).astype(np.float32)
    (y * torch.from_numpy(r)).sum().backward()
    npz(os.path.join(HERE, "pn_bimamba.npz"), x=x, y=y.detach().numpy(), r=r, dx=xt.grad.numpy(), **grads_of(enc))


def gen_fusion(DS):
    fu = DS.DualStreamFusion(wavlm_dim=32, sinc_dim=8, out_dim=16, reduction=4)
    seeded_fill_(fu, seed=31)
    fu.eval()
    fw = seeded_array("fusion.fw", (2, 20, 32)).astype(np.float32)
    fs_near = seeded_array("fusion.fs3", (2, 3, 8)).astype(np.float32)     # 20/3 > 4 -> nearest
    fs_lin = seeded_array("fusion.fs10", (2, 10, 8)).astype(np.float32)    # 20/10 <= 4 -> linear
    with torch.no_grad():
        o_near = fu(torch.from_numpy(fw), torch.from_numpy(fs_near)).numpy()
        o_lin = fu(torch.from_numpy(fw), torch.from_numpy(fs_lin)).numpy()
    npz(os.path.join(HERE, "fusion.npz"), fw=fw, fs_near=fs_near, fs_lin=fs_lin, out_near=o_near, out_lin=o_lin)


TINY_WAVLM = dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=128,
                  conv_dim=(32,) * 7, num_conv_pos_embeddings=16, num_conv_pos_embedding_groups=16,
                  do_stable_layer_norm=True, feat_extract_norm="layer", conv_bias=False, num_buckets=320,
                  max_bucket_distance=800)


def gen_model(DS):
    """Full reference Model (WavLM stream at reduced widths; 24 layers / 1024-d kept because the
    reference hard-codes out_dim=1024 and 25 layer weights), eval mode, seeded weights."""
    from transformers import WavLMConfig, WavLMModel
    cfg = WavLMConfig(**TINY_WAVLM)
    orig = WavLMModel.from_pretrained
    WavLMModel.from_pretrained = classmethod(lambda cls, *a, **k: WavLMModel(cfg))
    try:
        class Args:
            emb_size, num_encoders, d_state, sinc_channels, wavlm_freeze_layers = 144, 2, 16, 70, -1
        model = DS.Model(Args(), device="cpu")
    finally:
        WavLMModel.from_pretrained = orig
    seeded_fill_(model, seed=41)
    model.eval()
    x = seeded_array("model.x", (2, 16000), scale=0.1).astype(np.float32)
    xt = torch.from_numpy(x)
    feats, logits = model(xt, Freq_aug=False)
    (logits[:, 1].sum() - logits[:, 0].sum()).backward()
    keep = ["wavlm_stream.layer_weights", "classifier.weight", "attention_pool.weight", "fusion.sinc_proj.weight",
            "backbone_layers.0.mamba.A_log", "backbone_layers.1.mamba.in_proj.weight",
            "sinc_stream.first_bn.weight", "wavlm_stream.model.feature_projection.projection.bias",
            "wavlm_stream.model.encoder.layers.23.attention.q_proj.weight"]
    g = {k: v for k, v in grads_of(model).items() if k.split(":", 1)[1] in keep}
    npz(os.path.join(HERE, "model_tiny.npz"), x=x, feats=feats.detach().numpy(), logits=logits.detach().numpy(),
        wavlm_config=json.dumps(TINY_WAVLM), **g)


def gen_rawboost(ref_src):
    import rawboost as RB
    x = seeded_array("rawboost.x", (3000,), scale=0.2)
    cases = {}
    for algo in [1, 2, 3, 4]:
        for seed in [3, 4]:
            np.random.seed(seed)
            cases[f"a{algo}_s{seed}"] = RB.RawBoost(algo_id=[algo], fs=16000).process(x.copy())
    for seed in [5, 6, 7, 8]:
        np.random.seed(seed)
        cases[f"mix_s{seed}"] = RB.RawBoost(algo_id=[1, 2, 3, 4], fs=16000).process(x.copy())
    npz(os.path.join(HERE, "rawboost.npz"), x=x, **cases)


def gen_data(ref_src):
    import data_utils as DU
    lines_train = ["LA_0079 LA_T_1138215 - - bonafide", "LA_0079 LA_T_1271820 - A01 spoof",
                   "LA_0080 LA_T_1272637 - A06 spoof", "LA_0081 LA_T_1276960 - - bonafide",
                   "LA_0082 LA_T_1341447 - A04 spoof"]
    lines_2021 = ["LA_0023 DF_E_2000011 nocodec asvspoof A14 spoof notrim eval",
                  "LA_0043 DF_E_2000013 low_m4a vcc2020 - bonafide notrim eval", "", "DF_E_2000024"]
    tmp = os.path.join(HERE, "_tmp_proto.txt")
    res = {}
    try:
        with open(tmp, "w") as f:
            f.write("\n".join(lines_train) + "\n")
        lab, lst = DU.genSpoof_list(tmp, is_train=True)
        res["train"] = {"labels": lab, "list": lst}
        lab, lst = DU.genSpoof_list(tmp, is_train=False, is_eval=False)
        res["dev"] = {"labels": lab, "list": lst}
        res["eval"] = DU.genSpoof_list(tmp, is_train=False, is_eval=True)
        with open(tmp, "w") as f:
            f.write("\n".join(lines_2021) + "\n")
        res["df2021"] = DU.genSpoof_list(tmp, is_eval=True, is_2021=True)
    finally:
        os.remove(tmp)
    res["lines_train"] = lines_train
    res["lines_2021"] = lines_2021
    with open(os.path.join(HERE, "protocol.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("wrote protocol.json")
    pads = {}
    for n in [1000, 64599, 64600, 70000]:
        x = np.arange(n, dtype=np.float64)  # pad outputs are then the source-index maps
        idx = DU.pad(x).astype(np.int64)
        pads[f"pad_{n}_sha"] = np.frombuffer(hashlib.sha256(idx.tobytes()).digest(), np.uint8)
        pads[f"pad_{n}_head"] = idx[:256]
        if n != 64600:
            np.random.seed(n)
            idx = DU.pad_random(x).astype(np.int64)
            pads[f"padr_{n}_sha"] = np.frombuffer(hashlib.sha256(idx.tobytes()).digest(), np.uint8)
            pads[f"padr_{n}_head"] = idx[:256]
    try:
        DU.pad_random(np.zeros(64600))
        pads["padr_64600_raises"] = np.array(0)
    except ValueError:
        pads["padr_64600_raises"] = np.array(1)
    npz(os.path.join(HERE, "pad.npz"), **pads)


def _read_b0x(path):
    bona, spoof, attacks = [], [], []
    for ln in open(path):
        p = ln.split()
        if p[4] == "bonafide":
            bona.append(float(p[5]))
        else:
            spoof.append(float(p[5]))
            attacks.append(p[3])
    return np.array(bona), np.array(spoof), np.array(attacks)


def gen_eval(ref_root):
    import evaluation as EV
    import report_2021df_codec_breakdown as R21
    out = {}
    for name in ["B01", "B02"]:
        path = os.path.join(ref_root, f"tDCF_python_v2/scores/{name}_LA_primary_eval.txt")
        raw = open(path, "rb").read()
        bona, spoof, att = _read_b0x(path)
        eer, thr = EV.compute_eer(bona, spoof)
        per = {a: float(EV.compute_eer(bona, spoof[att == a])[0]) for a in sorted(set(att))}
        out[name] = {"sha256": hashlib.sha256(raw).hexdigest(), "n_bona": int(bona.size), "n_spoof": int(spoof.size),
                     "eer": float(eer), "threshold": float(thr), "eer_per_attack": per}
        # a 3000-trial subsample (with ties injected) as a committed, license-light vector
        rng = np.random.default_rng(5 if name == "B01" else 6)
        bi = rng.choice(bona.size, 400, replace=False)
        si = rng.choice(spoof.size, 2600, replace=False)
        b_s, s_s = np.round(bona[bi], 2), np.round(spoof[si], 2)
        e_s, t_s = EV.compute_eer(b_s, s_s)
        out[name]["subsample"] = {"bona": b_s.tolist(), "spoof": s_s.tolist(), "eer": float(e_s), "thr": float(t_s),
                                  "minflip_pct": float(R21.compute_eer_minflip(b_s, s_s))}
    # t-DCF on synthetic CM + ASV score files through calculate_tDCF_EER (file interface)
    rng = np.random.default_rng(9)
    attacks = [f"A{i:02d}" for i in range(7, 20)]
    cm_lines, asv_lines = [], []
    for i in range(1300):
        key = "bonafide" if i < 300 else "spoof"
        src = "-" if key == "bonafide" else attacks[i % 13]
        sc = rng.normal(1.5 if key == "bonafide" else -1.0, 1.0)
        cm_lines.append(f"LA_E_{i:07d} {src} {key} {sc}")
    for i in range(900):
        key = ["target", "nontarget", "spoof"][i % 3]
        sc = rng.normal({"target": 2.0, "nontarget": -2.0, "spoof": 0.5}[key], 1.0)
        asv_lines.append(f"LA_{i:04d} {key} {sc}")
    cm_p, asv_p, rep = (os.path.join(HERE, n) for n in ["_cm.txt", "_asv.txt", "_rep.txt"])
    try:
        open(cm_p, "w").write("\n".join(cm_lines) + "\n")
        open(asv_p, "w").write("\n".join(asv_lines) + "\n")
        import contextlib
        with contextlib.redirect_stdout(io.StringIO()):
            eer_cm, tdcf = EV.calculate_tDCF_EER(cm_p, asv_p, rep, printout=True)
        report = open(rep).read()
    finally:
        for p in (cm_p, asv_p, rep):
            if os.path.exists(p):
                os.remove(p)
    out["tdcf"] = {"cm_lines": cm_lines, "asv_lines": asv_lines, "eer_cm_pct": float(eer_cm), "min_tdcf": float(tdcf),
                   "report": report}
    with open(os.path.join(HERE, "eval_golden.json"), "w") as f:
        json.dump(out, f)
    print("wrote eval_golden.json")


def gen_eval21(ref_src):
    """2021-DF min-flip report (report_2021df_codec_breakdown.main) on a synthetic trial_metadata +
    score file, run in a scratch cwd with relative file names (the report prints the paths)."""
    import contextlib
    import report_2021df_codec_breakdown as R21
    rng = np.random.default_rng(21)
    codecs = ["nocodec", "low_mp3", "high_mp3", "low_m4a", "high_m4a", "mp3m4a", "oggm4a"]
    sources = ["asvspoof", "vcc2018", "vcc2020"]
    meta, scores = [], []
    for i in range(700):
        key = "bonafide" if rng.random() < 0.2 else "spoof"
        codec, src = codecs[i % 7], sources[(i // 7) % 3]
        meta.append(f"LA_{i % 40:04d} DF_E_{2000000 + i} {codec} {src} {'bonafide' if key == 'bonafide' else 'A14'} "
                    f"{key} notrim eval")
        if i % 50 == 17:
            continue                                   # unscored trial
        mu = 0.8 if key == "bonafide" else -0.6
        if codec in ("low_mp3", "mp3m4a"):
            mu = -mu                                   # a flipped-sign group
        sc = round(float(rng.normal(mu, 1.0)), 3)     # rounding -> ties
        scores.append(f"DF_E_{2000000 + i} {sc}")
    scores.append("garbage-line")
    scores.append("DF_E_9999999 notafloat")
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        try:
            open("trial_metadata.txt", "w").write("\n".join(meta) + "\n")
            open("scores.txt", "w").write("\n".join(scores) + "\n")
            argv = sys.argv
            sys.argv = ["r", "--score_file", "scores.txt", "--key_file", "trial_metadata.txt", "--out", "report.md"]
            try:
                with contextlib.redirect_stdout(io.StringIO()):
                    R21.main()
            finally:
                sys.argv = argv
            report = open("report.md").read()
        finally:
            os.chdir(cwd)
    with open(os.path.join(HERE, "eval21_golden.json"), "w") as f:
        json.dump({"meta": meta, "scores": scores, "report": report}, f)
    print("wrote eval21_golden.json")


def gen_scorefile(main):
    """produce_evaluation_file (src/main.py:958-995) with a toy model: the exact score-file bytes."""
    import contextlib
    rng = np.random.default_rng(22)
    n = 37
    x = rng.standard_normal((n, 6)).astype(np.float32)
    w = rng.standard_normal((6, 2)).astype(np.float32)
    trial = [f"LA_{i % 9:04d} LA_E_{1000000 + i} - {'-' if i % 4 == 0 else 'A1' + str(i % 10)} "
             f"{'bonafide' if i % 4 == 0 else 'spoof'}" for i in range(n)]

    class Toy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.from_numpy(w))

        def forward(self, xb, Freq_aug=False):
            return xb, xb @ self.w

    ids = [t.split()[1] for t in trial]
    batches = [(torch.from_numpy(x[i:i + 8]), ids[i:i + 8]) for i in range(0, n, 8)]
    with tempfile.TemporaryDirectory() as d:
        tp, sp = os.path.join(d, "trl.txt"), os.path.join(d, "score.txt")
        open(tp, "w").write("\n".join(trial) + "\n")
        with contextlib.redirect_stdout(io.StringIO()):
            main.produce_evaluation_file(batches, Toy(), torch.device("cpu"), sp, tp)
        text = open(sp).read()
    npz(os.path.join(HERE, "scorefile.npz"), x=x, w=w, trial=np.array("\n".join(trial)), text=np.array(text))
    print("wrote scorefile.npz")


def gen_train(main):
    """FGM attack/restore and a toy train_epoch trajectory through the reference driver."""
    class Toy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.feature_projection = torch.nn.Linear(6, 5)
            self.body = torch.nn.Linear(5, 4)
            self.classifier = torch.nn.Linear(4, 2)

        def forward(self, x, Freq_aug=False):
            h = torch.tanh(self.body(torch.tanh(self.feature_projection(x))))
            return h, self.classifier(h)

    toy = Toy()
    seeded_fill_(toy, seed=51)
    # FGM alone
    for p in toy.parameters():
        p.grad = torch.from_numpy(seeded_array("fgm.g." + str(p.shape), tuple(p.shape)).astype(np.float32))
    fgm = main.FGM(toy, emb_name="feature_projection", epsilon=0.5)
    before = {k: v.detach().clone().numpy() for k, v in toy.named_parameters()}
    fgm.attack()
    attacked = {k: v.detach().clone().numpy() for k, v in toy.named_parameters()}
    fgm.restore()
    restored = {k: v.detach().clone().numpy() for k, v in toy.named_parameters()}
    arrays = {}
    for k in before:
        arrays[f"fgm_grad:{k}"] = toy.get_parameter(k).grad.numpy()
        arrays[f"fgm_before:{k}"] = before[k]
        arrays[f"fgm_attacked:{k}"] = attacked[k]
        arrays[f"fgm_restored:{k}"] = restored[k]
    # train_epoch trajectory
    toy = Toy()
    seeded_fill_(toy, seed=52)
    init = {k: v.detach().clone().numpy() for k, v in toy.named_parameters()}
    B, nb, accum = 4, 6, 2
    xs = seeded_array("train.x", (nb, B, 6)).astype(np.float32)
    ys = (seeded_array("train.y", (nb, B)) > 0.4).astype(np.int64)
    loader = [(torch.from_numpy(xs[i]), torch.from_numpy(ys[i])) for i in range(nb)]
    opt = torch.optim.AdamW([{"params": [toy.feature_projection.weight, toy.feature_projection.bias], "lr": 1e-2},
                             {"params": list(toy.body.parameters()) + list(toy.classifier.parameters()), "lr": 5e-3}],
                            weight_decay=1e-4)
    total = 3
    warm = 1
    sched = torch.optim.lr_scheduler.SequentialLR(
        opt, [torch.optim.lr_scheduler.LinearLR(opt, start_factor=0.1, end_factor=1.0, total_iters=warm),
              torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=total - warm, eta_min=1e-6)], milestones=[warm])
    from torch.optim.swa_utils import AveragedModel, get_ema_multi_avg_fn
    ema = AveragedModel(toy, multi_avg_fn=get_ema_multi_avg_fn(0.999))
    crit = torch.nn.CrossEntropyLoss(weight=torch.tensor([0.1, 0.9]))
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        scaler = torch.cuda.amp.GradScaler(enabled=False)
        cfg = {"training_config": {"use_mixup": True, "mixup_alpha": 1.0}, "freq_aug": "False",
               "optim_config": {"scheduler": "cosine"}}
        np.random.seed(61)
        torch.manual_seed(61)
        loss = main.train_epoch(loader, toy, opt, "cpu", sched, cfg, crit, None, scaler, freeze_bn=True,
                                ema_model=ema, accumulation_steps=accum,
                                fgm=main.FGM(toy, emb_name="feature_projection", epsilon=0.5))
    arrays["train_x"] = xs
    arrays["train_y"] = ys
    arrays["train_loss"] = np.array(loss)
    arrays["train_lr_final"] = np.array([g["lr"] for g in opt.param_groups])
    for k in init:
        arrays[f"train_init:{k}"] = init[k]
        arrays[f"train_final:{k}"] = toy.get_parameter(k).detach().numpy()
        arrays[f"train_ema:{k}"] = ema.module.get_parameter(k).detach().numpy()
    npz(os.path.join(HERE, "train_toy.npz"), **arrays)


def gen_legacy(ref_root):
    """Legacy plugins (BASELINE configs 1-2): the reference's models/AASIST.py and models/RawNet2Spoof.py,
    built from their own confs (src/config/AASIST.conf, RawNet2_baseline.conf) with seeded weights, at the
    full 64 600-sample input. Two modes per model: eval (BatchNorm running statistics) and train with every
    Dropout at p = 0 (BatchNorm batch statistics + running-stat update, deterministic). Stores the outputs,
    every parameter gradient of sum(hidden * r_h) + sum(out * r_o), the updated running stats, and the
    state_dict key / shape list. The input is seeded_array(f"{arch}.x", (2, 64600), scale=0.1), recomputed
    by the tests rather than stored."""
    import copy
    import importlib.util
    for arch, conf in (("AASIST", "AASIST.conf"), ("RawNet2Spoof", "RawNet2_baseline.conf")):
        spec = importlib.util.spec_from_file_location(f"ref_{arch}", os.path.join(ref_root, "models", arch + ".py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        with open(os.path.join(ref_root, "src", "config", conf)) as f:
            mc = json.load(f)["model_config"]
        arrays = {}
        x = seeded_array(f"{arch}.x", (2, 64600), scale=0.1).astype(np.float32)
        for mode in ("eval", "train"):
            torch.manual_seed(0)
            m = mod.Model(copy.deepcopy(mc))
            seeded_fill_(m, seed=41)
            # float64 throughout: the block-0 weight gradients reduce over B x 24 x 21490 terms, where an
            # fp32 CPU oracle is itself ~0.5 % off; the fixture holds the exact values
            m = m.double()
            for c in ("conv_time", "Sinc_conv"):
                if hasattr(m, c):
                    getattr(m, c).band_pass = getattr(m, c).band_pass.double()
            if mode == "train":
                for d in m.modules():
                    if isinstance(d, torch.nn.Dropout):
                        d.p = 0.0
                m.train()
            else:
                m.eval()
            hid, out = m(torch.from_numpy(x).double(), Freq_aug=False)
            rh = seeded_array(f"{arch}.rh", tuple(hid.shape)).astype(np.float32)
            ro = seeded_array(f"{arch}.ro", tuple(out.shape)).astype(np.float32)
            rh64, ro64 = torch.from_numpy(rh).double(), torch.from_numpy(ro).double()
            ((hid * rh64).sum() + (out * ro64).sum()).backward()
            arrays[f"{mode}:hidden"] = hid.detach().numpy().astype(np.float32)
            arrays[f"{mode}:out"] = out.detach().numpy().astype(np.float32)
            arrays[f"{mode}:rh"] = rh
            arrays[f"{mode}:ro"] = ro
            for k, v in grads_of(m).items():
                arrays[f"{mode}:{k}"] = v
            if mode == "train":
                for k, v in m.state_dict().items():
                    if k.endswith("running_mean") or k.endswith("running_var"):
                        arrays[f"stat:{k}"] = v.numpy().astype(np.float32)
            else:
                sd = m.state_dict()
                arrays["keys"] = np.array(list(sd.keys()))
                arrays["shapes"] = np.array([json.dumps(list(v.shape)) for v in sd.values()])
                arrays["n_params"] = np.array(sum(p.numel() for p in m.parameters()))
        npz(os.path.join(HERE, f"legacy_{arch}.npz"), **arrays)


def gen_getitem(ref_src):
    """Gate order of Dataset_ASVspoof2019_train.__getitem__ (data_utils.py:163-184), run by the reference
    itself: RawBoost gate (python random) -> RawBoost draws (numpy) -> codec gate (python random) with
    apply_codec_aug's inner 0.5 gate and random.choice of the rate -> pad_random's crop start (numpy, on the
    post-codec length). soundfile and torchaudio are absent: sf.read is stubbed to return a ramp of a
    per-key length, and T.Resample by a stub that logs (orig, new) and returns torchaudio's output length
    ceil(new' * n / orig') (gcd-reduced rates, torchaudio's _apply_sinc_resample_kernel). RawBoost is the
    reference's own, with algo 1 (LnL), whose numpy draw sequence the product reproduces exactly (the ISD /
    SSI per-sample noise is a documented Philox deviation, so those algorithms would desynchronise the
    streams). Records per call: rawboost applied, codec rate (0 = none), crop start (-1 = tiled)."""
    import math
    import data_utils as DU
    lens = {f"LA_T_{i:07d}": n for i, n in enumerate([70000, 64601, 30000, 90000, 64000, 100000, 66000, 80000] * 8)}
    DU.sf.read = lambda path: (np.arange(lens[os.path.basename(str(path))[:-5]], dtype=np.float64) * 1e-5, 16000)
    log = []

    class Resample:
        def __init__(self, orig, new):
            g = math.gcd(int(orig), int(new))
            self.o, self.n = int(orig) // g, int(new) // g
            log.append(("resample", int(orig), int(new)))

        def __call__(self, sig):
            return torch.zeros(sig.shape[0], math.ceil(self.n * sig.shape[-1] / self.o))
    DU.T.Resample = Resample
    real_pad_random = DU.pad_random

    def pad_random(x, max_len=64600):
        st = np.random.get_state()
        out = real_pad_random(x, max_len)
        if x.shape[0] >= max_len:
            rs = np.random.RandomState()
            rs.set_state(st)
            log.append(("start", int(rs.randint(x.shape[0] - max_len)), int(x.shape[0])))
        else:
            log.append(("start", -1, int(x.shape[0])))
        return out
    DU.pad_random = pad_random
    keys = list(lens)
    ds = DU.Dataset_ASVspoof2019_train(keys, {k: 0 for k in keys}, __import__("pathlib").Path("/nonexistent"), algo=1, use_codec=True,
                                       codec_p=0.6, rawboost_p=0.8)
    real_process = ds.rawboost.process

    def process(x):
        log.append(("rawboost",))
        return real_process(x)
    ds.rawboost.process = process
    random.seed(2024)
    np.random.seed(2024)
    recs = []
    for k in keys:
        del log[:]
        ds[keys.index(k)]
        rb = int(any(e[0] == "rawboost" for e in log))
        rates = [e[2] for e in log if e[0] == "resample" and e[1] == 16000]
        st = [e for e in log if e[0] == "start"][0]
        recs.append([lens[k], rb, rates[0] if rates else 0, st[1], st[2]])
    DU.pad_random = real_pad_random
    with open(os.path.join(HERE, "getitem_order.json"), "w") as f:
        json.dump({"seed": 2024, "algo": 1, "rawboost_p": 0.8, "use_codec": True, "codec_p": 0.6,
                   "fields": ["len", "rawboost", "codec_rate", "start", "len_after_codec"], "records": recs}, f)
    print("wrote getitem_order.json")


def gen_dirty(ref_src):
    """src/filter_dirty_data.py run by the reference itself on a toy scorer: models.ToyScore (registered in
    sys.modules; logits [0, 40 * mean(x) + b]) loaded from a torch.save'd state dict, a 36-utterance train
    protocol, sf.read stubbed to the int16 / 32768 samples of dirty_audio(i), np.random seeded 77 before
    main() (the reference does not seed; pad_random crops long utterances with it). Stores the protocol,
    the per-utterance CE losses in protocol order, and the two output files' bytes."""
    import importlib
    import data_utils as DU
    FD = importlib.import_module("filter_dirty_data")

    class ToyScore(torch.nn.Module):
        def __init__(self, args, device):
            super().__init__()
            self.w = torch.nn.Parameter(torch.tensor([40.0, 0.05]))

        def forward(self, x, Freq_aug=False):
            z = self.w[0] * x.mean(dim=1) + self.w[1]
            return x[:, :4], torch.stack([torch.zeros_like(z), z], dim=1)
    mod = types.ModuleType("models.ToyScore")
    mod.Model = ToyScore
    sys.modules["models.ToyScore"] = mod
    keys = [f"LA_T_{9000000 + i:07d}" for i in range(36)]
    audio = {k: dirty_audio(i) for i, k in enumerate(keys)}
    DU.sf.read = lambda path: (audio[os.path.basename(str(path))[:-5]].astype(np.float64) / 32768.0, 16000)
    FD.tqdm = lambda it: it
    rows = [f"LA_{i % 7:04d} {k} - {'-' if i % 3 == 0 else 'A0%d' % (1 + i % 6)} {'bonafide' if i % 3 == 0 else 'spoof'}"
            for i, k in enumerate(keys)]
    losses = []
    real_ce = torch.nn.CrossEntropyLoss

    class CE(real_ce):
        def forward(self, a, b):
            out = super().forward(a, b)
            losses.extend(out.detach().float().tolist())
            return out
    FD.nn = types.SimpleNamespace(CrossEntropyLoss=CE)
    with tempfile.TemporaryDirectory() as td:
        db = os.path.join(td, "LA")
        os.makedirs(os.path.join(db, "ASVspoof2019_LA_cm_protocols"))
        with open(os.path.join(db, "ASVspoof2019_LA_cm_protocols", "ASVspoof2019.LA.cm.train.trn.txt"), "w") as f:
            f.write("\n".join(rows) + "\n")
        conf = os.path.join(td, "toy.conf")
        with open(conf, "w") as f:
            json.dump({"database_path": db, "track": "LA", "model_config": {"architecture": "ToyScore"}}, f)
        mp = os.path.join(td, "toy.pth")
        torch.save({"module.w": torch.tensor([40.0, 0.05])}, mp)
        out = os.path.join(td, "dirty_samples.txt")
        np.random.seed(77)
        import contextlib
        with contextlib.redirect_stdout(io.StringIO()):
            FD.main(argparse.Namespace(config=conf, model_path=mp, output_path=out, batch_size=5, filter_ratio=0.25,
                                       device="cpu", allow_cpu=True, amp=False))
        dirty = open(out).read()
        clean = open(out.replace(".txt", "_cleaned_protocol.txt")).read()
    del sys.modules["models.ToyScore"]
    with open(os.path.join(HERE, "dirty_filter.json"), "w") as f:
        json.dump({"keys": keys, "protocol": rows, "np_seed": 77, "batch_size": 5, "filter_ratio": 0.25,
                   "weights": [40.0, 0.05], "losses": losses, "dirty_txt": dirty, "cleaned_protocol_txt": clean}, f,
                  indent=0)
    print("wrote dirty_filter.json")


def main_():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    ref_src = os.path.join(args.ref, "src")
    MambaBlock = install_stubs(ref_src)
    torch.set_num_threads(8)
    import importlib
    DS = importlib.import_module("models.DualStreamSEMamba")
    only = set(args.only.split(",")) if args.only else None

    def want(n):
        return only is None or n in only
    if want("sinc"):
        gen_sinc(DS)
    if want("sincnet"):
        gen_sincnet(DS)
    if want("mamba"):
        gen_mamba(MambaBlock, DS)
    if want("fusion"):
        gen_fusion(DS)
    if want("rawboost"):
        gen_rawboost(ref_src)
    if want("data"):
        gen_data(ref_src)
    if want("eval"):
        gen_eval(args.ref)
    if want("eval21"):
        gen_eval21(ref_src)
    if want("train") or want("scorefile"):
        import contextlib
        with contextlib.redirect_stdout(io.StringIO()):
            main = importlib.import_module("main")
        if want("train"):
            gen_train(main)
        if want("scorefile"):
            gen_scorefile(main)
    if want("model"):
        gen_model(DS)
    if want("legacy"):
        gen_legacy(args.ref)
    if want("getitem"):
        gen_getitem(ref_src)
    if want("dirty"):
        gen_dirty(ref_src)


if __name__ == "__main__":
    main_()
