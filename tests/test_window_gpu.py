"""Accumulation-window execution (radhip/window.py) against the reference's per-micro-batch order
(Trainer.micro_step = train_epoch, src/main.py:998-1126): K clean passes batched into one, per-group
feature_projection gradients feeding the sequential FGM chain. With every random regulariser off,
the accumulated gradient of one window must equal K sequential micro-steps (fp32: to the atomic-
accumulation noise floor; bf16 / fp16: to their rounding), and the HIP-graph replay must equal the eager
window. The fp16 case is the bench's configuration: K = 4 micro-batches (the batched clean pass runs 4 x B
utterances through every fp16 kernel at its batched size), fp16 autocast with the reference's GradScaler
(src/main.py:28,1049,1077-1108), the FGM chain; gradients compared after the scaler's unscale."""
import json
import os

import numpy as np
import pytest
import torch

from seeded import seeded_fill_

pytestmark = pytest.mark.gpu
DEV = "cuda"
PROFILES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")


def _record(name, obj):
    """Keep a test's error table under profiles/ (the suite run's record of the measured ratios)."""
    os.makedirs(PROFILES, exist_ok=True)
    with open(os.path.join(PROFILES, name), "w") as f:
        json.dump(obj, f, indent=1)


def _model(golden, K=3):
    import models.DualStreamSEMamba as DS
    from radhip.build import apply_lora_to_wavlm, load_config
    g = golden("model_tiny.npz")
    wcfg = json.loads(str(g["wavlm_config"]))
    wcfg.update(hidden_dropout=0.0, attention_dropout=0.0, feat_proj_dropout=0.0, activation_dropout=0.0,
                layerdrop=0.0, mask_time_prob=0.0)

    class Args:
        emb_size, num_encoders, d_state, sinc_channels, wavlm_freeze_layers = 144, 2, 16, 70, -1
        wavlm_config = wcfg
    torch.manual_seed(0)
    m = DS.Model(Args(), device=DEV)
    seeded_fill_(m, seed=41)
    m = m.to(DEV)
    cfg = load_config("Phase6_Proposed.conf")
    cfg["training_config"]["lora_dropout"] = 0.0
    cfg["training_config"]["lora_mode"] = "active"     # the fused layer's folded LoRA columns take part
    cfg["training_config"]["accumulation_steps"] = K
    cfg["freq_aug"] = "False"
    m = apply_lora_to_wavlm(m, cfg["training_config"])
    with torch.no_grad():   # non-zero LoRA B so the adapters take part
        for n, p in m.named_parameters():
            if "lora_B" in n:
                p.normal_(0, 0.02)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    return m, cfg


def _batches(K, B, seed=5):
    rng = np.random.default_rng(seed)
    xs = [torch.from_numpy(np.clip(0.1 * rng.standard_normal((B, 64600)), -1, 1).astype(np.float32)).to(DEV)
          for _ in range(K)]
    ys = [rng.integers(0, 2, B) for _ in range(K)]
    lams = [0.3, 0.8, 1.0, 0.55][:K]
    perms = [list(rng.permutation(B)) for _ in range(K)]
    return xs, ys, lams, perms


def _unscaled(tr, flat):
    """The gradient as the optimizer sees it after GradScaler's unscale_ (scale 1 when the scaler is off)."""
    scale = float(tr.scaler.get_scale()) if tr.scaler.is_enabled() else 1.0
    return flat / scale


def _grads_sequential(golden, amp, K=3, B=4, seed=5):
    from radhip.train import Trainer
    m, cfg = _model(golden, K)
    tr = Trainer(m, cfg, DEV, total_steps=10, amp_dtype=amp)
    got = []
    tr.optimizer_step = lambda: got.append(_unscaled(tr, tr.grads.flat.clone()))
    xs, ys, lams, perms = _batches(K, B, seed)
    for k in range(K):
        tr.micro_step(xs[k], torch.from_numpy(ys[k]), lams[k], perms[k])
    torch.cuda.synchronize()
    return got[0], float(tr.loss_sum)


def _grads_window(golden, amp, graphs, K=3, B=4, seed=5):
    from radhip.train import Trainer
    from radhip.window import WindowStep
    m, cfg = _model(golden, K)
    tr = Trainer(m, cfg, DEV, total_steps=10, amp_dtype=amp)
    got = []
    w = WindowStep(tr, B, graphs=graphs)
    xs, ys, lams, perms = _batches(K, B, seed)
    def opt_step():                             # record the window's gradient, then zero it as
        got.append(_unscaled(tr, tr.grads.flat.clone()))   # optimizer_step would (the next window starts clean)
        tr.grads.zero()
    tr.optimizer_step = opt_step
    for rep in range(2 if graphs else 1):       # graphs: the second window is a pure replay
        got.clear()
        tr.loss_sum.zero_()
        for k in range(K):
            w.xslot(k).copy_(xs[k])
            w.add(k, ys[k], lams[k], perms[k])
        w.run()
    torch.cuda.synchronize()
    return got[0], float(tr.loss_sum)


def _rel(a, b):
    return float((a - b).norm() / b.norm())


def test_window_matches_sequential_fp32(golden):
    """fp32: the eager window and its HIP-graph replay both equal the reference-order micro-steps (to the
    fp32 atomic-accumulation noise floor)."""
    ref, lref = _grads_sequential(golden, torch.float32)
    got, lgot = _grads_window(golden, torch.float32, graphs=False)
    assert _rel(got, ref) < 1e-4
    assert lgot == pytest.approx(lref, rel=1e-5)
    graph, lgraph = _grads_window(golden, torch.float32, graphs=True)
    assert _rel(graph, ref) < 1e-4
    assert lgraph == pytest.approx(lref, rel=1e-5)


BF16_SEEDS = (5, 6, 7, 8, 9, 10)


def test_window_matches_sequential_bf16_and_graph_replay(golden):
    """bf16: the eager window is as close to the fp32 reference-order gradient as the bf16 reference-order run is,
    and its graph replay is as close as the eager window.

    Why over several input draws: FGM normalises the accumulated feature_projection gradient (g / ||g||, src/main.py:
    85-93), and on this 2-layer model that direction amplifies bf16 rounding chaotically. Over six draws the reference
    order's own bf16 error ranges 5 % to 239 % and the window's 4.8 % to 79 % (tools/diag_window_groups.py seeds,
    profiles/r06_window_bf16_seeds.jsonl); MIOpen's per-process algorithm choice changes the roundings too (draw 5: 3.6 %
    sequential / 7.4 % window in one process, 7.3 % / 4.8 % in another). The window / sequential ratio has median 0.93
    (0.33-1.14; fp16 0.61-1.05): no window-specific loss. Per group the window's error is uniform
    (profiles/r06_window_groups.jsonl), and at K = 1 or without FGM the window equals or beats the sequential run. So the
    bound is on the median ratio over the draws: <= 1.5."""
    rows, ratios = [], []
    for seed in BF16_SEEDS:
        ref32, lref = _grads_sequential(golden, torch.float32, seed=seed)
        seq16, _ = _grads_sequential(golden, torch.bfloat16, seed=seed)
        eager, leager = _grads_window(golden, torch.bfloat16, graphs=False, seed=seed)
        e_seq, e_win = _rel(seq16, ref32), _rel(eager, ref32)
        ratios.append(e_win / e_seq)
        rows.append({"seed": seed, "e_seq": e_seq, "e_window": e_win, "ratio": e_win / e_seq})
        if seed == BF16_SEEDS[0]:
            graph, lgraph = _grads_window(golden, torch.bfloat16, graphs=True, seed=seed)
            e_graph = _rel(graph, ref32)
            rows[-1]["e_graph"] = e_graph
            # the replay may run other MIOpen / hipBLASLt solutions than the eager window: held to the bf16 spread of
            # the two eager runs of the same draw, not to bit-equality
            assert e_graph < 1.5 * max(e_seq, e_win) + 1e-3, (e_graph, e_seq, e_win)
            assert lgraph == pytest.approx(leager, rel=1e-2)
            assert leager == pytest.approx(lref, rel=1e-2)
        print(f"[window bf16 draw {seed}] rel L2 vs fp32 reference order: sequential {e_seq:.3e}, window {e_win:.3e}")
    med = float(np.median(ratios))
    _record("r06_window_bf16_draws.json", {"draws": rows, "median_ratio": med})
    print(f"[window bf16] median window / sequential ratio over {len(ratios)} draws: {med:.3f}")
    assert med <= 1.5, rows


def test_window_matches_sequential_fp16_gradscaler_k4(golden):
    """The bench's arithmetic: fp16 autocast + GradScaler, K = 4 (the batched clean pass at 4 x B = 16 utterances,
    the fp16 kernels at their batched sizes, the scaled losses inside the captured graphs), then the four FGM chain
    links. The eager window and its graph replay are each as close to the fp32 reference-order gradient as the
    fp16 reference-order micro-steps are, and finite at the scaler's initial scale."""
    ref32, lref = _grads_sequential(golden, torch.float32, K=4)
    seq16, lseq = _grads_sequential(golden, torch.float16, K=4)
    eager, leager = _grads_window(golden, torch.float16, graphs=False, K=4)
    graph, lgraph = _grads_window(golden, torch.float16, graphs=True, K=4)
    for g in (seq16, eager, graph):
        assert torch.isfinite(g).all()
    e_seq = _rel(seq16, ref32)
    print(f"[window fp16 K=4] rel L2 vs fp32 reference order: sequential fp16 {e_seq:.3e}, window "
          f"{_rel(eager, ref32):.3e}, graph {_rel(graph, ref32):.3e}; window vs sequential fp16 {_rel(eager, seq16):.3e}")
    # measured: sequential fp16 2.9 %, window 2.9 %, graph 3.1 % (bf16's sequential run: 5.6 %); the window and
    # its replay within 1.5x the reference order's own fp16 error, under the bf16 level
    _record("r06_window_fp16_k4.json", {"e_seq": e_seq, "e_window": _rel(eager, ref32), "e_graph": _rel(graph, ref32),
                                        "window_vs_seq": _rel(eager, seq16)})
    assert e_seq < 0.05, e_seq
    for got in (eager, graph):
        assert _rel(got, ref32) < min(1.5 * e_seq + 1e-3, 0.05), (_rel(got, ref32), e_seq)
    assert lseq == pytest.approx(lref, rel=5e-3)
    assert leager == pytest.approx(lref, rel=5e-3)
    assert lgraph == pytest.approx(leager, rel=5e-3)
