"""Accumulation-window execution (radhip/window.py) against the reference's per-micro-batch order
(Trainer.micro_step = train_epoch, src/main.py:998-1126): K clean passes batched into one, per-group
feature_projection gradients feeding the sequential FGM chain. With every random regulariser off,
the accumulated gradient of one window must equal K sequential micro-steps (fp32: to the atomic-
accumulation noise floor; bf16 / fp16: to their rounding), and the HIP-graph replay must equal the eager
window. The fp16 case is the bench's configuration: K = 4 micro-batches (the batched clean pass runs 4 x B
utterances through every fp16 kernel at its batched size), fp16 autocast with the reference's GradScaler
(src/main.py:28,1049,1077-1108), the FGM chain; gradients compared after the scaler's unscale."""
import json

import numpy as np
import pytest
import torch

from seeded import seeded_fill_

pytestmark = pytest.mark.gpu
DEV = "cuda"


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


def _grads_sequential(golden, amp, K=3, B=4):
    from radhip.train import Trainer
    m, cfg = _model(golden, K)
    tr = Trainer(m, cfg, DEV, total_steps=10, amp_dtype=amp)
    got = []
    tr.optimizer_step = lambda: got.append(_unscaled(tr, tr.grads.flat.clone()))
    xs, ys, lams, perms = _batches(K, B)
    for k in range(K):
        tr.micro_step(xs[k], torch.from_numpy(ys[k]), lams[k], perms[k])
    torch.cuda.synchronize()
    return got[0], float(tr.loss_sum)


def _grads_window(golden, amp, graphs, K=3, B=4):
    from radhip.train import Trainer
    from radhip.window import WindowStep
    m, cfg = _model(golden, K)
    tr = Trainer(m, cfg, DEV, total_steps=10, amp_dtype=amp)
    got = []
    w = WindowStep(tr, B, graphs=graphs)
    xs, ys, lams, perms = _batches(K, B)
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


def test_window_matches_sequential_bf16_and_graph_replay(golden):
    """bf16: the eager window and its graph replay are each as close to the fp32 reference-order gradient
    as the bf16 reference-order run is (all differ from fp32 only by rounding; the captured graph may run
    other MIOpen / hipBLASLt solutions than the eager pass, so it is held to the same bound, not to
    bit-equality with the eager window)."""
    ref32, lref = _grads_sequential(golden, torch.float32)
    seq16, _ = _grads_sequential(golden, torch.bfloat16)
    eager, leager = _grads_window(golden, torch.bfloat16, graphs=False)
    graph, lgraph = _grads_window(golden, torch.bfloat16, graphs=True)
    e_seq = _rel(seq16, ref32)
    print(f"[window bf16] rel L2 vs fp32 reference order: sequential bf16 {e_seq:.3e}, window {_rel(eager, ref32):.3e}, "
          f"graph {_rel(graph, ref32):.3e}; window vs sequential bf16 {_rel(eager, seq16):.3e}")
    # the reference order's own bf16 error is itself noisy (fp32 atomic-order differences amplified by bf16
    # roundings): 3.4-5.6 % over runs of this test. The window and its replay are held to 1.5x the larger of this
    # run's and that 5.6 % level (measured 6.1-7.7 %), under an absolute cap of 10 %: a kernel bug shared by both
    # bf16 runs must not hide behind the relative bound
    assert e_seq < 0.1, e_seq
    for got in (eager, graph):
        assert _rel(got, ref32) < min(1.5 * max(e_seq, 0.056) + 1e-3, 0.1), (_rel(got, ref32), e_seq)
    assert lgraph == pytest.approx(leager, rel=1e-2)
    assert leager == pytest.approx(lref, rel=1e-2)


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
    assert e_seq < 0.05, e_seq
    for got in (eager, graph):
        assert _rel(got, ref32) < min(1.5 * e_seq + 1e-3, 0.05), (_rel(got, ref32), e_seq)
    assert lseq == pytest.approx(lref, rel=5e-3)
    assert leager == pytest.approx(lref, rel=5e-3)
    assert lgraph == pytest.approx(leager, rel=5e-3)
