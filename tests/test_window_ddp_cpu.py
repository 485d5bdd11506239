"""The accumulation window (radhip/window.py::WindowStep, the bench's and CLI's step) under data parallelism,
on CPU with gloo at world size 2, eager (no HIP graphs).

A toy model exposes exactly the hooks WindowStep drives on the dual-stream model: a SincConv-like
`sinc_stream.conv_time` (band-mask slot), and a WavLM-like core with a frozen "CNN" whose features the
adversarial passes reuse, a feature_projection (LayerNorm + Linear, the FGM target) that runs per group
through the window's leaf copies, a SpecAugment time-mask slot and encoder layers with a LayerDrop slot.

Checked: two ranks running WindowStep on half of every micro-batch end with the same parameters and EMA
as ONE process running the reference's sequential micro-steps (Trainer.micro_step: clean pass, FGM on the
accumulated gradient, adversarial pass, restore; step every K) on the whole micro-batches, so the window
batching, the FGM direction taken from the globally reduced gradient (fgm_global_grads at
radhip/window.py:_adv_chain) and the all-reduce in optimizer_step compose to the reference's math.
The HIP fgm_attack kernel is swapped for the same update in torch (no GPU here)."""
import os
import socket
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

L, FR = 48, 4                       # toy waveform length, "CNN" frame size -> T = 12 frames


class _Cfg:
    conv_kernel, conv_stride = [FR], [FR]
    mask_time_prob, mask_time_length, mask_time_min_masks = 0.0, 2, 0
    layerdrop, apply_spec_augment = 0.0, True


class _Conv(torch.nn.Module):
    out_channels = 6

    def __init__(self):
        super().__init__()
        self.mask_dev = None

    def draw_mask(self):
        return 0, 0


class _Sinc(torch.nn.Module):
    """A trainable stand-in for the SincNet stream: the window batches the adversarial passes' forwards and
    backwards of this stream (radhip/window.py::_sinc_adv_forward / _sinc_adv_backward)."""

    def __init__(self):
        super().__init__()
        self.conv_time = _Conv()
        self.proj = torch.nn.Linear(FR, 6)

    def forward(self, x, freq_aug=False):
        return torch.tanh(self.proj(x.view(x.shape[0], -1, FR)))


class _FP(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.layer_norm = torch.nn.LayerNorm(FR)
        self.projection = torch.nn.Linear(FR, 6)


class _Enc(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.layers = torch.nn.ModuleList([torch.nn.Linear(6, 6), torch.nn.Linear(6, 6)])
        self.keep_dev = None


class _Core(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.config = _Cfg()
        self.cnn = torch.nn.Linear(FR, FR)
        self.feature_projection = _FP()
        self.encoder = _Enc()
        self.fp_groups = self.cnn_reuse = self._cnn_feats = self.time_mask_dev = self.cnn_feats_given = None
        for p in self.cnn.parameters():
            p.requires_grad = False

    def forward(self, x):
        if self.cnn_feats_given is not None:
            f = self.cnn_feats_given
        elif self.cnn_reuse == "use" and self._cnn_feats is not None:
            f = self._cnn_feats[1]
        else:
            with torch.no_grad():
                f = torch.tanh(self.cnn(x.view(x.shape[0], -1, FR)))
            if self.cnn_reuse == "store":
                self._cnn_feats = ((x.data_ptr(), tuple(x.shape), x.dtype), f)
        fp = self.feature_projection
        if self.fp_groups is not None:
            parts = [F.linear(F.layer_norm(fk, (FR,), lw, lb, fp.layer_norm.eps), pw, pb)
                     for fk, (lw, lb, pw, pb) in zip(f.chunk(len(self.fp_groups)), self.fp_groups)]
            h = torch.cat(parts)
        else:
            h = fp.projection(fp.layer_norm(f))
        if self.time_mask_dev is not None:
            h = h.masked_fill(self.time_mask_dev[..., None], 0.0)
        for layer in self.encoder.layers:
            h = h + torch.tanh(layer(h))
        return h


class _WavLM(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.core = _Core()

    def _core(self):
        return self.core


class ToyDual(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.sinc_stream = _Sinc()
        self.wavlm_stream = _WavLM()
        self.classifier = torch.nn.Linear(6, 2)
        self.sinc_given = None

    def forward(self, x, Freq_aug=False):
        s = self.sinc_given if self.sinc_given is not None else self.sinc_stream(x, freq_aug=Freq_aug)
        h = self.wavlm_stream.core(x).mean(dim=1) + s.mean(dim=1)
        return h, self.classifier(h)


CFG = {"loss": "Focal", "freq_aug": "False",
       "optim_config": {"base_lr": 5e-3, "wavlm_lr": 1e-2, "weight_decay": 1e-4, "scheduler": "cosine",
                        "scheduler_config": {"eta_min": 1e-6}},
       "training_config": {"use_mixup": False, "accumulation_steps": 2, "use_ema": True, "ema_decay": 0.9,
                           "use_fgm": True, "fgm_epsilon": 0.5, "warmup_steps": 1, "warmup_init_factor": 0.1,
                           "freeze_bn": True, "focal_alpha": 0.9, "focal_gamma": 2.5,
                           "focal_alpha_mode": "scalar"}}


def _torch_fgm(params, grads, backups, eps):
    for p, g, b in zip(params, grads, backups):
        b.copy_(p)
        nrm = torch.linalg.vector_norm(g.double())
        if nrm != 0 and not torch.isnan(nrm):
            p.add_((eps * g.double() / nrm).to(p.dtype))


def _trainer(init):
    import radhip.train as T
    T.fgm_attack = _torch_fgm
    m = ToyDual()
    m.load_state_dict(init)
    return T.Trainer(m, CFG, "cpu", total_steps=4, amp_dtype=torch.float32), m


def _sequential(xs, ys, init):
    tr, m = _trainer(init)
    for i in range(xs.shape[0]):
        tr.micro_step(torch.from_numpy(xs[i]), torch.from_numpy(ys[i]), last_in_epoch=(i == xs.shape[0] - 1))
    return {k: v.detach().clone() for k, v in m.state_dict().items()}, tr.ema.state_dict()


def _windowed(rank, world, xs, ys, init):
    from radhip.window import WindowStep
    tr, m = _trainer(init)
    B = xs.shape[1] // world
    sl = slice(rank * B, (rank + 1) * B)
    w = WindowStep(tr, B, graphs=False, max_len=L)
    for i in range(xs.shape[0]):
        k = i % w.K
        w.xslot(k).copy_(torch.from_numpy(xs[i][sl]))
        w.add(k, ys[i][sl])
        if k == w.K - 1:
            w.run()
    return {k: v.detach().clone() for k, v in m.state_dict().items()}, tr.ema.state_dict()


def _worker(rank, world, port, xs, ys, init, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        params, ema = _windowed(rank, world, xs, ys, init)
        torch.save({"params": params, "ema": ema}, os.path.join(out, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    rng = np.random.default_rng(5)
    xs = rng.standard_normal((4, 4, L)).astype(np.float32)        # 4 micro-batches of 4 = 2 windows of K = 2
    ys = rng.integers(0, 2, (4, 4)).astype(np.int64)
    torch.manual_seed(2)
    init = {k: v.clone() for k, v in ToyDual().state_dict().items()}
    return xs, ys, init


def _close(a, b, what):
    for k, v in a.items():
        torch.testing.assert_close(b[k], v, rtol=2e-5, atol=1e-6, msg=f"{what} {k}")


def test_window_single_process_equals_sequential_micro_steps():
    xs, ys, init = _data()
    ref_p, ref_e = _sequential(xs, ys, init)
    got_p, got_e = _windowed(0, 1, xs, ys, init)
    _close(ref_p, got_p, "params")
    _close(ref_e, got_e, "ema")
    assert not torch.equal(ref_p["wavlm_stream.core.feature_projection.projection.weight"],
                           init["wavlm_stream.core.feature_projection.projection.weight"])


def test_window_two_ranks_equal_single_process_sequential():
    xs, ys, init = _data()
    ref_p, ref_e = _sequential(xs, ys, init)
    with tempfile.TemporaryDirectory() as out:
        mp.start_processes(_worker, args=(2, _free_port(), xs, ys, init, out), nprocs=2, join=True,
                           start_method="spawn")
        got = [torch.load(os.path.join(out, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    for r in range(2):
        _close(ref_p, got[r]["params"], f"rank{r}")
        _close(ref_e, got[r]["ema"], f"rank{r} ema")
    for k in ref_p:
        assert torch.equal(got[0]["params"][k], got[1]["params"][k]), k
