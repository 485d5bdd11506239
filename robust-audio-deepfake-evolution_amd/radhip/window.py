"""Accumulation-window execution of the Phase-6 step (same math as train_epoch, src/main.py:998-1126).

Within one gradient-accumulation window of K micro-batches the parameters do not change: FGM perturbs
feature_projection and restores it before the next micro-batch, and the optimizer steps only at the
end. So the K CLEAN passes are independent of each other and of the adversarial passes, and run here
as ONE batched forward/backward over K*B utterances (every norm is per-utterance: BN frozen, LN/SE/
Mamba per sample). What the FGM chain needs from them is each micro-batch's own feature_projection
gradient: group k of the batch runs feature_projection through its own leaf copy of those four
tensors, so after the batched backward the copies hold g_1..g_K. The K ADVERSARIAL passes stay
sequential, exactly as the reference orders them:
    for k: fp.grad += g_k; FGM.attack() (accumulated grad, incl. adversarial passes < k); adv pass k
           (B utterances, the clean pass's frozen-CNN features of group k); FGM.restore()
then one optimizer step. The SincNet stream does not depend on the FGM perturbation (it sees the same mixed
input; only its band mask is drawn per pass), so the K adversarial passes' SincNet forwards run as ONE batched
pass in the clean graph (each row with its pass's mask) and their backward as ONE batched pass after the last
adversarial pass, from the output gradients the K passes leave in a [K*B, T', 64] buffer (the SincNet backward
is linear in its output gradient at fixed activations; BN is frozen). Per-call random decisions (SincConv band mask, SpecAugment, LayerDrop,
mixup) are drawn on the host in the reference's per-micro-batch order and staged into device
buffers; the clean pass reads them per utterance row. With HIP graphs the window is 1 + K replays.
"""
import os

import numpy as np
import torch

from . import ops
from .linear import direct_grad
from .train import MAX_LEN, _PinnedRing, check_graph_memset_replay, layerdrop_draws, refuse_step_tuning  # noqa: F401
from .wavlm import compute_time_mask


def _add_many(dsts, srcs, copy=False):
    """dsts[k] += srcs[k] (copy: =) in one HIP launch per 64 tensors on the GPU (ops.add_many); torch's multi-tensor
    ops for the CPU runs of the window (the gloo tests of the host logic)."""
    if not dsts:
        return
    if dsts[0].is_cuda:
        ops.add_many(dsts, srcs, copy=copy)
    elif copy:
        torch._foreach_copy_(dsts, srcs)
    else:
        torch._foreach_add_(dsts, srcs)


def window_eligible(trainer):
    """True when batching the window's clean passes is exact: no BatchNorm computes batch statistics
    (freeze_bn, or a model without BatchNorm)."""
    if trainer.freeze_bn:
        return True
    return not any(isinstance(m, torch.nn.modules.batchnorm._BatchNorm) for m in trainer.model.modules())


class WindowStep:
    def __init__(self, trainer, batch, K=None, graphs=True, max_len=MAX_LEN):
        tr = trainer
        m = tr.model
        dev = tr.device
        self.tr, self.B, self.K = tr, int(batch), int(K or tr.accum)
        if self.K < 1:
            raise ValueError("window needs K >= 1")
        if not window_eligible(tr):
            raise ValueError("the accumulation window batches K micro-batches into one pass, which is the same "
                             "math only when every BatchNorm is frozen (freeze_bn) or absent")
        N = self.K * self.B
        self.N = N
        self.graphs_on = graphs
        self.x = torch.zeros(N, max_len, device=dev)
        self.ya = torch.zeros(N, dtype=torch.long, device=dev)
        self.yb = torch.zeros(N, dtype=torch.long, device=dev)
        self.lam = torch.ones(self.K, device=dev)
        self.conv = m.sinc_stream.conv_time
        self.core = m.wavlm_stream._core()
        cfg = self.core.config
        T = max_len
        for k, st in zip(cfg.conv_kernel, cfg.conv_stride):
            T = (T - k) // st + 1
        self.T = T
        nl = len(self.core.encoder.layers)
        self.nl = nl
        self.spec_on = bool(getattr(cfg, "apply_spec_augment", True)) and cfg.mask_time_prob > 0
        # device draws: clean rows (one per utterance) and one set per adversarial pass
        self.c_mask = torch.zeros(N, 2, dtype=torch.int32, device=dev)
        self.c_tmask = torch.zeros(N, T, dtype=torch.bool, device=dev)
        self.c_keep = torch.ones(N, nl, dtype=torch.bool, device=dev)
        self.a_mask = torch.zeros(self.K, 2, dtype=torch.int32, device=dev)
        self.a_mask_rows = torch.zeros(N, 2, dtype=torch.int32, device=dev)   # a_mask[k] on micro-batch k's rows
        self.a_tmask = torch.zeros(self.K, self.B, T, dtype=torch.bool, device=dev)
        self.a_keep = torch.ones(self.K, nl, dtype=torch.bool, device=dev)
        self.adv = tr.fgm is not None
        # batched adversarial SincNet passes (see the module docstring; RADHIP_SINC_BATCH=0: per pass)
        self.sinc_batched = (self.adv and hasattr(m, "sinc_given") and hasattr(m, "sinc_stream")
                             and os.environ.get("RADHIP_SINC_BATCH", "1") != "0")
        self.f_adv = None
        self.f_adv_leaf = None
        self.dfa = None
        # the model's SincNet stream: the clean pass's SincNet branch and this batched pass share the window's
        # SincNet weight layouts (ops.SCONV_WCACHE), so they must be ordered on one stream
        self._sinc_side = (m.sinc_side_stream(self.x) if self.sinc_batched and hasattr(m, "sinc_side_stream")
                           else None)
        # feature_projection: the real tensors and K leaf copies whose grads live in one flat buffer
        fp = self.core.feature_projection
        self.fp_real = [fp.layer_norm.weight, fp.layer_norm.bias, fp.projection.weight, fp.projection.bias]
        n = sum(p.numel() for p in self.fp_real)
        self.fp_grad = torch.zeros(self.K, n, device=dev)
        self.fp_copies = []
        for k in range(self.K):
            group, off = [], 0
            for p in self.fp_real:
                c = torch.empty_like(p, requires_grad=True)
                c.grad = self.fp_grad[k, off:off + p.numel()].view_as(p)
                off += p.numel()
                group.append(c)
            self.fp_copies.append(tuple(group))
        self._flat_copies = [c for g in self.fp_copies for c in g]
        self._flat_real = [p for _ in range(self.K) for p in self.fp_real]
        # parameters whose gradients autograd delivers (everything trainable but the LoRA weights, which
        # the fused WavLM layer accumulates into .grad itself): during a pass their .grad is unset, so
        # autograd hands each gradient over instead of launching one fp32 add per parameter into the flat
        # buffer; one multi-tensor add per pass then accumulates them (_pass_grads)
        self.handed = [p for n, p in m.named_parameters() if p.requires_grad and "lora_" not in n and not direct_grad(p)]
        self.ring = _PinnedRing(8192 + 2 * N * 8 + N * (T + nl + 16) + self.K * (self.B * T + nl + 64))
        self.graphs = None
        self._wcache = {}
        # the detector head's fp32 linear parameters (radhip.linear.SideLinear), cast to the autocast dtype once per
        # window by ONE launch into persistent buffers (_precast_linears) instead of one cast per tensor
        from .linear import SideLinear
        self._lin_src = [p for mod in m.modules() if isinstance(mod, SideLinear)
                         for p in (mod.weight, mod.bias) if p is not None and p.dtype == torch.float32]
        self._lin_dst = None
        self._sconv_w = None
        self.chain_captured = False
        self.feats = None
        self._host = None
        self.reset_host()

    # ------------------------------------------------------------------ host staging ----------
    def reset_host(self):
        N, K, B, T, nl = self.N, self.K, self.B, self.T, self.nl
        self._host = dict(ya=np.zeros(N, np.int64), yb=np.zeros(N, np.int64), lam=np.ones(K, np.float32),
                          c_mask=np.zeros((N, 2), np.int32), c_tmask=np.zeros((N, T), bool),
                          c_keep=np.ones((N, nl), bool), a_mask=np.zeros((K, 2), np.int32),
                          a_tmask=np.zeros((K, B, T), bool), a_keep=np.ones((K, nl), bool),
                          a_mask_rows=np.zeros((N, 2), np.int32))
        self._added = 0

    def _draw_pass(self):
        """One forward's host draws in the reference order: SpecAugment (numpy), LayerDrop (torch CPU),
        SincConv band mask (numpy + python random)."""
        c = self.core.config
        tm = (compute_time_mask(self.B, self.T, c.mask_time_prob, c.mask_time_length, c.mask_time_min_masks)
              if self.spec_on else np.zeros((self.B, self.T), dtype=bool))
        p = c.layerdrop
        keep = np.ones(self.nl, dtype=bool)
        r = layerdrop_draws(self.nl)
        if p > 0:
            keep[1:] = ~(r[1:] < p)
        lo, hi = self.conv.draw_mask() if self.tr.freq_aug else (0, 0)
        return tm, keep, np.array([lo, hi], dtype=np.int32)

    def xslot(self, k):
        """Row block of micro-batch k: Augmenter.run(..., out=window.xslot(k))."""
        return self.x[k * self.B:(k + 1) * self.B]

    def add(self, k, y, lam=1.0, perm=None):
        """Register micro-batch k (already mixed into xslot(k)) and make its clean-pass and
        adversarial-pass draws, in the order the reference makes them."""
        h, B = self._host, self.B
        y = np.asarray(y, dtype=np.int64).reshape(-1)
        if y.shape[0] != B or k != self._added:
            raise ValueError("window: micro-batches must be added in order with B labels each")
        sl = slice(k * B, (k + 1) * B)
        h["ya"][sl] = y
        h["yb"][sl] = y[np.asarray(perm)] if perm is not None else y
        h["lam"][k] = lam
        tm, keep, mk = self._draw_pass()
        h["c_tmask"][sl], h["c_keep"][sl], h["c_mask"][sl] = tm, keep[None, :], mk[None, :]
        if self.adv:
            tm, keep, mk = self._draw_pass()
            h["a_tmask"][k], h["a_keep"][k], h["a_mask"][k] = tm, keep, mk
            h["a_mask_rows"][sl] = mk[None, :]
        self._added += 1

    def _stage(self):
        h = self._host
        self.ring.stage([(h["ya"], self.ya), (h["yb"], self.yb), (h["lam"], self.lam), (h["c_mask"], self.c_mask),
                         (h["c_tmask"], self.c_tmask), (h["c_keep"], self.c_keep), (h["a_mask"], self.a_mask),
                         (h["a_tmask"], self.a_tmask), (h["a_keep"], self.a_keep),
                         (h["a_mask_rows"], self.a_mask_rows)])

    # ------------------------------------------------------------------ passes ----------------
    def _amp(self):
        """Autocast with its weight-cast cache on. Every pass of a window runs inside one outer context
        (run / capture), so each trainable fp32 weight is cast to the compute dtype once per window, by the
        clean pass (inside graph G0 when graphed), and the adversarial passes reuse that copy: the weights
        do not change within a window. The one exception, the FGM target feature_projection, is perturbed
        between passes and is cast without the cache (WavLMModel.forward, fp_nocache)."""
        tr = self.tr
        return torch.autocast("cuda", dtype=tr.amp_dtype, enabled=tr.amp_dtype != torch.float32, cache_enabled=True)

    def _loss(self, out, k):
        tr, B = self.tr, self.B
        lam = self.lam[k]
        ya, yb = self.ya[k * B:(k + 1) * B], self.yb[k * B:(k + 1) * B]
        return lam * tr.criterion(out, ya) + (1.0 - lam) * tr.criterion(out, yb)

    def _focal_fused(self, out):
        from .train import FocalLoss
        return isinstance(self.tr.criterion, FocalLoss) and out.is_cuda and out.shape[1] <= 16

    def _pass_loss(self, out, k=None):
        """The pass's loss / accum: micro-batch k's rows (adversarial pass) or all K (clean pass). The focal
        criterion is one HIP launch per pass (ops.mixup_focal); any other criterion runs as modules."""
        tr, B, K = self.tr, self.B, self.K
        if self._focal_fused(out):
            if k is None:
                return ops.mixup_focal(out, self.ya, self.yb, self.lam, B, tr.criterion, tr.accum)
            sl = slice(k * B, (k + 1) * B)
            return ops.mixup_focal(out, self.ya[sl], self.yb[sl], self.lam[k:k + 1], B, tr.criterion, tr.accum)
        if k is None:
            return sum(self._loss(out[j * B:(j + 1) * B], j) for j in range(K)) / tr.accum
        return self._loss(out, k) / tr.accum

    def _pass_grads(self, fn):
        """Run one forward/backward with the handed-over gradients unset, then add them into the flat
        fp32 buffer in one multi-tensor launch and point .grad back at its views."""
        views = [p.grad for p in self.handed]
        for p in self.handed:
            p.grad = None
        try:
            fn()
        finally:
            got = [(v, p.grad) for p, v in zip(self.handed, views) if p.grad is not None]
            if got:
                _add_many([v for v, _ in got], [g for _, g in got])
            for p, v in zip(self.handed, views):
                p.grad = v

    def _precast_linears(self):
        """Fill the window's weight-cast cache (radhip.linear._cast) for every SideLinear parameter with one
        multi-tensor launch (ops.cast_many); the parameters do not change within a window."""
        dt = self.tr.amp_dtype
        if dt not in ops.HALF or not self._lin_src or not self._lin_src[0].is_cuda:
            return
        if self._lin_dst is None or self._lin_dst[0].dtype != dt:
            self._lin_dst = [torch.empty_like(p, dtype=dt) for p in self._lin_src]
        ops.cast_many([p.detach() for p in self._lin_src], self._lin_dst)
        for p, c in zip(self._lin_src, self._lin_dst):
            self._wcache[("lin", id(p), c.dtype)] = (p, c)

    def _precast_sconv(self):
        """Both 16-bit layouts of every SincNet stack convolution weight into the window's cache in one launch
        (ops.sconv_prep_many); the convolutions' first use then finds them."""
        dt = self.tr.amp_dtype
        if dt not in ops.HALF or not hasattr(self.tr.model, "sinc_stream") or os.environ.get("RADHIP_SCONV_PREP") == "0":
            return
        if self._sconv_w is None:
            self._sconv_w = [mod.weight for mod in self.tr.model.sinc_stream.modules()
                             if isinstance(mod, torch.nn.Conv2d) and mod.weight.dim() == 4 and mod.weight.shape[-1] == 3]
        ops.sconv_prep_many(self._sconv_w, dt)    # the parameters themselves: the cache is keyed by them

    def _clean_pass(self):
        self._wcache = {}                  # weight layouts prepared by this pass, reused by the window's others
        ops.SCONV_WCACHE = self._wcache
        self._precast_linears()
        self._precast_sconv()
        self._pass_grads(self._clean_pass_body)

    def _sinc_adv_forward(self):
        """The K adversarial passes' SincNet forwards as one pass over the window's rows (row block k with
        adversarial pass k's band mask). Leaves one [B, T', 64] leaf per pass whose .grad is a view of dfa."""
        tr, B = self.tr, self.B
        self.conv.mask_dev = self.a_mask_rows
        side = self._sinc_side
        if side is not None:       # a parallel branch of the clean pass (joined at its end, _sinc_join)
            cur = torch.cuda.current_stream(self.x.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                f = tr.model.sinc_stream(self.x, freq_aug=tr.freq_aug)
            f.record_stream(cur)
        else:
            f = tr.model.sinc_stream(self.x, freq_aug=tr.freq_aug)
        if self.dfa is None or self.dfa.shape != f.shape or self.dfa.dtype != f.dtype:
            self.dfa = torch.zeros_like(f)
        else:
            self.dfa.zero_()
        self.f_adv = f
        self.f_adv_leaf = []
        for k in range(self.K):
            leaf = f[k * B:(k + 1) * B].detach().requires_grad_()
            leaf.grad = self.dfa[k * B:(k + 1) * B]
            self.f_adv_leaf.append(leaf)

    def _sinc_join(self):
        if self.sinc_batched and self._sinc_side is not None:
            torch.cuda.current_stream(self.x.device).wait_stream(self._sinc_side)

    def _sinc_adv_backward(self):
        """The batched SincNet backward of the K adversarial passes (after the last one)."""
        f, self.f_adv = self.f_adv, None
        torch.autograd.backward(f, self.dfa)

    def _clean_pass_body(self):
        tr, core, B = self.tr, self.core, self.B
        if self.sinc_batched:
            self._sinc_adv_forward()
        with torch.no_grad():
            _add_many(self._flat_copies, self._flat_real, copy=True)
            self.fp_grad.zero_()
        core.fp_groups = self.fp_copies
        core.cnn_reuse = "store"
        self.conv.mask_dev = self.c_mask
        core.time_mask_dev = self.c_tmask
        core.encoder.keep_dev = self.c_keep
        try:
            with self._amp():
                _, out = tr.model(self.x, Freq_aug=tr.freq_aug)
                loss = self._pass_loss(out)
            with ops.wgrad_batch():
                tr.scaler.scale(loss).backward()
            tr.loss_sum.add_(loss.detach().double() * (tr.accum * B))
        finally:
            self._sinc_join()
            core.fp_groups = None
            self.feats = core._cnn_feats[1] if core._cnn_feats is not None else None
            core.cnn_reuse = None

    def _adv_pass(self, k):
        ops.SCONV_WCACHE = self._wcache

        def body():
            self._adv_pass_body(k)
            if self.sinc_batched and k == self.K - 1:
                self._sinc_adv_backward()
        try:
            self._pass_grads(body)
        finally:
            ops.SCONV_WCACHE = None

    def _adv_pass_body(self, k):
        tr, core, B = self.tr, self.core, self.B
        self.conv.mask_dev = self.a_mask[k]
        core.time_mask_dev = self.a_tmask[k]
        core.encoder.keep_dev = self.a_keep[k]
        if self.feats is not None:
            core.cnn_feats_given = self.feats[k * B:(k + 1) * B]
        if self.sinc_batched:
            tr.model.sinc_given = self.f_adv_leaf[k]
        try:
            with self._amp():
                _, out = tr.model(self.x[k * B:(k + 1) * B], Freq_aug=tr.freq_aug)
                adv = self._pass_loss(out, k)
            with ops.wgrad_batch():
                tr.scaler.scale(adv).backward()
        finally:
            core.cnn_feats_given = None
            if self.sinc_batched:
                tr.model.sinc_given = None

    def _unbind(self):
        ops.SCONV_WCACHE = None
        self.conv.mask_dev = None
        self.core.time_mask_dev = None
        self.core.encoder.keep_dev = None

    def _prefix_grad(self, k):
        """feature_projection.grad += g_k (micro-batch k's clean gradient). Without FGM feature_projection
        is frozen (no .grad) and the copies' gradients are never used."""
        if not self.adv:
            return
        _add_many([p.grad for p in self.fp_real], [self.fp_copies[k][i].grad for i in range(4)])

    def _adv_step(self, k):
        """Micro-batch k's FGM chain link: its clean gradient into feature_projection.grad, the attack on the
        accumulated gradient, the adversarial pass, the restore. All device work, so with one process it is
        captured as ONE graph per k (no host round trip between the replays); with several ranks the attack's
        all-reduce (fgm_global_grads) stays outside the graphs."""
        tr = self.tr
        self._prefix_grad(k)
        if self.adv:
            tr.fgm.attack()
            self._adv_pass(k)
            tr.fgm.restore()

    def _adv_chain(self, run_adv):
        tr = self.tr
        for k in range(self.K):
            self._prefix_grad(k)
            if self.adv:
                tr.fgm.attack()
                run_adv(k)
                tr.fgm.restore()

    def _chain_in_graph(self):
        import torch.distributed as dist
        return self.adv and not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1)

    # ------------------------------------------------------------------ driver ----------------
    def capture(self, warmup=2):
        tr = self.tr
        refuse_step_tuning()
        check_graph_memset_replay(tr.device)
        tr.train_mode()
        saved_loss = tr.loss_sum.clone()
        self._stage()
        side = torch.cuda.Stream(device=tr.device)
        side.wait_stream(torch.cuda.current_stream(tr.device))
        chain = self._chain_in_graph()
        with torch.cuda.stream(side):
            for _ in range(warmup):
                with self._amp():
                    self._clean_pass()
                    self._adv_chain(self._adv_pass)
        torch.cuda.current_stream(tr.device).wait_stream(side)
        torch.cuda.synchronize(tr.device)
        if chain:   # capture must not leave the warm-up's FGM state behind: feature_projection was restored
            tr.fgm.backup = {}

        ops.reserve_graph_workspace(tr.device)   # split-K GEMMs of the captured passes (the warm-up sized it)
        def new_graph():
            if ops.CAPTURE_TIMING is not None:   # bench.py: stamp the first launch sites of each graph
                ops.CAPTURE_TIMING.new_graph()
            return torch.cuda.CUDAGraph()
        with self._amp():        # one cast cache for G0 and the adversarial graphs (see _amp)
            g0 = new_graph()
            with torch.cuda.graph(g0):
                self._clean_pass()
            gadv = []
            if self.adv:
                # the captured attack perturbs feature_projection in place: keep the real values to put back
                fp_saved = [p.detach().clone() for p in self.fp_real]
                if chain and os.environ.get("RADHIP_ADV_GRAPHS", "one") == "one":
                    # the K chain links back to back in ONE graph: every graph replay starts with the device
                    # waiting on the host's submission of its first nodes (≈80-100 µs per kernel for the first
                    # layer's launches in the rocprofv3 trace), once per window instead of once per link
                    g = new_graph()
                    with torch.cuda.graph(g):
                        for k in range(self.K):
                            self._adv_step(k)
                    gadv.append(g)
                else:
                    for k in range(self.K):
                        g = new_graph()
                        with torch.cuda.graph(g):
                            if chain:
                                self._adv_step(k)
                            else:
                                self._adv_pass(k)
                        gadv.append(g)
                with torch.no_grad():
                    for p, v in zip(self.fp_real, fp_saved):
                        p.copy_(v)
                tr.fgm.backup = {}
        ops.finalize_graph_workspace(tr.device)     # tickets grown inside a capture: zero before any replay
        self._unbind()
        tr.grads.zero()
        self.fp_grad.zero_()
        tr.loss_sum.copy_(saved_loss)
        self.graphs = (g0, gadv)
        self.chain_captured = chain

    def run(self, last_in_epoch=False):
        """Execute the window (every micro-batch added); ends with the optimizer step."""
        if self._added != self.K:
            raise RuntimeError(f"window has {self._added} of {self.K} micro-batches")
        tr = self.tr
        tr.train_mode()
        self._stage()
        if self.graphs_on:
            if self.graphs is None:
                self.capture()
            ops.SCONV_WCACHE = None
            g0, gadv = self.graphs
            g0.replay()
            if self.chain_captured:
                for g in gadv:
                    g.replay()
            else:
                self._adv_chain(lambda k: gadv[k].replay())
        else:
            with self._amp():
                self._clean_pass()
                self._adv_chain(self._adv_pass)
            self._unbind()
        tr.count_micro(self.K)      # a whole window: K micro-batches, then the step (epoch_micro % K == 0)
        tr.n_seen += self.N
        tr.optimizer_step()
        self.reset_host()
