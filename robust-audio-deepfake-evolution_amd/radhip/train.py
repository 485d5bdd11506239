"""Phase-6 training engine on MI355X: GPU augmentation, FGM, focal loss, EMA, DDP gradient reducer,
and the micro-batch / optimizer-step loop.

Reference semantics (src/main.py):
  train_epoch :998-1126  mixup -> autocast fwd -> loss/accum -> bwd -> [FGM attack -> fwd -> bwd ->
                         restore] -> every `accum` micro-batches: unscale, clip 3.0, step, zero_grad,
                         EMA update, scheduler step
  FGM :74-100, focal loss :297-305 (kornia), AdamW groups :416-457, schedule :460-483,
  EMA :491-496, FGM group :514-544; per-utterance augmentation data_utils.py:163-184.
Design differences (same math): augmentation runs batched on the GPU from utterances resident in
HBM; the loss is accumulated on the device (no per-micro-batch .item() sync); gradients of all
trainable tensors live in ONE flat fp32 buffer so a data-parallel step is one RCCL all-reduce.
"""
import math
import os
import random

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from . import _lib, ops
from .augment import CODEC_RATES, draw_rawboost
from .ops import add_many, fgm_attack, pad_mixup, rawboost_batch, resample_batch, resample_kernel
from .wavlm import compute_time_mask

MAX_LEN = 64600


# ------------------------------------------------------------------------------- losses ------
class FocalLoss(nn.Module):
    """kornia.losses.FocalLoss(alpha, gamma, reduction='mean') (src/main.py:297-305) for [B, C] logits.

    kornia is absent from the image and from the reference's requirements, and the two kornia
    generations differ, so both are restated (parity unpinned):
      'per_class' (kornia >= 0.7, default): loss_tmp[b, c] = -alpha_c (1 - p_bc)^gamma log p_bc onehot[b, c]
                  with alpha_c = [1 - alpha, alpha, alpha, ...]; 'mean' averages loss_tmp over all B*C
                  elements (the class axis is kept, so the mean divides by C as well).
      'scalar'    (kornia < 0.7): loss[b] = -alpha (1 - p_b,y)^gamma log p_b,y, mean over B.
    alpha None drops the factor. (1 - p)^gamma uses p = exp(log_softmax), so p -> 1 gives 0, not NaN."""

    def __init__(self, alpha=0.25, gamma=2.0, alpha_mode="per_class"):
        super().__init__()
        if alpha_mode not in ("per_class", "scalar"):
            raise ValueError(f"focal alpha_mode must be 'per_class' or 'scalar', got {alpha_mode!r}")
        self.alpha, self.gamma, self.alpha_mode = alpha, gamma, alpha_mode

    def forward(self, logits, target):
        logp = F.log_softmax(logits.float(), dim=1)
        lp = logp.gather(1, target[:, None]).squeeze(1)
        w = torch.pow(1.0 - lp.exp(), self.gamma)
        if self.alpha is None:
            a = 1.0
        elif self.alpha_mode == "per_class":
            a = torch.where(target == 0, 1.0 - self.alpha, self.alpha).to(lp.dtype)
        else:
            a = self.alpha
        per_utt = -a * w * lp
        if self.alpha_mode == "per_class":
            return per_utt.sum() / (logits.shape[0] * logits.shape[1])
        return per_utt.mean()


def build_criterion(config, device):
    """Loss selection of main.py:270-312 (focal when loss == 'Focal' or use_focal_loss, else weighted CE)."""
    tc = config.get("training_config", {})
    if config.get("loss") == "Focal" or tc.get("use_focal_loss", False):
        return FocalLoss(tc.get("focal_alpha", 0.25), tc.get("focal_gamma", 2.0),
                         tc.get("focal_alpha_mode", "per_class"))
    w = torch.tensor([0.1, 0.9], device=device)
    return nn.CrossEntropyLoss(weight=w, label_smoothing=tc.get("label_smoothing", 0.0))


def no_grad_params(model):
    """Trainable parameters the reference's forward never uses, so they never get a .grad there and AdamW (and
    its weight decay) and clip_grad_norm_ skip them: bypassed LoRA adapters (radhip.wavlm.LoraLinear) and the
    SincNet blocks' dead bn1 affine weights (Residual_block.dead_parameters)."""
    from .wavlm import inert_lora_params
    out = list(inert_lora_params(model))
    for m in model.modules():
        if hasattr(m, "dead_parameters"):
            out += [p for p in m.dead_parameters() if p.requires_grad]
    return out


# --------------------------------------------------------------------------------- FGM -------
class FGM:
    """FGM on parameters whose name contains `emb_name` (main.py:74-100), on the HIP kernel.
    `grad_hook(list_of_grads) -> list_of_grads` lets DDP hand in the globally reduced gradient."""

    def __init__(self, model, emb_name="feature_projection", epsilon=1.0, grad_hook=None):
        self.model, self.emb_name, self.epsilon = model, emb_name, epsilon
        self.grad_hook = grad_hook
        self.backup = {}

    def _targets(self):
        return [(n, p) for n, p in self.model.named_parameters() if p.requires_grad and self.emb_name in n]

    def attack(self):
        tg = self._targets()
        with_grad = [(n, p) for n, p in tg if p.grad is not None]
        for n, p in tg:
            if p.grad is None:
                self.backup[n] = p.data.clone()
        if not with_grad:
            return
        ps = [p.data for _, p in with_grad]
        gs = [p.grad.contiguous() for _, p in with_grad]
        if self.grad_hook is not None:
            gs = self.grad_hook(gs)
        bks = [torch.empty_like(p) for p in ps]
        fgm_attack(ps, gs, bks, self.epsilon)
        for (n, _), b in zip(with_grad, bks):
            self.backup[n] = b

    def restore(self):
        pairs = [(p.data, self.backup[n]) for n, p in self.model.named_parameters()
                 if p.requires_grad and self.emb_name in n and n in self.backup]
        if pairs and all(d.is_cuda and d.dtype == torch.float32 and d.is_contiguous() and b.is_contiguous()
                         for d, b in pairs):
            add_many([d for d, _ in pairs], [b for _, b in pairs], copy=True)   # one launch for every target
        else:
            for d, b in pairs:
                d.copy_(b)
        self.backup = {}


# --------------------------------------------------------------------------------- EMA -------
class EMA:
    """AveragedModel(model, multi_avg_fn=get_ema_multi_avg_fn(decay)) restricted to the tensors that
    can change (lerp(a, a, w) == a, so frozen tensors are unaffected in the reference as well).
    First update copies. Buffers are not averaged (use_buffers=False): like the reference's deep copy,
    the EMA model keeps the BatchNorm buffers it was constructed with (identical to the live ones
    whenever BN is frozen), and swap() exchanges those too."""

    def __init__(self, model, decay=0.999):
        self.model, self.decay = model, decay
        self.names = [n for n, p in model.named_parameters() if p.requires_grad]
        self.shadow = None
        self.n_averaged = 0
        self.buf_names = [n for n, _ in model.named_buffers()]
        self.buffers = [b.detach().clone() for _, b in model.named_buffers()]

    def refresh_names(self):
        self.names = [n for n, p in self.model.named_parameters() if p.requires_grad]
        self._cur_params = None
        self.shadow = None if self.n_averaged == 0 else self.shadow

    @torch.no_grad()
    def update(self):
        cur = getattr(self, "_cur_params", None)
        if cur is None:    # the name walk (~9000 modules) once; parameters are updated in place, refresh_names rebinds
            named = dict(self.model.named_parameters())
            cur = self._cur_params = [named[n].detach() for n in self.names]
        if self.shadow is None or self.n_averaged == 0:
            self.shadow = [c.clone() for c in cur]
        else:
            torch._foreach_lerp_(self.shadow, cur, 1.0 - self.decay)
        self.n_averaged += 1

    @torch.no_grad()
    def swap(self):
        """Exchange live and EMA values (call twice to restore)."""
        if self.shadow is None:
            return
        params = dict(self.model.named_parameters())
        bufs = dict(self.model.named_buffers())
        for n, s in list(zip(self.names, self.shadow)) + list(zip(self.buf_names, self.buffers)):
            live = params[n].data if n in params else bufs[n]
            tmp = live.clone()
            live.copy_(s)
            s.copy_(tmp)

    def state_dict(self):
        """Full model state dict with EMA values (the reference saves ema_model.state_dict()): EMA
        parameters, the construction-time buffers, live values for everything never averaged."""
        sd = {k: v.detach().clone() for k, v in self.model.state_dict().items()}
        for n, b in zip(self.buf_names, self.buffers):
            if n in sd:
                sd[n] = b.detach().clone()
        if self.shadow is not None:
            for n, s in zip(self.names, self.shadow):
                sd[n] = s.detach().clone()
        return sd

    def train_state(self):
        return {"names": list(self.names), "n_averaged": self.n_averaged,
                "shadow": None if self.shadow is None else [s.detach().clone() for s in self.shadow],
                "buf_names": list(self.buf_names), "buffers": [b.detach().clone() for b in self.buffers]}

    def load_train_state(self, st):
        if list(st["names"]) != self.names or list(st["buf_names"]) != self.buf_names:
            raise ValueError("EMA state was saved for a different set of tensors")
        self.n_averaged = int(st["n_averaged"])
        self.shadow = None if st["shadow"] is None else [s.to(b.device) for s, b in
                                                         zip(st["shadow"], self._live_params())]
        self.buffers = [b.to(l.device) for b, l in zip(st["buffers"], self.model.buffers())]

    def _live_params(self):
        params = dict(self.model.named_parameters())
        return [params[n] for n in self.names]


# ---------------------------------------------------------------------- flat gradients -------
class FlatGrads:
    """Every trainable tensor's .grad is a view into one contiguous fp32 buffer: zero_grad is one
    memset, clipping one norm, and a data-parallel step one all-reduce (11.9 MB for Phase 6)."""

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        total = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(total, device=dev, dtype=torch.float32)
        off = 0
        self._ptrs = []
        for p in self.params:
            n = p.numel()
            assert p.dtype == torch.float32
            p.grad = self.flat[off:off + n].view_as(p)
            self._ptrs.append(p.grad.data_ptr())
            off += n

    def bound(self):
        """True while every parameter's .grad is still its view of the flat buffer."""
        return all(p.grad is not None and p.grad.data_ptr() == q for p, q in zip(self.params, self._ptrs))

    def clip_norm_(self, max_norm):
        """torch.nn.utils.clip_grad_norm_ over the parameters (error_if_nonfinite off) on the flat buffer: the total
        2-norm in one reduction and min(1, max_norm / (norm + 1e-6)) applied in one multiply, instead of a norm per
        tensor (torch's multi-tensor kernels deal 64 K elements per block: ~0.1 ms per step for these ~3 M)."""
        norm = torch.linalg.vector_norm(self.flat, 2)
        self.flat.mul_(torch.clamp(max_norm / (norm + 1e-6), max=1.0))
        return norm

    def zero(self):
        self.flat.zero_()

    def all_reduce_mean(self, group=None):
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
            self.flat.div_(dist.get_world_size(group))


def fgm_global_grads(grads):
    """DDP: FGM direction from the globally accumulated gradient (sum over ranks; the direction is
    scale-invariant). One small all-reduce of the feature_projection grads per attack."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return grads
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat)
    out, off = [], 0
    for g in grads:
        out.append(flat[off:off + g.numel()].view_as(g))
        off += g.numel()
    return out


# ------------------------------------------------------------------------- augmentation -------
class Augmenter:
    """Per-utterance RawBoost + codec decisions drawn on the host in the reference's order
    (Dataset_ASVspoof2019_train.__getitem__, data_utils.py:163-184), executed as one batched kernel
    per stage on the GPU, then pad_random/tile + mixup gather into the [B, 64600] model input."""

    def __init__(self, device, algo=0, rawboost_p=1.0, use_codec=False, codec_p=0.5, max_len=MAX_LEN,
                 exact_noise=False):
        self.device = torch.device(device)
        self.algo, self.rawboost_p = int(algo), float(rawboost_p)
        # exact_noise: the ISD / SSI noise is the reference's own numpy draws (randn / choice per sample,
        # src/rawboost.py:66-95), uploaded per micro-batch; otherwise one numpy seed per call keys a device
        # Philox stream (the bench and the default train path)
        self.exact_noise = bool(exact_noise)
        self.use_codec, self.codec_p = bool(use_codec), float(codec_p)
        self.max_len = max_len
        self.algo_ids = [1, 2, 3, 4] if self.algo == 5 else [self.algo]
        kerns, self.kinfo, off = [], {}, 0
        for sr in CODEC_RATES:
            for a, b in ((16000, sr), (sr, 16000)):
                k, w, og, ng = resample_kernel(a, b)
                self.kinfo[(a, b)] = (off, w, og, ng)
                kerns.append(k.reshape(-1))
                off += k.numel()
        self.kernels = torch.cat(kerns).to(self.device)

    # --- host draws (mirror rawboost.py / data_utils.py draw order; per-sample noise -> Philox seed)
    def _draw_rawboost(self, n):
        """The record, or (record, isd noise, ssi noise) with exact_noise."""
        return draw_rawboost(n, self.algo_ids[np.random.randint(0, len(self.algo_ids))], exact=self.exact_noise)

    def codec_len(self, n, sr):
        _, _, ogd, ngd = self.kinfo[(16000, sr)]
        _, _, ogu, ngu = self.kinfo[(sr, 16000)]
        nd = -(-ngd * n // ogd)
        return -(-ngu * nd // ogu)

    def draw(self, lens):
        """Host decisions for a batch, per utterance in the reference's order: RawBoost gate + draws,
        codec gates + rate, then the pad_random crop start (on the post-codec length)."""
        plan = []
        for n in lens:
            rec = None
            if self.algo != 0 and random.random() < self.rawboost_p:
                rec = self._draw_rawboost(n)
            sr = None
            if self.use_codec and random.random() < self.codec_p:
                if random.random() < 0.5:                       # apply_codec_aug's inner gate (:35)
                    sr = random.choice(list(CODEC_RATES))
            m = self.codec_len(n, sr) if sr is not None else n
            # pad_random: crop at randint(len - max_len) (a length of exactly max_len, which makes the
            # reference's randint(0) raise, is taken whole)
            start = int(np.random.randint(m - self.max_len)) if m > self.max_len else 0
            plan.append((rec, sr, start))
        return plan

    def run(self, raw, offsets, lens, plan, perm=None, lam=1.0, out=None):
        """raw: flat fp32 device buffer holding the utterances at `offsets`; returns x [B, max_len].
        The batch is first packed contiguously (one gather launch), so every later stage addresses a
        compact [sum(lens)] buffer whatever the layout of the resident corpus."""
        B = len(lens)
        total = int(sum(lens))
        work = torch.cat([raw[int(o):int(o) + int(n)] for o, n in zip(offsets, lens)])
        offs, acc = [], 0
        for n in lens:
            offs.append(acc)
            acc += int(n)
        cur_lens = list(lens)
        packed = work
        recs, isd, ssi = [], None, None
        for b, (rec, _, _) in enumerate(plan):
            if isinstance(rec, tuple):          # exact_noise draws: (record, isd noise*mask, ssi noise)
                rec, nm, nz = rec
                for arr, name in ((nm, "isd"), (nz, "ssi")):
                    if arr is None:
                        continue
                    if name == "isd":
                        isd = np.zeros(total) if isd is None else isd
                        isd[offs[b]:offs[b] + lens[b]] = arr
                    else:
                        ssi = np.zeros(total) if ssi is None else ssi
                        ssi[offs[b]:offs[b] + lens[b]] = arr
            r = rec if rec is not None else _lib.RawboostUtt()
            r.offset, r.len = int(offs[b]), int(lens[b])
            if rec is None:
                r.algo = 0
            recs.append(r)
        if any(r.algo != 0 for r in recs):
            work = rawboost_batch(packed, recs,
                                  noise_isd=None if isd is None else torch.from_numpy(isd).to(self.device),
                                  noise_ssi=None if ssi is None else torch.from_numpy(ssi).to(self.device))
        codec = [(b, sr) for b, (_, sr, _) in enumerate(plan) if sr is not None]
        if codec:
            jobs_d, jobs_u, mid_off, out_off = [], [], 0, 0
            outs = []
            for b, sr in codec:
                kd, wd, ogd, ngd = self.kinfo[(16000, sr)]
                ku, wu, ogu, ngu = self.kinfo[(sr, 16000)]
                n = cur_lens[b]
                nd = -(-ngd * n // ogd)
                nu = -(-ngu * nd // ogu)
                jobs_d.append(_lib.ResampleJob(int(offs[b]), n, mid_off, nd, ogd, ngd, wd, kd))
                jobs_u.append(_lib.ResampleJob(mid_off, nd, total + out_off, nu, ogu, ngu, wu, ku))
                outs.append((b, total + out_off, nu))
                mid_off += nd
                out_off += nu
            mid = torch.empty(mid_off, device=self.device)
            ext = torch.empty(total + out_off, device=self.device)
            ext[:total].copy_(work[:total])
            for i in range(0, len(jobs_d), 64):
                resample_batch(work, mid, self.kernels, jobs_d[i:i + 64])
            for i in range(0, len(jobs_u), 64):
                resample_batch(mid, ext, self.kernels, jobs_u[i:i + 64])
            work = ext
            for b, o, nu in outs:
                offs[b], cur_lens[b] = o, nu
        starts = [st for (_, _, st) in plan]
        return pad_mixup(work, offs, cur_lens, starts, self.max_len, perm, lam, out=out)


# --------------------------------------------------------------------------- trainer ---------
def refuse_step_tuning():
    """PyTorch TunableOp tuning over the window's passes tries every rocBLAS solution rocBLAS accepts for the
    head's n = 1 strided-batched GEMM (tn_201_1_144_B_32: the attention-pooling bmm in the clean pass's backward),
    and one of them faults the GPU (gpurun_out/tune3: the fault follows the first accepted solution, 618385, in
    the eager warm-up before any capture). Every step kind runs that backward (the window, the
    graphed micro-step, the eager micro-step), so Trainer checks this at construction. Tune the WavLM shapes
    offline (tools/tune_wavlm_gemms.py) and run with tuning off."""
    tun = getattr(torch.cuda, "tunable", None)
    env_on = (os.environ.get("PYTORCH_TUNABLEOP_ENABLED", "0") == "1"
              and os.environ.get("PYTORCH_TUNABLEOP_TUNING", "1") == "1")
    api_on = tun is not None and torch.cuda.is_available() and tun.is_enabled() and tun.tuning_is_enabled()
    if env_on or api_on:
        raise RuntimeError("TunableOp tuning is on (PYTORCH_TUNABLEOP_TUNING): tuning inside the training step runs "
                           "rocBLAS solutions that fault on the head's n=1 batched GEMM; tune offline with "
                           "tools/tune_wavlm_gemms.py and set PYTORCH_TUNABLEOP_TUNING=0")


class Trainer:
    """One Phase-6 training process (one GPU). Mirrors main.py's optimizer/scheduler construction and
    train_epoch ordering."""

    def __init__(self, model, config, device, total_steps, amp_dtype=torch.bfloat16, world_group=None,
                 criterion=None, param_groups=None):
        self.model, self.config, self.device = model, config, torch.device(device)
        if self.device.type == "cuda":
            refuse_step_tuning()
        tc = config.get("training_config", {})
        oc = config["optim_config"]
        self.accum = max(1, int(tc.get("accumulation_steps", 1)))
        self.use_mixup = bool(tc.get("use_mixup", False))
        self.mixup_alpha = float(tc.get("mixup_alpha", 1.0))
        self.freq_aug = str(config.get("freq_aug", "False")).lower() in ("true", "1", "yes", "y", "t", "on")
        self.freeze_bn = bool(tc.get("freeze_bn", False))
        self.amp_dtype = amp_dtype
        self.criterion = criterion if criterion is not None else build_criterion(config, device)
        self.group = world_group
        # --- parameter groups (main.py:416-457): wavlm_stream* at wavlm_lr, the rest at base_lr
        wl, bb = [], []
        for n, p in model.named_parameters():
            if p.requires_grad:
                (wl if "wavlm_stream" in n else bb).append(p)
        wavlm_lr = oc.get("wavlm_lr", 1e-6)
        groups = [{"params": wl, "lr": wavlm_lr}, {"params": bb, "lr": oc["base_lr"]},
                  {"params": [], "lr": oc["base_lr"]}]
        if param_groups is not None:
            groups = param_groups
        if self.device.type == "cuda" and os.environ.get("RADHIP_ADAMW", "1") != "0":
            # torch.optim.AdamW's update on csrc/optim.hip (same state and GradScaler contract; radhip/optim.py)
            from .optim import AdamW as RdxAdamW
            self.opt = RdxAdamW(groups, weight_decay=oc["weight_decay"])
        else:
            try:
                self.opt = torch.optim.AdamW(groups, weight_decay=oc["weight_decay"], fused=True)
            except (RuntimeError, TypeError):
                self.opt = torch.optim.AdamW(groups, weight_decay=oc["weight_decay"])
        # --- FGM (main.py:514-544): unfreeze feature_projection, add it as its own group at wavlm_lr.
        # The reference adds this group AFTER building its LR schedulers; on torch >= 2.x that makes
        # SequentialLR's milestone step fail (strict zip over param groups), and on older torch the
        # group silently escaped the warmup. Here the group is added first, so it follows the same
        # warmup + cosine schedule as the other groups.
        self.fgm = None
        if tc.get("use_fgm", False):
            emb = tc.get("fgm_emb_name", "feature_projection")
            if "feature_projection" in emb and hasattr(model, "wavlm_stream"):
                fp = model.wavlm_stream._core().feature_projection
                fp.requires_grad_(True)
                in_opt = any(p is fp.projection.weight for g in self.opt.param_groups for p in g["params"])
                if not in_opt:
                    self.opt.add_param_group({"params": list(fp.parameters()), "lr": wavlm_lr})
            self.fgm = FGM(model, emb, tc.get("fgm_epsilon", 1.0), grad_hook=fgm_global_grads)
        warm = int(tc.get("warmup_steps", max(1, int(total_steps * float(tc.get("warmup_ratio", 0.05))))))
        warm = min(max(1, warm), max(1, total_steps - 1))
        # the reference reads optim_config["scheduler_config"]["eta_min"] (src/main.py:477) and KeyErrors on the
        # legacy AASIST / RawNet2 confs, which carry no scheduler_config: they fall back to their lr_min
        eta_min = oc.get("scheduler_config", {}).get("eta_min", oc.get("lr_min", 1e-6))
        w_sched = torch.optim.lr_scheduler.LinearLR(self.opt, start_factor=float(tc.get("warmup_init_factor", 0.1)),
                                                    end_factor=1.0, total_iters=warm)
        c_sched = torch.optim.lr_scheduler.CosineAnnealingLR(self.opt, T_max=max(1, total_steps - warm),
                                                             eta_min=eta_min)
        self.sched = torch.optim.lr_scheduler.SequentialLR(self.opt, [w_sched, c_sched], milestones=[warm])
        self.sched_on = oc.get("scheduler", "cosine") in ("cosine", "keras_decay")
        self.scaler = torch.amp.GradScaler("cuda", enabled=(amp_dtype == torch.float16))
        self.ema = EMA(model, tc.get("ema_decay", 0.999)) if tc.get("use_ema", False) else None
        inert = {id(p) for p in no_grad_params(model)}     # never in the reference's graph: no .grad, no step
        self.grads = FlatGrads([p for p in model.parameters() if id(p) not in inert])
        self.params = self.grads.params
        self.micro = 0              # micro-batches since construction (resume state)
        self.epoch_micro = 0        # micro-batches of the current epoch: the reference's i + 1 (begin_epoch)
        self.loss_sum = torch.zeros((), device=self.device, dtype=torch.float64)
        self.n_seen = 0

    def _loss(self, out, ya, yb, lam):
        if ya is yb or lam == 1.0:
            return self.criterion(out, ya)
        return lam * self.criterion(out, ya) + (1 - lam) * self.criterion(out, yb)

    def _fwd_loss(self, x, ya, yb, lam):
        with torch.autocast("cuda", dtype=self.amp_dtype, enabled=self.amp_dtype != torch.float32):
            _, out = self.model(x, Freq_aug=self.freq_aug)
            return self._loss(out, ya, yb, lam) / self.accum

    def mixup_draw(self, B):
        """lam ~ Beta(alpha, alpha) (numpy), perm = torch.randperm(B) (CPU generator) — main.py:1038-1046."""
        if self.use_mixup and B > 1:
            lam = float(np.random.beta(self.mixup_alpha, self.mixup_alpha))
            perm = torch.randperm(B).tolist()
            return lam, perm
        return 1.0, None

    def train_mode(self):
        """model.train() + freeze_batch_norm_stats (main.py:44-51,1016-1018). Walking the model's ~9000 modules
        costs ~6 ms of host time, once per window in front of its graph replays; when the model is still as the
        last call left it (top module training, every frozen BatchNorm in eval: any model.train() / eval() since
        flips those) the walk is skipped."""
        sent = getattr(self, "_mode_sentinel", None)
        if sent is not None and self.model.training and not any(m.training for m in sent):
            return
        self.model.train()
        if self.freeze_bn:
            for m in self.model.modules():
                if isinstance(m, (nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d)):
                    m.eval()
        self._mode_sentinel = [m for m in self.model.modules() if not m.training]

    def cnn_reuse(self, mode, drop=False):
        """FGM's adversarial pass reuses the frozen WavLM CNN features of the clean pass (identical input,
        eval-mode frozen CNN), saving one CNN forward per micro-batch."""
        wf = getattr(self.model, "wavlm_stream", None)
        core = wf._core() if wf is not None and hasattr(wf, "_core") else None
        if core is not None and hasattr(core, "cnn_reuse"):
            core.cnn_reuse = mode
            if drop:
                core._cnn_feats = None

    def begin_epoch(self):
        """train_epoch's loop index restarts every epoch (src/main.py:1030): the optimizer steps when
        (i + 1) % accumulation_steps == 0 or at the epoch's last micro-batch (:1100), counted per epoch."""
        self.epoch_micro = 0

    def count_micro(self, n=1, last_in_epoch=False):
        """Account n micro-batches; True when the optimizer steps after them (the reference's do_step)."""
        self.micro += n
        self.epoch_micro += n
        return self.epoch_micro % self.accum == 0 or last_in_epoch

    def micro_step(self, x, y, lam=1.0, perm=None, last_in_epoch=False):
        """One micro-batch: x [B, 64600] already mixed (perm/lam are those used for the mix)."""
        self.train_mode()
        y = y.view(-1).long().to(self.device, non_blocking=True)
        ya = y
        yb = y[torch.tensor(perm, device=self.device)] if perm is not None else y
        self.cnn_reuse("store" if self.fgm is not None else None)
        loss = self._fwd_loss(x, ya, yb, lam)
        with ops.wgrad_batch():
            self.scaler.scale(loss).backward()
        if self.fgm is not None:
            self.fgm.attack()
            self.cnn_reuse("use")
            adv = self._fwd_loss(x, ya, yb, lam)
            with ops.wgrad_batch():
                self.scaler.scale(adv).backward()
            self.fgm.restore()
        self.cnn_reuse(None, drop=True)
        B = x.shape[0]
        self.loss_sum += loss.detach().double() * self.accum * B
        self.n_seen += B
        if self.count_micro(1, last_in_epoch):
            self.optimizer_step()
        return loss

    def optimizer_step(self):
        self.grads.all_reduce_mean(self.group)
        self.scaler.unscale_(self.opt)
        if self.grads.bound():
            self.grads.clip_norm_(3.0)
        else:
            torch.nn.utils.clip_grad_norm_(self.params, max_norm=3.0, foreach=True)
        self.scaler.step(self.opt)
        self.scaler.update()
        self.grads.zero()
        if self.ema is not None:
            self.ema.update()
        if self.sched_on:
            self.sched.step()

    def epoch_loss(self):
        v = float(self.loss_sum.item()) / max(self.n_seen, 1)
        self.loss_sum.zero_()
        self.n_seen = 0
        return v

    # ---------------------------------------------------------------- full resume state -------
    def state_dict(self):
        """Everything an exact resume needs beyond the model weights (the reference saves weights only,
        src/main.py:649-664): optimizer moments, LR schedule position, grad scaler, EMA."""
        return {"optimizer": self.opt.state_dict(), "scheduler": self.sched.state_dict(),
                "scaler": self.scaler.state_dict(), "micro": self.micro,
                "ema": self.ema.train_state() if self.ema is not None else None}

    def load_state_dict(self, st):
        self.opt.load_state_dict(st["optimizer"])
        self.sched.load_state_dict(st["scheduler"])
        self.scaler.load_state_dict(st["scaler"])
        self.micro = int(st["micro"])
        if (st["ema"] is None) != (self.ema is None):
            raise ValueError("train state and config disagree on use_ema")
        if self.ema is not None:
            self.ema.load_train_state(st["ema"])


@torch.no_grad()
def swa_bn_update(model, feeder, augmenter, device):
    """torchcontrib SWA.bn_update(trn_loader, model) after swap_swa_sgd (src/main.py:669-672): reset every
    BatchNorm's running statistics and recompute them as a cumulative average (momentum b / (n + b)) over
    one pass of the augmented train loader in train mode. In the dual-stream model only the SincNet stream
    holds BatchNorm, and nothing else it computes is kept, so only that stream runs (the WavLM stream's
    forward does not touch any BatchNorm statistic); the legacy plugins run whole."""
    bns = [m for m in model.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)]
    if not bns:
        return 0
    was_training = model.training
    momenta = {}
    tracked0 = {m: m.num_batches_tracked.clone() for m in bns if m.num_batches_tracked is not None}
    for m in bns:
        m.running_mean.zero_()      # in place: captured HIP graphs keep pointing at the same buffers
        m.running_var.fill_(1.0)
        momenta[m] = m.momentum
    model.train()
    for m in bns:
        m.train()
    n = 0
    for keys in feeder.epoch():
        flat, offs, lens, _ = feeder.load(keys, device)
        x = augmenter.run(flat, offs, lens, augmenter.draw(lens))
        b = x.shape[0]
        for m in bns:
            m.momentum = b / float(n + b)
        if hasattr(model, "sinc_stream"):
            model.sinc_stream(x, freq_aug=False)
        else:                       # legacy plugins: BatchNorm all through the network
            model(x)
        n += b
    for m in bns:
        m.momentum = momenta[m]
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        # each rank averaged its own shard: the cumulative averages combine weighted by the ranks' sample
        # counts into the average over the whole train set, as the reference's single-process pass computes
        cnt = torch.tensor([float(n)], dtype=torch.float64, device=bns[0].running_mean.device)
        dist.all_reduce(cnt)
        total = float(cnt.item())
        for m in bns:
            st = torch.cat([m.running_mean.double(), m.running_var.double()]) * float(n)
            dist.all_reduce(st)
            st /= max(total, 1.0)
            c = m.running_mean.numel()
            m.running_mean.copy_(st[:c])
            m.running_var.copy_(st[c:])
            if m.num_batches_tracked is not None:       # batches counted by this pass, over all ranks
                nb = m.num_batches_tracked - tracked0[m]
                dist.all_reduce(nb)
                m.num_batches_tracked.copy_(tracked0[m] + nb)
        n = int(total)
    model.train(was_training)
    return n


def layerdrop_draws(n):
    """HF WavLM's LayerDrop draws, torch.rand([]) once per layer on the CPU generator, as ONE torch.rand(n): the
    same values and the same generator state afterwards (tests/test_recipe_cpu.py checks it), at 1/20 of the
    host time (24 scalar draws took ~80 us per forward)."""
    return torch.rand(n).numpy().astype(np.float64)


class _PinnedRing:
    """Small ring of pinned host slots for H2D copies of per-replay inputs (non_blocking, stream-ordered;
    a slot is reused only after the copy that read it has executed)."""

    def __init__(self, nbytes, slots=4):
        self.gpu = torch.cuda.is_available()
        self.bufs = [torch.empty(nbytes, dtype=torch.uint8, pin_memory=self.gpu) for _ in range(slots)]
        self.events = [None] * slots
        self.i = 0

    def stage(self, arrays):
        """arrays: list of (numpy array, device tensor); packs them into one slot and copies."""
        k = self.i
        self.i = (self.i + 1) % len(self.bufs)
        if self.events[k] is not None:
            self.events[k].synchronize()
        buf = self.bufs[k]
        off = 0
        views = []
        for a, dst in arrays:
            a = np.ascontiguousarray(a)
            nb = a.nbytes
            off = (off + 15) & ~15
            buf[off:off + nb].numpy()[:] = a.view(np.uint8).reshape(-1)
            views.append((buf[off:off + nb].view(dst.dtype).view(dst.shape), dst))
            off += nb
        for src, dst in views:
            dst.copy_(src, non_blocking=dst.is_cuda)
        if self.gpu:
            ev = torch.cuda.Event()
            ev.record()
            self.events[k] = ev


def check_graph_memset_replay(device):
    """Capture hipMemsetAsync(0) + add(1) and replay it three times: every replay must leave 1.
    Raises if the HIP runtime replays captured memset nodes wrongly (see radhip/__init__.py)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    buf = torch.zeros(64, dtype=torch.int32, device=device)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        rc = hip.hipMemsetAsync(buf.data_ptr(), 0, buf.numel() * 4, torch.cuda.current_stream().cuda_stream)
        buf.add_(1)
    if rc != 0:
        raise RuntimeError(f"hipMemsetAsync failed during capture ({rc})")
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize(device)
        if not bool((buf == 1).all()):
            raise RuntimeError(
                "HIP graph replays a captured memset with a wrong value; run with "
                "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 set before the HIP runtime initialises (radhip does this "
                "on import — import radhip before touching the GPU)")
    del g


class GraphedMicroStep:
    """The Phase-6 micro-batch as two replayed HIP graphs: G0 = clean forward + loss + backward,
    G1 = adversarial forward + backward; the FGM attack (and its DDP all-reduce) and the restore run
    eagerly between them, so no collective is captured. Every per-call random decision (SincConv band
    mask, SpecAugment time mask, LayerDrop, mixup lambda/permutation) is drawn on the host in the
    reference's order and staged into static device buffers before each replay; the model reads them
    through its *_dev hooks. ~9k kernel launches per micro-batch become 2 graph launches."""

    def __init__(self, trainer, batch, max_len=MAX_LEN):
        self.tr = trainer
        m = trainer.model
        dev = trainer.device
        self.B = batch
        self.x = torch.zeros(batch, max_len, device=dev)
        self.ya = torch.zeros(batch, dtype=torch.long, device=dev)
        self.yb = torch.zeros(batch, dtype=torch.long, device=dev)
        self.lam = torch.ones((), device=dev)
        self.conv = m.sinc_stream.conv_time
        self.core = m.wavlm_stream._core()
        cfg = self.core.config
        nl = len(self.core.encoder.layers)
        # frames after the WavLM feature extractor
        T = max_len
        for k, st in zip(cfg.conv_kernel, cfg.conv_stride):
            T = (T - k) // st + 1
        self.T = T
        self.mask = [torch.zeros(2, dtype=torch.int32, device=dev) for _ in range(2)]
        self.tmask = [torch.zeros(batch, T, dtype=torch.bool, device=dev) for _ in range(2)]
        self.keep = [torch.ones(nl, dtype=torch.bool, device=dev) for _ in range(2)]
        self.spec_on = bool(getattr(cfg, "apply_spec_augment", True)) and cfg.mask_time_prob > 0
        self.nl = nl
        self.ring = _PinnedRing(4096 + 2 * batch * (T + 16) + 64 * nl)
        self.adv = trainer.fgm is not None     # the adversarial pass exists only with FGM
        self.graphs = None
        self.pool = None

    # -- host draws, in the reference's per-forward order: SpecAugment (numpy), LayerDrop (torch CPU),
    #    SincConv band mask (numpy + python random)
    def _draw_pass(self):
        c = self.core.config
        tm = (compute_time_mask(self.B, self.T, c.mask_time_prob, c.mask_time_length, c.mask_time_min_masks)
              if self.spec_on else np.zeros((self.B, self.T), dtype=bool))
        p = c.layerdrop
        keep = np.ones(self.nl, dtype=bool)
        r = layerdrop_draws(self.nl)   # one CPU draw per layer, as HF
        if p > 0:
            keep[1:] = ~(r[1:] < p)
        lo, hi = self.conv.draw_mask() if self.tr.freq_aug else (0, 0)
        return tm, keep, np.array([lo, hi], dtype=np.int32)

    def _bind(self, k):
        self.conv.mask_dev = self.mask[k]
        self.core.time_mask_dev = self.tmask[k]
        self.core.encoder.keep_dev = self.keep[k]

    def _unbind(self):
        self.conv.mask_dev = None
        self.core.time_mask_dev = None
        self.core.encoder.keep_dev = None

    def _pass(self, k):
        tr = self.tr
        self._bind(k)
        tr.cnn_reuse(("use" if k == 1 else "store") if self.adv else None)
        with torch.autocast("cuda", dtype=tr.amp_dtype, enabled=tr.amp_dtype != torch.float32, cache_enabled=False):
            _, out = tr.model(self.x, Freq_aug=tr.freq_aug)
            loss = (self.lam * tr.criterion(out, self.ya) + (1.0 - self.lam) * tr.criterion(out, self.yb)) / tr.accum
        with ops.wgrad_batch():
            loss.backward()
        if k == 0:
            tr.loss_sum.add_(loss.detach().double() * (tr.accum * self.B))

    def _stage(self, y, lam, perm):
        y = np.asarray(y, dtype=np.int64).reshape(-1)
        yb = y[np.asarray(perm)] if perm is not None else y
        draws = [self._draw_pass()] + ([self._draw_pass()] if self.adv else [])
        arrs = [(y, self.ya), (yb, self.yb), (np.array(lam, dtype=np.float32), self.lam)]
        for k, (tm, keep, mk) in enumerate(draws):
            arrs += [(tm, self.tmask[k]), (keep, self.keep[k]), (mk, self.mask[k])]
        self.ring.stage(arrs)

    def _fgm(self):
        fgm = self.tr.fgm
        if fgm is not None:
            fgm.attack()

    def _restore(self):
        if self.tr.fgm is not None:
            self.tr.fgm.restore()

    def capture(self, warmup=2):
        tr = self.tr
        check_graph_memset_replay(tr.device)
        tr.train_mode()
        saved_loss = tr.loss_sum.clone()
        side = torch.cuda.Stream(device=tr.device)
        side.wait_stream(torch.cuda.current_stream(tr.device))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._pass(0)
                if self.adv:
                    self._fgm()
                    self._pass(1)
                    self._restore()
        torch.cuda.current_stream(tr.device).wait_stream(side)
        torch.cuda.synchronize(tr.device)
        gs = []
        from . import ops
        ops.reserve_graph_workspace(tr.device)
        for k in ((0, 1) if self.adv else (0,)):
            if ops.CAPTURE_TIMING is not None:
                ops.CAPTURE_TIMING.new_graph()
            g = torch.cuda.CUDAGraph()
            # one private memory pool per graph (sharing one pool between the clean and the adversarial
            # graph corrupted bias-gradient reductions of the clean graph on ROCm 7 / torch 2.10)
            with torch.cuda.graph(g):
                self._pass(k)
            gs.append(g)
            if k == 0 and self.adv:
                self._fgm()
        if self.adv:
            self._restore()
        ops.finalize_graph_workspace(tr.device)     # tickets grown inside a capture: zero before any replay
        self._unbind()
        # the graphs hold the "store"/"use" branches; eager calls (eval, tools) must recompute the CNN.
        # The stored feature tensor stays referenced: graph 1 reads it on every replay.
        tr.cnn_reuse(None)
        tr.grads.zero()
        tr.loss_sum.copy_(saved_loss)
        self.graphs = gs

    def run(self, y, lam=1.0, perm=None, last_in_epoch=False):
        """self.x must already hold the mixed batch (Augmenter.run(..., out=self.x))."""
        tr = self.tr
        self._stage(y, lam, perm)
        self.graphs[0].replay()
        if self.adv:
            self._fgm()
            self.graphs[1].replay()
            self._restore()
        tr.n_seen += self.B
        if tr.count_micro(1, last_in_epoch):
            tr.optimizer_step()


def ddp_micro_batches(batch_size, accum, world):
    """Per-rank (micro-batch, accumulation) that keeps the reference's global batch under data parallelism
    (SURVEY.md §8e): one optimizer step sees batch_size * accum utterances (src/main.py:1100-1117; 8 x 4 = 32
    for Phase 6) split evenly over `world` ranks, the per-rank micro-batch as large as possible (at most
    batch_size, mixup permutes within it) and at least 2 (mixup is skipped at B = 1, src/main.py:1038).
    1-4 ranks: 8 x 4/world; 8 ranks: 4 x 1."""
    batch_size, accum, world = int(batch_size), max(1, int(accum)), max(1, int(world))
    if world == 1:
        return batch_size, accum
    glob = batch_size * accum
    if glob % world:
        raise ValueError(f"global batch {batch_size} x {accum} = {glob} does not split over {world} ranks")
    share = glob // world
    for b in range(min(batch_size, share), 1, -1):
        if share % b == 0:
            return b, share // b
    raise ValueError(f"{share} utterances per rank and step: a per-rank micro-batch of at least 2 is needed")


def total_optimizer_steps(num_epochs, micro_batches_per_epoch, accum):
    return num_epochs * math.ceil(micro_batches_per_epoch / accum)
