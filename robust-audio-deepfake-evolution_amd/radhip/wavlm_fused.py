"""Fused WavLM encoder layer for the 16-bit (bf16 or fp16 autocast) training/eval step (csrc/wavlm_layer.hip +
attention.hip; fp16 runs the same kernels from libradhip_f16.so).

The LoRA weight gradients (four skinny reductions over the tokens) are one kernel that accumulates
into the fp32 .grad buffers directly (so the Function returns no gradient for those leaves).
One autograd Function per layer replaces the ~44 forward / ~100 backward framework kernels of the
module-by-module layer (casts, LN, gate MLP, LoRA GEMMs, dropouts, residual adds) with 9 forward and
11 backward launches: four hipBLASLt GEMMs (q/k/v with the LoRA update folded in as 16 extra K
columns, out_proj, FFN1, FFN2), the MFMA gated-bias attention, and wave-per-row fused kernels for
LN1 + gate + LoRA-A, dropout + residual + LN2, GELU, and their backwards. Same math as the
reference layer (HF WavLMEncoderLayerStableLayerNorm + peft LoRA q/v; DualStreamSEMamba.py:292-439,
main.py:103-158); dropout masks come from the device-seeded counter hash (graph replayable).

Used when: CUDA, bf16 or fp16 autocast, stable layer norm, E = 1024 with 64-dim heads, GELU FFN, a frozen
base layer, and either no LoRA or LoRA r = 8 on exactly q_proj and v_proj. Anything else takes the
module path (radhip/wavlm.py), which is what the fp32 parity tests exercise.
RADHIP_FUSED_WAVLM=0 disables the fused layer (A/B measurement).
"""
import ctypes
import os

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import check
from .ops import (HALF, _L, _p, _stream, _timed, attn_bwd_launch, attn_keep_mask, cast_many, half_dtype,
                  layer_gemm, rel_bias_table, wgemm_policy)

E_FUSED = 1024


def _off(t, elems):
    """Device address of element `elems` of t (a column offset into a row-major GEMM output)."""
    return ctypes.c_void_p(t.data_ptr() + elems * t.element_size())
SALT_BASE = 4096


def enabled():
    return os.environ.get("RADHIP_FUSED_WAVLM", "1") != "0"


def _lora_parts(attn):
    from .wavlm import LoraLinear
    q, k, v, o = attn.q_proj, attn.k_proj, attn.v_proj, attn.out_proj
    if isinstance(k, LoraLinear) or isinstance(o, LoraLinear):
        return "unsupported"
    if isinstance(q, LoraLinear) != isinstance(v, LoraLinear):
        return "unsupported"
    if not isinstance(q, LoraLinear):
        return None
    if not q.active and not v.active:
        return None                 # bypassed adapters (the reference's HF WavLM): the plain q/k/v GEMM
    if q.active != v.active:
        return "unsupported"
    r = q.r[q.adapter]
    if r != 8 or v.r[v.adapter] != 8 or q.scaling[q.adapter] != v.scaling[v.adapter]:
        return "unsupported"
    return q, v


def eligible(encoder, h):
    cfg = encoder.cfg
    if not (enabled() and h.is_cuda and encoder.stable and cfg.hidden_size == E_FUSED
            and cfg.hidden_size // cfg.num_attention_heads == 64 and cfg.hidden_act == "gelu"):
        return False
    if not (torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") in HALF):
        return False
    st = encoder.__dict__.get("_fused_ok")
    if st is not None and st[0] == _trainable_signature(encoder):
        return st[1]
    ok = True
    for layer in encoder.layers:
        lp = _lora_parts(layer.attention)
        if lp == "unsupported":
            ok = False
            break
        lora_params = set()
        from .wavlm import LoraLinear
        for ad in (layer.attention.q_proj, layer.attention.v_proj):
            if isinstance(ad, LoraLinear):      # active or bypassed: their gradients never come from autograd here
                lora_params |= {id(p) for p in ad.lora_A.parameters()} | {id(p) for p in ad.lora_B.parameters()}
        if any(p.requires_grad and id(p) not in lora_params for p in layer.parameters()):
            ok = False
            break
    encoder.__dict__["_fused_ok"] = (_trainable_signature(encoder), ok)
    return ok


def _trainable_signature(encoder):
    from .wavlm import LoraLinear
    return (tuple(p.requires_grad for p in encoder.parameters())
            + tuple(m.active for m in encoder.modules() if isinstance(m, LoraLinear)))


class _LayerCache:
    """16-bit (the autocast dtype) copies of a frozen layer's weights (rebuilt when a source tensor or the dtype
    changes) and the
    [3E, E + 2r] q/k/v operand whose last 2r columns receive s * lora_B every forward."""

    def __init__(self):
        self.key = None

    def refresh(self, layer, lora, hd):
        a, ff = layer.attention, layer.feed_forward
        from .wavlm import _base
        bq, bk, bv = _base(a.q_proj), _base(a.k_proj), _base(a.v_proj)
        src = [bq.weight, bk.weight, bv.weight, bq.bias, bk.bias, bv.bias, a.out_proj.weight, a.out_proj.bias,
               ff.intermediate_dense.weight, ff.intermediate_dense.bias, ff.output_dense.weight,
               ff.output_dense.bias]
        key = (lora is not None, hd) + tuple((t.data_ptr(), t._version) for t in src)
        if key == self.key:
            return
        E = bq.weight.shape[0]
        r2 = 16 if lora is not None else 0
        with torch.no_grad():
            w = torch.zeros(3 * E, E + r2, device=bq.weight.device, dtype=hd)
            w[:, :E] = torch.cat([bq.weight, bk.weight, bv.weight]).to(hd)
            self.wext = w
            self.bqkv = torch.cat([bq.bias, bk.bias, bv.bias]).to(hd)
            self.wo = a.out_proj.weight.to(hd)
            self.bo = a.out_proj.bias.to(hd)
            self.w1 = ff.intermediate_dense.weight.to(hd)
            self.b1 = ff.intermediate_dense.bias.to(hd)
            self.w2 = ff.output_dense.weight.to(hd)
            self.b2 = ff.output_dense.bias.to(hd)
            # transposed copies for the input-gradient GEMMs on csrc/wgemm.hip (B operand [N][K]; built lazily)
            self.woT = self.w1T = self.w2T = self.wqkvT = None
            self.hd = hd
            self.wg = a.gru_rel_pos_linear.weight.detach().float().contiguous()
            self.bg = a.gru_rel_pos_linear.bias.detach().float().contiguous()
            self.gconst = a.gru_rel_pos_const.detach().float().reshape(-1).contiguous()
        self.key = key

    def t(self, name):
        """The transposed frozen weight `name` ('wo', 'w1', 'w2', 'wqkv' = the q/k/v rows without LoRA columns)."""
        cur = getattr(self, name + "T")
        if cur is None:
            src = self.wext[:, :E_FUSED] if name == "wqkv" else getattr(self, name)
            cur = src.t().contiguous()
            setattr(self, name + "T", cur)
        return cur


def _gemm(name, M, N, K):
    """(tile, splits) of csrc/wgemm.hip for the layer GEMM `name` at M tokens, or None for hipBLASLt
    (radhip.ops.wgemm_policy)."""
    return wgemm_policy(name, M, N, K)


class EncoderChain:
    """Per-forward state of a fused encoder whose layers run back to back (no LayerDrop selection between them):
      * layer i leaves its residual h_{i+1} = h2 + drop(fo) to layer i+1's LN1 forward (rdx_wl_res_ln1_fwd),
        which computes it into layer i's (returned) output tensor: one pass instead of two;
      * the layer-weighted sum's backward does not write the gradients of states 0..n-1 (the layers' inputs);
        it leaves g and softmax(w) here and layer i's LN1 backward adds softmax(w)_i * g (rdx_wl_ln1_bwd_ex):
        no [M, E] gradient per layer and no autograd add;
      * layer i+1's LN1 backward also writes layer i's dropped FFN-output gradient drop_i(dh), which layer i's
        backward then takes instead of running its dropout backward."""

    def __init__(self, n):
        self.n = n
        self.indices = frozenset(range(n))
        self.pending_res = None
        self.g = None
        self.p = None
        self.dfo = {}


class WavLMLayerFn(torch.autograd.Function):
    """h_out = layer(h) for one stable-LN WavLM layer; inputs h fp32 [B, T, E] and the LoRA factors
    (lora_A q, lora_B q, lora_A v, lora_B v, fp32 leaves, or None)."""

    @staticmethod
    def forward(ctx, h, aq, bq, av, bv, layer, cache, rel, seed, index, p_hidden, p_attn, p_lora, scale, chain):
        B, T, E = h.shape
        H = E // 64
        M = B * T
        dev = h.device
        lora = aq is not None
        r2 = 16 if lora else 0
        ldx = E + r2
        hf = h.contiguous().view(M, E)
        st = _stream(hf)
        ln1, ln2 = layer.layer_norm, layer.final_layer_norm
        sd = seed if seed is not None else None
        sdp = _p(sd) if sd is not None else None
        salt = SALT_BASE + 8 * index
        hd = cache.hd
        L = _L(hd)
        x1 = torch.empty(M, ldx, device=dev, dtype=hd)
        gate = torch.empty(M, H, device=dev, dtype=torch.float32)
        mean1 = torch.empty(M, device=dev, dtype=torch.float32)
        rstd1 = torch.empty_like(mean1)
        a16 = cache.a16.view(2, 8, E) if lora else None    # the pass's 16-bit lora_A (FusedEncoderRunner.prepare)
        pend = chain.pending_res if chain is not None else None
        if pend is not None and pend[0] == hf.data_ptr():
            # the previous layer's residual, computed here into its output (= this layer's input) tensor
            chain.pending_res = None
            _, h2p, fop, salt_res, p_res = pend
            check(L.rdx_wl_res_ln1_fwd(_p(h2p), _p(fop), salt_res, float(p_res), _p(hf), _p(ln1.weight),
                                           _p(ln1.bias), float(ln1.eps), _p(cache.wg), _p(cache.bg), _p(cache.gconst),
                                           _p(a16[0]) if lora else None, _p(a16[1]) if lora else None, 8, sdp, salt + 3,
                                           salt + 4, float(p_lora), _p(x1), ldx, _p(gate), _p(mean1), _p(rstd1), M,
                                           E, st), "wl_res_ln1_fwd")
        else:
            check(L.rdx_wl_ln1_fwd(_p(hf), _p(ln1.weight), _p(ln1.bias), float(ln1.eps), _p(cache.wg),
                                       _p(cache.bg), _p(cache.gconst), _p(a16[0]) if lora else None,
                                       _p(a16[1]) if lora else None, 8, sdp, salt + 3, salt + 4, float(p_lora), _p(x1),
                                       ldx, _p(gate), _p(mean1), _p(rstd1), M, E, st), "wl_ln1_fwd")
        pol = _gemm("qkv", M, 3 * E, ldx)
        if pol is not None:
            qkv = layer_gemm(pol, x1, cache.wext, cache.bqkv)
        else:
            qkv = F.linear(x1, cache.wext, cache.bqkv)                      # [M, 3E] (LoRA folded in)
        o = torch.empty(M, E, device=dev, dtype=hd)
        lse = torch.empty(B, H, T, device=dev, dtype=torch.float32)
        zseed = sd if sd is not None else torch.zeros(1, dtype=torch.int64, device=dev)
        mask = attn_keep_mask(B, T, H, float(p_attn), dev)
        with _timed("attn_fwd", hf, 2.0 * 2 * B * H * T * T * 64):
            check(L.rdx_attn_fwd(_p(qkv), 3 * E, _off(qkv, E), 3 * E, _off(qkv, 2 * E), 3 * E, _p(gate), _p(rel),
                                     _p(zseed), int(index), float(p_attn), 0.125, _p(o), E, _p(lse),
                                     _p(mask) if mask is not None else None, B, T, H, 64, st), "attn_fwd")
        pol = _gemm("out", M, E, E)
        if pol is not None:
            aout = layer_gemm(pol, o, cache.wo, cache.bo)
        else:
            aout = F.linear(o, cache.wo, cache.bo)
        h2 = torch.empty(M, E, device=dev, dtype=torch.float32)
        x2 = torch.empty(M, E, device=dev, dtype=hd)
        mean2 = torch.empty_like(mean1)
        rstd2 = torch.empty_like(mean1)
        check(L.rdx_wl_add_ln_fwd(_p(hf), _p(aout), sdp, salt + 1, float(p_hidden), _p(h2), _p(ln2.weight),
                                      _p(ln2.bias), float(ln2.eps), _p(x2), _p(mean2), _p(rstd2), M, E, st),
              "wl_add_ln_fwd")
        F4 = cache.w1.shape[0]
        pol = _gemm("ffn1", M, F4, E)
        if pol is not None:                             # FFN1 + bias + GELU in one launch
            u, v = layer_gemm(pol, x2, cache.w1, cache.b1, epilogue=_lib.EPI_BIAS_GELU)
        else:
            u = F.linear(x2, cache.w1, cache.b1)
            v = torch.empty_like(u)
            check(L.rdx_wl_gelu(0, _p(u), None, _p(v), u.numel(), st), "wl_gelu")
        pol = _gemm("ffn2", M, E, F4)
        if pol is not None:
            fo = layer_gemm(pol, v, cache.w2, cache.b2)
        else:
            fo = F.linear(v, cache.w2, cache.b2)
        out = torch.empty(M, E, device=dev, dtype=torch.float32)
        if chain is not None and index < chain.n - 1:
            chain.pending_res = (out.data_ptr(), h2, fo, salt + 2, float(p_hidden))   # -> the next LN1 forward
        else:
            check(L.rdx_wl_residual(_p(h2), _p(fo), sdp, salt + 2, float(p_hidden), _p(out), M * E, st),
                  "wl_residual")
        ctx.save_for_backward(hf, x1, qkv, o, lse, gate, h2, mean1, rstd1, mean2, rstd2, u, zseed, rel, aq, av)
        ctx.layer, ctx.cache, ctx.mask, ctx.chain = layer, cache, mask, chain
        ctx.lora_b = (bq, bv)
        ctx.meta = (B, T, E, H, index, float(p_hidden), float(p_attn), float(p_lora), float(scale), lora,
                    sd is not None)
        return out.view(B, T, E)

    @staticmethod
    def backward(ctx, dout):
        hf, x1, qkv, o, lse, gate, h2, mean1, rstd1, mean2, rstd2, u, zseed, rel, aq, av = ctx.saved_tensors
        B, T, E, H, index, p_hidden, p_attn, p_lora, scale, lora, has_seed = ctx.meta
        layer, cache = ctx.layer, ctx.cache
        M = B * T
        dev = hf.device
        st = _stream(hf)
        sdp = _p(zseed) if has_seed else None
        salt = SALT_BASE + 8 * index
        ldx = x1.shape[1]
        a16 = cache.a16.view(2, 8, E) if lora else None
        g = dout.contiguous().view(M, E).float()
        hd = x1.dtype
        L = _L(hd)
        chain = ctx.chain
        rec = chain.dfo.pop(index, None) if chain is not None else None
        if rec is not None and rec[0] == g.data_ptr():
            dfo = rec[1]                  # written by the next layer's LN1 backward along with g
        else:
            dfo = torch.empty(M, E, device=dev, dtype=hd)
            check(L.rdx_wl_dropout_bwd(_p(g), sdp, salt + 2, p_hidden, _p(dfo), M * E, st), "wl_dropout_bwd")
        F4 = u.shape[1]
        pol = _gemm("d_ffn2", M, F4, E)
        if pol is not None:                             # FFN2's input gradient with the GELU backward fused
            du = layer_gemm(pol, dfo, cache.t("w2"), epilogue=_lib.EPI_GELU_BWD, aux=u)
        else:
            dv = torch.mm(dfo, cache.w2)
            du = torch.empty_like(u)
            check(L.rdx_wl_gelu(1, _p(u), _p(dv), _p(du), u.numel(), st), "wl_gelu_bwd")
        pol = _gemm("d_ffn1", M, E, F4)
        if pol is not None:
            dx2 = layer_gemm(pol, du, cache.t("w1"))
        else:
            dx2 = torch.mm(du, cache.w1)
        dh2 = torch.empty(M, E, device=dev, dtype=torch.float32)
        daout = torch.empty(M, E, device=dev, dtype=hd)
        ln1, ln2 = layer.layer_norm, layer.final_layer_norm
        check(L.rdx_wl_ln_bwd(_p(dx2), E, _p(h2), _p(mean2), _p(rstd2), _p(ln2.weight), _p(g), _p(dh2), sdp,
                                  salt + 1, p_hidden, _p(daout), M, E, st), "wl_ln_bwd")
        pol = _gemm("d_out", M, E, E)
        if pol is not None:
            do = layer_gemm(pol, daout, cache.t("wo"))
        else:
            do = torch.mm(daout, cache.wo)
        D = torch.empty(B, H, T, device=dev, dtype=torch.float32)
        dqkv = torch.empty(M, 3 * E, device=dev, dtype=hd)
        dgate = torch.empty(M, H, device=dev, dtype=torch.float32)
        with _timed("attn_bwd", hf, 2.0 * 5 * B * H * T * T * 64):
            attn_bwd_launch(_p(qkv), 3 * E, _off(qkv, E), 3 * E, _off(qkv, 2 * E), 3 * E, gate, rel, ctx.mask,
                            _p(zseed), int(index), p_attn, _p(o), E, lse, _p(do), E, D, _p(dqkv), _off(dqkv, E),
                            _off(dqkv, 2 * E), 3 * E, dgate, B, T, H, st, hd)
        pol = _gemm("d_qkv", M, ldx, 3 * E) if not lora else None   # (active LoRA: wext changes every step)
        if pol is not None:
            dx1 = layer_gemm(pol, dqkv, cache.t("wqkv"))
        else:
            dx1 = torch.mm(dqkv, cache.wext)                                 # [M, E + 2r]
        dh = torch.empty(M, E, device=dev, dtype=torch.float32)
        sgp = swp = ddp = None
        if chain is not None and chain.g is not None and index in chain.indices:
            sgp = _p(chain.g)                                   # this input's layer-weighted-sum gradient
            swp = ctypes.c_void_p(chain.p.data_ptr() + 4 * index)
        if chain is not None and index > 0:
            ddrop = torch.empty(M, E, device=dev, dtype=hd)
            ddp = _p(ddrop)
        check(L.rdx_wl_ln1_bwd_ex(_p(dx1), ldx, _p(dgate), _p(hf), _p(mean1), _p(rstd1), _p(ln1.weight),
                                      _p(ln1.bias), _p(cache.wg), _p(cache.bg), _p(cache.gconst),
                                      _p(a16[0]) if lora else None, _p(a16[1]) if lora else None, 8, sdp, salt + 3,
                                      salt + 4, p_lora, _p(dh2), _p(dh), None, sgp, swp, salt - 8 + 2, p_hidden, ddp, M,
                                      E, st),
              "wl_ln1_bwd")
        if ddp is not None:
            chain.dfo[index - 1] = (dh.data_ptr(), ddrop)
        if lora:
            # the four LoRA weight gradients in one launch, accumulated straight into .grad (fp32; with
            # FlatGrads these are views of the flat all-reduce buffer) instead of returned to autograd
            bq, bv = ctx.lora_b
            gs = []
            for prm in (aq, bq, av, bv):
                if prm.grad is None:
                    prm.grad = torch.zeros_like(prm)
                gs.append(prm.grad)
            check(L.rdx_wl_lora_grad(_p(dqkv), 3 * E, _p(x1), ldx, _p(dx1), ldx, sdp, salt + 3, salt + 4,
                                         p_lora, scale, _p(gs[0]), _p(gs[1]), _p(gs[2]), _p(gs[3]), M, E, 8, st),
                  "wl_lora_grad")
        return (dh.view(B, T, E),) + (None,) * 14


class FusedEncoderRunner:
    """Per-Encoder state of the fused path: weight caches, the LoRA-B pack tables, the position bias."""

    def __init__(self, encoder):
        self.encoder = encoder
        self.caches = [_LayerCache() for _ in encoder.layers]
        self.pack_key = None
        self.pb_key = None

    def position_bias(self, T, device):
        emb = self.encoder.layers[0].attention.rel_attn_embed.weight
        key = (T, emb.data_ptr(), emb._version)
        if key != self.pb_key:
            with torch.no_grad():
                self.pb = rel_bias_table(self.encoder.layers[0].attention.compute_bias(T, device).float())
            self.pb_key = key
        return self.pb

    def prepare(self, device):
        loras = [_lora_parts(layer.attention) for layer in self.encoder.layers]
        hd = half_dtype()
        for layer, cache, lp in zip(self.encoder.layers, self.caches, loras):
            cache.refresh(layer, lp, hd)
        if loras[0] is None:
            return loras
        key = tuple(c.wext.data_ptr() for c in self.caches) + tuple(
            lp[i].lora_B[lp[i].adapter].weight.data_ptr() for lp in loras for i in (0, 1))
        if key != self.pack_key:
            bq = [lp[0].lora_B[lp[0].adapter].weight for lp in loras]
            bv = [lp[1].lora_B[lp[1].adapter].weight for lp in loras]
            self.tab = torch.tensor([[t.data_ptr() for t in bq], [t.data_ptr() for t in bv],
                                     [c.wext.data_ptr() for c in self.caches]], dtype=torch.int64).to(device)
            self.pack_key = key
        # lora_A of every layer in the 16-bit dtype (autocast's cast of the fp32 weight), one launch per pass: the LN1
        # kernels stage it per workgroup with 16-byte loads instead of reading and converting 64 KB of fp32 each
        n = len(self.caches)
        if getattr(self, "a16", None) is None or self.a16.dtype != hd or self.a16.device != device:
            self.a16 = torch.empty(n, 16, E_FUSED, device=device, dtype=hd)
            for i, cache in enumerate(self.caches):
                cache.a16 = self.a16[i]
        srcs = [lp[i].lora_A[lp[i].adapter].weight.detach() for lp in loras for i in (0, 1)]
        cast_many(srcs, [self.a16[l, 8 * i:8 * (i + 1)] for l in range(n) for i in (0, 1)])
        lp0 = loras[0][0]
        check(_L(hd).rdx_wl_lora_pack(n, self.tab[0].data_ptr(), self.tab[1].data_ptr(), self.tab[2].data_ptr(),
                                     self.caches[0].wext.shape[1], 8, float(lp0.scaling[lp0.adapter]), E_FUSED,
                                     _stream(self.tab)), "wl_lora_pack")
        return loras

    def layer(self, i, h, pb, loras, seed, chain=None):
        layer = self.encoder.layers[i]
        cfg = self.encoder.cfg
        tr = layer.training
        lp = loras[i]
        p_hidden = cfg.hidden_dropout if tr else 0.0
        p_attn = layer.attention.dropout if tr else 0.0
        if lp is None:
            aq = bq = av = bv = None
            p_lora, scale = 0.0, 1.0
        else:
            q, v = lp
            aq, bq = q.lora_A[q.adapter].weight, q.lora_B[q.adapter].weight
            av, bv = v.lora_A[v.adapter].weight, v.lora_B[v.adapter].weight
            dp = q.lora_dropout[q.adapter]
            p_lora = float(getattr(dp, "p", 0.0)) if tr else 0.0
            scale = float(q.scaling[q.adapter])
        if (p_hidden > 0 or p_attn > 0 or p_lora > 0) and seed is None:
            raise RuntimeError("fused WavLM layer: dropout needs the encoder's device seed")
        return WavLMLayerFn.apply(h, aq, bq, av, bv, layer, self.caches[i], pb, seed, i, p_hidden, p_attn, p_lora,
                                  scale, chain)
