"""The WavLM-Large stream of the fp32 scoring pass on split-precision ("x3") kernels.

The reference scores without autocast (src/main.py:958-995; the comment at :974-975 keeps eval in fp32), through
WavLMFrontend (src/models/DualStreamSEMamba.py:392-439) over HF WavLMModel, and the north star holds the logits to
1e-3 of that fp32 path. gfx950 has no TF32, and its fp32 MFMA runs at 1/16 of the bf16 rate (157 TF). So every fp32
operand here is carried as two bf16 planes, hi = bf16(x) and lo = bf16(x - hi), and each GEMM sums three bf16 MFMA
products Ahi.Bhi + Alo.Bhi + Ahi.Blo with fp32 accumulation (csrc/hgemm.hip rdx_hgemm_x3): about 2^-16 relative error
per product against fp32's 2^-24, at a third of the bf16 MFMA rate. The rest of the stream stays fp32 (csrc/x3.hip):
  * CNN layer 0 + LayerNorm + GELU direct in fp32; layers 1-6 as strided implicit GEMMs over the token-major planes
    (rows overlapping at stride * 512, one launch over the batch), LayerNorm + GELU in fp32;
  * feature_projection: LayerNorm(512) -> planes -> x3 GEMM;
  * positional conv: the fp32 stream split as it is staged, 3 MFMA products per tap, + GELU + the residual add;
  * per layer: LN1 + gate -> planes; q|k|v x3 GEMM -> fp32; fp32 gated attention (v_mfma_f32_16x16x4_f32) -> planes;
    out_proj x3 -> fp32; residual + LN2 -> planes; FFN1 + GELU x3 (planes out) -> FFN2 x3 -> fp32; the residual
    add runs in the next layer's LN1 pass.
The frozen weights' planes are made once per weight version (LoRA in "active" mode merged into q / v first:
W + s B A, the same product the adapter adds). Everything else of the model (SincNet, fusion, Bi-Mamba, head) runs
its fp32 kernels.

Enabled by `scoring()` (radhip.infer._scores with amp="x3"); RADHIP_X3=0 disables it.
"""
import contextlib
import os
import threading

import torch

from . import _lib
from ._lib import check, lib
from .ops import _p, _stream, _timed, gemm_flops, rel_bias_table, _wgemm_workspace

_STATE = threading.local()

# (tile, splits, group_m) of rdx_hgemm_x3 per GEMM at the eval batch (32 x 201 tokens), from the standalone sweep
# (tools/bench_x3.py, profiles/r06_bench_x3.jsonl, us; bf16-equivalent rate / 2.5 PF): q|k|v 256 x 192 column order
# 124 (0.39), out_proj 128 x 256 48 (0.34), FFN1 + GELU planes 256 x 256 164 (0.39), FFN2 128 x 256 159 (0.41);
# hipBLASLt fp32 on the same shapes 393 / 138 / 434 / 454. The CNN convs take 256 x 256.
X3_POLICY = {"qkv": (1, 1, 0), "out": (2, 1, 4), "ffn1": (0, 1, 4), "ffn2": (2, 1, 4), "proj": (2, 1, 4),
             "cnn": (0, 1, 0)}


@contextlib.contextmanager
def scoring():
    """Within the block, an eligible WavLM stream in eval mode without grad runs on the x3 kernels."""
    prev = getattr(_STATE, "on", False)
    _STATE.on = True
    try:
        yield
    finally:
        _STATE.on = prev


def active():
    return getattr(_STATE, "on", False) and os.environ.get("RADHIP_X3", "1") != "0"


def planes(w):
    """fp32 tensor -> (hi, lo) bf16 tensors of its shape: hi = bf16(w), lo = bf16(w - hi)."""
    w = w.detach().float()
    hi = w.to(torch.bfloat16)
    lo = (w - hi.float()).to(torch.bfloat16)
    return hi.contiguous(), lo.contiguous()


def eligible(model, x):
    """The x3 stream applies to WavLM-Large geometry (layer-norm CNN of 512 channels with conv0 k 10, stable layer
    norm, 64-dim heads, GELU FFN, the 128-tap / 16-group positional conv), CUDA, eval mode, no grad."""
    c = model.config
    if not (active() and x.is_cuda and x.dim() == 2 and not model.training and not torch.is_grad_enabled()):
        return False
    if torch.is_autocast_enabled("cuda"):
        return False
    from .wavlm import LoraLinear
    ok = (c.feat_extract_norm == "layer" and c.feat_extract_activation == "gelu" and c.hidden_act == "gelu"
          and all(d == 512 for d in c.conv_dim) and c.conv_kernel[0] == 10 and c.conv_dim[0] == 512
          and c.do_stable_layer_norm and c.hidden_size == 1024 and c.hidden_size // c.num_attention_heads == 64
          and c.num_conv_pos_embeddings == 128 and c.num_conv_pos_embedding_groups == 16 and x.shape[1] >= 400)
    if not ok:
        return False
    for layer in model.encoder.layers:
        a = layer.attention
        for name in ("k_proj", "out_proj"):
            if isinstance(getattr(a, name), LoraLinear) and getattr(a, name).active:
                return False
    return True


def _merged(lin):
    """Weight of a (possibly LoRA-wrapped) projection as the forward applies it: W, or W + s B A for an active
    adapter (peft lora.Linear without dropout in eval: y = W x + b + s B A x)."""
    from .wavlm import LoraLinear
    if isinstance(lin, LoraLinear):
        w = lin.base_layer.weight.detach().float()
        if lin.active:
            a = lin.adapter
            w = w + lin.scaling[a] * (lin.lora_B[a].weight.detach().float() @ lin.lora_A[a].weight.detach().float())
        return w, lin.base_layer.bias
    return lin.weight.detach().float(), lin.bias


def _src(model):
    """Every tensor the planes are made from (weights, LoRA factors) with its version: the cache key."""
    ts = [p for p in model.parameters()] + [b for b in model.buffers()]
    return tuple((t.data_ptr(), t._version) for t in ts)


class X3Weights:
    """Planes and fp32 parameters of one WavLM model for the x3 stream."""

    def __init__(self, model):
        c = model.config
        dev = next(model.parameters()).device
        f = lambda t: t.detach().float().contiguous() if t is not None else None   # noqa: E731
        with torch.no_grad():
            fe = model.feature_extractor.conv_layers
            self.fe0 = (f(fe[0].conv.weight.reshape(512, -1)), f(fe[0].conv.bias), f(fe[0].layer_norm.weight),
                        f(fe[0].layer_norm.bias), float(fe[0].layer_norm.eps), fe[0].conv.kernel_size[0],
                        fe[0].conv.stride[0])
            self.fe = []
            for ly in fe[1:]:
                w = ly.conv.weight.detach().float().permute(0, 2, 1).reshape(512, -1)     # [C_out][k][C_in]
                self.fe.append((planes(w), f(ly.conv.bias), f(ly.layer_norm.weight), f(ly.layer_norm.bias),
                                float(ly.layer_norm.eps), ly.conv.kernel_size[0], ly.conv.stride[0]))
            fp = model.feature_projection
            self.fp = (f(fp.layer_norm.weight), f(fp.layer_norm.bias), float(fp.layer_norm.eps),
                       planes(fp.projection.weight), f(fp.projection.bias))
            pce = model.encoder.pos_conv_embed
            W = pce._weight().detach().float().reshape(16, 64, 64, 128)                 # [g, n, c, k]
            wk = W.permute(0, 3, 1, 2).contiguous()                                     # [g][k][n][c]
            self.pos = (planes(wk), f(pce.conv.bias))
            self.layers = []
            for layer in model.encoder.layers:
                a, ff = layer.attention, layer.feed_forward
                (wq, bq), (wk_, bk), (wv, bv) = _merged(a.q_proj), _merged(a.k_proj), _merged(a.v_proj)
                wo, bo = _merged(a.out_proj)
                self.layers.append(dict(
                    ln1=(f(layer.layer_norm.weight), f(layer.layer_norm.bias), float(layer.layer_norm.eps)),
                    gate=(f(a.gru_rel_pos_linear.weight), f(a.gru_rel_pos_linear.bias),
                          f(a.gru_rel_pos_const.reshape(-1))),
                    wqkv=planes(torch.cat([wq, wk_, wv])), bqkv=f(torch.cat([bq, bk, bv])),
                    wo=planes(wo), bo=f(bo),
                    ln2=(f(layer.final_layer_norm.weight), f(layer.final_layer_norm.bias),
                         float(layer.final_layer_norm.eps)),
                    w1=planes(ff.intermediate_dense.weight), b1=f(ff.intermediate_dense.bias),
                    w2=planes(ff.output_dense.weight), b2=f(ff.output_dense.bias)))
            ln = model.encoder.layer_norm
            self.ln_f = (f(ln.weight), f(ln.bias), float(ln.eps))
            self.rel_emb = model.encoder.layers[0].attention
            self.H = c.num_attention_heads
        self.dev = dev
        self.pb_key = None

    def position_bias(self, T):
        emb = self.rel_emb.rel_attn_embed.weight
        key = (T, emb.data_ptr(), emb._version)
        if key != self.pb_key:
            with torch.no_grad():
                self.pb = rel_bias_table(self.rel_emb.compute_bias(T, self.dev).float())
            self.pb_key = key
        return self.pb


def weights(model):
    key = _src(model)
    cur = model.__dict__.get("_x3w")
    if cur is None or cur[0] != key:
        cur = (key, X3Weights(model))
        model.__dict__["_x3w"] = cur
    return cur[1]


def gemm(a, a_lo, w, bias, out=None, out_lo=None, epilogue=_lib.EPI_F32, pol="qkv", M=None, lda=None, sa=0,
         batch=1, sc=0, K=None, name="hgemm_x3"):
    """C = (a + a_lo) (w_hi + w_lo)^T + bias on rdx_hgemm_x3. a / a_lo bf16 planes (row stride lda, default a's),
    w the (hi, lo) planes [N, K]; EPI_F32 returns fp32 C [M, N]; EPI_F32_GELU_SPLIT returns the planes of
    gelu(C)."""
    wh, wl = w
    N, Kw = wh.shape
    K = Kw if K is None else K
    M = a.shape[0] if M is None else M
    lda = a.stride(0) if lda is None else lda
    tile, splits, group_m = X3_POLICY[pol]
    dev = a.device
    if epilogue == _lib.EPI_F32:
        if out is None:
            out = torch.empty(M, N, device=dev, dtype=torch.float32)
    elif out is None:
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        out_lo = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ldc = N if batch == 1 else out.stride(-2)
    ws = cnt = None
    ws_bytes = n_cnt = 0
    if splits > 1:
        ws_bytes = int(lib().rdx_hgemm_ws_bytes(M, N, tile, splits))
        n_cnt = int(lib().rdx_hgemm_counters(M, N, tile))
        ws, cnt = _wgemm_workspace(dev, ws_bytes, n_cnt)
        ws_bytes, n_cnt = ws.numel(), cnt.numel()
    with _timed(name, a, 3 * gemm_flops(M * batch, N, K), shape=(M * batch, N, K)):
        check(lib().rdx_hgemm_x3(_p(a), _p(a_lo), int(lda), int(sa), _p(wh), _p(wl), wh.stride(0), _p(out),
                                 _p(out_lo) if out_lo is not None else None, int(ldc), int(sc), int(M), int(N), int(K),
                                 int(batch), _p(bias) if bias is not None else None, int(epilogue), tile, splits,
                                 group_m, _p(ws) if ws is not None else None, ws_bytes,
                                 _p(cnt) if cnt is not None else None, n_cnt, _stream(a)), "hgemm_x3")
    return out if epilogue == _lib.EPI_F32 else (out, out_lo)


def _ln(a, ln, out_planes=True, b=None, sum_out=None, y32=None, gate=None, gate_out=None):
    M, E = a.shape
    hi = lo = None
    if out_planes:
        hi = torch.empty(M, E, device=a.device, dtype=torch.bfloat16)
        lo = torch.empty_like(hi)
    g, bt, eps = ln
    wg = bg = gc = None
    if gate is not None:
        wg, bg, gc = gate
    check(lib().rdx_x3_ln_split(_p(a), _p(b) if b is not None else None, _p(sum_out) if sum_out is not None else None,
                                _p(g), _p(bt), float(eps), _p(hi) if hi is not None else None,
                                _p(lo) if lo is not None else None, E, _p(y32) if y32 is not None else None,
                                _p(wg) if wg is not None else None, _p(bg) if bg is not None else None,
                                _p(gc) if gc is not None else None, _p(gate_out) if gate_out is not None else None,
                                M, E, _stream(a)), "x3_ln_split")
    return hi, lo


def feature_encoder(W, x):
    """x [B, L] fp32 -> fp32 [B, T, 512] token-major (the CNN's output before feature_projection)."""
    B, L = x.shape
    dev = x.device
    w0, b0, g0, be0, eps0, k0, s0 = W.fe0
    T = (L - k0) // s0 + 1
    hi = torch.empty(B, T, 512, device=dev, dtype=torch.bfloat16)
    lo = torch.empty_like(hi)
    with _timed("x3_fe_conv0", x, 4.0 * B * L + 4.0 * B * T * 512):
        check(lib().rdx_x3_fe_conv0(_p(x), B, L, _p(w0), _p(b0) if b0 is not None else None, _p(g0), _p(be0),
                                    float(eps0), k0, s0, _p(hi), _p(lo), _stream(x)), "x3_fe_conv0")
    out = None
    for i, (wp, b, g, be, eps, k, s) in enumerate(W.fe):
        To = (T - k) // s + 1
        y = torch.empty(B, To, 512, device=dev, dtype=torch.float32)
        gemm(hi, lo, wp, b, out=y, M=To, lda=s * 512, sa=T * 512, batch=B, sc=To * 512, K=k * 512, pol="cnn",
             name="x3_fe_conv")
        last = i == len(W.fe) - 1
        if last:
            out = torch.empty(B, To, 512, device=dev, dtype=torch.float32)
            nh = nl = None
        else:
            nh = torch.empty(B, To, 512, device=dev, dtype=torch.bfloat16)
            nl = torch.empty_like(nh)
        check(lib().rdx_x3_fe_ln_gelu(_p(y), B * To, None, _p(g), _p(be), float(eps),
                                      _p(nh) if nh is not None else None, _p(nl) if nl is not None else None,
                                      _p(out) if out is not None else None, _stream(x)), "x3_fe_ln_gelu")
        hi, lo, T = nh, nl, To
    return out


@torch.no_grad()
def forward(model, x):
    """WavLMEncoderModel.forward (eval, output_hidden_states) on the x3 kernels: (last, states) with the 25 hidden
    states of HF WavLMEncoderStableLayerNorm (each layer's input, then the final LayerNorm's output), fp32."""
    W = weights(model)
    x = x.contiguous().float()
    feats = feature_encoder(W, x)                                   # [B, T, 512]
    B, T, _ = feats.shape
    M, E = B * T, 1024
    dev = x.device
    g, bt, eps, wp, bp = W.fp
    fh, fl = _ln(feats.view(M, 512), (g, bt, eps))
    h = gemm(fh, fl, wp, bp, pol="proj")                            # [M, 1024]
    hp = torch.empty_like(h)
    (pkh, pkl), pbias = W.pos
    check(lib().rdx_x3_posconv_fwd(_p(h), _p(pkh), _p(pkl), _p(pbias), _p(hp), B, T, _stream(h)), "x3_posconv")
    h = hp
    rel = W.position_bias(T)
    states = []
    prev = None                                                     # (h2, fo) of the previous layer
    H = W.H
    n = len(W.layers)
    for i, L in enumerate(W.layers):
        gate = torch.empty(M, H, device=dev, dtype=torch.float32)
        if prev is None:
            states.append(h.view(B, T, E))
            x1h, x1l = _ln(h, L["ln1"], gate=L["gate"], gate_out=gate)
        else:
            h = torch.empty(M, E, device=dev, dtype=torch.float32)
            x1h, x1l = _ln(prev[0], L["ln1"], b=prev[1], sum_out=h, gate=L["gate"], gate_out=gate)
            states.append(h.view(B, T, E))
        qkv = gemm(x1h, x1l, L["wqkv"], L["bqkv"], pol="qkv")        # [M, 3E]
        oh = torch.empty(M, E, device=dev, dtype=torch.bfloat16)
        ol = torch.empty_like(oh)
        with _timed("x3_attn", h, 2.0 * 2 * B * H * T * T * 64):
            check(lib().rdx_x3_attn_fwd(_p(qkv), _p(qkv[:, E:]), _p(qkv[:, 2 * E:]), 3 * E, _p(gate), _p(rel), 0.125,
                                        _p(oh), _p(ol), E, B, T, H, 1 if B * H >= 256 else 2, _stream(h)), "x3_attn")
        aout = gemm(oh, ol, L["wo"], L["bo"], pol="out")
        h2 = torch.empty(M, E, device=dev, dtype=torch.float32)
        x2h, x2l = _ln(h, L["ln2"], b=aout, sum_out=h2)
        vh, vl = gemm(x2h, x2l, L["w1"], L["b1"], epilogue=_lib.EPI_F32_GELU_SPLIT, pol="ffn1")
        fo = gemm(vh, vl, L["w2"], L["b2"], pol="ffn2")
        prev = (h2, fo)
    last = torch.empty(M, E, device=dev, dtype=torch.float32)
    _ln(prev[0], W.ln_f, out_planes=False, b=prev[1], y32=last)
    states.append(last.view(B, T, E))
    return last.view(B, T, E), states
