"""Dual-Stream SE-Mamba (Phase-5/6 detector) on the radhip MI355X path.

Drop-in for the reference plugin src/models/DualStreamSEMamba.py::Model(args, device): same
constructor, same attribute names (wavlm_stream / sinc_stream / fusion / backbone_layers / norm_f /
attention_pool / dropout / classifier) and the same state_dict keys, so reference checkpoints load
strictly. forward(x[B, T], Freq_aug) -> (features[B, emb], logits[B, 2]).

What runs where:
  WavLM stream   radhip.wavlm (fused frozen QKV GEMM, SDPA) + HIP layer-weighted sum
  SincNet stream HIP fused SincConv+|.|+maxpool, then the residual Conv2d encoder (csrc/sconv.hip), on a
                 side stream so that it is a parallel branch of the captured graphs
  Bi-Mamba       radhip.mamba.Mamba.bidirectional: HIP conv / selective scan / gate, both
                 directions per launch, one shared out_proj
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch import Tensor

from radhip.head import attn_pool, pool_eligible, se_eligible, se_layer, upcat, upcat_eligible
from radhip.linear import RowLayerNorm, SideLinear, ffn_residual
from radhip.mamba import Mamba
from radhip.ops import layer_weighted_sum
from radhip.sinc import CONV, Residual_block, SincNetEncoder  # noqa: F401  (re-exported like the reference)
from radhip.wavlm import PeftWrapped, WavLMConfigLite, WavLMEncoderModel

_SE_FUSED = os.environ.get("RADHIP_SE_FUSED", "1") != "0"    # 0: the module path (A/B)
_POOL_FUSED = os.environ.get("RADHIP_POOL_FUSED", "1") != "0"   # 0: the module path (A/B)
_UPCAT_FUSED = os.environ.get("RADHIP_UPCAT_FUSED", "1") != "0"  # 0: the module path (A/B)

_LOCAL_WAVLM = [
    os.environ.get("RADHIP_WAVLM_DIR", ""),
    os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pretrained", "microsoft", "wavlm-large"),
    os.path.join(os.getcwd(), "pretrained", "microsoft", "wavlm-large"),
]


def _load_hf_weights(model, path):
    """Load a local HF checkpoint (safetensors or torch .bin with weights_only=True) strictly."""
    st = os.path.join(path, "model.safetensors")
    if os.path.exists(st):
        from safetensors.torch import load_file
        sd = load_file(st)
    else:
        sd = torch.load(os.path.join(path, "pytorch_model.bin"), map_location="cpu", weights_only=True)
    sd = {k[len("wavlm."):] if k.startswith("wavlm.") else k: v for k, v in sd.items()}
    ren = {}
    for k, v in sd.items():  # torch<2.1 weight_norm naming in older HF checkpoints
        k = k.replace("pos_conv_embed.conv.weight_g", "pos_conv_embed.conv.parametrizations.weight.original0")
        k = k.replace("pos_conv_embed.conv.weight_v", "pos_conv_embed.conv.parametrizations.weight.original1")
        ren[k] = v
    own = model.state_dict()
    ren = {k: v for k, v in ren.items() if k in own}
    missing = [k for k in own if k not in ren]
    if missing:
        raise RuntimeError(f"WavLM checkpoint at {path} lacks {len(missing)} tensors, e.g. {missing[:3]}")
    model.load_state_dict(ren, strict=True)


_SIDE = {}


def _side_stream(x):
    """Per-device side stream for the SincNet branch (RADHIP_SINC_BRANCH=0 runs both streams in order)."""
    if not x.is_cuda or os.environ.get("RADHIP_SINC_BRANCH", "1") == "0":
        return None
    d = x.device.index if x.device.index is not None else torch.cuda.current_device()
    if d not in _SIDE:
        _SIDE[d] = torch.cuda.Stream(device=d)
    return _SIDE[d]


class WavLMFrontend(nn.Module):
    """WavLM stream + softmax layer weighting (reference :276-439). With no local checkpoint (no network
    here) the encoder is random-initialised with the wavlm-large architecture."""

    def __init__(self, model_path="microsoft/wavlm-large", freeze_layers=18, config=None):
        super().__init__()
        local = next((p for p in _LOCAL_WAVLM if p and os.path.exists(os.path.join(p, "config.json"))), None)
        if config is not None:
            cfg = WavLMConfigLite(**config)
        elif local:
            cfg = WavLMConfigLite.from_dir(local)
        else:
            cfg = WavLMConfigLite()
        self.model = WavLMEncoderModel(cfg)
        if local and config is None and (os.path.exists(os.path.join(local, "model.safetensors"))
                                          or os.path.exists(os.path.join(local, "pytorch_model.bin"))):
            _load_hf_weights(self.model, local)
            self.pretrained_from = local
        else:
            self.pretrained_from = None
        self.out_dim = 1024
        self.layer_weights = nn.Parameter(torch.zeros(cfg.num_hidden_layers + 1))
        self.apply_freezing_strategy(freeze_layers)

    def _core(self):
        return self.model.base_model.model if isinstance(self.model, PeftWrapped) else self.model

    def apply_freezing_strategy(self, freeze_layers):
        core = self._core()
        core.feature_extractor.requires_grad_(False)
        core.feature_projection.requires_grad_(False)
        for i, layer in enumerate(core.encoder.layers):
            layer.requires_grad_(freeze_layers < 0 or i >= freeze_layers)

    def train(self, mode=True):
        super().train(mode)
        if mode:
            core = self._core()
            core.feature_extractor.eval()
            core.feature_projection.eval()
            for m in core.modules():
                if isinstance(m, (nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d)):
                    m.eval()
        return self

    def forward(self, x, layerdrop=None):
        if x.ndim == 3:
            x = x.squeeze(-1)
        core = self._core()
        _, states = core(x.float(), layerdrop=layerdrop)
        # fused encoder layers take their hidden-state gradients from the sum's backward (radhip/wavlm_fused.py)
        return layer_weighted_sum(states, self.layer_weights, deferred=getattr(core.encoder, "state_defer", None))


class PN_BiMambas_Encoder(nn.Module):
    """Pre-norm Bi-Mamba layer (reference :445-486); the two directions run fused."""

    def __init__(self, d_model, n_state):
        super().__init__()
        self.d_model = d_model
        self.mamba = Mamba(d_model, n_state)
        self.norm1 = RowLayerNorm(d_model, to_linear=True)
        self.norm2 = RowLayerNorm(d_model, to_linear=True)
        self.feed_forward = nn.Sequential(SideLinear(d_model, d_model * 4), nn.GELU(), SideLinear(d_model * 4, d_model))

    def forward(self, x):
        m = self.mamba.bidirectional(self.norm1(x))     # == mamba(n) + flip(mamba(flip(n)))
        # x + feed_forward(norm2(m)).to(x.dtype): on the GPU two csrc/lgemm.hip launches each way (FFN1's bias +
        # GELU and FFN2's bias + widening + residual add in the GEMM epilogues)
        return ffn_residual(x, self.norm2(m), self.feed_forward[0], self.feed_forward[2])


class SELayer(nn.Module):
    """Squeeze-excitation over time for [B, T, C] (reference :492-531)."""

    def __init__(self, channel: int, reduction: int = 16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool1d(1)
        self.fc = nn.Sequential(SideLinear(channel, channel // reduction, bias=False), nn.ReLU(inplace=True),
                                SideLinear(channel // reduction, channel, bias=False), nn.Sigmoid())

    def forward(self, x: Tensor) -> Tensor:
        w1, w2 = self.fc[0].weight, self.fc[2].weight
        if _SE_FUSED and se_eligible(x, w1, w2):
            return se_layer(x, w1, w2)       # radhip/head.py: one launch forward, two backward
        b, t, c = x.size()
        y = self.avg_pool(x.permute(0, 2, 1)).view(b, c)
        return x * self.fc(y).view(b, 1, c)


class DualStreamFusion(nn.Module):
    """LN both streams, project, align SincNet time to WavLM time (nearest if the ratio > 4 else
    linear), concat -> Linear -> SE -> LN -> Dropout (reference :537-637)."""

    def __init__(self, wavlm_dim: int, sinc_dim: int, out_dim: int, reduction: int = 16):
        super().__init__()
        self.ln_wavlm = RowLayerNorm(wavlm_dim, to_linear=True)
        self.ln_sinc = RowLayerNorm(sinc_dim, to_linear=True)
        self.wavlm_proj = SideLinear(wavlm_dim, out_dim)
        self.sinc_proj = SideLinear(sinc_dim, out_dim)
        self.fusion_proj = SideLinear(out_dim * 2, out_dim)
        self.se_layer = SELayer(out_dim, reduction=reduction)
        self.norm = RowLayerNorm(out_dim)
        self.dropout = nn.Dropout(0.1)

    def forward(self, f_wavlm: Tensor, f_sinc: Tensor) -> Tensor:
        f_w = self.wavlm_proj(self.ln_wavlm(f_wavlm))
        f_s = self.sinc_proj(self.ln_sinc(f_sinc))
        T1 = f_w.size(1)
        if _UPCAT_FUSED and upcat_eligible(f_w, f_s):       # radhip/head.py: one gather each way
            return self.dropout(self.norm(self.se_layer(self.fusion_proj(upcat(f_w, f_s)))))
        if f_s.size(1) != T1:
            mode = "nearest" if T1 / f_s.size(1) > 4.0 else "linear"
            kw = {} if mode == "nearest" else {"align_corners": False}
            f_s = F.interpolate(f_s.permute(0, 2, 1), size=T1, mode=mode, **kw).permute(0, 2, 1)
        f = self.fusion_proj(torch.cat([f_w, f_s.to(f_w.dtype)], dim=-1))
        return self.dropout(self.norm(self.se_layer(f)))


class Model(nn.Module):
    def __init__(self, args=None, device="cuda"):
        super().__init__()
        self.device = device
        g = (lambda k, d: getattr(args, k, d)) if args is not None else (lambda k, d: d)
        emb_size = g("emb_size", 144)
        num_encoders = g("num_encoders", 4)
        d_state = g("d_state", 16)
        sinc_channels = g("sinc_channels", 70)
        freeze_layers = g("wavlm_freeze_layers", 18)
        self.wavlm_stream = WavLMFrontend(freeze_layers=freeze_layers, config=g("wavlm_config", None))
        self.sinc_stream = SincNetEncoder(sinc_channels=sinc_channels)
        self.fusion = DualStreamFusion(wavlm_dim=self.wavlm_stream.out_dim, sinc_dim=self.sinc_stream.out_dim,
                                       out_dim=emb_size, reduction=16)
        self.backbone_layers = nn.ModuleList([PN_BiMambas_Encoder(d_model=emb_size, n_state=d_state)
                                              for _ in range(num_encoders)])
        self.norm_f = RowLayerNorm(emb_size, to_linear=True)
        self.attention_pool = SideLinear(emb_size, 1)
        self.dropout = nn.Dropout(0.1)
        self.classifier = SideLinear(emb_size, 2)
        # set by radhip/window.py for an adversarial pass: its SincNet output (a leaf), from one batched pass
        self.sinc_given = None

    @staticmethod
    def sinc_side_stream(x):
        """The stream the SincNet branch runs on (None: in order on the current stream). radhip/window.py puts
        its batched adversarial SincNet pass on it too, so every SincNet launch of a window (and the per-window
        weight layouts they share through radhip.ops.SCONV_WCACHE) is ordered on one stream."""
        return _side_stream(x)

    def _streams(self, x, Freq_aug):
        """The two streams are independent until the fusion. On the GPU the SincNet stream runs on a side
        stream forked from the current one (reference order: WavLM, then SincNet, :728-750), so inside a
        captured HIP graph it is a parallel branch: its kernels (and, because autograd runs each backward
        op on its forward op's stream, its backward) fill the CUs the latency-bound WavLM kernels leave idle.
        The branch is taken only when no RNG is drawn inside the SincNet stream (band mask off, or staged in
        device memory by the graphed trainers): an eager Freq_aug forward draws its mask in the stream, after
        the WavLM stream's SpecAugment / LayerDrop draws, so it runs the streams in the reference order."""
        if self.sinc_given is not None:      # radhip/window.py: this pass's SincNet output, computed batched
            return self.wavlm_stream(x), self.sinc_given
        if os.environ.get("RADHIP_PROBE_NO_SINC") == "1":   # timing probe only (tools): WavLM stream alone
            T2 = (x.shape[-1] - self.sinc_stream.conv_time.kernel_size + 1) // 3
            for _ in range(6):
                T2 //= 3
            return self.wavlm_stream(x), x.new_zeros(x.shape[0], T2, self.sinc_stream.out_dim)
        side = _side_stream(x)
        if Freq_aug and self.sinc_stream.conv_time.mask_dev is None:
            side = None
        if side is None:
            return self.wavlm_stream(x), self.sinc_stream(x, freq_aug=Freq_aug)
        cur = torch.cuda.current_stream(x.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            f_sinc = self.sinc_stream(x, freq_aug=Freq_aug)
        f_wavlm = self.wavlm_stream(x)
        cur.wait_stream(side)
        f_sinc.record_stream(cur)
        return f_wavlm, f_sinc

    def forward(self, x, Freq_aug=False):
        if x.ndim == 3:
            x = x.squeeze(-1)
        f_wavlm, f_sinc = self._streams(x, Freq_aug)
        f = self.fusion(f_wavlm, f_sinc)
        for layer in self.backbone_layers:
            f = layer(f)
        f = self.norm_f(f)
        if _POOL_FUSED and pool_eligible(f, self.attention_pool):
            features = attn_pool(f, self.attention_pool.weight, self.attention_pool.bias)   # radhip/head.py
        else:
            attn = F.softmax(self.attention_pool(f), dim=1)                  # [B, T, 1]
            features = torch.matmul(attn.transpose(1, 2), f).squeeze(1)      # [B, emb]
        features = self.dropout(features)
        return features, self.classifier(features)
