"""CPU restatement of the reference Model (src/models/DualStreamSEMamba.py:49-769).

WavLM stream = transformers' WavLMModel (the reference's own dependency, installed in the image)
with the reference's softmax layer weighting; SincNet / fusion / Bi-Mamba / head restated with the
sequential Mamba of oracle.mamba. State-dict keys equal the reference's (and the product's).
Pinned by tests/golden/model_tiny.npz (reference forward + gradients on seeded weights).
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .mamba import PNBiMambaRef
from .sinc import sinc_filterbank


class OWavLM(nn.Module):
    def __init__(self, cfg_dict):
        super().__init__()
        from transformers import WavLMConfig, WavLMModel
        self.model = WavLMModel(WavLMConfig(**cfg_dict))
        self.layer_weights = nn.Parameter(torch.zeros(self.model.config.num_hidden_layers + 1))

    def forward(self, x, time_mask=None):
        """time_mask: the SpecAugment mask of a training forward ([B, T] bool; HF _mask_hidden_states), given
        explicitly so the oracle uses the product's host draw."""
        hs = self.model(x, output_hidden_states=True, mask_time_indices=time_mask).hidden_states
        w = F.softmax(self.layer_weights, dim=0)
        return (w.view(-1, 1, 1, 1) * torch.stack(hs)).sum(0)


class OConv(nn.Module):
    def __init__(self):
        super().__init__()
        self.band_pass = sinc_filterbank(70, 128, 16000)

    def forward(self, x, mask=None):
        w = self.band_pass.clone().to(device=x.device, dtype=x.dtype)
        if mask is not None:
            w[mask[0]:mask[1]] = 0
        return F.conv1d(x, w.view(70, 1, 129))


class ORes(nn.Module):
    """Residual_block (:144-200) incl. the dead bn1/selu branch."""

    def __init__(self, nb, first=False):
        super().__init__()
        self.first = first
        if not first:
            self.bn1 = nn.BatchNorm2d(nb[0])
        self.conv1 = nn.Conv2d(nb[0], nb[1], (2, 3), padding=(1, 1))
        self.selu = nn.SELU()
        self.bn2 = nn.BatchNorm2d(nb[1])
        self.conv2 = nn.Conv2d(nb[1], nb[1], (2, 3), padding=(0, 1))
        self.downsample = nb[0] != nb[1]
        if self.downsample:
            self.conv_downsample = nn.Conv2d(nb[0], nb[1], (1, 3), padding=(0, 1))
        self.mp = nn.MaxPool2d((1, 3))

    def forward(self, x):
        if not self.first:
            self.selu(self.bn1(x))   # computed and discarded, as in the reference (:185-189)
        out = self.conv2(self.selu(self.bn2(self.conv1(x))))
        idn = self.conv_downsample(x) if self.downsample else x
        return self.mp(out + idn)


class OSinc(nn.Module):
    def __init__(self):
        super().__init__()
        f = [70, [1, 32], [32, 32], [32, 64], [64, 64]]
        self.conv_time = OConv()
        self.first_bn = nn.BatchNorm2d(1)
        self.selu = nn.SELU()
        self.encoder = nn.Sequential(*[nn.Sequential(ORes(nb, first=(i == 0)))
                                       for i, nb in enumerate([f[1], f[2], f[3], f[4], f[4], f[4]])])

    def forward(self, x, mask=None):
        x = self.conv_time(x.unsqueeze(1), mask).unsqueeze(1)
        x = self.selu(self.first_bn(F.max_pool2d(torch.abs(x), (3, 3))))
        e = self.encoder(x)
        return torch.max(torch.abs(e), dim=2)[0].transpose(1, 2)


class OSE(nn.Module):
    def __init__(self, c, r):
        super().__init__()
        self.fc = nn.Sequential(nn.Linear(c, c // r, bias=False), nn.ReLU(), nn.Linear(c // r, c, bias=False),
                                nn.Sigmoid())

    def forward(self, x):
        return x * self.fc(x.mean(1)).unsqueeze(1)


class OFusion(nn.Module):
    def __init__(self, wd, sd, od, red):
        super().__init__()
        self.ln_wavlm, self.ln_sinc = nn.LayerNorm(wd), nn.LayerNorm(sd)
        self.wavlm_proj, self.sinc_proj = nn.Linear(wd, od), nn.Linear(sd, od)
        self.fusion_proj = nn.Linear(2 * od, od)
        self.se_layer = OSE(od, red)
        self.norm = nn.LayerNorm(od)
        self.dropout = nn.Dropout(0.1)

    def forward(self, fw, fs):
        fw = self.wavlm_proj(self.ln_wavlm(fw))
        fs = self.sinc_proj(self.ln_sinc(fs))
        T1, T2 = fw.shape[1], fs.shape[1]
        if T1 != T2:
            if T1 / T2 > 4.0:      # nearest: source index floor(i * T2 / T1)
                idx = torch.floor(torch.arange(T1, dtype=torch.float64) * (T2 / T1)).long()
                fs = fs[:, idx]
            else:
                fs = F.interpolate(fs.transpose(1, 2), size=T1, mode="linear", align_corners=False).transpose(1, 2)
        f = self.se_layer(self.fusion_proj(torch.cat([fw, fs], -1)))
        return self.dropout(self.norm(f))


class OracleModel(nn.Module):
    def __init__(self, wavlm_cfg, emb_size=144, num_encoders=4, d_state=16):
        super().__init__()
        self.wavlm_stream = OWavLM(wavlm_cfg)
        self.sinc_stream = OSinc()
        self.fusion = OFusion(1024, 64, emb_size, 16)
        self.backbone_layers = nn.ModuleList([PNBiMambaRef(emb_size, d_state) for _ in range(num_encoders)])
        self.norm_f = nn.LayerNorm(emb_size)
        self.attention_pool = nn.Linear(emb_size, 1)
        self.dropout = nn.Dropout(0.1)
        self.classifier = nn.Linear(emb_size, 2)

    def forward(self, x, mask=None, time_mask=None):
        f = self.fusion(self.wavlm_stream(x, time_mask), self.sinc_stream(x, mask))
        for layer in self.backbone_layers:
            f = layer(f)
        f = self.norm_f(f)
        a = F.softmax(self.attention_pool(f), dim=1)
        feats = self.dropout(torch.matmul(a.transpose(1, 2), f).squeeze(1))
        return feats, self.classifier(feats)


class OLoraLinear(nn.Module):
    """peft lora.Linear as the reference injects it (src/main.py:103-158: LoraConfig(r, lora_alpha,
    target_modules=[q_proj, v_proj], lora_dropout) + get_peft_model), with peft's state-dict layout
    (base_layer, lora_A.default, lora_B.default). peft's tuner layer exposes its base layer's `weight` and
    `bias` as properties (BaseTunerLayer.weight / .bias; in peft < 0.7 the layer subclasses nn.Linear and
    keeps the base tensors itself): transformers' WavLMAttention reads exactly those (q_proj.weight and the
    concatenated biases go to F.multi_head_attention_forward) and never calls the layer, so in the reference
    the adapter does not enter the forward and its weights get no gradient.

    merged=True is the oracle of the product's lora_mode "active": `weight` returns base + (alpha/r) B A, the
    adapter's contribution with dropout off, so HF's attention applies it."""

    def __init__(self, base, r=8, alpha=32, merged=False):
        super().__init__()
        self.base_layer = base
        self.lora_A = nn.ModuleDict({"default": nn.Linear(base.in_features, r, bias=False)})
        self.lora_B = nn.ModuleDict({"default": nn.Linear(r, base.out_features, bias=False)})
        self.scaling = alpha / r
        self.merged = merged

    @property
    def weight(self):
        w = self.base_layer.weight
        if self.merged:
            w = w + self.scaling * (self.lora_B["default"].weight @ self.lora_A["default"].weight)
        return w

    @property
    def bias(self):
        return self.base_layer.bias

    def forward(self, x):
        return self.base_layer(x) + self.lora_B["default"](self.lora_A["default"](x)) * self.scaling


def apply_lora(model, r=8, alpha=32, targets=("q_proj", "v_proj"), merged=False):
    """Wrap every target linear of the oracle's WavLM in OLoraLinear (base weights frozen, as peft does)."""
    wl = model.wavlm_stream.model
    for p in wl.parameters():
        p.requires_grad_(False)
    for layer in wl.encoder.layers:
        att = layer.attention
        for t in targets:
            setattr(att, t, OLoraLinear(getattr(att, t), r, alpha, merged))
    return model


def from_peft_state(sd):
    """The product's peft-wrapped WavLM keys (wavlm_stream.model.base_model.model.<path>) -> the oracle's."""
    return {k.replace("wavlm_stream.model.base_model.model.", "wavlm_stream.model."): v for k, v in sd.items()}


def focal_loss(logits, y, alpha=0.9, gamma=2.5):
    """kornia FocalLoss(alpha, gamma, reduction='mean') with per-class alpha [1 - alpha, alpha] (src/main.py:
    297-305; the default 'per_class' restatement of radhip.train.FocalLoss): the mean runs over B x C."""
    lp = F.log_softmax(logits, dim=1).gather(1, y[:, None]).squeeze(1)
    a = torch.where(y == 0, 1.0 - alpha, alpha).to(lp.dtype)
    return (-a * (1.0 - lp.exp()) ** gamma * lp).sum() / (logits.shape[0] * logits.shape[1])


def tiny_wavlm_config(js):
    import json
    d = json.loads(str(js)) if not isinstance(js, dict) else dict(js)
    d["conv_dim"] = tuple(d["conv_dim"])
    return d


def np_seed_everything(seed):
    np.random.seed(seed)
    torch.manual_seed(seed)
