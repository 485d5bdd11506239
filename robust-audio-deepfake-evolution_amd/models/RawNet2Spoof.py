"""RawNet2 (legacy plugin, BASELINE config 1) on the radhip MI355X path.

Drop-in for the reference's models/RawNet2Spoof.py::Model(d_args): same constructor, attribute names
and state_dict keys (Sinc_conv has no parameters; block0..block5, fc_attention0..5, bn_before_gru, gru,
fc1_gru, fc2_gru), forward(x[B, 64600], Freq_aug=None) -> (last_hidden[B, nb_fc_node], log-probs[B, 2]).

What runs where:
  front end   SincConv (20 x 1025 taps) + |.| + MaxPool1d(3) in ONE HIP launch
              (rdx_sincconv_abspool1d_fwd, csrc/sincconv.hip): the [B, 20, 63576] conv output is never
              written (reference :77-103, :244-245); the bank is fixed (not a Parameter), so nothing
              flows back through it
  blocks      Conv1d / BatchNorm1d / LeakyReLU(0.3) residual blocks with the filter-wise feature
              map scaling (FMS: x * s + s, s = sigmoid(fc(avgpool(x)))) (reference :106-165, :249-295)
  back end    BatchNorm1d + SELU, 3-layer GRU(1024) (MIOpen RNN, fp32 under autocast), last step -> fc1 -> fc2 -> log-softmax

Reference quirks kept: `out = self.conv1(x)` discards the bn1/LeakyReLU branch of non-first blocks
(:155), but bn1 still updates its running statistics in training mode; blocks 3-5 are built after the
reference rewrites filts[2][0] := filts[2][1] (:189) — here on a copy, so the caller's config is not
mutated.
"""
import copy

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from radhip.ops import sincconv_abspool1d
from radhip.sinc import mel_edges


def sinc_bank_rawnet(out_channels, kernel_size, sample_rate=16000):
    """[C, K] fp32 bank of SincConv.forward (:77-93): hamming(K) x (hHigh - hLow) on the float32 tap grid,
    numpy sinc evaluated on it, float32 products — the same numeric path as the reference."""
    K = kernel_size
    edges = mel_edges(out_channels, sample_rate)
    n = torch.arange(-(K - 1) / 2, (K - 1) / 2 + 1)
    win = torch.from_numpy(np.hamming(K)).float()
    rows = []
    for lo, hi in zip(edges[:-1], edges[1:]):
        h = (2 * hi / sample_rate) * np.sinc(2 * hi * n / sample_rate)
        l = (2 * lo / sample_rate) * np.sinc(2 * lo * n / sample_rate)
        rows.append(win * torch.from_numpy(np.asarray(h - l)).float())
    return torch.stack(rows)


class SincConv(nn.Module):
    """Reference SincConv (:15-103): fixed mel-spaced band-pass bank, no parameters."""

    def __init__(self, out_channels, kernel_size, in_channels=1, sample_rate=16000, stride=1, padding=0,
                 dilation=1, bias=False, groups=1):
        super().__init__()
        if in_channels != 1:
            raise ValueError("SincConv only support one input channel (here, in_channels = {%i})" % in_channels)
        if bias:
            raise ValueError("SincConv does not support bias.")
        if groups > 1:
            raise ValueError("SincConv does not support groups.")
        self.out_channels = out_channels
        self.kernel_size = kernel_size + 1 if kernel_size % 2 == 0 else kernel_size
        self.sample_rate = sample_rate
        self.stride, self.padding, self.dilation = stride, padding, dilation
        self.register_buffer("band_pass", sinc_bank_rawnet(out_channels, self.kernel_size, sample_rate),
                             persistent=False)

    def forward(self, x):
        """The raw conv (reference API): x [B, 1, L] -> [B, C, L - K + 1]."""
        return F.conv1d(x, self.band_pass.view(self.out_channels, 1, self.kernel_size), stride=self.stride,
                        padding=self.padding, dilation=self.dilation)

    def abspool(self, x):
        """max_pool1d(|conv(x)|, 3) on the HIP kernel: x [B, L] -> [B, C, (L - K + 1) // 3]."""
        if self.stride != 1 or self.padding != 0 or self.dilation != 1:
            raise ValueError("radhip SincConv front end: stride 1, no padding, no dilation (the RawNet2 setup)")
        return sincconv_abspool1d(x, self.band_pass)


class Residual_block(nn.Module):
    """Reference :106-165 (1-D residual block)."""

    def __init__(self, nb_filts, first=False):
        super().__init__()
        self.first = first
        if not self.first:
            self.bn1 = nn.BatchNorm1d(num_features=nb_filts[0])
        self.lrelu = nn.LeakyReLU(negative_slope=0.3)
        self.conv1 = nn.Conv1d(nb_filts[0], nb_filts[1], kernel_size=3, padding=1, stride=1)
        self.bn2 = nn.BatchNorm1d(num_features=nb_filts[1])
        self.conv2 = nn.Conv1d(nb_filts[1], nb_filts[1], padding=1, kernel_size=3, stride=1)
        self.downsample = nb_filts[0] != nb_filts[1]
        if self.downsample:
            self.conv_downsample = nn.Conv1d(nb_filts[0], nb_filts[1], padding=0, kernel_size=1, stride=1)
        self.mp = nn.MaxPool1d(3)

    def dead_parameters(self):
        """bn1's affine weights: the reference discards bn1's output (models/RawNet2Spoof.py:150-155), so they
        never get a gradient or an optimizer step there (radhip.train.no_grad_params)."""
        return [] if self.first else list(self.bn1.parameters())

    def forward(self, x):
        if not self.first and self.bn1.training:
            with torch.no_grad():           # the discarded bn1 branch: only its running-stat update survives
                self.bn1(x)
        out = self.conv2(self.lrelu(self.bn2(self.conv1(x))))
        identity = self.conv_downsample(x) if self.downsample else x
        return self.mp(out + identity)


class Model(nn.Module):
    def __init__(self, d_args):
        super().__init__()
        filts = copy.deepcopy(d_args["filts"])
        self.Sinc_conv = SincConv(out_channels=filts[0], kernel_size=d_args["first_conv"],
                                  in_channels=d_args["in_channels"])
        self.first_bn = nn.BatchNorm1d(num_features=filts[0])
        self.selu = nn.SELU(inplace=True)
        self.block0 = nn.Sequential(Residual_block(nb_filts=filts[1], first=True))
        self.block1 = nn.Sequential(Residual_block(nb_filts=filts[1]))
        self.block2 = nn.Sequential(Residual_block(nb_filts=filts[2]))
        filts[2][0] = filts[2][1]
        self.block3 = nn.Sequential(Residual_block(nb_filts=filts[2]))
        self.block4 = nn.Sequential(Residual_block(nb_filts=filts[2]))
        self.block5 = nn.Sequential(Residual_block(nb_filts=filts[2]))
        self.avgpool = nn.AdaptiveAvgPool1d(1)
        c1, c2 = filts[1][-1], filts[2][-1]
        for i, c in enumerate([c1, c1, c2, c2, c2, c2]):
            setattr(self, f"fc_attention{i}", nn.Sequential(nn.Linear(c, c)))
        self.bn_before_gru = nn.BatchNorm1d(num_features=c2)
        self.gru = nn.GRU(input_size=c2, hidden_size=d_args["gru_node"], num_layers=d_args["nb_gru_layer"],
                          batch_first=True)
        self.fc1_gru = nn.Linear(d_args["gru_node"], d_args["nb_fc_node"])
        self.fc2_gru = nn.Linear(d_args["nb_fc_node"], d_args["nb_classes"], bias=True)
        self.sig = nn.Sigmoid()
        self.logsoftmax = nn.LogSoftmax(dim=1)

    def _fms(self, x, fc):
        """Filter-wise feature map scaling (reference :250-255): s = sigmoid(fc(mean_t x)); x * s + s."""
        s = self.sig(fc(x.mean(dim=2))).unsqueeze(-1)
        return x * s + s

    def forward(self, x, Freq_aug=None):
        x = self.Sinc_conv.abspool(x.reshape(x.shape[0], -1).float())    # [B, 20, (L - 1024) / 3]
        x = self.selu(self.first_bn(x))
        for i in range(6):
            x = self._fms(getattr(self, f"block{i}")(x), getattr(self, f"fc_attention{i}"))
        x = self.selu(self.bn_before_gru(x))
        self.gru.flatten_parameters()
        with torch.autocast(x.device.type, enabled=False):   # GRU kept in fp32 (no bf16 RNN path relied on)
            x, _ = self.gru(x.float().permute(0, 2, 1))
        last_hidden = self.fc1_gru(x[:, -1, :])
        return last_hidden, self.logsoftmax(self.fc2_gru(last_hidden))
