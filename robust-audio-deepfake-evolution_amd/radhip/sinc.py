"""SincNet stream: SincConv front end on the HIP kernel + the residual 2-D encoder.

Reference: CONV (src/models/DualStreamSEMamba.py:49-138), Residual_block (:144-200) and
SincNetEncoder (:206-270), themselves taken from AASIST (models/AASIST.py:325-466).
"""
import os
import random

import numpy as np
import torch
import torch.nn as nn

import torch.nn.functional as F

from .ops import (HALF, Block0Convs, Block0Front, Block0Fused, BnSelu, ResBlockIdentity, BnSeluSConv, ResTail, SConv, SConvBnSelu, SConvBnSeluSConv, sconv_ok,
                  sconv_weight_ok, sincconv_absmaxpool)


def _half_autocast(x):
    """CUDA autocast to bf16 or fp16: the 16-bit NHWC kernels (libradhip.so / libradhip_f16.so) apply."""
    return x.is_cuda and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") in HALF


def mel_edges(out_channels, sample_rate, nfft=512):
    """Band edges equally spaced on the mel scale over 0..fs/2 (CONV.__init__ :95-101)."""
    f = int(sample_rate / 2) * np.linspace(0, 1, int(nfft / 2) + 1)
    mel = 2595 * np.log10(1 + f / 700)
    m = np.linspace(np.min(mel), np.max(mel), out_channels + 1)
    return 700 * (10 ** (m / 2595) - 1)


def sinc_bank(out_channels=70, kernel_size=129, sample_rate=16000):
    """[C, K] float32 Hamming-windowed band-pass bank. Follows the reference's numeric path exactly
    (float32 tap grid, numpy sinc on it, float32 window x float32 ideal response; :104-117) so the
    bank is bit-identical to the reference's `band_pass` (checked against tests/golden)."""
    K = kernel_size
    edges = mel_edges(out_channels, sample_rate)
    n = torch.arange(-(K - 1) / 2, (K - 1) / 2 + 1, device="cpu")   # float32 grid, as the reference
    win = torch.from_numpy(np.hamming(K)).float()
    rows = []
    for lo, hi in zip(edges[:-1], edges[1:]):
        h = (2 * hi / sample_rate) * np.sinc(2 * hi * n / sample_rate)
        l = (2 * lo / sample_rate) * np.sinc(2 * lo * n / sample_rate)
        rows.append(win * torch.from_numpy(np.asarray(h - l)).float())
    return torch.stack(rows)


class CONV(nn.Module):
    """Drop-in of the reference CONV: fixed (non-learnable) sinc filter bank. `forward` keeps the
    reference's API (x [B,1,T] -> [B,C,T-K+1]) for callers that need the raw conv; SincNetEncoder uses
    `absmaxpool`, the fused HIP path that never materialises the [B, 70, 64472] conv output."""

    def __init__(self, out_channels, kernel_size, sample_rate=16000, in_channels=1, stride=1, padding=0,
                 dilation=1, bias=False, groups=1, mask=False):
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
        self.stride, self.padding, self.dilation, self.mask = stride, padding, dilation, mask
        self.register_buffer("band_pass", sinc_bank(out_channels, self.kernel_size, sample_rate), persistent=False)
        # HIP-graph mode: when set (int32 [2] on the device), the Freq_aug mask is read from here at
        # execution time; the trainer draws it on the host (same RNG order) before each replay.
        self.mask_dev = None

    def draw_mask(self):
        """Freq_aug: zero A = int(U(0,20)) consecutive filters at A0 = randint(0, C-A) (:121-125),
        numpy then python RNG, exactly as the reference draws them."""
        A = int(np.random.uniform(0, 20))
        A0 = random.randint(0, self.out_channels - A)
        return A0, A0 + A

    def forward(self, x, mask=False):
        w = self.band_pass.clone()
        if mask:
            lo, hi = self.draw_mask()
            w[lo:hi] = 0
        return torch.nn.functional.conv1d(x, w.view(self.out_channels, 1, self.kernel_size), stride=self.stride,
                                          padding=self.padding, dilation=self.dilation)

    def absmaxpool(self, x, mask=False):
        """max_pool2d(|conv(x)|, (3,3)) on the HIP kernel: x [B, T] -> [B, C//3, (T-K+1)//3]."""
        if mask and self.mask_dev is not None:
            return sincconv_absmaxpool(x, self.band_pass, mask_dev=self.mask_dev)
        lo, hi = self.draw_mask() if mask else (0, 0)
        return sincconv_absmaxpool(x, self.band_pass, lo, hi)


class Residual_block(nn.Module):
    """Same parameters and forward as the reference block. The reference computes bn1+selu and then
    discards them (`out = self.conv1(x)`, :189); here only bn1's running-stat side effect is kept
    (when bn1 is in training mode), without the dead activation."""

    def __init__(self, nb_filts, first=False):
        super().__init__()
        self.first = first
        if not self.first:
            self.bn1 = nn.BatchNorm2d(num_features=nb_filts[0])
        self.conv1 = nn.Conv2d(nb_filts[0], nb_filts[1], kernel_size=(2, 3), padding=(1, 1), stride=1)
        self.selu = nn.SELU(inplace=True)
        self.bn2 = nn.BatchNorm2d(num_features=nb_filts[1])
        self.conv2 = nn.Conv2d(nb_filts[1], nb_filts[1], kernel_size=(2, 3), padding=(0, 1), stride=1)
        self.downsample = nb_filts[0] != nb_filts[1]
        if self.downsample:
            self.conv_downsample = nn.Conv2d(nb_filts[0], nb_filts[1], padding=(0, 1), kernel_size=(1, 3), stride=1)
        self.mp = nn.MaxPool2d((1, 3))

    def dead_parameters(self):
        """bn1's affine weights: the reference's forward discards bn1's output, so they never receive a
        gradient there (AdamW skips them, weight decay included); radhip.train leaves them out likewise."""
        return [] if self.first else list(self.bn1.parameters())

    def _fused_ok(self, x):
        return (x.is_cuda and not self.bn2.training and x.dim() == 4
                and x.is_contiguous(memory_format=torch.channels_last) and self.conv2.out_channels % 8 == 0)

    def forward(self, x):
        if not self.first and self.bn1.training:
            with torch.no_grad():
                self.bn1(x)
        if self._fused_ok(x):
            # NHWC fused epilogues (csrc/sincnet.hip): conv1's bias is folded into the frozen-BN+SELU pass,
            # conv2 / conv_downsample biases into the add + MaxPool2d((1,3)) pass. Under bf16 / fp16 autocast the
            # 32/64-channel convolutions run on csrc/sconv.hip (conv1 with the BN+SELU in its epilogue).
            bn = self.bn2
            bf = _half_autocast(x)
            invstd = _frozen_invstd(bn)
            bnp = (self.conv1.bias, bn.running_mean, invstd, bn.weight, bn.bias)
            w2 = self.conv2.weight
            # conv1 -> bn2 -> selu -> conv2 as one autograd op on csrc/sconv.hip (its backward reaches conv1's
            # pre-activation in one pass for the 32-channel blocks)
            pair = bf and sconv_weight_ok(w2) and os.environ.get("RADHIP_SCONV_PAIR", "1") != "0"
            idn, a = None, None
            if (self.first and self.downsample and x.shape[1] == 1 and bf and pair and x.shape[3] >= 3
                    and self.conv1.out_channels == 32 and os.environ.get("RADHIP_B0X", "1") != "0"):
                # the whole block in one HIP pass each way (radhip.ops.Block0Fused): no full-size intermediates
                return Block0Fused.apply(x, self.conv1.weight, self.conv_downsample.weight, *bnp, w2, self.conv2.bias,
                                         self.conv_downsample.bias)
            if (self.first and self.downsample and x.shape[1] == 1 and bf
                    and os.environ.get("RADHIP_FUSED_B0", "1") != "0"):
                # one input channel: both convolutions (and conv1's BN + SELU) in one HIP pass each way
                # (radhip.ops.Block0Front; Block0Convs + BnSeluSConv with RADHIP_B0_FWD=0)
                if pair and os.environ.get("RADHIP_B0_FWD", "1") != "0":
                    a, idn = Block0Front.apply(x, self.conv1.weight, self.conv_downsample.weight, *bnp, w2)
                else:
                    c, idn = Block0Convs.apply(x, self.conv1.weight, self.conv_downsample.weight)
                    if pair:
                        a = BnSeluSConv.apply(c, *bnp, w2)
                    else:
                        out = BnSelu.apply(c, *bnp)
            elif bf and sconv_ok(x, self.conv1.weight):
                if pair and not self.downsample and os.environ.get("RADHIP_RES_FUSED", "1") != "0":
                    # the whole block as one autograd op: the block input's gradient in one pass
                    # (conv1's input gradient + the identity branch's, radhip.ops.ResBlockIdentity)
                    return ResBlockIdentity.apply(x, self.conv1.weight, *bnp, w2, self.conv2.bias)
                if pair:
                    a = SConvBnSeluSConv.apply(x, self.conv1.weight, 1, *bnp, w2)
                else:
                    out = SConvBnSelu.apply(x, self.conv1.weight, 1, *bnp)
            else:
                c = F.conv2d(x, self.conv1.weight, None, self.conv1.stride, self.conv1.padding)
                out = BnSelu.apply(c, *bnp)
            if a is None:
                if bf and sconv_ok(out, w2):
                    a = SConv.apply(out, w2, 0)
                else:
                    a = F.conv2d(out, w2, None, self.conv2.stride, self.conv2.padding)
            if self.downsample:
                if idn is None and bf and sconv_ok(x, self.conv_downsample.weight):
                    idn = SConv.apply(x, self.conv_downsample.weight, 0)
                elif idn is None:
                    idn = F.conv2d(x, self.conv_downsample.weight, None, self.conv_downsample.stride,
                                   self.conv_downsample.padding)
                bias = self.conv2.bias + self.conv_downsample.bias
            else:
                idn, bias = x, self.conv2.bias
            return ResTail.apply(a, idn, bias)
        out = self.conv1(x)
        out = self.selu(self.bn2(out))
        out = self.conv2(out)
        identity = self.conv_downsample(x) if self.downsample else x
        return self.mp(out + identity)


def _frozen_invstd(bn):
    """rsqrt(running_var + eps) of a frozen BatchNorm, once per accumulation window (ops.SCONV_WCACHE)."""
    from . import ops as _ops
    cache = _ops.SCONV_WCACHE
    if cache is None:
        return torch.rsqrt(bn.running_var + bn.eps)
    key = ("invstd", id(bn.running_var))
    hit = cache.get(key)
    if hit is not None and hit[0] is bn.running_var:
        return hit[1]
    v = torch.rsqrt(bn.running_var + bn.eps)
    cache[key] = (bn.running_var, v)
    return v


class SincNetEncoder(nn.Module):
    def __init__(self, sinc_channels=70, sinc_kernel=128):
        super().__init__()
        filts = [sinc_channels, [1, 32], [32, 32], [32, 64], [64, 64]]
        self.conv_time = CONV(out_channels=filts[0], kernel_size=sinc_kernel, in_channels=1)
        self.first_bn = nn.BatchNorm2d(num_features=1)
        self.selu = nn.SELU(inplace=True)
        self.encoder = nn.Sequential(
            nn.Sequential(Residual_block(nb_filts=filts[1], first=True)),
            nn.Sequential(Residual_block(nb_filts=filts[2])),
            nn.Sequential(Residual_block(nb_filts=filts[3])),
            nn.Sequential(Residual_block(nb_filts=filts[4])),
            nn.Sequential(Residual_block(nb_filts=filts[4])),
            nn.Sequential(Residual_block(nb_filts=filts[4])))
        self.out_dim = filts[-1][-1]
        # NHWC activations for the residual Conv2d stack: MIOpen's NHWC implicit-GEMM solvers are
        # ~1.4x faster than its NCHW path on these [B, C, 23, T] shapes (measured on MI355X).
        self.channels_last = True

    def forward(self, x, freq_aug=False):
        """x [B, T] -> e_T [B, T', 64] (SincNetEncoder.forward :238-270)."""
        x = self.conv_time.absmaxpool(x.float(), mask=freq_aug).unsqueeze(1)    # [B, 1, 23, T/3]
        x = self.selu(self.first_bn(x))
        if self.channels_last and x.is_cuda:
            x = x.contiguous()
            # C == 1: NCHW memory is already NHWC, but torch keeps the NCHW strides and its layout
            # heuristic would then run block 0's convs in NCHW (and copy every gradient back and forth).
            # Restride to the channels_last form (same bytes) so MIOpen picks its NHWC kernels.
            N, C, H, W = x.shape
            x = x.as_strided((N, C, H, W), (C * H * W, 1, W * C, C)) if C == 1 else \
                x.contiguous(memory_format=torch.channels_last)
        e = self.encoder(x)
        e_T, _ = torch.max(torch.abs(e), dim=2)
        return e_T.transpose(1, 2)
