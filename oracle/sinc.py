"""SincConv restatement: filter bank, Freq_aug band mask, valid conv, |.| + 3x3 max-pool.

Restates CONV.__init__ / CONV.forward (src/models/DualStreamSEMamba.py:55-138) and the first step
of SincNetEncoder.forward (:250-253).
"""
import random

import numpy as np
import torch


def _mel(hz):
    return 2595 * np.log10(1 + hz / 700)


def _hz(mel):
    return 700 * (10 ** (mel / 2595) - 1)


def sinc_filterbank(out_channels=70, kernel_size=128, sample_rate=16000):
    """[C, K] float32 bank with the reference's exact numeric path (DualStreamSEMamba.py:83-117):
    mel-spaced edges over 0..fs/2 (NFFT 512), torch-float32 tap positions, numpy sinc, float32 Hamming
    window times float32 ideal band-pass."""
    K = kernel_size + 1 if kernel_size % 2 == 0 else kernel_size
    f = int(sample_rate / 2) * np.linspace(0, 1, int(512 / 2) + 1)
    fm = _mel(f)
    edges = _hz(np.linspace(np.min(fm), np.max(fm), out_channels + 1))
    taps = torch.arange(-(K - 1) / 2, (K - 1) / 2 + 1, device="cpu")   # float32, as in the reference
    bank = torch.zeros(out_channels, K, device="cpu")
    win = torch.from_numpy(np.hamming(K)).float()
    for i in range(out_channels):
        lo, hi = edges[i], edges[i + 1]
        ideal = (2 * hi / sample_rate) * np.sinc(2 * hi * taps / sample_rate) - \
                (2 * lo / sample_rate) * np.sinc(2 * lo * taps / sample_rate)
        bank[i, :] = win * torch.from_numpy(np.asarray(ideal)).float()
    return bank


def draw_band_mask(n_channels=70):
    """Freq_aug mask draw (DualStreamSEMamba.py:121-125): numpy uniform then python randint."""
    A = int(np.random.uniform(0, 20))
    A0 = random.randint(0, n_channels - A)
    return A0, A0 + A


def sincconv_absmaxpool(x, bank, mask_lo=0, mask_hi=0):
    """float64 numpy: x [B, L], bank [C, K] -> max_pool(|conv|, 3x3) [B, C//3, (L-K+1)//3]."""
    x = np.asarray(x, dtype=np.float64)
    w = np.array(bank, dtype=np.float64)
    w[mask_lo:mask_hi] = 0.0
    C, K = w.shape
    win = np.lib.stride_tricks.sliding_window_view(x, K, axis=1)      # [B, T, K]
    conv = np.abs(np.einsum("btk,ck->bct", win, w))                     # [B, C, T]
    B, _, T = conv.shape
    C3, T3 = C // 3, T // 3
    conv = conv[:, :3 * C3, :3 * T3].reshape(B, C3, 3, T3, 3)
    return conv.max(axis=(2, 4))
