"""Per-utterance augmentation API of the reference, on the same HIP kernels as the batched train path.

  RawBoost(algo_id, fs).process(x)         src/rawboost.py:9-33  (algorithms :36-95)
  apply_codec_aug(waveform, sample_rate)   src/data_utils.py:31-59

Same names, arguments and host RNG consumption as the reference: every random parameter is drawn from
numpy's global RNG (RawBoost) or python's `random` (codec gates) in the reference's order, so a caller
interleaving these calls with its own draws sees the same stream. `RawBoost.process` draws the ISD noise
(`np.random.randn(len)` then `np.random.choice([0, 1], len, p)`) and the SSI noise (`randn(len)` before the
SNR) on the host exactly as src/rawboost.py:66-95 does, uploads them, and applies them on the GPU
(csrc/augment.hip: fp64 arithmetic, fp64 IIR for the LnL filters; batched polyphase resampling), one
utterance per launch. `exact=False` selects the batched train path's draw instead: one 62-bit seed per
ISD / SSI call keys a device Philox stream (statistically equivalent, not sample-identical; the numpy
stream then differs from the reference's after such a call — DESIGN.md §2, deviation 6).

Signals are read as fp32 (the model consumes fp32; FLAC samples are exact in fp32); `process` returns
float64 like the reference, `apply_codec_aug` float32 like the reference's torch round trip.
Errors are raised, not swallowed: the reference's try/except fallbacks (rawboost in __getitem__,
codec :55-57) would hide a missing HIP library.
"""
import random

import numpy as np
import torch

from . import _lib
from .ops import rawboost_batch, resample_batch, resample_kernel

CODEC_RATES = (8000, 6000, 4000)


def draw_rawboost(n, algo, exact=False):
    """Host draws of one RawBoost call for an utterance of n samples, after the algorithm choice, in
    the order of rawboost.py:36-95 (LnL: n_a, the unused `a`, 5 numerator and n_a denominator taps, f;
    ISD: beta; SSI: SNR).

    exact=False: one Philox seed for the ISD / SSI noise (drawn last); returns the record.
    exact=True: the reference's own noise draws (ISD: beta, randn(n), choice([0, 1], n, p=[1 - 1/beta,
    1/beta]); SSI: randn(n), then the SNR); returns (record, isd noise*mask or None, ssi noise or None) as
    float64 host arrays."""
    r = _lib.RawboostUtt()
    r.len = n
    r.algo = algo
    if algo in (1, 4):
        n_a = [1, 2, 3, 4, 5][np.random.randint(0, 5)]
        np.random.randint(0, 90)                          # the unused `a` draw (rawboost.py:40)
        b = np.array([1.0])
        for _ in range(5):
            b = np.convolve(b, [1.0, np.random.uniform(-1, 1)])
        a = np.array([1.0])
        for _ in range(n_a):
            a = np.convolve(a, [1.0, np.random.uniform(-0.1, 0.1)])
        r.n_a = n_a
        r.b[:] = list(b)
        aa = np.zeros(6)
        aa[:len(a)] = a
        r.a[:] = list(aa)
        r.f = float(np.random.randn())
    nm = ssi = None
    if algo in (2, 4):
        beta = list(range(5, 10))[np.random.randint(0, 5)]
        r.beta = float(beta)
        if exact:                                         # rawboost.py:71-73
            noise = np.random.randn(n)
            nm = noise * np.random.choice([0, 1], size=n, p=[1 - 1 / beta, 1 / beta])
    if algo == 3:
        if exact:
            ssi = np.random.randn(n)                      # rawboost.py:82, before the SNR (:88)
        r.snr_db = float(np.random.uniform(10, 40))
    if exact:
        return r, nm, ssi
    if algo in (2, 3, 4):
        r.seed = int(np.random.randint(0, 2 ** 62, dtype=np.int64))
    return r


def _device(device):
    return torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())


class RawBoost:
    """Drop-in of src/rawboost.py::RawBoost: process(x) picks one of algo_id per call (np.random.randint,
    :18) — 0 = none, 1 LnL convolutive, 2 ISD impulsive, 3 SSI stationary, 4 LnL then ISD.
    exact (default True): the reference's numpy draws for the ISD / SSI noise (see the module docstring)."""

    def __init__(self, algo_id=(0, 1, 2, 3, 4), fs=16000, device=None, exact=True):
        self.algo_id = list(algo_id)
        self.fs = fs
        self.device = device
        self.exact = bool(exact)

    def process(self, x):
        algo = self.algo_id[np.random.randint(0, len(self.algo_id))]
        if algo not in (1, 2, 3, 4):
            return x
        x = np.asarray(x).reshape(-1)
        dev = _device(self.device)
        isd = ssi = None
        if self.exact:
            rec, nm, nz = draw_rawboost(len(x), algo, exact=True)
            isd = torch.from_numpy(nm).to(dev) if nm is not None else None
            ssi = torch.from_numpy(nz).to(dev) if nz is not None else None
        else:
            rec = draw_rawboost(len(x), algo)
        rec.offset = 0
        out = rawboost_batch(torch.from_numpy(x.astype(np.float32)).to(dev), [rec], noise_isd=isd, noise_ssi=ssi)
        return out.cpu().numpy().astype(np.float64)


_KERNELS = {}


def _resample_kernel_dev(a, b, dev):
    key = (a, b, str(dev))
    if key not in _KERNELS:
        k, w, og, ng = resample_kernel(a, b)
        _KERNELS[key] = (k.reshape(-1).to(dev), w, og, ng)
    return _KERNELS[key]


def apply_codec_aug(waveform_np, sample_rate=16000, device=None):
    """Band-limiting "codec" augmentation (data_utils.py:31-59): with probability 0.5, resample to
    8/6/4 kHz (random.choice) and back with torchaudio's default sinc-Hann kernel (width 6, rolloff 0.99),
    on the GPU. Returns the input object unchanged when the gate is not taken."""
    if random.random() < 0.5:
        target_sr = random.choice(list(CODEC_RATES))
        dev = _device(device)
        x = waveform_np.reshape(-1) if isinstance(waveform_np, torch.Tensor) else np.asarray(waveform_np).reshape(-1)
        x = torch.as_tensor(x, dtype=torch.float32).to(dev)
        kd, wd, ogd, ngd = _resample_kernel_dev(sample_rate, target_sr, dev)
        ku, wu, ogu, ngu = _resample_kernel_dev(target_sr, sample_rate, dev)
        n = x.numel()
        nd = -(-ngd * n // ogd)
        nu = -(-ngu * nd // ogu)
        mid = torch.empty(nd, device=dev)
        out = torch.empty(nu, device=dev)
        resample_batch(x, mid, kd, [_lib.ResampleJob(0, n, 0, nd, ogd, ngd, wd, 0)])
        resample_batch(mid, out, ku, [_lib.ResampleJob(0, nd, 0, nu, ogu, ngu, wu, 0)])
        return out.cpu().numpy()
    return waveform_np
