"""Audio file reading for the data path: ctypes binding of libradio.so (include/radio.h).

`read(path)` mirrors `soundfile.read(path)` as the reference calls it (src/data_utils.py:165, :200,
:221): it returns (float64 array, sample_rate), mono as [n], multi-channel as [n, channels], values
x / 2^(bits-1). `read_batch(paths)` is the native multi-threaded loader the train/eval pipelines use:
every file of a micro-batch is decoded in parallel into one float32 buffer (optionally pinned) that
then goes to the GPU in a single copy. `.wav` files (the In-the-Wild set, data_utils.py:262) are read
with scipy.io.wavfile, normalised the same way.

There is no Python fallback decoder: a missing libradio.so raises.
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RADIO_LIB", os.path.join(_HERE, "libradio.so"))

c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_vp = ctypes.c_void_p
c_str = ctypes.c_char_p

SIGNATURES = {
    "rdx_io_strerror": (c_str, [c_int]),
    "rdx_flac_probe": (c_int, [c_str, ctypes.POINTER(c_i64), ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                               ctypes.POINTER(c_int)]),
    "rdx_flac_read": (c_int, [c_str, c_vp, c_i64, ctypes.POINTER(c_i64)]),
    "rdx_flac_decode_mem": (c_int, [c_vp, c_i64, c_vp, c_i64, ctypes.POINTER(c_i64), ctypes.POINTER(c_int),
                                    ctypes.POINTER(c_int)]),
    "rdx_flac_read_batch": (c_int, [ctypes.POINTER(c_str), c_int, c_vp, ctypes.POINTER(c_i64),
                                    ctypes.POINTER(c_i64), ctypes.POINTER(c_i64), ctypes.POINTER(c_int), c_int]),
}

_lock = threading.Lock()
_lib = None


def header_symbols():
    import re
    text = open(os.path.join(_HERE, "..", "..", "include", "radio.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int64_t|int)\s+(rdx_\w+)\s*\(", text, re.M)))


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"libradio.so not found at {LIB_PATH}: build it with `make -C csrc`")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


class AudioReadError(RuntimeError):
    pass


def _check(code, what):
    if code != 0:
        raise AudioReadError(f"{what}: {lib().rdx_io_strerror(int(code)).decode()} (code {code})")


def probe(path):
    """(frames, channels, sample_rate, bits) from STREAMINFO."""
    fr, ch, sr, bits = c_i64(), c_int(), c_int(), c_int()
    _check(lib().rdx_flac_probe(os.fsencode(str(path)), ctypes.byref(fr), ctypes.byref(ch), ctypes.byref(sr),
                                ctypes.byref(bits)), str(path))
    return fr.value, ch.value, sr.value, bits.value


def decode_bytes(data):
    """Decode an in-memory FLAC stream -> (float64 [n] or [n, ch], sample_rate)."""
    buf = np.frombuffer(data, dtype=np.uint8)
    fr, ch, sr = c_i64(), c_int(), c_int()
    code = lib().rdx_flac_decode_mem(buf.ctypes.data, buf.size, None, 0, ctypes.byref(fr), ctypes.byref(ch),
                                     ctypes.byref(sr))
    if code not in (0, -104):
        _check(code, "flac stream")
    out = np.empty((fr.value, ch.value), dtype=np.float64)
    _check(lib().rdx_flac_decode_mem(buf.ctypes.data, buf.size, out.ctypes.data, fr.value, ctypes.byref(fr),
                                     ctypes.byref(ch), ctypes.byref(sr)), "flac stream")
    return (out[:, 0] if ch.value == 1 else out), sr.value


def read(path):
    """soundfile.read(path) equivalent for .flac (native) and .wav (scipy): (float64 data, sr)."""
    path = str(path)
    if path.lower().endswith(".wav"):
        from scipy.io import wavfile
        sr, x = wavfile.read(path)
        if x.dtype.kind == "i":
            x = x.astype(np.float64) / float(2 ** (8 * x.dtype.itemsize - 1))
        elif x.dtype == np.uint8:
            x = (x.astype(np.float64) - 128.0) / 128.0
        else:
            x = x.astype(np.float64)
        return x, sr
    frames, ch, sr, _ = probe(path)
    if frames == 0:  # length unknown to the encoder: decode from memory
        with open(path, "rb") as f:
            return decode_bytes(f.read())
    out = np.empty((frames, ch), dtype=np.float64)
    got = c_i64()
    _check(lib().rdx_flac_read(os.fsencode(path), out.ctypes.data, frames, ctypes.byref(got)), path)
    return (out[:, 0] if ch == 1 else out), sr


def read_batch(paths, out=None, threads=8):
    """Decode mono .flac files in parallel. Returns (flat float32 buffer, offsets[int64], lens[int64]).
    `out` may be a preallocated (e.g. pinned torch) float32 buffer large enough for all files."""
    n = len(paths)
    lens = np.empty(n, dtype=np.int64)
    for i, p in enumerate(paths):
        fr, ch, _, _ = probe(p)
        if ch != 1:
            raise AudioReadError(f"{p}: batch loader expects mono files, got {ch} channels")
        if fr == 0:
            raise AudioReadError(f"{p}: STREAMINFO has no sample count")
        lens[i] = fr
    offsets = np.zeros(n, dtype=np.int64)
    if n:
        offsets[1:] = np.cumsum(lens)[:-1]
    total = int(lens.sum())
    if out is None:
        out = np.empty(total, dtype=np.float32)
    if hasattr(out, "data_ptr"):
        if out.numel() < total:
            raise ValueError("read_batch: output buffer too small")
        ptr = out.data_ptr()
    else:
        if out.size < total:
            raise ValueError("read_batch: output buffer too small")
        ptr = out.ctypes.data
    cpaths = (c_str * n)(*[os.fsencode(str(p)) for p in paths])
    frames = np.zeros(n, dtype=np.int64)
    status = np.zeros(n, dtype=np.int32)
    code = lib().rdx_flac_read_batch(cpaths, n, ptr, offsets.ctypes.data_as(ctypes.POINTER(c_i64)),
                                     lens.ctypes.data_as(ctypes.POINTER(c_i64)),
                                     frames.ctypes.data_as(ctypes.POINTER(c_i64)),
                                     status.ctypes.data_as(ctypes.POINTER(c_int)), int(threads))
    if code != 0:
        bad = int(np.nonzero(status)[0][0])
        _check(int(status[bad]), str(paths[bad]))
    return out, offsets, lens
