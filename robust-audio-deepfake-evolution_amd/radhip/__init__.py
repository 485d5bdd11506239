"""radhip — MI355X-native (gfx950) engine for the Phase-6 audio-deepfake hot path.

Hand-written HIP kernels live in ../csrc (C ABI: ../../include/radhip.h, built into libradhip.so);
this package binds them (ctypes), wraps them as torch autograd ops, and provides the drop-in
modules (Mamba, SincConv front end, WavLM stream with LoRA) used by models/DualStreamSEMamba.py.
"""
from ._lib import lib  # noqa: F401

__all__ = ["lib"]
