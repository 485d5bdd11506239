"""radhip — MI355X-native (gfx950) engine for the Phase-6 audio-deepfake hot path.

Hand-written HIP kernels live in ../csrc (C ABI: ../../include/radhip.h, built into libradhip.so);
this package binds them (ctypes), wraps them as torch autograd ops, and provides the drop-in
modules (Mamba, SincConv front end, WavLM stream with LoRA) used by models/DualStreamSEMamba.py.
"""
import os

# ROCm 7 graph "packet capture" replays a captured hipMemsetAsync with a wrong fill value from the
# second replay on (tools/graph_memset_repro.py), which silently corrupts every torch op that zeroes
# scratch with a memset inside a HIP graph. The flag is read when the HIP runtime initialises, so it
# is set here, before any device call; GraphedMicroStep re-checks the behaviour before capturing.
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

from ._lib import lib  # noqa: F401,E402

__all__ = ["lib"]
