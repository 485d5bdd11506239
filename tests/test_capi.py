"""libradhip.so (and libradhip_f16.so) load, export every symbol include/radhip.h declares, and its host-only entry
points behave (no GPU needed: argument checks return before any HIP call)."""
import ctypes
import os

import numpy as np
import pytest

from radhip import _lib


def test_library_loads_and_exports_header_symbols():
    L = _lib.lib()
    declared = _lib.header_symbols()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), f"libradhip.so does not export {name}"
        assert name in _lib.SIGNATURES, f"no ctypes signature for {name}"
    assert L.rdx_version().decode().startswith("radhip")


def test_f16_library_exports_the_same_entry_points():
    """libradhip_f16.so: the same sources built with -DRDX_F16 (fp16 16-bit storage), the same C ABI, loaded
    beside libradhip.so with its own bindings (-Bsymbolic, RTLD_LOCAL)."""
    L, L16 = _lib.lib(), _lib.lib16()
    for name in _lib.header_symbols():
        assert hasattr(L16, name), f"libradhip_f16.so does not export {name}"
    assert L16._handle != L._handle
    # a host-only entry point answers from the f16 library itself
    assert L16.rdx_strerror(-2) == b"unsupported shape"
    assert L16.rdx_scan_nblk_d(288) == L.rdx_scan_nblk_d(288)


def test_ops_pick_the_library_by_storage_dtype():
    import torch
    from radhip import ops
    assert ops._L(torch.bfloat16) is _lib.lib() and ops._L(torch.float32) is _lib.lib()
    assert ops._L(torch.float16) is _lib.lib16() and ops._L(torch.float32, torch.float16) is _lib.lib16()
    with pytest.raises(TypeError):
        ops._L(torch.bfloat16, torch.float16)
    assert ops._dtype_code(torch.empty(0, dtype=torch.float16)) == ops._dtype_code(torch.empty(0, dtype=torch.bfloat16))


def test_error_codes():
    L = _lib.lib()
    assert L.rdx_strerror(0) == b"ok"
    assert L.rdx_strerror(-1) == b"invalid argument"
    assert L.rdx_strerror(-2) == b"unsupported shape"
    # null pointers are rejected before any device work
    assert L.rdx_sincconv_absmaxpool_fwd(None, 1, 64600, None, 70, 129, 0, 0, None, None) == -1
    assert L.rdx_selective_scan_fwd(0, None, None, None, None, None, 41, None, None, None, None, 1, 10, 8, 16, 2,
                                    None) == -1
    assert L.rdx_fgm_attack(0, None, None, None, None, 0.5, None, None) == -1


def test_workspace_queries():
    L = _lib.lib()
    assert L.rdx_scan_nblk_d(288) == 24
    nck = (201 + 15) // 16
    assert L.rdx_scan_ckpt_elems(8, 201, 288, 16, 2) == 2 * 8 * (nck - 1) * 288 * 16
    assert L.rdx_layer_wsum_nblk(8 * 201 * 1024) >= 1
    assert L.rdx_rawboost_workspace_bytes(8, 8 * 64000) > 0


@pytest.mark.parametrize("orig,new", [(16000, 8000), (16000, 6000), (16000, 4000), (8000, 16000), (6000, 16000),
                                      (4000, 16000)])
def test_resample_kernel_matches_oracle(orig, new):
    from oracle.resample import sinc_kernel
    from radhip.ops import resample_kernel
    k, width, og, ng = resample_kernel(orig, new)
    kr, wr, ogr, ngr = sinc_kernel(orig, new)
    assert (width, og, ng) == (wr, ogr, ngr)
    np.testing.assert_allclose(k.numpy(), kr, rtol=1e-6, atol=1e-7)


def test_bench_knows_the_bound_of_every_timed_kernel():
    """bench.py's roofline prices the dominant kernel by KERNEL_BOUND; a kernel timed in radhip/ops.py but absent
    there would be priced as HBM-bound bytes (round 3 found wgemm's FLOPs read as bytes)."""
    import ast
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, "robust-audio-deepfake-evolution_amd", "radhip", "ops.py")).read()
    names = set(re.findall(r'_timed\("([a-z0-9_]+)"', src)) | set(re.findall(r'name="([a-z0-9_]*gemm)"', src))
    tree = ast.parse(open(os.path.join(root, "bench.py")).read())
    bound = next(ast.literal_eval(n.value) for n in tree.body
                 if isinstance(n, ast.Assign) and getattr(n.targets[0], "id", "") == "KERNEL_BOUND")
    assert names and names <= set(bound), sorted(names - set(bound))
