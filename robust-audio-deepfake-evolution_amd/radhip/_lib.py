"""ctypes binding of libradhip.so and libradhip_f16.so (C ABI declared in include/radhip.h).

Both are built in-tree from the same sources (csrc/Makefile -> radhip/libradhip.so with bf16 16-bit storage,
radhip/libradhip_f16.so with fp16 storage, -DRDX_F16) and export the same entry points; radhip.ops picks the
one matching a tensor's 16-bit dtype. There is no CPU fallback: if a library is missing or a call fails, a
RuntimeError is raised.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RADHIP_LIB", os.path.join(_HERE, "libradhip.so"))
LIB16_PATH = os.environ.get("RADHIP_LIB16", os.path.join(_HERE, "libradhip_f16.so"))

RDX_F32 = 0
RDX_BF16 = 1
EPI_BIAS, EPI_BIAS_GELU, EPI_GELU_BWD, EPI_RESID_DROP = 0, 1, 2, 3
EPI_F32, EPI_F32_GELU_SPLIT = 4, 5          # rdx_hgemm_x3

c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_f32 = ctypes.c_float
c_f64 = ctypes.c_double
c_vp = ctypes.c_void_p
c_fp = ctypes.c_void_p  # float* passed as raw address


class RawboostUtt(ctypes.Structure):
    """Mirror of rdx_rawboost_utt (include/radhip.h)."""

    _fields_ = [
        ("offset", c_i64),
        ("len", c_i64),
        ("algo", ctypes.c_int32),
        ("n_a", ctypes.c_int32),
        ("b", c_f64 * 6),
        ("a", c_f64 * 6),
        ("f", c_f64),
        ("beta", c_f64),
        ("snr_db", c_f64),
        ("seed", ctypes.c_uint64),
    ]


class ResampleJob(ctypes.Structure):
    """Mirror of rdx_resample_job (include/radhip.h)."""

    _fields_ = [
        ("in_offset", c_i64),
        ("in_len", c_i64),
        ("out_offset", c_i64),
        ("out_len", c_i64),
        ("orig_g", ctypes.c_int32),
        ("new_g", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("kern_offset", ctypes.c_int32),
    ]


# name -> (restype, argtypes)
SIGNATURES = {
    "rdx_version": (ctypes.c_char_p, []),
    "rdx_strerror": (ctypes.c_char_p, [c_int]),
    "rdx_sincconv_absmaxpool_fwd": (c_int, [c_vp, c_i64, c_i64, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp]),
    "rdx_sincconv_abspool1d_fwd": (c_int, [c_vp, c_i64, c_i64, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp]),
    "rdx_sincconv_absmaxpool_fwd_devmask": (c_int, [c_vp, c_i64, c_i64, c_vp, c_int, c_int, c_vp, c_int, c_vp,
                                                    c_vp]),
    "rdx_dwconv_bidir_fwd": (c_int, [c_int, c_vp, c_i64, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "rdx_dwconv_bidir_bwd_parts": (c_int, [c_int]),
    "rdx_dwconv_bidir_bwd": (c_int, [c_int, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64,
                                     c_int, c_int, c_int, c_int, c_int, c_vp]),
    "rdx_scan_ckpt_elems": (c_i64, [c_int, c_int, c_int, c_int, c_int]),
    "rdx_scan_nblk_d": (c_int, [c_int]),
    "rdx_selective_scan_fwd": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                       c_int, c_int, c_int, c_int, c_int, c_vp]),
    "rdx_selective_scan_bwd": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64,
                                       c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "rdx_bigate_fwd": (c_int, [c_int, c_vp, c_int, c_vp, c_i64, c_vp, c_vp, c_int, c_int, c_int, c_vp]),
    "rdx_bigate_bwd": (c_int, [c_int, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_vp]),
    "rdx_layer_wsum_fwd": (c_int, [c_int, c_int, ctypes.POINTER(c_vp), c_vp, c_vp, c_i64, c_vp]),
    "rdx_layer_wsum_nblk": (c_int, [c_i64]),
    "rdx_cast_f32_many": (c_int, [c_int, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), ctypes.POINTER(c_i64), c_vp]),
    "rdx_add_f32_many": (c_int, [c_int, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), ctypes.POINTER(c_i64), c_int,
                                 c_vp]),
    "rdx_layer_wsum_bwd": (c_int, [c_int, c_int, ctypes.POINTER(c_vp), c_vp, c_vp, ctypes.POINTER(c_vp), c_vp,
                                   c_i64, c_vp]),
    "rdx_rawboost_workspace_bytes": (c_i64, [c_int, c_i64]),
    "rdx_rawboost_batch": (c_int, [c_vp, c_vp, ctypes.POINTER(RawboostUtt), c_int, c_vp, c_vp, c_vp, c_vp]),
    "rdx_resample_kernel": (c_int, [c_int, c_int, c_int, c_f64, ctypes.POINTER(c_f32), c_int,
                                    ctypes.POINTER(c_int), ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "rdx_resample_batch": (c_int, [c_vp, c_vp, c_vp, ctypes.POINTER(ResampleJob), c_int, c_vp]),
    "rdx_pad_mixup": (c_int, [c_vp, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64), ctypes.POINTER(c_i64), c_int,
                              c_i64, ctypes.POINTER(c_int), c_f32, c_vp, c_vp]),
    "rdx_bnselu_fwd": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp]),
    "rdx_bnselu_bwd": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp]),
    "rdx_res_tail_fwd": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp]),
    "rdx_res_tail_bwd": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp]),
    "rdx_row_ln_fwd": (c_int, [c_int, c_vp, c_vp, c_vp, c_f32, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_vp]),
    "rdx_row_ln_bwd": (c_int, [c_int, c_vp, c_int] + [c_vp] * 7 + [c_i64, c_int, c_vp]),
    "rdx_sincnet_b0_fwd": (c_int, [c_vp] * 7 + [c_int, c_int, c_int, c_int, c_vp]),
    "rdx_sincnet_b0_nblk": (c_int, [c_i64]),
    "rdx_sincnet_b0_bwd": (c_int, [c_vp] * 7 + [c_int, c_int, c_int, c_int, c_vp]),
    "rdx_b0x_fwd": (c_int, [c_vp] * 8 + [c_int, c_int, c_int, c_vp]),
    "rdx_b0x_bwd_nblk": (c_int, [c_int, c_int]),
    "rdx_b0x_bwd": (c_int, [c_vp] * 9 + [c_int, c_int, c_int, c_vp]),
    "rdx_posconv_fwd": (c_int, [c_vp] * 5 + [c_int, c_int, c_vp]),
    "rdx_posconv_bwd": (c_int, [c_vp] * 4 + [c_int, c_int, c_vp]),
    "rdx_gemm_bf16": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_int, c_vp, c_i64,
                              c_vp, c_i64, c_vp, c_int, c_f32, c_vp]),
    "rdx_wgemm_bf16": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_int, c_vp, c_i64,
                               c_vp, c_i64, c_int, c_vp]),
    "rdx_wgemm_pick": (c_int, [c_int, c_int, c_int]),
    "rdx_wgemm_bf16_ex": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_int, c_vp,
                                  c_i64, c_vp, c_i64, c_int, c_int, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "rdx_wgemm_ws_bytes": (c_i64, [c_int, c_int, c_int, c_int]),
    "rdx_wgrad_chunk": (c_int, [c_int, c_int, c_int]),
    "rdx_wgrad_ws_floats": (c_i64, [c_int, c_int, c_int]),
    "rdx_wgrad_acc": (c_int, [c_vp, c_i64, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "rdx_wgrad_many_ws_floats": (c_i64, [c_int, c_vp, c_vp, c_vp, c_vp]),
    "rdx_wgrad_acc_many": (c_int, [c_int] + [c_vp] * 10 + [c_vp, c_i64, c_vp]),
    "rdx_adamw_many_max": (c_int, []),
    "rdx_adamw_many": (c_int, [c_int] + [c_vp] * 6 + [c_f64] * 5 + [c_vp, c_vp, c_vp]),
    "rdx_wgemm_counters": (c_i64, [c_int, c_int, c_int]),
    "rdx_sincconv_absmaxpool_f16mfma": (c_int, [c_vp, c_i64, c_i64, c_vp, c_int, c_int, c_int, c_int, c_vp, c_int,
                                                c_vp, c_vp]),
    "rdx_scan2_chunks": (c_int, [c_int]),
    "rdx_scan2_rec_elems": (c_i64, [c_int, c_int, c_int, c_int, c_int]),
    "rdx_scan2_fwd": (c_int, [c_int] + [c_vp] * 5 + [c_i64] + [c_vp] * 6 + [c_int] * 5 + [c_vp]),
    "rdx_scan2_bwd": (c_int, [c_int] + [c_vp] * 5 + [c_i64] + [c_vp] * 5 + [c_i64] + [c_vp] * 6 + [c_i64, c_vp]
                      + [c_int] * 5 + [c_vp]),
    "rdx_pgemm_bf16": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_int, c_vp, c_i64,
                               c_vp, c_i64, c_int, c_int, c_vp]),
    "rdx_pgemm_prof": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_int, c_int, c_vp,
                               c_vp]),
    "rdx_hgemm": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_int, c_vp, c_i64, c_vp,
                          c_i64, c_int, c_int, c_int, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "rdx_hgemm_ws_bytes": (c_i64, [c_int, c_int, c_int, c_int]),
    "rdx_colsum_many": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rdx_lgemm": (c_int, [c_vp, c_i64, c_int, c_vp, c_i64, c_vp, c_i64, c_int, c_int, c_int, c_int, c_vp, c_int,
                          c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "rdx_hgemm_counters": (c_i64, [c_int, c_int, c_int]),
    "rdx_hgemm_sk_ws_bytes": (c_i64, [c_int, c_int, c_int, c_int]),
    "rdx_gemm_bf16_strided": (c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_int, c_int,
                                      c_vp, c_vp]),
    "rdx_fe_conv0": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_int, c_int, c_vp, c_vp]),
    "rdx_fe_ln_gelu": (c_int, [c_vp, c_i64, c_vp, c_vp, c_f32, c_vp, c_vp]),
    "rdx_sconv_dgrad_bnselu": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                                       c_int, c_vp]),
    "rdx_sconv_fwd": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "rdx_sconv_fwd_res": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "rdx_sconv_wgrad_nblk": (c_int, [c_int, c_int, c_int]),
    "rdx_sconv_wgrad": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp]),
    "rdx_sconv_wprep_many": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "rdx_se_fwd": (c_int, [c_vp] * 7 + [c_int] * 4 + [c_vp]),
    "rdx_se_bwd_part_floats": (c_i64, [c_int, c_int, c_int]),
    "rdx_se_bwd": (c_int, [c_vp] * 11 + [c_int] * 4 + [c_vp]),
    "rdx_attn_pool_fwd": (c_int, [c_vp] * 5 + [c_int] * 3 + [c_vp]),
    "rdx_attn_pool_bwd": (c_int, [c_vp] * 8 + [c_int] * 3 + [c_vp]),
    "rdx_upcat_fwd": (c_int, [c_vp] * 3 + [c_int] * 4 + [c_vp]),
    "rdx_upcat_bwd": (c_int, [c_vp] * 2 + [c_int] * 4 + [c_vp]),
    "rdx_attn_fwd": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_int, c_f32, c_f32, c_vp, c_i64,
                             c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp]),
    "rdx_attn_keep_mask_words": (c_i64, [c_int, c_int, c_int]),
    "rdx_attn_bwd": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_int, c_f32, c_f32, c_vp, c_i64,
                             c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_int, c_int, c_int, c_int, c_vp]),
    "rdx_attn_bwd_fused": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_f32, c_f32, c_vp, c_i64,
                                   c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_int, c_int, c_int, c_int,
                                   c_vp]),
    "rdx_attn_bwd_split_ws": (c_i64, [c_int, c_int]),
    "rdx_attn_bwd_fused_split": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_f32, c_f32, c_vp,
                                         c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64,
                                         c_vp, c_i64, c_int, c_int, c_int, c_int, c_vp]),
    "rdx_attn_dropout_mask": (c_int, [c_vp, c_int, c_f32, c_vp, c_i64, c_int, c_vp]),
    "rdx_dropout_mask": (c_int, [c_vp, c_int, c_f32, c_vp, c_i64, c_vp]),
    "rdx_wl_ln1_fwd": (c_int, [c_vp] * 3 + [c_f32] + [c_vp] * 5 + [c_int, c_vp,
                       c_int, c_int, c_f32, c_vp, c_i64] + [c_vp] * 3
                       + [c_i64, c_int, c_vp]),
    "rdx_wl_add_ln_fwd": (c_int, [c_vp, c_vp, c_vp, c_int, c_f32, c_vp, c_vp,
                          c_vp, c_f32, c_vp, c_vp, c_vp, c_i64, c_int,
                          c_vp]),
    "rdx_wl_residual": (c_int, [c_vp, c_vp, c_vp, c_int, c_f32, c_vp, c_i64,
                        c_vp]),
    "rdx_wl_dropout_bwd": (c_int, [c_vp, c_vp, c_int, c_f32, c_vp, c_i64,
                           c_vp]),
    "rdx_wl_gelu": (c_int, [c_int, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "rdx_wl_ln_bwd": (c_int, [c_vp, c_i64] + [c_vp] * 7 + [c_int, c_f32, c_vp,
                      c_i64, c_int, c_vp]),
    "rdx_wl_ln1_bwd": (c_int, [c_vp, c_i64] + [c_vp] * 11 + [c_int, c_vp, c_int,
                       c_int, c_f32, c_vp, c_vp, c_vp, c_i64, c_int, c_vp]),
    "rdx_wl_ln1_bwd_ex": (c_int, [c_vp, c_i64] + [c_vp] * 11 + [c_int, c_vp, c_int, c_int, c_f32] + [c_vp] * 3
                          + [c_vp, c_vp, c_int, c_f32, c_vp, c_i64, c_int, c_vp]),
    "rdx_wl_res_ln1_fwd": (c_int, [c_vp, c_vp, c_int, c_f32, c_vp, c_vp, c_vp, c_f32] + [c_vp] * 5
                           + [c_int, c_vp, c_int, c_int, c_f32, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_int, c_vp]),
    "rdx_wl_lora_grad": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_int, c_int, c_f32, c_f32,
                                 c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp]),
    "rdx_wl_lora_pack": (c_int, [c_int, c_vp, c_vp, c_vp, c_i64, c_int,
                         c_f32, c_int, c_vp]),
    "rdx_timestamp_acc": (c_int, [c_vp, c_int, c_vp]),
    "rdx_wallclock_khz": (c_int, [c_int]),
    "rdx_focal_mixup_fwd": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_f32, c_f32, c_int,
                                    c_f32, c_vp, c_vp, c_vp]),
    "rdx_focal_mixup_bwd": (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_vp]),
    "rdx_hgemm_x3": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_i64, c_int, c_int, c_int,
                             c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "rdx_hgemm_batched": (c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_int, c_int,
                                  c_vp, c_int, c_int, c_vp]),
    "rdx_x3_split": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_i64, c_vp]),
    "rdx_x3_ln_split": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                c_i64, c_int, c_vp]),
    "rdx_x3_attn_fwd": (c_int, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_f32, c_vp, c_vp, c_i64, c_int, c_int, c_int,
                                c_int, c_vp]),
    "rdx_x3_posconv_fwd": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp]),
    "rdx_x3_fe_conv0": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_int, c_int, c_vp, c_vp, c_vp]),
    "rdx_x3_fe_ln_gelu": (c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_vp]),
    "rdx_fgm_attack": (c_int, [c_int, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), ctypes.POINTER(c_vp),
                               ctypes.POINTER(c_i64), c_f32, c_vp, c_vp]),
}

_lock = threading.Lock()
_lib = None
_lib16 = None


def header_symbols():
    """Function names declared in include/radhip.h (used by the export test)."""
    import re
    hdr = os.path.join(_HERE, "..", "..", "include", "radhip.h")
    text = open(hdr).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int64_t|int)\s+(rdx_\w+)\s*\(", text, re.M)))


def _load(path, mode):
    if not os.path.exists(path):
        raise RuntimeError(
            f"{os.path.basename(path)} not found at {path}: build it with `make -C csrc` "
            "(or __graft_entry__.build()); there is no CPU fallback for the HIP path")
    L = ctypes.CDLL(path, mode=mode)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def lib():
    """Load libradhip.so (bf16 storage) once; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            _lib = _load(LIB_PATH, ctypes.RTLD_GLOBAL)
    return _lib


def lib16():
    """Load libradhip_f16.so (the same entry points over fp16 storage) once, with its symbols kept local (both
    libraries are linked -Bsymbolic); raise loudly if it is absent."""
    global _lib16
    if _lib16 is not None:
        return _lib16
    lib()
    with _lock:
        if _lib16 is None:
            _lib16 = _load(LIB16_PATH, ctypes.RTLD_LOCAL)
    return _lib16


def check(code, what=""):
    if code != 0:
        msg = lib().rdx_strerror(int(code)).decode()
        raise RuntimeError(f"radhip {what} failed: code {code} ({msg})")


def ptr_array(ptrs):
    arr = (c_vp * len(ptrs))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr
