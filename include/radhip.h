/*
 * radhip.h — C ABI of libradhip.so (and libradhip_f16.so), the hand-written HIP (gfx950 / MI355X) kernels of the
 * Phase-6 audio-deepfake hot path (lux-liang/Robust-Audio-Deepfake-Evolution).
 *
 * Conventions ("C-ABI conventions"):
 *   - extern "C", plain pointers and sizes, no torch types.
 *   - Every entry point returns int: 0 = ok, > 0 = hipError_t of the failing launch,
 *     < 0 = argument error (RDX_E*). rdx_strerror() names a code.
 *   - All device pointers are caller-owned; no entry point allocates device memory
 *     (workspace sizes are queried with the *_workspace / *_elems helpers).
 *   - `stream` is a hipStream_t (0 = legacy default stream). Nothing synchronises the host,
 *     so every launch function is graph-capturable.
 *   - Tensors are row-major and contiguous unless a leading dimension (ld*) is given.
 *   - dtype selects the storage type of the "activation" operands (RDX_F32 or RDX_BF16 = the library's
 *     16-bit type); arithmetic is fp32 (fp64 for the RawBoost filters and reductions).
 *   - Two libraries export this same ABI from the same sources: libradhip.so stores 16-bit operands
 *     as bf16, libradhip_f16.so (built with -DRDX_F16) as IEEE fp16 — the reference trains under
 *     torch.cuda.amp.autocast(), i.e. fp16 (src/main.py:28,1049). In libradhip_f16.so every "bf16"
 *     in a comment or an entry-point name (rdx_gemm_bf16, rdx_wgemm_bf16_ex, ...) reads "fp16"; the
 *     MFMA forms (v_mfma_f32_*_f16 vs *_bf16) take the same cycles. Both are linked -Bsymbolic so one
 *     process can load both (radhip/_lib.py: lib() and lib16()).
 *   - No global state: thread-compatible, one process per GPU.
 *
 * Each function names the reference interface it replaces (file:line into the reference).
 */
#ifndef RADHIP_H
#define RADHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RDX_OK 0
#define RDX_EINVAL (-1)        /* bad shape / pointer / argument */
#define RDX_EUNSUPPORTED (-2)  /* shape outside what the kernel is built for */

typedef enum { RDX_F32 = 0, RDX_BF16 = 1 } rdx_dtype;

const char* rdx_version(void);
const char* rdx_strerror(int code);

/* ------------------------------------------------------------------------------------------
 * SincConv front end.
 * Replaces CONV.__init__ filter bank (src/models/DualStreamSEMamba.py:95-117), CONV.forward
 * (:119-138) and the first step of SincNetEncoder.forward, `max_pool2d(abs(conv), (3,3))` (:251-253).
 *   x       [batch, len] fp32 waveform
 *   filters [channels, ksize] fp32 band-pass bank (unmasked)
 *   channels in [mask_lo, mask_hi) are treated as zeroed filters (the Freq_aug band mask, :121-125)
 *   out     [batch, channels/3, (len-ksize+1)/3] fp32  = max over 3x3 windows of |conv|
 * ------------------------------------------------------------------------------------------ */
int rdx_sincconv_absmaxpool_fwd(const float* x, int64_t batch, int64_t len, const float* filters,
                                int channels, int ksize, int mask_lo, int mask_hi, float* out,
                                void* stream);
/* Same, with the band mask [lo, hi) read from device memory at execution time, so a captured HIP
 * graph can be replayed with a fresh mask per call: utterance b uses mask_dev[b*mask_stride + {0,1}]
 * (mask_stride 0: one int32[2] mask for the batch, as one CONV.forward call draws; 2: one mask per
 * utterance, for several forward calls batched into one launch). */
int rdx_sincconv_absmaxpool_fwd_devmask(const float* x, int64_t batch, int64_t len,
                                        const float* filters, int channels, int ksize,
                                        const int32_t* mask_dev, int mask_stride, float* out,
                                        void* stream);
/* f16 MFMA form for the autocast paths (the reference's autocast runs this F.conv1d in fp16, src/main.py:1049):
 * x and the bank rounded to fp16, fp32 accumulation, fp32 pooled output. mask_dev null: the band mask
 * [mask_lo, mask_hi); else per-batch / per-utterance as rdx_sincconv_absmaxpool_fwd_devmask (mask_stride 0 / 2).
 * ksize <= 160, channels <= 80 (csrc/sincconv.hip sincconv_mfma_kernel). */
int rdx_sincconv_absmaxpool_f16mfma(const float* x, int64_t batch, int64_t len, const float* filters, int channels,
                                    int ksize, int mask_lo, int mask_hi, const int32_t* mask_dev, int mask_stride,
                                    float* out, void* stream);
/* RawNet2 front end (legacy plugin, models/RawNet2Spoof.py:77-103 SincConv.forward and :244-245
 * `F.max_pool1d(torch.abs(x), 3)`): the same fused sinc conv + |.|, pooled over time only.
 *   out [batch, channels, (len-ksize+1)/3] fp32 = max over 3 consecutive conv times of |conv| */
int rdx_sincconv_abspool1d_fwd(const float* x, int64_t batch, int64_t len, const float* filters,
                               int channels, int ksize, int mask_lo, int mask_hi, float* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * Bidirectional Mamba (replaces mamba_ssm Mamba.forward -> mamba_inner_fn, called twice per
 * PN_BiMambas_Encoder.forward with a flip, src/models/DualStreamSEMamba.py:467-486; semantics of
 * the reference-owned MambaBlock, src/models/modules/mamba_block.py:41-122).
 * Direction 0 scans t = 0..L-1; direction 1 scans the flipped sequence, with every tensor kept at
 * ORIGINAL positions (no flip is ever materialised). `dirs` = 1 (plain Mamba) or 2 (Bi-Mamba).
 * ------------------------------------------------------------------------------------------ */

/* Depthwise causal conv (kernel K, bias) + SiLU, for both scan directions.
 *   x  [B, L, D] with row stride ldx (the x half of in_proj's xz [B, L, 2D])
 *   w  [D, K] fp32, bias [D] fp32
 *   u  [dirs, B, L, D]   u[0] causal, u[1] anti-causal (= flip(conv(flip(x)))) */
int rdx_dwconv_bidir_fwd(int dtype, const void* x, int64_t ldx, const float* w, const float* bias,
                         void* u, int B, int L, int D, int K, int dirs, void* stream);
/* Backward. du [dirs, B, L, D]; writes dx (row stride lddx, overwritten), and partial weight / bias
 * gradients per (time chunk, batch): dw_part [P, D, K], db_part [P, D] with P = rdx_dwconv_bidir_bwd_parts(L)
 * * B (fp32; caller sums dim 0), rows of ld_part floats (0: dense; D * K + D packs both into one [P][D * K + D]
 * buffer, db_part = dw_part + D * K, summed with one reduction). */
int rdx_dwconv_bidir_bwd_parts(int L);
int rdx_dwconv_bidir_bwd(int dtype, const void* x, int64_t ldx, const float* w, const float* bias,
                         const void* du, void* dx, int64_t lddx, float* dw_part, float* db_part, int64_t ld_part,
                         int B, int L, int D, int K, int dirs, void* stream);

/* Selective scan, replaces selective_scan_cuda.fwd (mamba_ssm) / MambaBlock.ssm_step
 * (mamba_block.py:65-122):  dt = softplus(delta + dt_bias);  h = exp(dt*A) h + dt*B*u;
 * y = C.h + Dp*u, A = -exp(A_log).  N (d_state) must be 16; L <= 640.
 *   u, delta  [dirs, B, L, D]
 *   Bm, Cm    [dirs, B, L, N] with row stride ldbc (views into x_proj's [dirs, B, L, R+2N])
 *   A_log [D, N], Dp [D], dt_bias [D] fp32
 *   y     [dirs, B, L, D] fp32 out
 *   ckpt  [dirs, B, nck-1, D, N] fp32 out (state checkpoints for bwd; see rdx_scan_ckpt_elems) */
int64_t rdx_scan_ckpt_elems(int B, int L, int D, int N, int dirs);
int rdx_scan_nblk_d(int D);
int rdx_selective_scan_fwd(int dtype, const void* u, const void* delta, const float* A_log,
                           const void* Bm, const void* Cm, int64_t ldbc, const float* Dp,
                           const float* dt_bias, float* y, float* ckpt, int B, int L, int D, int N,
                           int dirs, void* stream);
/* Backward. dy [dirs, B, L, D] fp32 with direction stride dy_dir_stride (0 = both directions see
 * the same dy, the Bi-Mamba case). Outputs:
 *   du, ddelta [dirs, B, L, D] (dtype)           — overwritten
 *   dBC        [dirs, B, L, 2N] fp32 — dB|dC, ACCUMULATED with atomics: the caller zeroes it
 *   dA_part    [dirs*B, D, N] fp32 (d/dA_log)    — caller sums dim 0
 *   dD_part, dbias_part [dirs*B, D] fp32         — caller sums dim 0
 * Needs dynamic LDS of 4*L*24 + L*12*es + L*32*es + 30 KB bytes (es = dtype size) <= 160 KB:
 * L <= 640 for bf16, L <= 460 for f32; RDX_EUNSUPPORTED beyond. */
int rdx_selective_scan_bwd(int dtype, const void* u, const void* delta, const float* A_log,
                           const void* Bm, const void* Cm, int64_t ldbc, const float* Dp,
                           const float* dt_bias, const float* ckpt, const float* dy,
                           int64_t dy_dir_stride, void* du, void* ddelta, float* dBC,
                           float* dA_part, float* dD_part, float* dbias_part, int B, int L, int D,
                           int N, int dirs, void* stream);

/* Gate shared by both directions: g = (sum_dir y[dir]) * silu(z);  ysum = sum_dir y[dir].
 *   y [dirs, B, L, D] fp32, z [B, L, D] with row stride ldz, g [B, L, D] (dtype), ysum fp32. */
int rdx_bigate_fwd(int dtype, const float* y, int dirs, const void* z, int64_t ldz, void* g,
                   float* ysum, int B, int L, int D, void* stream);
/* dy = dg * silu(z) (fp32, [B, L, D]);  dz = dg * ysum * silu'(z) (dtype, row stride lddz). */
int rdx_bigate_bwd(int dtype, const void* dg, const void* z, int64_t ldz, const float* ysum,
                   float* dy, void* dz, int64_t lddz, int B, int L, int D, void* stream);

/* ------------------------------------------------------------------------------------------
 * LayerNorm over the last dimension, C <= 1024 (the detector head's norms: PN-BiMamba norm1/norm2, the
 * fusion's ln_wavlm / ln_sinc / norm, norm_f; src/models/DualStreamSEMamba.py:445-486,537-637,700-770).
 * Forward: x [M, C] (dtype_x) -> y (dtype_y; bf16 when the consumer is a bf16 linear), mean / rstd [M] fp32
 * (biased variance, as torch). Backward: dx (dtype_x) = rstd (g - mean(g) - xhat mean(g xhat)), g = dy gamma;
 * dgamma += sum dy xhat, dbeta += sum dy (fp32, ACCUMULATED into the caller's buffers). C > 1024:
 * RDX_EUNSUPPORTED.
 * ------------------------------------------------------------------------------------------ */
int rdx_row_ln_fwd(int dtype_x, const void* x, const float* gamma, const float* beta, float eps, int dtype_y, void* y,
                   float* mean, float* rstd, int64_t M, int C, void* stream);
int rdx_row_ln_bwd(int dtype_dy, const void* dy, int dtype_x, const void* x, const float* mean, const float* rstd,
                   const float* gamma, void* dx, float* dgamma, float* dbeta, int64_t M, int C, void* stream);

/* ------------------------------------------------------------------------------------------
 * WavLM layer-weighted sum, replaces WavLMFrontend.forward's stack + softmax-weighted sum
 * (src/models/DualStreamSEMamba.py:427-437).  hs: host array of `nl` device pointers, each
 * [n] elements; w: device [nl] fp32 raw layer weights (softmax taken in-kernel). nl <= 64.
 * ------------------------------------------------------------------------------------------ */
int rdx_layer_wsum_fwd(int dtype, int nl, const void* const* hs, const float* w, void* out,
                       int64_t n, void* stream);
/* Backward: dhs[l] = softmax(w)_l * g (dtype, overwritten; dhs[l] == NULL: not written, the consumer
 * applies softmax(w)_l * g itself, e.g. rdx_wl_ln1_bwd's state gradient), dot_part [nblk, nl] fp32 partial
 * sums of <g, h_l>; nblk = rdx_layer_wsum_nblk(n). dw follows on the host side from the dots. */
int rdx_layer_wsum_nblk(int64_t n);
int rdx_layer_wsum_bwd(int dtype, int nl, const void* const* hs, const float* w, const void* g,
                       void* const* dhs, float* dot_part, int64_t n, void* stream);
/* fp32 -> the library's 16-bit type (bf16 / fp16) of n <= 64 tensors in one launch: dst[k][i] = src[k][i] for
 * i < numel[k] (round to nearest even). The accumulation window casts the detector head's fp32 linear weights to the
 * autocast dtype once per window with it (radhip/window.py; autocast's own cast cache: one launch per tensor). */
int rdx_cast_f32_many(int n, const float* const* src, void* const* dst, const int64_t* numel, void* stream);
/* dst[k][i] += src[k][i] (copy = 0) or dst[k][i] = src[k][i] (copy = 1), i < numel[k], over n <= 64 fp32 tensors in
 * one launch (4096 elements per workgroup). Replaces torch._foreach_add_ / _foreach_copy_ in the window's gradient
 * hand-over (radhip/window.py; the reference accumulates each .grad by autograd, src/main.py:1077-1108). */
int rdx_add_f32_many(int n, void* const* dst, const float* const* src, const int64_t* numel, int copy, void* stream);

/* ------------------------------------------------------------------------------------------
 * RawBoost, batched over utterances with host-drawn parameters. Replaces RawBoost.process and
 * its three algorithms (src/rawboost.py:15-95) as called per utterance by
 * Dataset_ASVspoof2019_train.__getitem__ (src/data_utils.py:169-174).
 * One record per utterance; arithmetic in fp64.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  int64_t offset;   /* first sample of this utterance in x / out (flat buffers)            */
  int64_t len;      /* samples                                                             */
  int32_t algo;     /* 0 copy, 1 LnL convolutive, 2 ISD impulsive, 3 SSI stationary, 4 = 1+2 */
  int32_t n_a;      /* IIR order (1..5) for LnL                                            */
  double b[6];      /* FIR numerator (product of five (1 + c z^-1))                        */
  double a[6];      /* IIR denominator, a[0] = 1                                           */
  double f;         /* non-linearity coefficient  y += f*y^2                               */
  double beta;      /* ISD: impulse probability 1/beta                                     */
  double snr_db;    /* SSI: target SNR (dB)                                                */
  uint64_t seed;    /* Philox key for the per-sample noise of ISD / SSI                    */
} rdx_rawboost_utt;

/* Workspace: fp64 partial sums [nutt][ceil(total_samples/4096)][2]. */
int64_t rdx_rawboost_workspace_bytes(int nutt, int64_t total_samples);
/* noise_isd / noise_ssi: optional device fp64 arrays laid out like x that replace the in-kernel
 * Philox draws (ISD: the product noise*mask; SSI: the Gaussian noise). Pass NULL in production;
 * tests pass the reference's numpy draws to get exact parity. */
int rdx_rawboost_batch(const float* x, float* out, const rdx_rawboost_utt* utts, int nutt,
                       void* workspace, const double* noise_isd, const double* noise_ssi,
                       void* stream);

/* ------------------------------------------------------------------------------------------
 * "Poor man's codec": windowed-sinc polyphase resampling, restating
 * torchaudio.transforms.Resample (sinc_interp_hann, lowpass width 6, rolloff 0.99) as called by
 * apply_codec_aug (src/data_utils.py:31-59).
 * rdx_resample_kernel fills the [new_g, 2*width + orig_g] fp32 kernel on the HOST
 * (orig_g/new_g = orig/new divided by their gcd); returns width via *width_out.
 * rdx_resample_batch: one launch for all records; out_len = ceil(new_g * len / orig_g).
 * ------------------------------------------------------------------------------------------ */
int rdx_resample_kernel(int orig_freq, int new_freq, int lowpass_width, double rolloff,
                        float* host_kernel, int host_kernel_cap, int* width_out, int* orig_g_out,
                        int* new_g_out);
typedef struct {
  int64_t in_offset, in_len, out_offset, out_len;
  int32_t orig_g, new_g, width, kern_offset; /* kern_offset into the packed kernel buffer */
} rdx_resample_job;
int rdx_resample_batch(const float* in, float* out, const float* kernels,
                       const rdx_resample_job* jobs, int njobs, void* stream);

/* ------------------------------------------------------------------------------------------
 * pad_random / pad + mixup gather: builds the model input batch [nutt, max_len] from
 * variable-length signals. Replaces pad_random (src/data_utils.py:116-127) / pad (:107-113) and
 * the mixup blend of train_epoch (src/main.py:1038-1042):
 *   base[b][i] = sig_b[ start_b + i ]          if len_b >= max_len (crop at start_b)
 *              = sig_b[ i mod len_b ]          otherwise (tile)
 *   out[b] = lam * base[b] + (1 - lam) * base[perm[b]]   (perm = NULL -> out = base)
 * offsets/lens/starts are host arrays of nutt entries; nutt <= 64.
 * ------------------------------------------------------------------------------------------ */
int rdx_pad_mixup(const float* sig, const int64_t* offsets, const int64_t* lens,
                  const int64_t* starts, int nutt, int64_t max_len, const int* perm, float lam,
                  float* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * FGM attack, replaces FGM.attack (src/main.py:85-94): for each tensor i,
 *   backup_i = p_i;  if (||g_i|| != 0 && !isnan(||g_i||))  p_i += eps * g_i / ||g_i||
 * Host arrays of ntensors (<= 32) device pointers, fp32. workspace: fp64 [ntensors * 256].
 * ------------------------------------------------------------------------------------------ */
int rdx_fgm_attack(int ntensors, float* const* params, const float* const* grads,
                   float* const* backup, const int64_t* numels, float eps, double* workspace,
                   void* stream);

/* ------------------------------------------------------------------------------------------
 * Mixup focal loss, replaces criterion(out, y_a) * lam + criterion(out, y_b) * (1 - lam), divided by the
 * accumulation steps (src/main.py:297-305 kornia FocalLoss, :1040-1050 mixup + accumulation):
 *   loss = scale * sum_b [ lam_b f(z_b, ya_b) + (1 - lam_b) f(z_b, yb_b) ],  lam_b = lam[b / rows_per_lam]
 *   f(z, y) = -a_y (1 - p_y)^gamma log p_y,  p = softmax(z);  mode 0: a_y = y == 0 ? 1 - alpha : alpha
 *   (kornia >= 0.7 'per_class'), mode 1: a_y = alpha; alpha < 0: a = 1.
 * logits [B, C] (row stride ld, bf16 when logits_bf16 else fp32), C <= 16; yb NULL: no mixup (lam ignored
 * for the weight of ya when lam is NULL, = 1). One workgroup writes loss (fp32 scalar) and dlogits (fp32
 * [B, C], d loss / d logits). rdx_focal_mixup_bwd: out = grad[0] * dlogits in the logits' dtype (n = B*C).
 * ------------------------------------------------------------------------------------------ */
int rdx_focal_mixup_fwd(const void* logits, int logits_bf16, int ld, int B, int C, const int64_t* ya,
                        const int64_t* yb, const float* lam, int rows_per_lam, float alpha, float gamma,
                        int mode, float scale, float* loss, float* dlogits, void* stream);
int rdx_focal_mixup_bwd(const float* grad, const float* dlogits, void* out, int out_bf16, int n, void* stream);

/* ---- SincNet residual stack, NHWC fused epilogues (Residual_block.forward,
 * src/models/DualStreamSEMamba.py:182-200, with freeze_bn: src/main.py:44-51,1016-1018) -----------
 * Activations are [npix, C] row-major (channels_last), C % 8 == 0, C <= 512, 256 % (C/8) == 0.
 * rdx_bnselu_fwd: y = selu(((c + conv_bias) - mean) * invstd * weight + bias)  (conv1 bias folded in,
 *   frozen BN statistics). rdx_bnselu_bwd: dc = dy * selu'(u) * invstd * weight and ACCUMULATES into
 *   sums[3][C] (caller zeroes): sum(dc) = d conv_bias, sum(dy selu' xhat) = d weight, sum(dy selu') = d bias.
 * rdx_res_tail_fwd: y[r, wo, :] = max_{k<3} (a + identity + bias)[r, 3wo + k, :]  (MaxPool2d((1,3)) of
 *   conv2 + identity; rows = N*H, W input columns, Wo = W/3); argmax one byte per output element.
 * rdx_res_tail_bwd: dx[r, w, :] = dy at the argmax, 0 elsewhere (incl. the W % 3 tail); ACCUMULATES
 *   sum(dy) per channel into dbias[C] (caller zeroes) = d conv2.bias = d conv_downsample.bias. */
int rdx_bnselu_fwd(int dtype, const void* c, const float* conv_bias, const float* mean, const float* invstd,
                   const float* weight, const float* bias, void* y, int64_t npix, int C, void* stream);
int rdx_bnselu_bwd(int dtype, const void* c, const void* dy, const float* conv_bias, const float* mean,
                   const float* invstd, const float* weight, const float* bias, void* dc, float* sums,
                   int64_t npix, int C, void* stream);
int rdx_res_tail_fwd(int dtype, const void* a, const void* identity, const float* bias, void* y,
                     uint8_t* argmax, int64_t rows, int W, int C, void* stream);
int rdx_res_tail_bwd(int dtype, const void* dy, const uint8_t* argmax, void* dx, float* dbias, int64_t rows,
                     int W, int C, void* stream);
/* SincNet block 0 (ONE input channel, C = 32 output channels): backward of conv1 (2 x 3, padding (1, 1)) and
 * conv_downsample (1 x 3, padding (0, 1)) (Residual_block.forward, src/models/DualStreamSEMamba.py:182-200) in
 * one pass. x bf16 [N, H, W] (the block input); dc bf16 [N, H+1, W, C] = d conv1 output (NHWC); di bf16
 * [N, H, W, C] = d conv_downsample output (NHWC); w1 fp32 [C][2][3], wd fp32 [C][3]. Writes dx fp32 [N, H, W]
 * and per-block partial weight gradients part fp32 [nblk][C][9] (taps 0..5 = conv1 kh*3+kw, 6..8 =
 * conv_downsample kw; the caller sums dim 0), nblk = rdx_sincnet_b0_nblk(N*H*W). C != 32: RDX_EUNSUPPORTED. */
/* SincNet block 0 forward (same block, C = 32): conv1 and conv_downsample of the bf16 input x [N, H, W] with the
 * bf16-valued weights w1 fp32 [C][2][3], wd fp32 [C][3] (fp32 accumulation), and conv1's frozen BN + SELU:
 * bn fp32 [4][C] = (conv1 bias, running mean, invstd * gamma, beta). Writes NHWC bf16 c [N, H+1, W, C] (conv1
 * output without bias), y [N, H+1, W, C] = selu((c + bias - mean) * invstd * gamma + beta) and idn [N, H, W, C]
 * (conv_downsample output without bias). C != 32: RDX_EUNSUPPORTED. */
int rdx_sincnet_b0_fwd(const void* x, const float* w1, const float* wd, const float* bn, void* c, void* y, void* idn,
                       int N, int H, int W, int C, void* stream);
int rdx_sincnet_b0_nblk(int64_t npix);
/* SincNet block 0 forward in one pass (csrc/b0fused.hip; Residual_block.forward with one input channel,
 * src/models/DualStreamSEMamba.py:182-200, frozen BN): y = MaxPool2d((1,3))(conv2(selu(bn2(conv1(x) + cb))) +
 * conv_downsample(x) + bias), NHWC bf16 [N, H, W/3, 32], and arg = the window argmax byte per output element,
 * equal bit for bit to rdx_sincnet_b0_fwd + rdx_sconv_fwd + rdx_res_tail_fwd without their four full-size
 * intermediates. x [N, H, W] bf16 (one channel); w1 [32][6] / wd [32][3] fp32 (bf16 values); bn [4][32]
 * (conv1 bias, mean, invstd * gamma, beta); w2 [6][32 co][32 ci] bf16 tap-major; bias [32] = conv2.bias +
 * conv_downsample.bias. */
int rdx_b0x_fwd(const void* x, const float* w1, const float* wd, const float* bn, const void* w2, const float* bias,
                void* y, uint8_t* arg, int N, int H, int W, void* stream);
/* Its backward in one pass (recomputing c and out1 from x, one exp for both out1 and the SELU derivative): dx fp32 [N, H, W] and one partial row per
 * workgroup, part [rdx_b0x_bwd_nblk(N, W)][6560] fp32 = d conv2.weight [6 taps][32 co][32 ci] | d conv1.weight
 * [32][6] | d conv_downsample.weight [32][3] | d bias [32] (both conv biases) | BN sums [3][32] (d conv1.bias,
 * d gamma, d beta); the caller sums the rows. dp = the pooled output gradient (NHWC bf16), arg = the forward's
 * argmax, bn [5][32] (conv1 bias, mean, invstd * gamma, beta, invstd), w2f = [6][32 ci][32 co] conv2 weights
 * flipped in both axes (the input-gradient layout of rdx_sconv_fwd). */
int rdx_b0x_bwd_nblk(int N, int W);
int rdx_b0x_bwd(const void* x, const void* dp, const uint8_t* arg, const float* w1, const float* wd, const float* bn,
                const void* w2f, float* dx, float* part, int N, int H, int W, void* stream);
int rdx_sincnet_b0_bwd(const void* x, const void* dc, const void* di, const float* w1, const float* wd, float* dx,
                       float* part, int N, int H, int W, int C, void* stream);

/* ---- WavLM positional convolution (HF WavLMPositionalConvEmbedding inside WavLMFrontend,
 * src/models/DualStreamSEMamba.py:292-439): grouped Conv1d 1024 -> 1024, 16 groups x 64 channels, 128 taps,
 * padding 64, last frame dropped, + bias, GELU (erf), MFMA bf16 with fp32 accumulation ----------------------
 * h, y, u, dy, dh: bf16 [B, T, 1024] token-major rows, 16-byte aligned.
 * rdx_posconv_fwd: u = conv(h) + bias (kept for the backward), y = gelu(u); wk bf16 [16][128][64][64] holds
 *   W[g*64+n, c, k] at [g][k][n][c]; bias fp32 [1024].
 * rdx_posconv_bwd: dh = conv^T(dy * gelu'(u)); wkt bf16 [16][128][64][64] holds W[g*64+n, c, 127-k] at
 *   [g][k][c][n]. The weights are frozen in Phase 6: no weight gradient. */
int rdx_posconv_fwd(const void* h, const void* wk, const float* bias, void* y, void* u, int B, int T, void* stream);
int rdx_posconv_bwd(const void* dy, const void* u, const void* wkt, void* dh, int B, int T, void* stream);

/* ---- WavLM self-attention with the gated relative-position bias (HF WavLMAttention as used by
 * WavLMFrontend, src/models/DualStreamSEMamba.py:292-439), MFMA bf16, 64-dim heads -------------------
 * q, k, v: bf16 [B, T, H*64] row views (row strides ldq/ldk/ldv, 16-byte aligned); gate [B, T, H] fp32;
 * rel_bias [H, 2T-1] fp32 (frozen): WavLM's position bias of (query i, key j) depends on j - i only
 * (bucketed relative position, compute_bias), so it is passed as rel_bias[h][j - i + T - 1].
 * S = q k^T * scale + gate[b,i,h] * rel_bias[h, j-i+T-1]; P = softmax(S);
 * O = dropout_p(P) v -> o [B, T, H*64] bf16 (row stride ldo); lse [B, H, T] fp32 (saved for bwd).
 * Dropout: one hash per key pair (2m, 2m+1) of score row (b*H+h)*T+i, pair id row*ceil(T/2)+m, seed =
 * f(seed_dev[0], salt) read on the device (HIP-graph replayable); key 2m keeps iff the hash's low 16 bits
 * >= round(p*2^16), key 2m+1 iff its high 16 bits are. rdx_attn_dropout_mask materialises that mask over
 * n = rows*T elements (tests). keep_mask (nullable; rdx_attn_keep_mask_words(B, T, H) uint32 words) receives
 * the forward's keep bits for rdx_attn_bwd_fused.
 * rdx_attn_bwd: D [B, H, T] fp32 workspace; dq, dk, dv bf16 [B, T, H*64] (row stride ldg), dgate
 * [B, T, H] fp32 (all overwritten); recomputes the dropout hash. */
int rdx_attn_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                 const float* gate, const float* rel_bias, const int64_t* seed_dev, int salt, float p_drop,
                 float scale, void* o, int64_t ldo, float* lse, uint32_t* keep_mask, int B, int T, int H, int head_dim,
                 void* stream);
int64_t rdx_attn_keep_mask_words(int B, int T, int H);
int rdx_attn_bwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                 const float* gate, const float* rel_bias, const int64_t* seed_dev, int salt, float p_drop, float scale,
                 const void* o, int64_t ldo, const float* lse, const void* dout, int64_t lddo, float* D, void* dq,
                 void* dk, void* dv, int64_t ldg, float* dgate, int B, int T, int H, int head_dim, void* stream);
/* rdx_attn_bwd_fused: the same gradients as rdx_attn_bwd from ONE launch of one workgroup per (b, h)
 * (S and dP computed once per tile pair; dS kept in LDS for dQ). T <= 224 (RDX_EUNSUPPORTED above);
 * keep_mask is the forward's (required when p_drop > 0). */
int rdx_attn_bwd_fused(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                       const float* gate, const float* rel_bias, const uint32_t* keep_mask, float p_drop, float scale,
                       const void* o, int64_t ldo, const float* lse, const void* dout, int64_t lddo, float* D,
                       void* dq, void* dk, void* dv, int64_t ldg, float* dgate, int B, int T, int H, int head_dim,
                       void* stream);
/* The same for grids of fewer (b, h) than CUs: two workgroups per (b, h) split the key tiles; each writes its
 * fp32 partial dQ / d gate to ws (>= rdx_attn_bwd_split_ws(B, H) floats) and the second to finish adds them in
 * part order (an agent-scope ticket per (b, h) in counters, zero before the first launch, left zero). B * H % 8
 * == 0. One workspace per stream. */
int64_t rdx_attn_bwd_split_ws(int B, int H);
int rdx_attn_bwd_fused_split(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                             const float* gate, const float* rel_bias, const uint32_t* keep_mask, float p_drop,
                             float scale, const void* o, int64_t ldo, const float* lse, const void* dout,
                             int64_t lddo, float* D, void* dq, void* dk, void* dv, int64_t ldg, float* dgate,
                             float* ws, int64_t ws_floats, int* counters, int64_t n_counters, int B, int T, int H,
                             int head_dim, void* stream);
int rdx_attn_dropout_mask(const int64_t* seed_dev, int salt, float p_drop, uint8_t* keep, int64_t n, int T,
                          void* stream);
/* the element-wise dropout of the fused WavLM layer kernels below (element t kept iff
 * hash(seed, t) >= p*2^32): its keep mask over n elements (tests) */
int rdx_dropout_mask(const int64_t* seed_dev, int salt, float p_drop, uint8_t* keep, int64_t n, void* stream);

/* ---- Fused WavLM encoder layer pieces (HF WavLMEncoderLayerStableLayerNorm + peft LoRA q/v as
 * run by WavLMFrontend, src/models/DualStreamSEMamba.py:292-439 and src/main.py:103-158). Row-major
 * fp32 residual stream h [M, E] (M = B*T tokens, E = 1024, one wave per row), bf16 GEMM operands.
 * Dropouts use the attention's counter hash keyed by (seed_dev[0], salt, m*E + e); p = 0 or a null
 * seed_dev disables one.
 * rdx_wl_ln1_fwd: x1 = LN1(h) -> bf16 x1[:, 0:E] (row stride ldx); gate[m, h] = ga (gb c_h - 1) + 2 with
 *   (ga, gb) = sigmoid of the 4-sums of wg [8, 64] x1_head + bg (gconst = c [H]); with lora_aq/lora_av
 *   [r, E] (r = 8; in the library's 16-bit storage type, the value autocast's cast gives lora_A's fp32 weight;
 *   16-byte aligned) also x1[:, E + k] = sum_e A_k[e] drop_k(x1)[e] (k < r: q adapter, else v); mean/rstd [M]
 *   saved. The LN1 backward entries take lora_aq/lora_av the same way.
 * rdx_wl_add_ln_fwd: h2 = h + drop(delta) (fp32 out), x = LN(h2) bf16, mean/rstd saved.
 * rdx_wl_residual: out = h + drop(delta) over n elements.  rdx_wl_dropout_bwd: out = drop(g) in bf16.
 * rdx_wl_gelu: mode 0 out = gelu(u) (erf form); mode 1 out = dy * gelu'(u).
 * rdx_wl_ln_bwd: dh = dres + LN_bwd(dx) (dres nullable); ddrop = drop(dh) bf16 when non-null.
 * rdx_wl_ln1_bwd: dx1 = dX1[:, :E] + gate and LoRA-A backward terms, dh = dres + LN1_bwd(dx1); with LoRA
 *   also (xd non-null) xd [2, M, E] bf16 = the dropped x1 of each adapter.
 * rdx_wl_lora_grad: LoRA weight gradients ACCUMULATED into fp32 daq/dav [r, E] and dbq/dbv [E, r]:
 *   dB += scale * d{q,v}^T a_{q,v}, dA += d a_{q,v}^T drop(x1) (dqkv [M, ldq] bf16, x1/dx1 [M, ld] bf16 with
 *   a / d a in columns E..E+2r).
 * rdx_wl_lora_pack: for every layer l, wext[l] [3E, ldw] bf16 columns E..E+2r <- scale * lora_B
 *   (q rows 0..E-1, v rows 2E..3E-1); bq, bv, wext are DEVICE arrays of nl pointers. */
int rdx_wl_ln1_fwd(const float* h, const float* gamma, const float* beta, float eps, const float* wg,
                   const float* bg, const float* gconst, const void* lora_aq, const void* lora_av, int r,
                   const int64_t* seed_dev, int salt_q, int salt_v, float p_lora, void* x1, int64_t ldx, float* gate, float* mean,
                   float* rstd, int64_t M, int E, void* stream);
int rdx_wl_add_ln_fwd(const float* h, const void* delta, const int64_t* seed_dev, int salt, float p, float* h2,
                      const float* gamma, const float* beta, float eps, void* x, float* mean, float* rstd,
                      int64_t M, int E, void* stream);
int rdx_wl_residual(const float* h, const void* delta, const int64_t* seed_dev, int salt, float p, float* out,
                    int64_t n, void* stream);
int rdx_wl_dropout_bwd(const float* g, const int64_t* seed_dev, int salt, float p, void* out, int64_t n,
                       void* stream);
int rdx_wl_gelu(int mode, const void* u, const void* dy, void* out, int64_t n, void* stream);
int rdx_wl_ln_bwd(const void* dx, int64_t ldd, const float* h, const float* mean, const float* rstd,
                  const float* gamma, const float* dres, float* dh, const int64_t* seed_dev, int salt, float p,
                  void* ddrop, int64_t M, int E, void* stream);
int rdx_wl_ln1_bwd(const void* dx1, int64_t ldx, const float* dgate, const float* h, const float* mean,
                   const float* rstd, const float* gamma, const float* beta, const float* wg, const float* bg,
                   const float* gconst, const void* lora_aq, const void* lora_av, int r,
                   const int64_t* seed_dev, int salt_q, int salt_v, float p_lora, const float* dres, float* dh, void* xd, int64_t M, int E,
                   void* stream);
/* rdx_wl_res_ln1_fwd: rdx_wl_ln1_fwd of h = h2 + drop(delta) (the residual of the previous layer, computed here
 *   and written to hout): one pass instead of rdx_wl_residual then rdx_wl_ln1_fwd. */
int rdx_wl_res_ln1_fwd(const float* h2, const void* delta, int salt_res, float p_res, float* hout,
                       const float* gamma, const float* beta, float eps, const float* wg, const float* bg,
                       const float* gconst, const void* lora_aq, const void* lora_av, int r, const int64_t* seed_dev,
                       int salt_q, int salt_v, float p_lora, void* x1, int64_t ldx, float* gate, float* mean,
                       float* rstd, int64_t M, int E, void* stream);
/* rdx_wl_ln1_bwd_ex: rdx_wl_ln1_bwd plus (state_grad, state_weight non-null) dh += state_weight[0] * state_grad,
 *   the gradient the layer input receives as a hidden state of the layer-weighted sum (see
 *   rdx_layer_wsum_bwd's NULL dhs[l]), and (ddrop_prev non-null) ddrop_prev = drop(dh) bf16 with the previous
 *   layer's hidden dropout (salt_prev, p_prev): that layer's rdx_wl_dropout_bwd, fused. */
int rdx_wl_ln1_bwd_ex(const void* dx1, int64_t ldx, const float* dgate, const float* h, const float* mean,
                      const float* rstd, const float* gamma, const float* beta, const float* wg, const float* bg,
                      const float* gconst, const void* lora_aq, const void* lora_av, int r, const int64_t* seed_dev,
                      int salt_q, int salt_v, float p_lora, const float* dres, float* dh, void* xd,
                      const float* state_grad, const float* state_weight, int salt_prev, float p_prev,
                      void* ddrop_prev, int64_t M, int E, void* stream);
int rdx_wl_lora_grad(const void* dqkv, int64_t ldq, const void* x1, int64_t ldx, const void* dx1, int64_t ldd,
                     const int64_t* seed_dev, int salt_q, int salt_v, float p_lora, float scale, float* daq,
                     float* dbq, float* dav, float* dbv, int64_t M, int E, int r, void* stream);
int rdx_wl_lora_pack(int nl, const float* const* bq, const float* const* bv, void* const* wext, int64_t ldw,
                     int r, float scale, int E, void* stream);

/* ---- bf16 MFMA GEMM with fused epilogues: the WavLM layer's projections (q|k|v + LoRA columns,
 * out_proj, FFN1, FFN2 of HF WavLMEncoderLayerStableLayerNorm, src/models/DualStreamSEMamba.py:292-439)
 * and their input gradients (the transposed frozen weight as B) --------------------------------------
 * C[M, N] = A[M, K] . B[N, K]^T, bf16 rows (lda, ldb multiples of 8, 16-byte aligned), fp32 accumulate.
 * epilogue RDX_EPI_BIAS: C bf16 = acc + bias (bias bf16 [N] or NULL);
 *          RDX_EPI_BIAS_GELU: C = u = bf16(acc + bias), aux_out bf16 [M, ldao] = gelu(u) (erf form);
 *          RDX_EPI_GELU_BWD: C bf16 = bf16(acc) * gelu'(aux), aux = u bf16 [M, ldaux];
 *          RDX_EPI_RESID_DROP: C fp32 = aux fp32 [M, ldaux] + bf16(acc + bias) * dropout_p, the
 *            element-wise hash of element m * N + n with seed f(seed_dev[0], salt) (rdx_dropout_mask).
 * Requires K % 8 == 0, N % 4 == 0. */
#define RDX_EPI_BIAS 0
#define RDX_EPI_BIAS_GELU 1
#define RDX_EPI_GELU_BWD 2
#define RDX_EPI_RESID_DROP 3
int rdx_gemm_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N, int K,
                  const void* bias, int epilogue, const void* aux, int64_t ldaux, void* aux_out, int64_t ldao,
                  const int64_t* seed_dev, int salt, float p_drop, void* stream);

/* ---- Chunked two-level selective scan (csrc/scan2.hip) -----------------------------------------------------
 * Same operands and results as rdx_selective_scan_fwd / _bwd (src/models/modules/mamba_block.py:65-122, both
 * directions at original positions, the same checkpoint layout), the steps cut into rdx_scan2_chunks(L) chunks of
 * 16: per-chunk local states and decay products, then every chunk from its composed carry. Forward: P (the
 * per-chunk decay products, kept for the backward) and hloc (a workspace: it ends holding every chunk's carry-in)
 * are [dirs][B][chunks][D][N] fp32 (rdx_scan2_rec_elems). Backward: gloc is a workspace of the same size; dA_part [dirs * B * chunks][D][N],
 * dD_part / dbias_part [dirs * B * chunks][D] (summed by the caller), rows of ld_part floats (0: dense; D * N + 2D
 * packs the three into one buffer summed with one reduction); dBC [dirs][B][L][2N] fp32 is zeroed and accumulated
 * by the call. */
int rdx_scan2_chunks(int L);
int64_t rdx_scan2_rec_elems(int B, int L, int D, int N, int dirs);
int rdx_scan2_fwd(int dtype, const void* u, const void* delta, const float* A_log, const void* Bm, const void* Cm,
                  int64_t ldbc, const float* Dp, const float* dt_bias, float* y, float* ckpt, float* P, float* hloc,
                  int B, int L, int D, int N, int dirs, void* stream);
int rdx_scan2_bwd(int dtype, const void* u, const void* delta, const float* A_log, const void* Bm, const void* Cm,
                  int64_t ldbc, const float* Dp, const float* dt_bias, const float* ckpt, const float* P,
                  const float* dy, int64_t dy_dir_stride, void* du, void* ddelta, float* dBC, float* dA_part,
                  float* dD_part, float* dbias_part, int64_t ld_part, float* gloc, int B, int L, int D, int N,
                  int dirs, void* stream);

/* ---- bf16 MFMA GEMM of the WavLM encoder projections, LDS-DMA pipeline (csrc/wgemm.hip) ---------------
 * Same contract as rdx_gemm_bf16 for the RDX_EPI_BIAS / _BIAS_GELU / _GELU_BWD epilogues, with K % 64 == 0;
 * the projections and input gradients of HF WavLMEncoderLayerStableLayerNorm (src/models/DualStreamSEMamba.py:
 * 292-439: q/k/v, out_proj, FFN1, FFN2 at M = B x 201 tokens). tile codes (csrc/wgemm.hip wg_geometry):
 * 0 / 6 / 14 = 128 x 128, 1 / 11 / 17 = 64 x 128, 5 = 64 x 64, 12 / 16 = 128 x 256, 13 = 256 x 128,
 * 15 = 64 x 256, 18 = 256 x 256, 20 / 21 = 128 x 192 output tiles (4- or 8-wave, 2-4 deep LDS rings);
 * -1 = rdx_wgemm_pick(M, N, K). The epilogue stages the tile through LDS and stores whole rows. */
int rdx_wgemm_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N, int K,
                   const void* bias, int epilogue, const void* aux, int64_t ldaux, void* aux_out, int64_t ldao,
                   int tile, void* stream);
int rdx_wgemm_pick(int M, int N, int K);
/* Split-K form: `splits` (1 ..= K / 64) workgroups share each output tile, split s taking k-steps
 * [s*nk/splits, (s+1)*nk/splits); each publishes an fp32 partial to `ws` and the last arriver (an agent-scope
 * ticket in `counters`, one int per tile, zero before the first launch and left zero after each) sums the
 * partials in split order (deterministic) and runs the epilogue. ws_bytes >= rdx_wgemm_ws_bytes(M, N, tile,
 * splits), n_counters >= rdx_wgemm_counters(M, N, tile). One workspace per stream: two launches in flight at
 * once must not share it. Rows of C / aux / aux_out 16-byte aligned (ld % 8 == 0) take 16-byte accesses. */
int rdx_wgemm_bf16_ex(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N,
                      int K, const void* bias, int epilogue, const void* aux, int64_t ldaux, void* aux_out,
                      int64_t ldao, int tile, int splits, void* ws, int64_t ws_bytes, int* counters,
                      int64_t n_counters, void* stream);
int64_t rdx_wgemm_ws_bytes(int M, int N, int tile, int splits);
int64_t rdx_wgemm_counters(int M, int N, int tile);

/* ---- Deep-pipelined bf16 MFMA GEMM of the WavLM encoder projections (csrc/pgemm.hip) ------------------------
 * Same operands, layouts and epilogues as rdx_wgemm_bf16 (K % 64 == 0; the q/k/v, out_proj, FFN1, FFN2 GEMMs and
 * their input gradients of HF WavLMEncoderLayerStableLayerNorm, src/models/DualStreamSEMamba.py:292-439), on
 * one 512-thread workgroup per output tile: 8 waves, an NST-deep LDS-DMA ring kept in flight across the one
 * barrier per K step, fragment reads one phase ahead of the MFMAs. tile codes (csrc/pgemm.hip pg::geometry):
 * 0 / 8 / 9 = 256 x 256, 1 / 6 = 256 x 128, 2 / 5 = 128 x 256, 3 / 7 = 128 x 128, 4 = 128 x 192 output tiles
 * (0-3, 8, 9: 32-deep K steps, 4-8 stage rings; 4-7: 64-deep, 3-4 stages); + 100 raises the wave priority around the MFMA clusters. group_m: tiles are dealt to XCDs in
 * contiguous runs and ordered group_m row tiles x every column tile (0 = all row tiles: column-panel order). */
int rdx_pgemm_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N, int K,
                   const void* bias, int epilogue, const void* aux, int64_t ldaux, void* aux_out, int64_t ldao,
                   int tile, int group_m, void* stream);
/* Diagnostic form (bias epilogue, tiles 0 / 2 / 4; + 10 = without refills in the K loop, + 20 = without MFMA;
 * group_m -1 puts every workgroup on tile (0, 0)): also stores 8 words per workgroup into prof [grid][8]: shader-clock
 * stamps at entry / stage 0 landed / main loop done / exit, 100 MHz real-time stamps at entry / exit, the
 * (XCC id << 32 | HW_ID) word and (row tile << 32 | column tile). */
int rdx_pgemm_prof(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N, int K,
                   const void* bias, int tile, int group_m, void* prof, void* stream);

/* ---- Ping-pong MFMA GEMM of the WavLM encoder projections (csrc/hgemm.hip) -------------------------------------
 * Same operands, layouts and epilogues as rdx_wgemm_bf16_ex (K % 64 == 0; q/k/v, out_proj, FFN1, FFN2 and their input
 * gradients of HF WavLMEncoderLayerStableLayerNorm, src/models/DualStreamSEMamba.py:292-439, under the autocast of
 * src/main.py:1049), on one 512-thread workgroup per output tile (or per split of one): 8 waves as 2 x 4, the two row
 * groups one barrier apart so each SIMD pairs one wave's MFMA segment with its partner's LDS reads and LDS-DMA issue,
 * a ring of 8 KB slabs refilled one phase after they are read (counted vmcnt, never drained in the loop). tile codes
 * (csrc/hgemm.hip hg::geometry): 0 = 256 x 256, 1 = 256 x 192, 2 = 128 x 256, 3 = 128 x 192, 4 = 128 x 128,
 * 5 = 256 x 128, 6 = 64 x 128, 7 = 64 x 256; + 100: s_setprio(1) around every MFMA segment, + 200: static priority 1 for the second row group.
 * group_m: XCD-contiguous runs ordered group_m row tiles x every column tile (0 = column-panel order); -R (R = 1, 2,
 * 4, 8): the tiles cut into an R x 8/R grid of blocks, one per XCD (each XCD's L2 sees 1/R of A's rows and R/8 of
 * B's panels). splits > 1:
 * split-K with an in-launch last-arriver sum in split order (deterministic); ws / counters as rdx_wgemm_bf16_ex
 * (rdx_hgemm_ws_bytes, rdx_hgemm_counters), one workspace per stream. */
int rdx_hgemm(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N, int K,
              const void* bias, int epilogue, const void* aux, int64_t ldaux, void* aux_out, int64_t ldao, int tile,
              int splits, int group_m, void* ws, int64_t ws_bytes, int* counters, int64_t n_counters, void* stream);
int64_t rdx_hgemm_ws_bytes(int M, int N, int tile, int splits);
int64_t rdx_hgemm_counters(int M, int N, int tile);
/* splits == 0 (tiles 2 / 3 / 4): stream-K. One workgroup per CU; the grid's workgroups take equal contiguous runs of
 * the (tile, 64-deep K step) units in tile order, and a tile shared by several runs is summed by the last of them to
 * arrive, its fp32 partials in K order (deterministic). ws_bytes >= rdx_hgemm_sk_ws_bytes(M, N, K, tile). */
int64_t rdx_hgemm_sk_ws_bytes(int M, int N, int K, int tile);
/* Batched form (RDX_EPI_BIAS, splits 1): `batch` problems C_y [M, ldc] = A_y . B^T + bias in one launch, A_y = A + y sa
 * (rows may overlap, lda < K: a token-major activation read as a strided convolution's im2col matrix), C_y = C + y sc.
 * The frozen WavLM CNN's layers 1-6 (HF WavLMFeatureEncoder, src/models/DualStreamSEMamba.py:392-439; csrc/featconv.hip
 * layout). tile 0-7 as rdx_hgemm, group_m >= 0. */
int rdx_hgemm_batched(const void* A, int64_t lda, int64_t sa, const void* B, int64_t ldb, void* C, int64_t ldc,
                      int64_t sc, int M, int N, int K, int batch, const void* bias, int tile, int group_m, void* stream);

/* ---- Split-precision ("x3") GEMM for the fp32 scoring pass (csrc/hgemm.hip) ------------------------------------
 * The reference scores in fp32 without autocast (src/main.py:958-995, comment at :974-975) and the north star holds the
 * logits to 1e-3 of its CPU path. gfx950 has no TF32 and its fp32 MFMA runs at 1/16 of the bf16 rate, so an fp32
 * operand x is carried as two bf16 planes, hi = bf16(x) and lo = bf16(x - hi) (|x - hi - lo| <= 2^-17 |x|), and
 *   C = A . B^T ~= Ahi . Bhi^T + Alo . Bhi^T + Ahi . Blo^T      (the dropped Alo . Blo^T is <= 2^-16 |A||B|)
 * runs as one ping-pong launch of rdx_hgemm whose K loop makes three passes over the planes (3K/64 steps, fp32
 * accumulation throughout). A / A_lo [M, lda], B / B_lo [N, ldb] (the frozen weight's planes), same strides; batch
 * > 1: blockIdx.y walks `batch` problems, A planes advanced by sa and C / C_lo by sc elements (the WavLM CNN's
 * per-utterance strided convolutions), splits must then be 1. bias fp32 [N] or NULL.
 * epilogue RDX_EPI_F32: C fp32 [M, ldc] = acc + bias (C_lo unused);
 *          RDX_EPI_F32_GELU_SPLIT: v = gelu(acc + bias) (erf form), C = bf16(v), C_lo = bf16(v - C) (the planes of the
 *          next GEMM's A: FFN1 -> FFN2).
 * tile 0-5 as rdx_hgemm; splits >= 1 with rdx_hgemm_ws_bytes / rdx_hgemm_counters workspaces. libradhip.so only
 * (libradhip_f16.so returns RDX_EINVAL: fp16 lo planes of small values fall into fp16's subnormal range). */
#define RDX_EPI_F32 4
#define RDX_EPI_F32_GELU_SPLIT 5
int rdx_hgemm_x3(const void* A, const void* A_lo, int64_t lda, int64_t sa, const void* B, const void* B_lo,
                 int64_t ldb, void* C, void* C_lo, int64_t ldc, int64_t sc, int M, int N, int K, int batch,
                 const float* bias, int epilogue, int tile, int splits, int group_m, void* ws, int64_t ws_bytes,
                 int* counters, int64_t n_counters, void* stream);

/* ---- The rest of the fp32 scoring pass's WavLM stream on the x3 planes (csrc/x3.hip; libradhip.so only) ---------
 * Planes: hi = bf16(x), lo = bf16(x - hi), same shape and strides. Reference: HF WavLMModel under
 * WavLMFrontend.forward (src/models/DualStreamSEMamba.py:392-439) as the fp32 eval runs it (src/main.py:958-995).
 *   rdx_x3_split: x fp32 [rows, cols] (row stride ldx) -> hi / lo [rows, ldo]; cols % 4 == 0.
 *   rdx_x3_ln_split: x = a (+ b when b != NULL; x written to sum_out when != NULL: the residual stream), rows of E = 512
 *     or 1024 fp32; y = LayerNorm(x; gamma, beta, eps) -> planes hi / lo [M, ldo] and / or fp32 y32 [M, E]. wg != NULL
 *     (E = 1024, 64-dim heads): the HF WavLMAttention gate of y, gate[m, h] = ga (gb gconst[h] - 1) + 2 with (ga, gb)
 *     = sigmoid of the two 4-sums of gru_rel_pos_linear(y_head) (wg [8, 64], bg [8]), gate fp32 [M, H].
 *   rdx_x3_attn_fwd: o = softmax(scaling q k^T + gate[b, i, h] rel[h, j - i + T - 1]) v per (utterance, head) in fp32
 *     (v_mfma_f32_16x16x4_f32), q / k / v fp32 [B*T, ld] column blocks of 64 per head, rel the [H, 2T - 1] table of
 *     the relative position bias (radhip.ops.rel_bias_table), output planes [B*T, ldo]; T <= 256; qsplit workgroups
 *     per (utterance, head) share its query tiles.
 *   rdx_x3_posconv_fwd: out = h + gelu(conv1d(h, W, bias, padding 64, groups 16)[:, :T]) (HF
 *     WavLMPositionalConvEmbedding + the encoder's residual add), h / out fp32 [B, T, 1024] (out != h); wk_hi / wk_lo
 *     the bf16 planes of W in rdx_posconv_fwd's [16][128][64][64] layout, bias fp32 [1024].
 *   rdx_x3_fe_conv0: CNN layer 0 of rdx_fe_conv0 in fp32 (unrounded waveform and weights w fp32 [512, 10], bias fp32
 *     [512] or NULL) + LayerNorm(512) + GELU -> planes [B, T0, 512].
 *   rdx_x3_fe_ln_gelu: LayerNorm(512) + GELU of in fp32 [rows, 512] (+ bias fp32 [512] when != NULL) -> planes
 *     [rows, 512], or fp32 out32 when != NULL (the last layer). */
int rdx_x3_split(const float* x, int64_t ldx, int64_t rows, int cols, void* hi, void* lo, int64_t ldo, void* stream);
int rdx_x3_ln_split(const float* a, const float* b, float* sum_out, const float* gamma, const float* beta, float eps,
                    void* hi, void* lo, int64_t ldo, float* y32, const float* wg, const float* bg, const float* gconst,
                    float* gate, int64_t M, int E, void* stream);
int rdx_x3_attn_fwd(const float* q, const float* k, const float* v, int64_t ld, const float* gate, const float* rel,
                    float scaling, void* ohi, void* olo, int64_t ldo, int B, int T, int H, int qsplit, void* stream);
int rdx_x3_posconv_fwd(const float* h, const void* wk_hi, const void* wk_lo, const float* bias, float* out, int B,
                       int T, void* stream);
int rdx_x3_fe_conv0(const float* x, int64_t batch, int64_t len, const float* w, const float* bias, const float* gamma,
                    const float* beta, float eps, int ksize, int stride, void* out_hi, void* out_lo, void* stream);
int rdx_x3_fe_ln_gelu(const float* in, int64_t rows, const float* bias, const float* gamma, const float* beta,
                      float eps, void* out_hi, void* out_lo, float* out32, void* stream);

/* Column sums of fp32 row-partial buffers, up to 4 problems per launch: out_k[c] = sum_r in_k[r * ld_k + c] (rows
 * in order, fixed-order combine: deterministic). Replaces the torch reductions of the scan / depthwise-conv backward
 * partials (csrc/layersum.hip). */
int rdx_colsum_many(int n, const float* const* in, const int* rows, const int* cols, const int64_t* ld,
                    float* const* out, void* stream);

/* ---- Small GEMMs of the detector head (csrc/lgemm.hip) -----------------------------------------------------------
 * C[M, N] = A[M, K] W[N, K]^T for the fusion / PN-BiMamba / pooling / classifier linears (replaces F.linear and the
 * input-gradient torch.matmul of src/models/DualStreamSEMamba.py:445-531,537-637,700-770 under the autocast of
 * src/main.py:1049): A 16-bit, or fp32 when a_f32 (rounded to 16 bits on load: autocast's input cast); W 16-bit
 * [N, ldw]; any K and any row strides (16-byte loads where rows are aligned). C 16-bit, or fp32 when c_f32 (the
 * 16-bit result widened); R [M, ldr] of C's type or NULL: C = R + C (16-bit: rounded; C may alias R). RDX_EPI_BIAS: C = acc +
 * bias (bias 16-bit [N] or NULL); RDX_EPI_BIAS_GELU (16-bit C): C = u = round(acc + bias), aux_out [M, ldao] =
 * gelu(u); RDX_EPI_GELU_BWD: C = round(round(acc) * gelu'(aux)), aux = u [M, ldaux], no bias. */
int rdx_lgemm(const void* A, int64_t lda, int a_f32, const void* W, int64_t ldw, void* C, int64_t ldc, int c_f32,
              int M, int N, int K, const void* bias, int epilogue, const void* aux, int64_t ldaux, void* aux_out,
              int64_t ldao, const void* R, int64_t ldr, void* stream);

/* ---- Weight / bias gradients of the head's linears, accumulated in fp32 (csrc/wgrad.hip) ----------------
 * dW[n][k] += sum_m dY[m][n] X[m][k], db[n] += sum_m dY[m][n] (db may be NULL): bf16 dY [M, ldy] and X [M, ldx],
 * fp32 dW [N, ldw] (the flat gradient buffer's views), the token rows split over the chip in chunks of
 * rdx_wgrad_chunk(M, N, K) rows and the chunk partials (ws, >= rdx_wgrad_ws_floats fp32) added in a fixed order:
 * deterministic. Replaces the addmm(out_dtype = fp32) + sum + add of SideLinear's backward
 * (radhip/linear.py; the linears of src/models/DualStreamSEMamba.py:445-531, 537-637, 700-770). */
int rdx_wgrad_chunk(int M, int N, int K);
int64_t rdx_wgrad_ws_floats(int M, int N, int K);
int rdx_wgrad_acc(const void* dy, int64_t ldy, const void* x, int64_t ldx, int M, int N, int K, float* dw, int64_t ldw,
                  float* db, float* ws, int64_t ws_floats, void* stream);
/* Batched form: n <= 32 problems (arrays of n entries; db[k] may be NULL), every dw / db distinct, in two launches:
 * one workgroup per (problem, 64 x 64 output block, run of 128-row sub-chunks), then one fixed-order reduction of
 * the runs' partials into each dW / db. ws >= rdx_wgrad_many_ws_floats (has_db[k] = db[k] != NULL). radhip.ops.
 * wgrad_batch collects a backward pass's SideLinear gradients into one call. */
int64_t rdx_wgrad_many_ws_floats(int n, const int* M, const int* N, const int* K, const int* has_db);
int rdx_wgrad_acc_many(int n, const void* const* dy, const int64_t* ldy, const void* const* x, const int64_t* ldx,
                       const int* M, const int* N, const int* K, float* const* dw, const int64_t* ldw,
                       float* const* db, float* ws, int64_t ws_floats, void* stream);

/* ---- AdamW over a list of fp32 tensors (csrc/optim.hip) ------------------------------------------------------
 * torch.optim.AdamW's update (decoupled weight decay; the reference's optimizer, src/main.py:416-457) for up to
 * rdx_adamw_many_max() tensors per call: params, grads, exp_avg, exp_avg_sq [numel[k]] fp32, step[k] the tensor's
 * step count (a device fp32 scalar, already incremented). grad_scale (may be NULL): grads are divided by it and
 * stored back; found_inf (may be NULL): nonzero skips the update (GradScaler's fused-optimizer contract). Each
 * block owns 4096 elements of one tensor; the element math follows torch's fused AdamW functor (double
 * hyper-parameters). radhip.optim.AdamW drives it and keeps torch's state layout. */
int rdx_adamw_many_max(void);
int rdx_adamw_many(int n, float* const* params, float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                   const float* const* step, const int64_t* numel, double lr, double beta1, double beta2,
                   double weight_decay, double eps, const float* grad_scale, const float* found_inf, void* stream);

/* ---- Timing inside replayed HIP graphs (bench instrumentation; no reference counterpart) -------
 * rdx_timestamp_acc: one-lane kernel, acc[0] += sign * wall_clock64(); acc[1] += 1 when sign == +1.
 * Launch with sign -1 before and +1 after a kernel on the same stream: acc[0] accumulates its
 * duration in device wall-clock ticks (rdx_wallclock_khz(device) kHz), acc[1] the launch count. */
int rdx_timestamp_acc(int64_t* acc, int sign, void* stream);
int rdx_wallclock_khz(int device);

/* ------------------------------------------------------------------------------------------
 * Batched / implicit-GEMM form of rdx_gemm_bf16 (bias epilogue): for z < batch,
 *   C[z*crow + m, n] = bf16(sum_k A[z*sA + m*lda + k] * B[n*ldb + k] + bias[n])
 * lda may be smaller than K (overlapping rows): a stride-s convolution over token-major [T, C]
 * activations is then a GEMM over its input in place (lda = s*C, K = ksize*C), no im2col copy.
 * ------------------------------------------------------------------------------------------ */
int rdx_gemm_bf16_strided(const void* A, int64_t lda, int64_t sA, const void* B, int64_t ldb, void* C, int64_t ldc,
                          int64_t crow, int batch, int M, int N, int K, const void* bias, void* stream);

/* ------------------------------------------------------------------------------------------
 * WavLM frozen CNN feature encoder (HF WavLMFeatureEncoder, feat_extract_norm "layer", conv_dim 512),
 * replacing the MIOpen conv + transpose + LayerNorm + GELU chain of WavLMFrontend's frozen CNN
 * (src/models/DualStreamSEMamba.py:392-439). Activations token-major [B, T_l, 512].
 *   rdx_fe_conv0: layer 0 (C_in 1, ksize 10): out bf16 [B, (len-ksize)/stride+1, 512] =
 *     gelu(LayerNorm(conv(bf16(x)) + bias)); w [512][ksize] and bias [512] fp32 holding bf16 values.
 *   rdx_fe_ln_gelu: LayerNorm(512) + GELU of rows [rows, 512] bf16, in place, or into out32 (fp32).
 * Layers 1-6 are rdx_gemm_bf16_strided over the previous layer's output (lda = stride*512).
 * ------------------------------------------------------------------------------------------ */
int rdx_fe_conv0(const float* x, int64_t batch, int64_t len, const float* w, const float* bias, const float* gamma,
                 const float* beta, float eps, int ksize, int stride, void* out, void* stream);
int rdx_fe_ln_gelu(void* io, int64_t rows, const float* gamma, const float* beta, float eps, float* out32,
                   void* stream);

/* ------------------------------------------------------------------------------------------
 * SincNet residual-stack convolutions (Residual_block conv1 2x3 pad (1,1), conv2 2x3 pad (0,1),
 * conv_downsample 1x3 pad (0,1); src/models/DualStreamSEMamba.py:144-200), NHWC bf16, C_in, C_out in
 * {32, 64}, kh in {1, 2}, stride 1, column padding 1, row padding ph; replaces MIOpen's solvers.
 *   rdx_sconv_fwd:   y [N, H+2ph-kh+1, W, co] = conv(x [N, H, W, ci], w), w tap-major [kh*3][co][ci] bf16.
 *                    With y2 and bn = [conv bias | running mean | invstd*gamma | beta] (4 x co fp32) also
 *                    y2 = bf16(selu(((bf16(y) + cb) - mean) * invstd*gamma + beta)).
 *                    The input gradient is this call on dY with the flipped kernel [kh*3][ci][co] and
 *                    row padding kh-1-ph.
 *   rdx_sconv_wgrad: dw [kh*3][co][ci] fp32 from x and dy; part: rdx_sconv_wgrad_nblk(N, Ho, W) rows of
 *                    kh*3*co*ci fp32 scratch (per-workgroup partials and the two-stage reduction's
 *                    slices, summed in a fixed order: deterministic).
 * ------------------------------------------------------------------------------------------ */
int rdx_sconv_fwd(const void* x, const void* w, void* y, void* y2, const float* bn, int N, int H, int W, int ci,
                  int co, int kh, int ph, void* stream);
/* rdx_sconv_fwd with a residual added in the epilogue: y = bf16(bf16(conv(x, w)) + res), res bf16 [N, Ho, W, co]
 * NHWC (16-byte aligned). A residual block's input gradient in one pass: conv1's input gradient plus the identity
 * branch's gradient, the bits autograd's add would produce (radhip.ops.ResBlockIdentity). */
int rdx_sconv_fwd_res(const void* x, const void* w, void* y, const void* res, int N, int H, int W, int ci, int co,
                      int kh, int ph, void* stream);
/* conv2's input gradient continued through conv1's frozen BN + SELU backward (Residual_block.forward,
 * src/models/DualStreamSEMamba.py:182-200; replaces rdx_sconv_fwd on dY followed by rdx_bnselu_bwd): the
 * 32-channel blocks (ci = co = 32, kh = 2). dO1 = conv(dy, w) (w: conv2's flipped, transposed kernel
 * [kh*3][co][ci]; ph = kh - 1 - conv2's row padding) stays on chip; dc = bf16(dO1) * selu'(u) * invstd*gamma
 * with the saved pre-activation c [N, Ho, W, co]; sums[3][co] += d conv1.bias | d bn.weight | d bn.bias.
 * bn = [cb | mean | invstd*gamma | beta | invstd] (5 x co fp32); sums zeroed by the caller. */
int rdx_sconv_dgrad_bnselu(const void* dy, const void* w, const void* c, void* dc, const float* bn, float* sums,
                           int N, int H, int W, int ci, int co, int kh, int ph, void* stream);
int rdx_sconv_wgrad_nblk(int N, int Ho, int W);
int rdx_sconv_wgrad(const void* x, const void* dy, float* dw, float* part, int N, int H, int W, int ci, int co,
                    int kh, int ph, void* stream);
/* ---- The detector head's squeeze-excitation (src/models/DualStreamSEMamba.py:492-531) under autocast, csrc/head.hip.
 * rdx_se_fwd: x [B, T, C] 16-bit (C % 8 == 0, C <= 256, 16-byte aligned), w1 [R, C], w2 [C, R] 16-bit (R <= 16):
 *   m = mean_t x, h = relu(m w1^T), s = sigmoid(h w2^T) (each rounded to 16 bits as autocast leaves them; saved to
 *   m [B, C], h [B, R], s [B, C]) and y = x * s [B, T, C].
 * rdx_se_bwd: from dy [B, T, C] and the saved tensors: dx [B, T, C] (both branches' gradients added in 16 bits) and
 *   the fc weight gradients ADDED in fp32 into dw1 [R, C] and dw2 [C, R] (per-utterance partial rows in part,
 *   rdx_se_bwd_part_floats(B, C, R) floats, summed in utterance order). */
int rdx_se_fwd(const void* x, const void* w1, const void* w2, void* y, void* m, void* h, void* s, int B, int T, int C,
               int R, void* stream);
int64_t rdx_se_bwd_part_floats(int B, int C, int R);
int rdx_se_bwd(const void* dy, const void* x, const void* w1, const void* w2, const void* m, const void* h, const void* s,
               void* dx, float* part, float* dw1, float* dw2, int B, int T, int C, int R, void* stream);
/* rdx_attn_pool_fwd: the head's attention pooling under autocast (src/models/DualStreamSEMamba.py:700-770):
 *   z = round(f w^T + bias) (f [B, T, C] 16-bit, w [C], bias [1] 16-bit or NULL), a = softmax_t(z) fp32 (saved to
 *   a [B, T]), feat [B, C] = round(round(a)^T f). T <= 1024, C <= 1024.
 * rdx_attn_pool_bwd: from dfeat [B, C]: df [B, T, C] (the weighted sum's and the scores' gradients added in 16 bits)
 *   and dw [C] / db [1] (db may be NULL) ADDED in fp32 (part: B * (C + 1) floats of per-utterance partials). */
int rdx_attn_pool_fwd(const void* f, const void* w, const void* bias, void* feat, float* a, int B, int T, int C,
                      void* stream);
int rdx_attn_pool_bwd(const void* f, const void* w, const float* a, const void* dfeat, void* df, float* part, float* dw,
                      float* db, int B, int T, int C, void* stream);
/* rdx_upcat_fwd: DualStreamFusion's alignment + concat (src/models/DualStreamSEMamba.py:537-637): out [B, T1, 2C] =
 *   [fw [B, T1, C] | fs [B, T2, C] at F.interpolate's 'nearest' index min(floor(t * (T2 / T1)), T2 - 1)], 16-bit,
 *   C % 8 == 0, 16-byte aligned.
 * rdx_upcat_bwd: dfs [B, T2, C] = the nearest upsample's backward of dout[..., C:2C] (fp32 sums, rounded once). */
int rdx_upcat_fwd(const void* fw, const void* fs, void* out, int B, int T1, int T2, int C, void* stream);
int rdx_upcat_bwd(const void* dout, void* dfs, int B, int T1, int T2, int C, void* stream);
/* rdx_sconv_wprep_many: for n <= 32 fp32 convolution weights src[k] [co][ci][kh][3] (kh 1 or 2), both 16-bit operand
 *   layouts in one launch: wf[k] [kh*3][co][ci] (rdx_sconv_fwd's w) and wd[k] [kh*3][ci][co] of the kernel flipped in
 *   both axes (the input gradient's w). src / wf / wd are host arrays of device pointers. */
int rdx_sconv_wprep_many(int n, const float* const* src, void* const* wf, void* const* wd, const int* co,
                         const int* ci, const int* kh, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RADHIP_H */
