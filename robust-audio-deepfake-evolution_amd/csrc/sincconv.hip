// Fused SincConv front end for gfx950: valid 1-D conv of the waveform with the fixed band-pass bank,
// |.|, and the 3x3 (channel x time) max-pool, in one pass.
//
// Reference: CONV.forward (src/models/DualStreamSEMamba.py:119-138) -> F.conv1d [B,70,T-128], then
// SincNetEncoder.forward: unsqueeze, F.max_pool2d(torch.abs(x), (3, 3)) (:250-253).  The conv output
// [B, 70, 64472] (18 MB/utt fp32) is never written: each thread keeps its 3 channels x 3 times of
// accumulators in registers and stores one pooled value per channel triple.
//
// Work split: block = (256 pooled time positions, utterance).  The 3*256+K-1 sample window is staged
// in LDS once (coalesced); each lane owns one pooled time position t3 (conv times 3t3..3t3+2) and
// sweeps all channel triples.  Filter taps are wave-uniform -> scalar (SMEM) loads, so the inner
// loop is 1 LDS read + 9 FMAs per tap (the x window slides through registers).
#include "common.h"

namespace rdx {

constexpr int SINC_T3 = 256;  // pooled outputs per block (= threads)

// kPoolC = true : MaxPool2d((3, 3)) over (channel, time) of |conv|  -> out [B, C/3, T/3]   (AASIST / SincNet)
// kPoolC = false: MaxPool1d(3) over time of |conv|, per channel      -> out [B, C, T/3]     (RawNet2)
// Either way a lane sweeps channel triples with 3 channels x 3 conv times of accumulators; in the
// per-channel form a trailing partial triple clamps its filter rows and skips their stores.
template <bool kPoolC>
__global__ __launch_bounds__(SINC_T3) void sincconv_absmaxpool_kernel(
    const float* __restrict__ x, int64_t len, const float* __restrict__ filters, int channels, int K,
    int mask_lo, int mask_hi, const int32_t* __restrict__ mask_dev, int mask_stride, float* __restrict__ out,
    int64_t T3, int C3) {
  extern __shared__ float s_x[];
  const int b = blockIdx.y;
  if (mask_dev != nullptr) {  // band mask read from device memory (HIP-graph replayable), per utterance
    mask_lo = mask_dev[(int64_t)b * mask_stride];
    mask_hi = mask_dev[(int64_t)b * mask_stride + 1];
  }
  const int64_t t3_0 = (int64_t)blockIdx.x * SINC_T3;
  const int64_t base = 3 * t3_0;                 // first conv time of the block
  const int win = 3 * SINC_T3 + K - 1;
  const float* xb = x + (int64_t)b * len;
  for (int i = threadIdx.x; i < win; i += SINC_T3) {
    int64_t g = base + i;
    s_x[i] = (g < len) ? xb[g] : 0.f;
  }
  __syncthreads();
  const int64_t t3 = t3_0 + threadIdx.x;
  const bool valid = t3 < T3;
  const float* sx = s_x + 3 * threadIdx.x;
  float* ob = out + (int64_t)b * (kPoolC ? C3 : channels) * T3;
  for (int c3 = 0; c3 < C3; ++c3) {
    const int c0 = 3 * c3;
    const float* w0 = filters + (int64_t)c0 * K;
    const float* w1 = filters + (int64_t)min(c0 + 1, channels - 1) * K;
    const float* w2 = filters + (int64_t)min(c0 + 2, channels - 1) * K;
    const bool m0 = (c0 >= mask_lo && c0 < mask_hi);
    const bool m1 = (c0 + 1 >= mask_lo && c0 + 1 < mask_hi);
    const bool m2 = (c0 + 2 >= mask_lo && c0 + 2 < mask_hi);
    float a00 = 0.f, a01 = 0.f, a02 = 0.f;
    float a10 = 0.f, a11 = 0.f, a12 = 0.f;
    float a20 = 0.f, a21 = 0.f, a22 = 0.f;
    float x0 = sx[0], x1 = sx[1];
    for (int k = 0; k < K; ++k) {
      const float x2 = sx[k + 2];
      const float f0 = w0[k], f1 = w1[k], f2 = w2[k];
      a00 = fmaf(f0, x0, a00); a01 = fmaf(f0, x1, a01); a02 = fmaf(f0, x2, a02);
      a10 = fmaf(f1, x0, a10); a11 = fmaf(f1, x1, a11); a12 = fmaf(f1, x2, a12);
      a20 = fmaf(f2, x0, a20); a21 = fmaf(f2, x1, a21); a22 = fmaf(f2, x2, a22);
      x0 = x1;
      x1 = x2;
    }
    float r0 = m0 ? 0.f : fmaxf(fabsf(a00), fmaxf(fabsf(a01), fabsf(a02)));
    float r1 = m1 ? 0.f : fmaxf(fabsf(a10), fmaxf(fabsf(a11), fabsf(a12)));
    float r2 = m2 ? 0.f : fmaxf(fabsf(a20), fmaxf(fabsf(a21), fabsf(a22)));
    if (!valid) continue;
    if (kPoolC) {
      ob[(int64_t)c3 * T3 + t3] = fmaxf(r0, fmaxf(r1, r2));
    } else {
      ob[(int64_t)c0 * T3 + t3] = r0;
      if (c0 + 1 < channels) ob[(int64_t)(c0 + 1) * T3 + t3] = r1;
      if (c0 + 2 < channels) ob[(int64_t)(c0 + 2) * T3 + t3] = r2;
    }
  }
}

// ------------------------------------------------------------------------------------------------------
// The same fused conv + |.| + 3x3 max-pool on the f16 MFMA, for the autocast paths: under the reference's
// torch.cuda.amp.autocast (src/main.py:1049) F.conv1d runs in fp16, so x and the filter bank are rounded to
// fp16 here as well (fp32 accumulation; the pooled output stays fp32). The conv is a GEMM with a Hankel
// operand, conv[c][p] = sum_k W[c][k] x[p + k]: M = channels (70 -> 5 x 16-row fragments), K = taps (129 ->
// 5 x 32, zero-padded), N = positions.
//   * block = 4 waves over SM_RANGE conv positions of one utterance; every wave keeps the whole filter bank as
//     MFMA A fragments in registers (25 x 8 f16, read once per block);
//   * the sample window is staged in LDS as 8 f16 copies shifted by 0..7 samples, so the B fragment of
//     v_mfma_f32_16x16x32_f16 (lane: 8 consecutive samples from p + (lane & 15) + 8 (lane >> 4)) is ONE
//     16-byte aligned ds_read from copy (lane & 7);
//   * per sub-tile of SM_SUB positions (12 fragments, 3 per wave) |conv| goes to an LDS image [70][SM_SUB]
//     fp32 (band-masked channels as 0, the reference zeroes those filter rows), and the 3 x 3 max-pool of the
//     image is stored as coalesced pooled rows.
constexpr int SM_SUB = 192;                  // conv positions per sub-tile (64 pooled)
constexpr int SM_NSUB = 6;
constexpr int SM_RANGE = SM_SUB * SM_NSUB;   // conv positions per block
constexpr int SM_KP = 160;                   // taps padded to 5 x 32
constexpr int SM_XW = SM_RANGE + SM_KP;      // staged samples per copy (multiple of 8)
constexpr int SM_CF = 5;                     // 16-channel fragments (80 >= 70)

typedef __attribute__((ext_vector_type(8))) _Float16 h16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4s;

__global__ __launch_bounds__(256, 2) void sincconv_mfma_kernel(
    const float* __restrict__ x, int64_t len, const float* __restrict__ filters, int channels, int K,
    int mask_lo, int mask_hi, const int32_t* __restrict__ mask_dev, int mask_stride, float* __restrict__ out,
    int64_t T3, int C3) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  _Float16* xc = reinterpret_cast<_Float16*>(smem);                       // [8][SM_XW]
  float* s_c = reinterpret_cast<float*>(smem + 8 * SM_XW * 2);             // [channels][SM_SUB + 4]
  constexpr int CP = SM_SUB + 4;
  const int b = blockIdx.y;
  if (mask_dev != nullptr) {
    mask_lo = mask_dev[(int64_t)b * mask_stride];
    mask_hi = mask_dev[(int64_t)b * mask_stride + 1];
  }
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t p0 = (int64_t)blockIdx.x * SM_RANGE;
  const float* xb = x + (int64_t)b * len;
  // 8 shifted copies: xc[s][i] = x[p0 + i + s] (0 past the utterance). A thread owns one 8-sample group i0 of every
  // copy: it reads the 15 samples p0 + i0 .. + 14 once (float4 loads when aligned) and writes 8 16-byte vectors
  const bool al16 = ((reinterpret_cast<uintptr_t>(xb) | (uintptr_t)(p0 * 4)) & 15) == 0;
  for (int g = tid; g < SM_XW / 8; g += 256) {
    const int64_t base = p0 + 8 * g;
    float v[16];
    if (al16 && base + 16 <= len) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 t = *reinterpret_cast<const float4*>(xb + base + 4 * q);
        v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = base + j < len ? xb[base + j] : 0.f;
    }
#pragma unroll
    for (int sft = 0; sft < 8; ++sft) {
      h16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (_Float16)v[sft + j];
      *reinterpret_cast<h16x8*>(xc + sft * SM_XW + 8 * g) = o;
    }
  }
  // the filter bank, rounded to f16 and zero-padded to [80][SM_KP], staged once per block in the s_c region
  // (coalesced along the taps), then read as A fragments: lane (row = lane & 15, kq = lane >> 4) holds
  // W[16 cf + row][32 ks + 8 kq + j], one 16-byte LDS read each
  _Float16* bank = reinterpret_cast<_Float16*>(s_c);
  for (int q = tid; q < 16 * SM_CF * SM_KP; q += 256) {
    const int c = q / SM_KP, k = q - c * SM_KP;
    bank[q] = (_Float16)((c < channels && k < K) ? filters[(int64_t)c * K + k] : 0.f);
  }
  __syncthreads();
  h16x8 wf[SM_CF][5];
  {
    const int row = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int cf = 0; cf < SM_CF; ++cf)
#pragma unroll
      for (int ks = 0; ks < 5; ++ks)
        wf[cf][ks] = *reinterpret_cast<const h16x8*>(bank + (16 * cf + row) * SM_KP + 32 * ks + 8 * kq);
  }
  __syncthreads();   // the s_c region is the conv image from here on
  float* ob = out + (int64_t)b * C3 * T3;
  const int col = lane & 15, kq = lane >> 4;
  for (int sub = 0; sub < SM_NSUB; ++sub) {
    // 12 position fragments of 16 per sub-tile, 3 per wave
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      const int pl = sub * SM_SUB + (wave * 3 + f) * 16;     // block-local position of the fragment
      f32x4s acc[SM_CF];
#pragma unroll
      for (int cf = 0; cf < SM_CF; ++cf) acc[cf] = f32x4s{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 5; ++ks) {
        const int e = pl + (col & ~7) + 32 * ks + 8 * kq;     // multiple of 8: 16-byte aligned in copy col & 7
        const h16x8 xv = *reinterpret_cast<const h16x8*>(xc + (col & 7) * SM_XW + e);
#pragma unroll
        for (int cf = 0; cf < SM_CF; ++cf)
          acc[cf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[cf][ks], xv, acc[cf], 0, 0, 0);
      }
      // lane holds conv[16 cf + 4 kq + i][pl + col]
      const int pc = pl - sub * SM_SUB + col;
#pragma unroll
      for (int cf = 0; cf < SM_CF; ++cf)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 16 * cf + 4 * kq + i;
          if (c < channels) s_c[c * CP + pc] = (c >= mask_lo && c < mask_hi) ? 0.f : fabsf(acc[cf][i]);
        }
    }
    __syncthreads();
    // 3 x 3 max-pool of the sub-tile: C3 x (SM_SUB / 3) outputs
    const int64_t t3b = (p0 + (int64_t)sub * SM_SUB) / 3;
    for (int q = tid; q < C3 * (SM_SUB / 3); q += 256) {
      const int c3 = q / (SM_SUB / 3), u = q - c3 * (SM_SUB / 3);
      const int64_t t3 = t3b + u;
      if (t3 >= T3) continue;
      const float* r0 = s_c + (3 * c3) * CP + 3 * u;
      float m = fmaxf(fmaxf(r0[0], r0[1]), r0[2]);
      m = fmaxf(m, fmaxf(fmaxf(r0[CP], r0[CP + 1]), r0[CP + 2]));
      m = fmaxf(m, fmaxf(fmaxf(r0[2 * CP], r0[2 * CP + 1]), r0[2 * CP + 2]));
      ob[(int64_t)c3 * T3 + t3] = m;
    }
    __syncthreads();
  }
}

static int sincconv_mfma_launch(const float* x, int64_t batch, int64_t len, const float* filters, int channels,
                                int ksize, int mask_lo, int mask_hi, const int32_t* mask_dev, int mask_stride,
                                float* out, hipStream_t st) {
  const int64_t T = len - ksize + 1, T3 = T / 3;
  const int C3 = channels / 3;
  if (T3 <= 0) return RDX_EINVAL;
  if (ksize > SM_KP || channels > 16 * SM_CF) return RDX_EUNSUPPORTED;
  const size_t img = (size_t)channels * (SM_SUB + 4) * 4, stage = (size_t)16 * SM_CF * SM_KP * 2;   // bank staging
  const size_t smem = (size_t)8 * SM_XW * 2 + (img > stage ? img : stage);
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&sincconv_mfma_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  dim3 grid((unsigned)((3 * T3 + SM_RANGE - 1) / SM_RANGE), (unsigned)batch);
  hipLaunchKernelGGL(sincconv_mfma_kernel, grid, dim3(256), smem, st, x, len, filters, channels, ksize, mask_lo,
                     mask_hi, mask_dev, mask_stride, out, T3, C3);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

}  // namespace rdx

using namespace rdx;

extern "C" int rdx_sincconv_absmaxpool_fwd(const float* x, int64_t batch, int64_t len,
                                           const float* filters, int channels, int ksize,
                                           int mask_lo, int mask_hi, float* out, void* stream) {
  RDX_REQUIRE(x && filters && out && batch > 0 && channels >= 3 && ksize > 0 && len >= ksize);
  RDX_REQUIRE(batch <= 65535);
  const int64_t T = len - ksize + 1;
  const int64_t T3 = T / 3;
  const int C3 = channels / 3;
  if (T3 <= 0) return RDX_EINVAL;
  if (ksize > 4096) return RDX_EUNSUPPORTED;
  dim3 grid((unsigned)((T3 + SINC_T3 - 1) / SINC_T3), (unsigned)batch);
  size_t smem = sizeof(float) * (3 * SINC_T3 + ksize - 1 + 2);
  hipLaunchKernelGGL(sincconv_absmaxpool_kernel<true>, grid, dim3(SINC_T3), smem, as_stream(stream), x, len,
                     filters, channels, ksize, mask_lo, mask_hi, (const int32_t*)nullptr, 0, out, T3, C3);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_sincconv_absmaxpool_fwd_devmask(const float* x, int64_t batch, int64_t len,
                                                   const float* filters, int channels, int ksize,
                                                   const int32_t* mask_dev, int mask_stride, float* out,
                                                   void* stream) {
  RDX_REQUIRE(x && filters && out && mask_dev && batch > 0 && channels >= 3 && ksize > 0 && len >= ksize);
  RDX_REQUIRE(mask_stride == 0 || mask_stride == 2);
  RDX_REQUIRE(batch <= 65535);
  const int64_t T3 = (len - ksize + 1) / 3;
  const int C3 = channels / 3;
  if (T3 <= 0) return RDX_EINVAL;
  if (ksize > 4096) return RDX_EUNSUPPORTED;
  dim3 grid((unsigned)((T3 + SINC_T3 - 1) / SINC_T3), (unsigned)batch);
  size_t smem = sizeof(float) * (3 * SINC_T3 + ksize - 1 + 2);
  hipLaunchKernelGGL(sincconv_absmaxpool_kernel<true>, grid, dim3(SINC_T3), smem, as_stream(stream), x, len,
                     filters, channels, ksize, 0, 0, mask_dev, mask_stride, out, T3, C3);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

// RawNet2 front end: |SincConv| then MaxPool1d(3) over time, channel by channel (no channel pooling).
//   reference models/RawNet2Spoof.py:95-103 (F.conv1d with the sinc bank) and :244-245
//   (F.max_pool1d(torch.abs(x), 3)).  x [B, len] -> out [B, channels, (len-ksize+1)/3].
extern "C" int rdx_sincconv_abspool1d_fwd(const float* x, int64_t batch, int64_t len, const float* filters,
                                          int channels, int ksize, int mask_lo, int mask_hi, float* out,
                                          void* stream) {
  RDX_REQUIRE(x && filters && out && batch > 0 && channels >= 1 && ksize > 0 && len >= ksize);
  RDX_REQUIRE(batch <= 65535);
  const int64_t T3 = (len - ksize + 1) / 3;
  const int C3 = (channels + 2) / 3;
  if (T3 <= 0) return RDX_EINVAL;
  if (ksize > 4096) return RDX_EUNSUPPORTED;
  dim3 grid((unsigned)((T3 + SINC_T3 - 1) / SINC_T3), (unsigned)batch);
  size_t smem = sizeof(float) * (3 * SINC_T3 + ksize - 1 + 2);
  hipLaunchKernelGGL(sincconv_absmaxpool_kernel<false>, grid, dim3(SINC_T3), smem, as_stream(stream), x, len,
                     filters, channels, ksize, mask_lo, mask_hi, (const int32_t*)nullptr, 0, out, T3, C3);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

// f16 MFMA form (autocast paths; see sincconv_mfma_kernel): same output as rdx_sincconv_absmaxpool_fwd[_devmask]
// with x and the bank rounded to fp16. mask_dev null: the band mask [mask_lo, mask_hi); else mask_dev as in
// rdx_sincconv_absmaxpool_fwd_devmask. ksize <= 160, channels <= 80.
extern "C" int rdx_sincconv_absmaxpool_f16mfma(const float* x, int64_t batch, int64_t len, const float* filters,
                                               int channels, int ksize, int mask_lo, int mask_hi,
                                               const int32_t* mask_dev, int mask_stride, float* out, void* stream) {
  RDX_REQUIRE(x && filters && out && batch > 0 && channels >= 3 && ksize > 0 && len >= ksize);
  RDX_REQUIRE(batch <= 65535 && (mask_stride == 0 || mask_stride == 2));
  return sincconv_mfma_launch(x, batch, len, filters, channels, ksize, mask_lo, mask_hi, mask_dev, mask_stride, out,
                              as_stream(stream));
}
