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
