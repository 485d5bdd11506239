// SincNet residual stack, NHWC (channels_last) fused epilogues for gfx950.
//
// Residual_block.forward (src/models/DualStreamSEMamba.py:182-200) with frozen batch-norm
// (freeze_bn, src/main.py:44-51,1016-1018):
//     out = selu(bn2(conv1(x)));  out = conv2(out);  out = maxpool_(1,3)(out + identity)
// Two fused passes replace torch's bias-add / batch_norm / selu / add / max_pool2d kernels and the
// three separate bias-gradient reductions:
//   bnselu   y = selu(((c + cb) - mean) * invstd * w + b)           (conv1 bias cb folded in)
//            bwd: dc = dy * selu'(u) * invstd * w, and per channel  sum(dc) (= d cb),
//                 sum(dy*selu'(u) * xhat) (= d w),  sum(dy*selu'(u)) (= d b)
//   tail     y[n,h,wo,c] = max_k (a + id + bias)[n,h,3wo+k,c]  (first maximum wins, NaN propagates,
//            as torch's max_pool2d), argmax kept as one byte per output element
//            bwd: dx scattered to the argmax (zero elsewhere, incl. the W % 3 tail), sum(dy) (= d bias)
// Layout: activations [npix = N*H*W, C] row-major (NHWC), C % 8 == 0; every lane owns 8 consecutive
// channels (one 16-byte bf16 vector), so per-channel sums stay in registers across the grid-stride
// loop and are reduced once per block (LDS) and once per grid (fp32 atomics into a zeroed buffer).
#include "common.h"

namespace rdx {

constexpr float SELU_ALPHA = 1.6732632423543772848170429916717f;
constexpr float SELU_SCALE = 1.0507009873554804934193349852946f;
constexpr int SN_THREADS = 256;
constexpr int SN_VEC = 8;

template <typename T> struct Vec8;
template <> struct Vec8<hst> {
  using raw = uint4;  // 8 x bf16
  static __device__ __forceinline__ void load(const hst* p, float* v) {
    uint4 r = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = hlo(w[i]);
      v[2 * i + 1] = hhi(w[i]);
    }
  }
  static __device__ __forceinline__ void store(hst* p, const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t lo = hbits_of(f2h(v[2 * i]));
      const uint32_t hi = hbits_of(f2h(v[2 * i + 1]));
      w[i] = lo | (hi << 16);
    }
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float* v) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

__device__ __forceinline__ float selu_f(float u) { return SELU_SCALE * (u > 0.f ? u : SELU_ALPHA * expm1f(u)); }
// selu with exp(u) - 1 on the hardware exp for the forward-only passes whose output is rounded to bf16 (b0_fwd):
// the absolute error of exp(u) - 1 near u = 0 (~1e-7) is far below a bf16 ulp of the result
__device__ __forceinline__ float selu_fast(float u) {
  return SELU_SCALE * (u > 0.f ? u : SELU_ALPHA * (__expf(u) - 1.0f));
}
__device__ __forceinline__ float selu_d(float u) { return u > 0.f ? SELU_SCALE : SELU_SCALE * SELU_ALPHA * __expf(u); }

// per-channel constants of the frozen BN with the conv bias folded: zc = c + cb - mean,
// xhat = zc * invstd, u = zc * s + t with s = invstd * w, t = b
struct BnAffine {
  float s[SN_VEC], t[SN_VEC], cb[SN_VEC], m[SN_VEC], is[SN_VEC];
};
__device__ __forceinline__ void bn_affine(BnAffine& a, int c0, const float* cb, const float* mean, const float* invstd,
                                          const float* w, const float* b) {
#pragma unroll
  for (int i = 0; i < SN_VEC; ++i) {
    const int c = c0 + i;
    a.cb[i] = cb[c];
    a.m[i] = mean[c];
    a.is[i] = invstd[c];
    a.s[i] = invstd[c] * w[c];
    a.t[i] = b[c];
  }
}

template <typename T>
__global__ __launch_bounds__(SN_THREADS) void bnselu_fwd_kernel(const T* __restrict__ c, const float* __restrict__ cb,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ invstd,
                                                                 const float* __restrict__ w,
                                                                 const float* __restrict__ b, T* __restrict__ y,
                                                                 int64_t nvec, int cvec) {
  const int64_t stride = (int64_t)gridDim.x * SN_THREADS;  // multiple of cvec: channel group fixed per lane
  int64_t i = (int64_t)blockIdx.x * SN_THREADS + threadIdx.x;
  if (i >= nvec) return;
  BnAffine a;
  bn_affine(a, (int)(i % cvec) * SN_VEC, cb, mean, invstd, w, b);
  for (; i < nvec; i += stride) {
    float v[SN_VEC];
    Vec8<T>::load(c + i * SN_VEC, v);
#pragma unroll
    for (int k = 0; k < SN_VEC; ++k) v[k] = selu_f(fmaf((v[k] + a.cb[k]) - a.m[k], a.s[k], a.t[k]));
    Vec8<T>::store(y + i * SN_VEC, v);
  }
}

// block-level per-channel reduction of NS sums per lane-channel, then one atomic per (sum, channel)
template <int NS>
__device__ __forceinline__ void flush_channel_sums(float (*acc)[SN_VEC], int c0, bool has, int C,
                                                   float* __restrict__ sums) {
  __shared__ float red[NS * 512];  // NS x C (C <= 512)
  for (int i = threadIdx.x; i < NS * C; i += SN_THREADS) red[i] = 0.f;
  __syncthreads();
  if (has) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int k = 0; k < SN_VEC; ++k) atomicAdd(&red[s * C + c0 + k], acc[s][k]);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NS * C; i += SN_THREADS) atomicAdd(&sums[i], red[i]);
}

template <typename T>
__global__ __launch_bounds__(SN_THREADS) void bnselu_bwd_kernel(
    const T* __restrict__ c, const T* __restrict__ dy, const float* __restrict__ cb, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ w, const float* __restrict__ b, T* __restrict__ dc,
    float* __restrict__ sums, int64_t nvec, int cvec, int C) {
  const int64_t stride = (int64_t)gridDim.x * SN_THREADS;
  int64_t i = (int64_t)blockIdx.x * SN_THREADS + threadIdx.x;
  const bool has = i < nvec;
  const int c0 = (int)(i % cvec) * SN_VEC;
  float acc[3][SN_VEC];
#pragma unroll
  for (int k = 0; k < SN_VEC; ++k) acc[0][k] = acc[1][k] = acc[2][k] = 0.f;
  if (has) {
    BnAffine a;
    bn_affine(a, c0, cb, mean, invstd, w, b);
    for (; i < nvec; i += stride) {
      float v[SN_VEC], g[SN_VEC];
      Vec8<T>::load(c + i * SN_VEC, v);
      Vec8<T>::load(dy + i * SN_VEC, g);
#pragma unroll
      for (int k = 0; k < SN_VEC; ++k) {
        const float zc = (v[k] + a.cb[k]) - a.m[k];
        const float xhat = zc * a.is[k];
        const float u = fmaf(zc, a.s[k], a.t[k]);
        const float du = g[k] * selu_d(u);
        const float dz = du * a.s[k];
        acc[0][k] += dz;
        acc[1][k] = fmaf(du, xhat, acc[1][k]);
        acc[2][k] += du;
        v[k] = dz;
      }
      Vec8<T>::store(dc + i * SN_VEC, v);
    }
  }
  flush_channel_sums<3>(acc, c0, has, C, sums);
}

template <typename T>
__global__ __launch_bounds__(SN_THREADS) void tail_fwd_kernel(const T* __restrict__ a, const T* __restrict__ id,
                                                              const float* __restrict__ bias, T* __restrict__ y,
                                                              uint8_t* __restrict__ arg, int64_t nout, int Wo, int W,
                                                              int cvec) {
  const int64_t stride = (int64_t)gridDim.x * SN_THREADS;
  int64_t i = (int64_t)blockIdx.x * SN_THREADS + threadIdx.x;
  if (i >= nout) return;
  const int c0 = (int)(i % cvec) * SN_VEC;
  float bs[SN_VEC];
#pragma unroll
  for (int k = 0; k < SN_VEC; ++k) bs[k] = bias[c0 + k];
  for (; i < nout; i += stride) {
    const int64_t pix = i / cvec;                // output pixel (n, h, wo)
    const int64_t row = pix / Wo;                // (n, h)
    const int wo = (int)(pix - row * Wo);
    const int64_t in0 = ((row * W + 3 * wo) * cvec + (i % cvec)) * SN_VEC;
    float best[SN_VEC];
    uint8_t bi[SN_VEC];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float v[SN_VEC], u[SN_VEC];
      Vec8<T>::load(a + in0 + (int64_t)j * cvec * SN_VEC, v);
      Vec8<T>::load(id + in0 + (int64_t)j * cvec * SN_VEC, u);
#pragma unroll
      for (int k = 0; k < SN_VEC; ++k) {
        const float s = v[k] + u[k] + bs[k];
        if (j == 0 || s > best[k] || s != s) {  // torch max_pool2d: val > max || isnan(val)
          best[k] = s;
          bi[k] = (uint8_t)j;
        }
      }
    }
    Vec8<T>::store(y + i * SN_VEC, best);
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(arg + i * SN_VEC) = packed;
  }
}

template <typename T>
__global__ __launch_bounds__(SN_THREADS) void tail_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                              T* __restrict__ dx, float* __restrict__ sums,
                                                              int64_t nout, int Wo, int W, int cvec, int C) {
  const int64_t stride = (int64_t)gridDim.x * SN_THREADS;
  int64_t i = (int64_t)blockIdx.x * SN_THREADS + threadIdx.x;
  const bool has = i < nout;
  const int c0 = (int)(i % cvec) * SN_VEC;
  float acc[1][SN_VEC];
#pragma unroll
  for (int k = 0; k < SN_VEC; ++k) acc[0][k] = 0.f;
  for (; i < nout; i += stride) {
    const int64_t pix = i / cvec;
    const int64_t row = pix / Wo;
    const int wo = (int)(pix - row * Wo);
    const int64_t in0 = ((row * W + 3 * wo) * cvec + (i % cvec)) * SN_VEC;
    float g[SN_VEC];
    Vec8<T>::load(dy + i * SN_VEC, g);
    const uint2 packed = *reinterpret_cast<const uint2*>(arg + i * SN_VEC);
    uint8_t bi[SN_VEC];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bi[k] = (packed.x >> (8 * k)) & 0xff;
      bi[4 + k] = (packed.y >> (8 * k)) & 0xff;
    }
#pragma unroll
    for (int k = 0; k < SN_VEC; ++k) acc[0][k] += g[k];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float o[SN_VEC];
#pragma unroll
      for (int k = 0; k < SN_VEC; ++k) o[k] = (bi[k] == j) ? g[k] : 0.f;
      Vec8<T>::store(dx + in0 + (int64_t)j * cvec * SN_VEC, o);
    }
    if (wo == Wo - 1) {  // columns 3*Wo .. W-1 are dropped by the pool: zero gradient
      float z[SN_VEC];
#pragma unroll
      for (int k = 0; k < SN_VEC; ++k) z[k] = 0.f;
      for (int wc = 3 * Wo; wc < W; ++wc)
        Vec8<T>::store(dx + ((row * W + wc) * cvec + (i % cvec)) * SN_VEC, z);
    }
  }
  flush_channel_sums<1>(acc, c0, has, C, sums);
}

// Block 0 of the residual stack (the only block with one input channel): the input gradient and the
// weight gradients of conv1 (2 x 3, padding (1, 1)) and conv_downsample (1 x 3, padding (0, 1)) in ONE
// pass over the two output gradients, instead of MIOpen's two backward-data convolutions with a single
// output channel (an implicit GEMM with N = 1, ~0.5 ms each at B = 8) and two weight-gradient passes:
//   dx[n,h,w]      = sum_c [ sum_{kh,kw} dc[n, h+1-kh, w+1-kw, c] W1[c,kh,kw] + sum_kw di[n, h, w+1-kw, c] Wd[c,kw] ]
//   dW1[c,kh,kw]  += x[n,h,w] dc[n, h+1-kh, w+1-kw, c],    dWd[c,kw] += x[n,h,w] di[n, h, w+1-kw, c]
// Output columns outside [0, W) are the zero padding; conv1's output has H + 1 rows, so row h+1-kh always
// exists. A work unit is one utterance x one strip of 64 columns, walked top-down: conv1 output row h+1
// is loaded once (as the kh = 0 taps of input row h) and kept in registers as the kh = 1 taps of row
// h+1, so every dc row comes from HBM once. Lane = (column, 4 channels): the eight lanes of a column add
// their dx partials with three xor-shuffles; the three column taps are loaded from clamped addresses and
// zeroed by a select (no divergent branch between the loads). Each lane's 36 weight-gradient sums are
// reduced per block in LDS and written as one partial row per block (the caller sums the rows: no
// same-address atomics across blocks); blocks without a unit write zeros.
constexpr int B0_C = 32;
constexpr int B0_TAPS = 9;  // conv1 taps kh * 3 + kw, then conv_downsample taps 6 + kw
constexpr int B0_BLOCKS = 4096;
constexpr int B0_CPL = 4;                         // channels per lane
constexpr int B0_LPC = B0_C / B0_CPL;             // lanes per column
constexpr int B0_STRIP = SN_THREADS / B0_LPC;     // columns per unit

__device__ __forceinline__ uint2 b0_tap(const hst* __restrict__ row, int wo, int W, int cg) {
  const int wc = wo < 0 ? 0 : (wo >= W ? W - 1 : wo);
  const uint2 v = *reinterpret_cast<const uint2*>(row + (int64_t)wc * B0_C + B0_CPL * cg);
  const bool ok = wo >= 0 && wo < W;
  return ok ? v : make_uint2(0u, 0u);
}

__device__ __forceinline__ float b0_lo(unsigned u) { return hlo(u); }
__device__ __forceinline__ float b0_hi(unsigned u) { return hhi(u); }

// pdx += sum_k v[k] wt[k][t];  acc[k][t] += xq v[k]
__device__ __forceinline__ void b0_fma(const uint2 v, int t, float xq, const float (&wt)[B0_CPL][B0_TAPS],
                                       float (&acc)[B0_CPL][B0_TAPS], float& pdx) {
  const unsigned u[2] = {v.x, v.y};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float a = b0_lo(u[j]), b = b0_hi(u[j]);
    pdx = fmaf(a, wt[2 * j][t], pdx);
    pdx = fmaf(b, wt[2 * j + 1][t], pdx);
    acc[2 * j][t] = fmaf(xq, a, acc[2 * j][t]);
    acc[2 * j + 1][t] = fmaf(xq, b, acc[2 * j + 1][t]);
  }
}

__global__ __launch_bounds__(SN_THREADS) void b0_bwd_kernel(const hst* __restrict__ x,
                                                            const hst* __restrict__ dc,
                                                            const hst* __restrict__ di,
                                                            const float* __restrict__ w1, const float* __restrict__ wd,
                                                            float* __restrict__ dx, float* __restrict__ part, int N,
                                                            int H, int W) {
  __shared__ float red[B0_C * B0_TAPS];
  for (int i = threadIdx.x; i < B0_C * B0_TAPS; i += SN_THREADS) red[i] = 0.f;
  const int cg = threadIdx.x & (B0_LPC - 1);  // channels 4 cg .. 4 cg + 3
  float wt[B0_CPL][B0_TAPS], acc[B0_CPL][B0_TAPS];
#pragma unroll
  for (int k = 0; k < B0_CPL; ++k) {
    const int c = B0_CPL * cg + k;
#pragma unroll
    for (int t = 0; t < 6; ++t) wt[k][t] = w1[c * 6 + t];
#pragma unroll
    for (int t = 0; t < 3; ++t) wt[k][6 + t] = wd[c * 3 + t];
#pragma unroll
    for (int t = 0; t < B0_TAPS; ++t) acc[k][t] = 0.f;
  }
  const int strips = (W + B0_STRIP - 1) / B0_STRIP;
  const int units = N * strips;
  for (int u = blockIdx.x; u < units; u += gridDim.x) {
    const int n = u / strips;
    const int w = (u - n * strips) * B0_STRIP + threadIdx.x / B0_LPC;
    const bool live = w < W;
    const int wl = live ? w : W - 1;  // dead lanes load a valid column and contribute nothing
    const hst* dcn = dc + (int64_t)n * (H + 1) * W * B0_C;
    const hst* din = di + (int64_t)n * H * W * B0_C;
    const int64_t xrow0 = (int64_t)n * H * W;
    uint2 cur[3];  // conv1 output row h: the kh = 1 taps of input row h
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) cur[kw] = b0_tap(dcn, wl + 1 - kw, W, cg);
    for (int h = 0; h < H; ++h) {
      uint2 nxt[3], dv[3];
      const hst* rn = dcn + (int64_t)(h + 1) * W * B0_C;
      const hst* ri = din + (int64_t)h * W * B0_C;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) nxt[kw] = b0_tap(rn, wl + 1 - kw, W, cg);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) dv[kw] = b0_tap(ri, wl + 1 - kw, W, cg);
      const float xq = live ? h2f(x[xrow0 + (int64_t)h * W + wl]) : 0.f;
      float pdx = 0.f;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        b0_fma(nxt[kw], kw, xq, wt, acc, pdx);     // kh = 0: conv1 output row h + 1
        b0_fma(cur[kw], 3 + kw, xq, wt, acc, pdx); // kh = 1: conv1 output row h
        b0_fma(dv[kw], 6 + kw, xq, wt, acc, pdx);  // conv_downsample output row h
      }
      pdx += __shfl_xor(pdx, 1, 64);
      pdx += __shfl_xor(pdx, 2, 64);
      pdx += __shfl_xor(pdx, 4, 64);
      if (cg == 0 && live) dx[xrow0 + (int64_t)h * W + w] = pdx;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) cur[kw] = nxt[kw];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < B0_CPL; ++k)
#pragma unroll
    for (int t = 0; t < B0_TAPS; ++t) atomicAdd(&red[(B0_CPL * cg + k) * B0_TAPS + t], acc[k][t]);
  __syncthreads();
  for (int i = threadIdx.x; i < B0_C * B0_TAPS; i += SN_THREADS)
    part[(int64_t)blockIdx.x * B0_C * B0_TAPS + i] = red[i];
}

inline unsigned sn_grid(int64_t n, int cvec) {
  // enough blocks to fill 256 CUs several times; keeps gridDim*256 a multiple of cvec (256 % cvec == 0)
  int64_t blocks = (n + SN_THREADS - 1) / SN_THREADS;
  if (blocks > 4096) blocks = 4096;
  return (unsigned)(blocks > 0 ? blocks : 1);
}

}  // namespace rdx

using namespace rdx;

#define SN_DISPATCH(dtype, ...)                                     \
  do {                                                              \
    if ((dtype) == RDX_F32) {                                       \
      using T = float;                                              \
      __VA_ARGS__;                                                  \
    } else if ((dtype) == RDX_BF16) {                               \
      using T = hst;                                     \
      __VA_ARGS__;                                                  \
    } else {                                                        \
      return RDX_EINVAL;                                            \
    }                                                               \
  } while (0)

static bool sn_shape_ok(int64_t npix, int C) { return npix > 0 && C > 0 && C % SN_VEC == 0 && C <= 512 && 256 % (C / SN_VEC) == 0; }

extern "C" int rdx_bnselu_fwd(int dtype, const void* c, const float* conv_bias, const float* mean,
                              const float* invstd, const float* weight, const float* bias, void* y,
                              int64_t npix, int C, void* stream) {
  RDX_REQUIRE(c && conv_bias && mean && invstd && weight && bias && y);
  if (!sn_shape_ok(npix, C)) return RDX_EUNSUPPORTED;
  const int cvec = C / SN_VEC;
  const int64_t nvec = npix * cvec;
  SN_DISPATCH(dtype, hipLaunchKernelGGL(bnselu_fwd_kernel<T>, dim3(sn_grid(nvec, cvec)), dim3(SN_THREADS), 0,
                                        as_stream(stream), (const T*)c, conv_bias, mean, invstd, weight, bias, (T*)y,
                                        nvec, cvec));
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_bnselu_bwd(int dtype, const void* c, const void* dy, const float* conv_bias, const float* mean,
                              const float* invstd, const float* weight, const float* bias, void* dc, float* sums,
                              int64_t npix, int C, void* stream) {
  RDX_REQUIRE(c && dy && conv_bias && mean && invstd && weight && bias && dc && sums);
  if (!sn_shape_ok(npix, C)) return RDX_EUNSUPPORTED;
  const int cvec = C / SN_VEC;
  const int64_t nvec = npix * cvec;
  SN_DISPATCH(dtype, hipLaunchKernelGGL(bnselu_bwd_kernel<T>, dim3(sn_grid(nvec, cvec)), dim3(SN_THREADS), 0,
                                        as_stream(stream), (const T*)c, (const T*)dy, conv_bias, mean, invstd, weight,
                                        bias, (T*)dc, sums, nvec, cvec, C));
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_res_tail_fwd(int dtype, const void* a, const void* identity, const float* bias, void* y,
                                uint8_t* argmax, int64_t rows, int W, int C, void* stream) {
  RDX_REQUIRE(a && identity && bias && y && argmax && rows > 0 && W >= 3);
  if (!sn_shape_ok(rows * W, C)) return RDX_EUNSUPPORTED;
  const int cvec = C / SN_VEC;
  const int Wo = W / 3;
  const int64_t nout = rows * Wo * cvec;
  SN_DISPATCH(dtype, hipLaunchKernelGGL(tail_fwd_kernel<T>, dim3(sn_grid(nout, cvec)), dim3(SN_THREADS), 0,
                                        as_stream(stream), (const T*)a, (const T*)identity, bias, (T*)y, argmax, nout,
                                        Wo, W, cvec));
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_res_tail_bwd(int dtype, const void* dy, const uint8_t* argmax, void* dx, float* dbias,
                                int64_t rows, int W, int C, void* stream) {
  RDX_REQUIRE(dy && argmax && dx && dbias && rows > 0 && W >= 3);
  if (!sn_shape_ok(rows * W, C)) return RDX_EUNSUPPORTED;
  const int cvec = C / SN_VEC;
  const int Wo = W / 3;
  const int64_t nout = rows * Wo * cvec;
  SN_DISPATCH(dtype, hipLaunchKernelGGL(tail_bwd_kernel<T>, dim3(sn_grid(nout, cvec)), dim3(SN_THREADS), 0,
                                        as_stream(stream), (const T*)dy, argmax, (T*)dx, dbias, nout, Wo, W, cvec, C));
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

// SincNet block 0 forward (one input channel, 32 output channels): conv1 (2 x 3, padding (1, 1)) and
// conv_downsample (1 x 3, padding (0, 1)) of the bf16 input with bf16-valued weights and fp32 accumulation (what
// autocast runs), plus conv1's frozen BN + SELU on the bf16-rounded conv1 output (bnselu_fwd_kernel's
// arithmetic, exp(u) - 1 on the hardware exp). Lane = (8-pixel run, 8-channel group): the lane's 104 weight /
// BN constants are loaded once into registers, and it walks B0F_RUN consecutive conv1 output pixels of a row
// with a sliding 2 x 3 input window (two new input values per pixel; index math once per run). Each store
// instruction of a wave writes 16 runs' 64-byte NHWC rows: c (pre-activation, kept for the backward),
// y = selu(bn(c + cb)) and, for h < H, idn (the bottom row of conv1's window is the downsample's window).
// Replaces two MIOpen convolutions (each with its own output-zeroing pass) and the separate BN + SELU pass.
constexpr int B0F_RUN = 8;
__device__ __forceinline__ float b0_x(const hst* x, int n, int r, int cc, int H, int W) {
  return (r >= 0 && r < H && cc >= 0 && cc < W) ? h2f(x[((int64_t)n * H + r) * W + cc]) : 0.f;
}
__global__ __launch_bounds__(SN_THREADS) void b0_fwd_kernel(
    const hst* __restrict__ x, const float* __restrict__ w1, const float* __restrict__ wd,
    const float* __restrict__ bn, hst* __restrict__ c, hst* __restrict__ y,
    hst* __restrict__ idn, int N, int H, int W) {
  const int g = threadIdx.x & 3;
  float t1[SN_VEC][6], td[SN_VEC][3], cb[SN_VEC], mu[SN_VEC], sc[SN_VEC], sh[SN_VEC];
#pragma unroll
  for (int k = 0; k < SN_VEC; ++k) {
    const int co = g * SN_VEC + k;
#pragma unroll
    for (int j = 0; j < 6; ++j) t1[k][j] = w1[co * 6 + j];
#pragma unroll
    for (int j = 0; j < 3; ++j) td[k][j] = wd[co * 3 + j];
    cb[k] = bn[co];
    mu[k] = bn[B0_C + co];
    sc[k] = bn[2 * B0_C + co];
    sh[k] = bn[3 * B0_C + co];
  }
  const int runs_per_row = (W + B0F_RUN - 1) / B0F_RUN;
  const int run = blockIdx.x * (SN_THREADS / 4) + (threadIdx.x >> 2);   // over N * (H + 1) * runs_per_row
  const int nrow = run / runs_per_row;
  if (nrow >= N * (H + 1)) return;
  const int n = nrow / (H + 1), h = nrow - n * (H + 1);
  const int w0 = (run - nrow * runs_per_row) * B0F_RUN;
  float v0[3], v1[3];   // input rows h - 1 and h, columns w - 1 .. w + 1
#pragma unroll
  for (int kw = 0; kw < 3; ++kw) {
    v0[kw] = b0_x(x, n, h - 1, w0 - 1 + kw, H, W);
    v1[kw] = b0_x(x, n, h, w0 - 1 + kw, H, W);
  }
  const int64_t pbase = (int64_t)nrow * W;
  const int64_t ibase = ((int64_t)n * H + h) * W;
#pragma unroll
  for (int st = 0; st < B0F_RUN; ++st) {
    const int w = w0 + st;
    if (w >= W) break;
    float cv[SN_VEC], yv[SN_VEC], iv[SN_VEC];
#pragma unroll
    for (int k = 0; k < SN_VEC; ++k) {
      float acc = v0[0] * t1[k][0];
      acc = fmaf(v0[1], t1[k][1], acc);
      acc = fmaf(v0[2], t1[k][2], acc);
      acc = fmaf(v1[0], t1[k][3], acc);
      acc = fmaf(v1[1], t1[k][4], acc);
      acc = fmaf(v1[2], t1[k][5], acc);
      cv[k] = h2f(f2h(acc));
      yv[k] = selu_fast(fmaf((cv[k] + cb[k]) - mu[k], sc[k], sh[k]));
      iv[k] = fmaf(v1[0], td[k][0], fmaf(v1[1], td[k][1], v1[2] * td[k][2]));
    }
    Vec8<hst>::store(c + (pbase + w) * B0_C + g * SN_VEC, cv);
    Vec8<hst>::store(y + (pbase + w) * B0_C + g * SN_VEC, yv);
    if (h < H) Vec8<hst>::store(idn + (ibase + w) * B0_C + g * SN_VEC, iv);
    v0[0] = v0[1]; v0[1] = v0[2]; v0[2] = b0_x(x, n, h - 1, w + 2, H, W);
    v1[0] = v1[1]; v1[1] = v1[2]; v1[2] = b0_x(x, n, h, w + 2, H, W);
  }
}

extern "C" int rdx_sincnet_b0_fwd(const void* x, const float* w1, const float* wd, const float* bn, void* c, void* y,
                                  void* idn, int N, int H, int W, int C, void* stream) {
  RDX_REQUIRE(x && w1 && wd && bn && c && y && idn && N > 0 && H > 0 && W > 0);
  if (C != B0_C) return RDX_EUNSUPPORTED;
  const int64_t nruns = (int64_t)N * (H + 1) * ((W + B0F_RUN - 1) / B0F_RUN);
  RDX_REQUIRE(nruns * 4 < ((int64_t)1 << 31));
  hipLaunchKernelGGL(b0_fwd_kernel, dim3((unsigned)((nruns + SN_THREADS / 4 - 1) / (SN_THREADS / 4))), dim3(SN_THREADS),
                     0, as_stream(stream), (const hst*)x, w1, wd, bn, (hst*)c, (hst*)y,
                     (hst*)idn, N, H, W);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_sincnet_b0_nblk(int64_t npix) {
  // about one block per (utterance, 32-column strip) unit at the bench shapes; the kernel grid-strides over units
  const int64_t b = (npix + B0_STRIP - 1) / B0_STRIP;
  return (int)(b < 1 ? 1 : (b > B0_BLOCKS ? B0_BLOCKS : b));
}

extern "C" int rdx_sincnet_b0_bwd(const void* x, const void* dc, const void* di, const float* w1, const float* wd,
                                  float* dx, float* part, int N, int H, int W, int C, void* stream) {
  RDX_REQUIRE(x && dc && di && w1 && wd && dx && part && N > 0 && H > 0 && W > 0);
  RDX_REQUIRE(((uintptr_t)dc & 15) == 0 && ((uintptr_t)di & 15) == 0);
  if (C != B0_C) return RDX_EUNSUPPORTED;
  const int64_t npix = (int64_t)N * H * W;
  hipLaunchKernelGGL(b0_bwd_kernel, dim3(rdx_sincnet_b0_nblk(npix)), dim3(SN_THREADS), 0, as_stream(stream),
                     (const hst*)x, (const hst*)dc, (const hst*)di, w1, wd, dx, part,
                     N, H, W);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
