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
template <> struct Vec8<__hip_bfloat16> {
  using raw = uint4;  // 8 x bf16
  static __device__ __forceinline__ void load(const __hip_bfloat16* p, float* v) {
    uint4 r = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void store(__hip_bfloat16* p, const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t lo = __bfloat16_as_ushort(__float2bfloat16(v[2 * i]));
      const uint32_t hi = __bfloat16_as_ushort(__float2bfloat16(v[2 * i + 1]));
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
// exists. Lane = (input pixel, 8 channels): the four lanes of a pixel add their dx partials with two
// xor-shuffles; each lane's 72 weight-gradient sums are reduced per block in LDS and written as one partial
// row per block (the caller sums the rows: no same-address atomics across blocks).
constexpr int B0_C = 32;
constexpr int B0_TAPS = 9;  // conv1 taps kh * 3 + kw, then conv_downsample taps 6 + kw
constexpr int B0_BLOCKS = 1024;

__global__ __launch_bounds__(SN_THREADS) void b0_bwd_kernel(const __hip_bfloat16* __restrict__ x,
                                                            const __hip_bfloat16* __restrict__ dc,
                                                            const __hip_bfloat16* __restrict__ di,
                                                            const float* __restrict__ w1, const float* __restrict__ wd,
                                                            float* __restrict__ dx, float* __restrict__ part,
                                                            int64_t npix, int H, int W) {
  __shared__ float red[B0_C * B0_TAPS];
  for (int i = threadIdx.x; i < B0_C * B0_TAPS; i += SN_THREADS) red[i] = 0.f;
  const int cg = threadIdx.x & 3;  // channels 8 cg .. 8 cg + 7
  float wt[SN_VEC][B0_TAPS], acc[SN_VEC][B0_TAPS];
#pragma unroll
  for (int k = 0; k < SN_VEC; ++k) {
    const int c = SN_VEC * cg + k;
#pragma unroll
    for (int t = 0; t < 6; ++t) wt[k][t] = w1[c * 6 + t];
#pragma unroll
    for (int t = 0; t < 3; ++t) wt[k][6 + t] = wd[c * 3 + t];
#pragma unroll
    for (int t = 0; t < B0_TAPS; ++t) acc[k][t] = 0.f;
  }
  const int64_t step = (int64_t)gridDim.x * (SN_THREADS / 4);
  for (int64_t q = (int64_t)blockIdx.x * (SN_THREADS / 4) + (threadIdx.x >> 2); q < npix; q += step) {
    const int64_t nh = q / W;  // n * H + h
    const int w = (int)(q - nh * W);
    const int64_t n = nh / H;
    const float xq = __bfloat162float(x[q]);
    float pdx = 0.f;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int64_t orow = (nh + n + 1 - kh) * W;  // conv1 output row (n, h + 1 - kh) of H + 1
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int wo = w + 1 - kw;
        if (wo < 0 || wo >= W) continue;
        float v[SN_VEC];
        Vec8<__hip_bfloat16>::load(dc + (orow + wo) * B0_C + SN_VEC * cg, v);
#pragma unroll
        for (int k = 0; k < SN_VEC; ++k) {
          pdx = fmaf(v[k], wt[k][kh * 3 + kw], pdx);
          acc[k][kh * 3 + kw] = fmaf(xq, v[k], acc[k][kh * 3 + kw]);
        }
      }
    }
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int wo = w + 1 - kw;
      if (wo < 0 || wo >= W) continue;
      float v[SN_VEC];
      Vec8<__hip_bfloat16>::load(di + (nh * W + wo) * B0_C + SN_VEC * cg, v);
#pragma unroll
      for (int k = 0; k < SN_VEC; ++k) {
        pdx = fmaf(v[k], wt[k][6 + kw], pdx);
        acc[k][6 + kw] = fmaf(xq, v[k], acc[k][6 + kw]);
      }
    }
    pdx += __shfl_xor(pdx, 1, 64);
    pdx += __shfl_xor(pdx, 2, 64);
    if (cg == 0) dx[q] = pdx;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < SN_VEC; ++k)
#pragma unroll
    for (int t = 0; t < B0_TAPS; ++t) atomicAdd(&red[(SN_VEC * cg + k) * B0_TAPS + t], acc[k][t]);
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
      using T = __hip_bfloat16;                                     \
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

extern "C" int rdx_sincnet_b0_nblk(int64_t npix) {
  const int64_t b = (npix + SN_THREADS / 4 - 1) / (SN_THREADS / 4);
  return (int)(b < 1 ? 1 : (b > B0_BLOCKS ? B0_BLOCKS : b));
}

extern "C" int rdx_sincnet_b0_bwd(const void* x, const void* dc, const void* di, const float* w1, const float* wd,
                                  float* dx, float* part, int N, int H, int W, int C, void* stream) {
  RDX_REQUIRE(x && dc && di && w1 && wd && dx && part && N > 0 && H > 0 && W > 0);
  RDX_REQUIRE(((uintptr_t)dc & 15) == 0 && ((uintptr_t)di & 15) == 0);
  if (C != B0_C) return RDX_EUNSUPPORTED;
  const int64_t npix = (int64_t)N * H * W;
  hipLaunchKernelGGL(b0_bwd_kernel, dim3(rdx_sincnet_b0_nblk(npix)), dim3(SN_THREADS), 0, as_stream(stream),
                     (const __hip_bfloat16*)x, (const __hip_bfloat16*)dc, (const __hip_bfloat16*)di, w1, wd, dx, part,
                     npix, H, W);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
