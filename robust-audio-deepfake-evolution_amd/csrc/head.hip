// Fused pieces of the detector head (src/models/DualStreamSEMamba.py:492-531, SELayer inside DualStreamFusion) for
// the training passes under autocast: the squeeze-excitation over time as one launch forward and two backward.
//
//   m = mean_t(x)              [B, C]   (AdaptiveAvgPool1d(1) of the 16-bit x: fp32 sum, one rounding)
//   h = relu(m W1^T)           [B, R]   (fc1, R = C / 16, no bias; the GEMM rounds once to 16 bits)
//   s = sigmoid(h W2^T)        [B, C]   (fc2, no bias; rounded, sigmoid rounded)
//   y = x * s                  [B, T, C]
// Every value autocast keeps in 16 bits is rounded to the storage type where autocast's op would round it, so the
// launches reproduce the module path's values up to the order of fp32 sums. Backward (one workgroup per utterance,
// then a fixed-order reduction): ds = sum_t round(dy x), dz = round(ds s (1 - s)), dh = round(dz W2) (relu'),
// dm = round(dh W1), dx = round(dy s) + round(dm / T) (the two branches' gradients added in 16 bits, as autograd
// adds them); dW2 = sum_b dz^T h and dW1 = sum_b dh^T m in fp32, per-utterance partial rows summed in utterance
// order and ADDED into the caller's fp32 .grad buffers.
// The torch ops this replaces (mean, two small GEMMs, relu, sigmoid, the product; their backward kernels, the
// broadcast-sum and cast, the two-branch add) were ~20 launches per pass for ~58 KB of activations per utterance.
#include "common.h"

namespace rdx {

constexpr int SE_T = 256;        // threads
constexpr int SE_CMAX = 256;     // channels
constexpr int SE_RMAX = 16;      // squeeze width
constexpr int SE_CH = 8;         // channels per 16-byte chunk

struct SeArgs {
  const hst* x;     // [B, T, C]
  const hst* w1;    // [R, C] (16-bit, autocast's cast of fc1.weight)
  const hst* w2;    // [C, R]
  hst* y;           // [B, T, C]
  hst* m;           // [B, C] saved for the backward
  hst* h;           // [B, R]
  hst* s;           // [B, C]
  int B, T, C, R;
};

// column sums over t of rows [T, C] (16-byte chunks): thread (chunk q, row group g) sums rows g, g + G, ...; the
// G partial sums of a chunk reduced through LDS. f(t, chunk j) -> 8 fp32 values added.
template <class F>
__device__ __forceinline__ void se_colsum(float* red, float* out, int T, int C, F f) {
  const int nq = C / SE_CH, G = SE_T / nq;   // nq <= 32 chunks, G >= 8 row groups
  const int q = threadIdx.x % nq, g = threadIdx.x / nq;
  float acc[SE_CH];
#pragma unroll
  for (int k = 0; k < SE_CH; ++k) acc[k] = 0.f;
  if (g < G)
    for (int t = g; t < T; t += G) f(t, q, acc);
  __syncthreads();
  if (g < G)
#pragma unroll
    for (int k = 0; k < SE_CH; ++k) red[(g * nq + q) * SE_CH + k] = acc[k];
  __syncthreads();
  if (threadIdx.x < C) {
    const int c = threadIdx.x, qq = c / SE_CH, k = c % SE_CH;
    float sum = 0.f;
    for (int gg = 0; gg < G; ++gg) sum += red[(gg * nq + qq) * SE_CH + k];
    out[c] = sum;
  }
  __syncthreads();
}

__device__ __forceinline__ void se_unpack(uint4 u, float* v) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = hlo(w[j]);
    v[2 * j + 1] = hhi(w[j]);
  }
}

__global__ __launch_bounds__(SE_T) void se_fwd_kernel(SeArgs a) {
  __shared__ float red[SE_T * SE_CH];
  __shared__ float sm[SE_CMAX], sh[SE_RMAX], ss[SE_CMAX];
  const int b = blockIdx.x, T = a.T, C = a.C, R = a.R;
  const hst* xb = a.x + (int64_t)b * T * C;
  se_colsum(red, sm, T, C, [&](int t, int q, float* acc) {
    float v[SE_CH];
    se_unpack(*reinterpret_cast<const uint4*>(xb + (int64_t)t * C + q * SE_CH), v);
#pragma unroll
    for (int k = 0; k < SE_CH; ++k) acc[k] += v[k];
  });
  if (threadIdx.x < C) {
    const int c = threadIdx.x;
    const float mv = hround(sm[c] * (1.0f / (float)T));
    sm[c] = mv;
    a.m[(int64_t)b * C + c] = f2h(mv);
  }
  __syncthreads();
  if (threadIdx.x < R) {   // fc1 + relu
    const int j = threadIdx.x;
    float acc = 0.f;
    for (int c = 0; c < C; ++c) acc = fmaf(sm[c], h2f(a.w1[(int64_t)j * C + c]), acc);
    const float hv = fmaxf(hround(acc), 0.f);
    sh[j] = hv;
    a.h[(int64_t)b * R + j] = f2h(hv);
  }
  __syncthreads();
  if (threadIdx.x < C) {   // fc2 + sigmoid
    const int c = threadIdx.x;
    float acc = 0.f;
    for (int j = 0; j < R; ++j) acc = fmaf(sh[j], h2f(a.w2[(int64_t)c * R + j]), acc);
    const float z = hround(acc);
    const float sv = hround(1.0f / (1.0f + __expf(-z)));
    ss[c] = sv;
    a.s[(int64_t)b * C + c] = f2h(sv);
  }
  __syncthreads();
  // y = x * s: 16-byte chunks, consecutive threads on consecutive chunks
  const int nq = C / SE_CH;
  hst* yb = a.y + (int64_t)b * T * C;
  for (int i = threadIdx.x; i < T * nq; i += SE_T) {
    const int t = i / nq, q = i % nq;
    float v[SE_CH];
    se_unpack(*reinterpret_cast<const uint4*>(xb + (int64_t)t * C + q * SE_CH), v);
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = hpack2(v[2 * j] * ss[q * SE_CH + 2 * j], v[2 * j + 1] * ss[q * SE_CH + 2 * j + 1]);
    *reinterpret_cast<uint4*>(yb + (int64_t)t * C + q * SE_CH) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

struct SeBwdArgs {
  const hst* dy;    // [B, T, C]
  const hst* x;
  const hst* w1;
  const hst* w2;
  const hst* m;
  const hst* h;
  const hst* s;
  hst* dx;          // [B, T, C]
  float* part;      // [B, R * C + C * R]: dW1 [R, C] then dW2 [C, R], per utterance
  int B, T, C, R;
};

__global__ __launch_bounds__(SE_T) void se_bwd_kernel(SeBwdArgs a) {
  __shared__ float red[SE_T * SE_CH];
  __shared__ float sds[SE_CMAX], sdz[SE_CMAX], sdh[SE_RMAX], sdm[SE_CMAX], ssv[SE_CMAX];
  const int b = blockIdx.x, T = a.T, C = a.C, R = a.R;
  const hst* dyb = a.dy + (int64_t)b * T * C;
  const hst* xb = a.x + (int64_t)b * T * C;
  // ds = sum_t round(dy * x)
  se_colsum(red, sds, T, C, [&](int t, int q, float* acc) {
    float d[SE_CH], v[SE_CH];
    se_unpack(*reinterpret_cast<const uint4*>(dyb + (int64_t)t * C + q * SE_CH), d);
    se_unpack(*reinterpret_cast<const uint4*>(xb + (int64_t)t * C + q * SE_CH), v);
#pragma unroll
    for (int k = 0; k < SE_CH; ++k) acc[k] += hround(d[k] * v[k]);
  });
  float* prow = a.part + (int64_t)b * (2 * R * C);
  if (threadIdx.x < C) {   // sigmoid backward; dW2 [C, R] row c = dz[c] h
    const int c = threadIdx.x;
    const float sv = h2f(a.s[(int64_t)b * C + c]);
    ssv[c] = sv;
    const float dz = hround(hround(sds[c]) * (sv * (1.0f - sv)));
    sdz[c] = dz;
    for (int j = 0; j < R; ++j) prow[R * C + c * R + j] = dz * h2f(a.h[(int64_t)b * R + j]);
  }
  __syncthreads();
  if (threadIdx.x < R) {   // fc2's input gradient, relu'
    const int j = threadIdx.x;
    float acc = 0.f;
    for (int c = 0; c < C; ++c) acc = fmaf(sdz[c], h2f(a.w2[(int64_t)c * R + j]), acc);
    sdh[j] = h2f(a.h[(int64_t)b * R + j]) > 0.f ? hround(acc) : 0.f;
  }
  __syncthreads();
  if (threadIdx.x < C) {   // fc1's input gradient; dW1 [R, C] column c = dh m[c]; the mean's backward
    const int c = threadIdx.x;
    float acc = 0.f;
    const float mv = h2f(a.m[(int64_t)b * C + c]);
    for (int j = 0; j < R; ++j) {
      acc = fmaf(sdh[j], h2f(a.w1[(int64_t)j * C + c]), acc);
      prow[j * C + c] = sdh[j] * mv;
    }
    sdm[c] = hround(hround(acc) / (float)T);
  }
  __syncthreads();
  const int nq = C / SE_CH;
  hst* dxb = a.dx + (int64_t)b * T * C;
  for (int i = threadIdx.x; i < T * nq; i += SE_T) {
    const int t = i / nq, q = i % nq;
    float d[SE_CH];
    se_unpack(*reinterpret_cast<const uint4*>(dyb + (int64_t)t * C + q * SE_CH), d);
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c0 = q * SE_CH + 2 * j;
      o[j] = hpack2(hround(d[2 * j] * ssv[c0]) + sdm[c0], hround(d[2 * j + 1] * ssv[c0 + 1]) + sdm[c0 + 1]);
    }
    *reinterpret_cast<uint4*>(dxb + (int64_t)t * C + q * SE_CH) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// grad[i] += sum_b part[b][i] (utterance order), i < n: dW1 into g1 [R * C], then dW2 into g2 [C * R]
__global__ __launch_bounds__(256) void se_wgrad_kernel(const float* __restrict__ part, int B, int n1, int n2,
                                                       float* __restrict__ g1, float* __restrict__ g2) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n1 + n2) return;
  float sum = 0.f;
  for (int b = 0; b < B; ++b) sum += part[(int64_t)b * (n1 + n2) + i];
  if (i < n1) g1[i] += sum;
  else g2[i - n1] += sum;
}


// ---- Attention pooling of the head (src/models/DualStreamSEMamba.py:700-770, Model.forward's tail) under autocast:
//   z = round(f w^T + b) [B, T] (attention_pool, a 1-output linear), a = softmax_t(z) in fp32, a16 = round(a),
//   feat = round(a16^T f) [B, C] (autocast's bmm on the 16-bit attention weights).
// One workgroup per utterance, f [T, C] read twice (scores, then the weighted sum). Backward from dfeat [B, C]:
//   da = round(f dfeat) [T], df1 = round(a16 dfeat^T); dz = round(a (da - sum_t a da)) (softmax backward in fp32 on the
//   fp32 output, then the cast back to z's dtype); df2 = round(dz w); df = round(df1 + df2) (the two branches' 16-bit
//   add); dw = sum dz f, db = sum dz in fp32, per-utterance partials summed in utterance order into .grad.
constexpr int AP_T = 256;
constexpr int AP_TMAX = 1024;

struct ApArgs {
  const hst* f;      // [B, T, C]
  const hst* w;      // [C] (16-bit)
  const hst* bias;   // [1] (16-bit) or null
  hst* feat;         // [B, C]
  float* a;          // [B, T] fp32 softmax (saved)
  int B, T, C;
};

__device__ __forceinline__ float ap_block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < AP_T / 64; ++i) s += red[i];
  return s;
}
__device__ __forceinline__ float ap_block_max(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = red[0];
#pragma unroll
  for (int i = 1; i < AP_T / 64; ++i) s = fmaxf(s, red[i]);
  return s;
}

__global__ __launch_bounds__(AP_T) void attn_pool_fwd_kernel(ApArgs a) {
  __shared__ float sz[AP_TMAX], red[AP_T / 64];
  const int b = blockIdx.x, T = a.T, C = a.C;
  const hst* fb = a.f + (int64_t)b * T * C;
  const float bias = a.bias ? h2f(a.bias[0]) : 0.f;
  // scores: one wave per row, lanes over channels
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int t = w; t < T; t += AP_T / 64) {
    float acc = 0.f;
    for (int c = lane; c < C; c += 64) acc = fmaf(h2f(fb[(int64_t)t * C + c]), h2f(a.w[c]), acc);
    acc = wave_sum(acc);
    if (lane == 0) sz[t] = hround(acc + bias);
  }
  __syncthreads();
  float mx = -INFINITY;
  for (int t = threadIdx.x; t < T; t += AP_T) mx = fmaxf(mx, sz[t]);
  mx = ap_block_max(mx, red);
  float sum = 0.f;
  for (int t = threadIdx.x; t < T; t += AP_T) {
    const float e = __expf(sz[t] - mx);
    sz[t] = e;
    sum += e;
  }
  sum = ap_block_sum(sum, red);
  const float inv = 1.0f / sum;
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += AP_T) {
    const float av = sz[t] * inv;
    a.a[(int64_t)b * T + t] = av;
    sz[t] = hround(av);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += AP_T) {
    float acc = 0.f;
    for (int t = 0; t < T; ++t) acc = fmaf(sz[t], h2f(fb[(int64_t)t * C + c]), acc);
    a.feat[(int64_t)b * C + c] = f2h(acc);
  }
}

struct ApBwdArgs {
  const hst* f;
  const hst* w;
  const float* a;
  const hst* dfeat;   // [B, C]
  hst* df;            // [B, T, C]
  float* part;        // [B, C + 1]: dw then db per utterance
  int B, T, C;
};

__global__ __launch_bounds__(AP_T) void attn_pool_bwd_kernel(ApBwdArgs a) {
  __shared__ float sa[AP_TMAX], sdz[AP_TMAX], sdf[1024], red[AP_T / 64];
  const int b = blockIdx.x, T = a.T, C = a.C;
  const hst* fb = a.f + (int64_t)b * T * C;
  for (int c = threadIdx.x; c < C; c += AP_T) sdf[c] = h2f(a.dfeat[(int64_t)b * C + c]);
  for (int t = threadIdx.x; t < T; t += AP_T) sa[t] = a.a[(int64_t)b * T + t];
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int t = w; t < T; t += AP_T / 64) {   // da = round(f dfeat)
    float acc = 0.f;
    for (int c = lane; c < C; c += 64) acc = fmaf(h2f(fb[(int64_t)t * C + c]), sdf[c], acc);
    acc = wave_sum(acc);
    if (lane == 0) sdz[t] = hround(acc);
  }
  __syncthreads();
  float dot = 0.f;
  for (int t = threadIdx.x; t < T; t += AP_T) dot = fmaf(sa[t], sdz[t], dot);
  dot = ap_block_sum(dot, red);
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += AP_T) sdz[t] = hround(sa[t] * (sdz[t] - dot));
  __syncthreads();
  // df = round(round(a16 dfeat) + round(dz w)); dw = sum_t dz f, db = sum_t dz
  float* prow = a.part + (int64_t)b * (C + 1);
  for (int c = threadIdx.x; c < C; c += AP_T) {
    const float wc = h2f(a.w[c]), dc = sdf[c];
    float acc = 0.f;
    for (int t = 0; t < T; ++t) {
      const float fv = h2f(fb[(int64_t)t * C + c]);
      acc = fmaf(sdz[t], fv, acc);
      a.df[((int64_t)b * T + t) * C + c] = f2h(hround(hround(sa[t]) * dc) + hround(sdz[t] * wc));
    }
    prow[c] = acc;
  }
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int t = 0; t < T; ++t) s += sdz[t];
    prow[C] = s;
  }
}

__global__ __launch_bounds__(256) void ap_wgrad_kernel(const float* __restrict__ part, int B, int C,
                                                       float* __restrict__ dw, float* __restrict__ db) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i > C) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += part[(int64_t)b * (C + 1) + i];
  if (i < C) dw[i] += s;
  else if (db) db[0] += s;
}

// ---- DualStreamFusion's time alignment and concatenation (src/models/DualStreamSEMamba.py:537-637) under autocast:
//   out[b, t] = [fw[b, t, :] | fs[b, idx(t), :]],  idx(t) = min(floor(t * (T2 / T1)), T2 - 1)  (F.interpolate's
// 'nearest' index, the scale in fp32 as torch computes it; the fp32 round trip autocast makes through the upsample is
// exact for 16-bit values). One launch instead of the casts, the upsample and the cat. Backward of the SincNet half:
//   dfs[b, t2, c] = round(sum_{t: idx(t) = t2} dout[b, t, C + c]) (fp32 sum, one rounding: the upsample's backward
//   in fp32 and autocast's cast back); the WavLM half's gradient is a view of dout.
__device__ __forceinline__ int up_idx(int t, float scale, int T2) {
  const int i = (int)floorf((float)t * scale);
  return i < T2 - 1 ? i : T2 - 1;
}

__global__ __launch_bounds__(256) void upcat_fwd_kernel(const hst* __restrict__ fw, const hst* __restrict__ fs,
                                                        hst* __restrict__ out, int B, int T1, int T2, int C,
                                                        float scale) {
  const int nq = C / 8;                      // 16-byte chunks per half row
  const int64_t n = (int64_t)B * T1 * 2 * nq;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int q2 = (int)(i % (2 * nq));
    const int64_t bt = i / (2 * nq);
    const int t = (int)(bt % T1), b = (int)(bt / T1);
    const hst* src = q2 < nq ? fw + bt * C + q2 * 8
                             : fs + ((int64_t)b * T2 + up_idx(t, scale, T2)) * C + (q2 - nq) * 8;
    *reinterpret_cast<uint4*>(out + bt * 2 * C + q2 * 8) = *reinterpret_cast<const uint4*>(src);
  }
}

__global__ __launch_bounds__(256) void upcat_bwd_kernel(const hst* __restrict__ dout, hst* __restrict__ dfs, int B,
                                                        int T1, int T2, int C, float scale) {
  const int64_t n = (int64_t)B * T2 * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    const int64_t bt2 = i / C;
    const int t2 = (int)(bt2 % T2), b = (int)(bt2 / T2);
    // the t with idx(t) == t2: a run around t2 * T1 / T2 (checked with the forward's own index arithmetic)
    int t0 = (int)((int64_t)t2 * T1 / T2) - 4;
    t0 = t0 < 0 ? 0 : t0;
    float acc = 0.f;
    for (int t = t0; t < T1; ++t) {
      const int k = up_idx(t, scale, T2);
      if (k > t2) break;
      if (k == t2) acc += h2f(dout[((int64_t)b * T1 + t) * 2 * C + C + c]);
    }
    dfs[i] = f2h(acc);
  }
}

}  // namespace rdx

using namespace rdx;

static bool se_shape_ok(int B, int T, int C, int R) {
  return B > 0 && T > 0 && C > 0 && C % SE_CH == 0 && C <= SE_CMAX && R > 0 && R <= SE_RMAX && C / SE_CH <= 32;
}

extern "C" int rdx_se_fwd(const void* x, const void* w1, const void* w2, void* y, void* m, void* h, void* s, int B,
                          int T, int C, int R, void* stream) {
  RDX_REQUIRE(x && w1 && w2 && y && m && h && s && se_shape_ok(B, T, C, R));
  RDX_REQUIRE((((uintptr_t)x | (uintptr_t)y) & 15) == 0);
  SeArgs a{(const hst*)x, (const hst*)w1, (const hst*)w2, (hst*)y, (hst*)m, (hst*)h, (hst*)s, B, T, C, R};
  hipLaunchKernelGGL(se_fwd_kernel, dim3((unsigned)B), dim3(SE_T), 0, as_stream(stream), a);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int64_t rdx_se_bwd_part_floats(int B, int C, int R) { return (int64_t)B * 2 * R * C; }

extern "C" int rdx_se_bwd(const void* dy, const void* x, const void* w1, const void* w2, const void* m, const void* h,
                          const void* s, void* dx, float* part, float* dw1, float* dw2, int B, int T, int C, int R,
                          void* stream) {
  RDX_REQUIRE(dy && x && w1 && w2 && m && h && s && dx && part && dw1 && dw2 && se_shape_ok(B, T, C, R));
  RDX_REQUIRE((((uintptr_t)dy | (uintptr_t)x | (uintptr_t)dx) & 15) == 0);
  SeBwdArgs a{(const hst*)dy, (const hst*)x, (const hst*)w1, (const hst*)w2, (const hst*)m, (const hst*)h,
              (const hst*)s, (hst*)dx, part, B, T, C, R};
  hipLaunchKernelGGL(se_bwd_kernel, dim3((unsigned)B), dim3(SE_T), 0, as_stream(stream), a);
  RDX_LAUNCH_CHECK();
  const int n = 2 * R * C;
  hipLaunchKernelGGL(se_wgrad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), part, B,
                     R * C, R * C, dw1, dw2);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_attn_pool_fwd(const void* f, const void* w, const void* bias, void* feat, float* a, int B, int T,
                                 int C, void* stream) {
  RDX_REQUIRE(f && w && feat && a && B > 0 && T > 0 && T <= AP_TMAX && C > 0 && C <= 1024);
  ApArgs g{(const hst*)f, (const hst*)w, (const hst*)bias, (hst*)feat, a, B, T, C};
  hipLaunchKernelGGL(attn_pool_fwd_kernel, dim3((unsigned)B), dim3(AP_T), 0, as_stream(stream), g);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_attn_pool_bwd(const void* f, const void* w, const float* a, const void* dfeat, void* df, float* part,
                                 float* dw, float* db, int B, int T, int C, void* stream) {
  RDX_REQUIRE(f && w && a && dfeat && df && part && dw && B > 0 && T > 0 && T <= AP_TMAX && C > 0 && C <= 1024);
  ApBwdArgs g{(const hst*)f, (const hst*)w, a, (const hst*)dfeat, (hst*)df, part, B, T, C};
  hipLaunchKernelGGL(attn_pool_bwd_kernel, dim3((unsigned)B), dim3(AP_T), 0, as_stream(stream), g);
  RDX_LAUNCH_CHECK();
  hipLaunchKernelGGL(ap_wgrad_kernel, dim3((unsigned)((C + 1 + 255) / 256)), dim3(256), 0, as_stream(stream), part, B,
                     C, dw, db);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_upcat_fwd(const void* fw, const void* fs, void* out, int B, int T1, int T2, int C, void* stream) {
  RDX_REQUIRE(fw && fs && out && B > 0 && T1 > 0 && T2 > 0 && C > 0 && C % 8 == 0);
  RDX_REQUIRE((((uintptr_t)fw | (uintptr_t)fs | (uintptr_t)out) & 15) == 0);
  const int64_t n = (int64_t)B * T1 * (C / 4);
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(upcat_fwd_kernel, dim3((unsigned)grid), dim3(256), 0, as_stream(stream), (const hst*)fw,
                     (const hst*)fs, (hst*)out, B, T1, T2, C, (float)T2 / (float)T1);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_upcat_bwd(const void* dout, void* dfs, int B, int T1, int T2, int C, void* stream) {
  RDX_REQUIRE(dout && dfs && B > 0 && T1 > 0 && T2 > 0 && C > 0);
  const int64_t n = (int64_t)B * T2 * C;
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(upcat_bwd_kernel, dim3((unsigned)grid), dim3(256), 0, as_stream(stream), (const hst*)dout,
                     (hst*)dfs, B, T1, T2, C, (float)T2 / (float)T1);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
