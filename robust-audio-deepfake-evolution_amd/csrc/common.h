// Shared helpers for the radhip HIP kernels (gfx950 only: wave64, CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include "../../include/radhip.h"

#define RDX_WAVE 64

#define RDX_LAUNCH_CHECK()                          \
  do {                                              \
    hipError_t e_ = hipGetLastError();              \
    if (e_ != hipSuccess) return (int)e_;           \
  } while (0)

#define RDX_REQUIRE(cond)                           \
  do {                                              \
    if (!(cond)) return RDX_EINVAL;                 \
  } while (0)

namespace rdx {

// ---- The 16-bit storage type of this build ----------------------------------------------------------------------
// libradhip.so keeps activations and GEMM / conv operands in bf16; libradhip_f16.so is the same sources built with
// -DRDX_F16 and keeps them in IEEE fp16, the reference's autocast dtype (src/main.py:28,1049). On gfx950 both MFMA
// forms (v_mfma_f32_{32x32x16,16x16x32}_{bf16,f16}) take the same cycles. Kernels reach the storage type only
// through the names below: hst (the element), hel (the MFMA vector element), hx8 / hx4v (operand vectors),
// h2f / f2h / hround (conversion, round to nearest even), hlo / hhi (the value of the low / high half-word of a
// packed pair), hbits / hpack2 (the rounded 16-bit pattern of a float, two of them packed), the MFMA wrappers and
// the transposed LDS read. All arithmetic stays fp32.
#ifdef RDX_F16
typedef __half hst;
typedef _Float16 hel;
#else
typedef __hip_bfloat16 hst;
typedef __bf16 hel;
#endif
typedef __attribute__((ext_vector_type(8))) hel hx8;
typedef __attribute__((__vector_size__(4 * sizeof(hel)))) hel hx4v;
typedef __attribute__((__vector_size__(4 * sizeof(short)))) short rdx_s4v;
typedef __attribute__((address_space(3))) rdx_s4v rdx_lds_s4v;
typedef __attribute__((ext_vector_type(16))) float rdx_f32x16;
typedef __attribute__((ext_vector_type(4))) float rdx_f32x4;

#ifdef RDX_F16
__device__ __forceinline__ float h2f(hst x) { return __half2float(x); }
__device__ __forceinline__ hst f2h(float x) { return __float2half(x); }
__device__ __forceinline__ uint32_t hbits_of(hst x) { return (uint32_t)__half_as_ushort(x); }
__device__ __forceinline__ float hlo(uint32_t u) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(u & 0xffffu)); }
__device__ __forceinline__ float hhi(uint32_t u) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(u >> 16)); }
__device__ __forceinline__ rdx_f32x16 mfma32x32x16(hx8 a, hx8 b, rdx_f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ rdx_f32x4 mfma16x16x32(hx8 a, hx8 b, rdx_f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// c + a.lo * b.lo + a.hi * b.hi of two packed 16-bit pairs, fp32 accumulate (v_dot2c_f32_f16)
__device__ __forceinline__ float hdot2(uint32_t a, uint32_t b, float c) {
  typedef __attribute__((ext_vector_type(2))) _Float16 rdx_h2;
  return __builtin_amdgcn_fdot2(__builtin_bit_cast(rdx_h2, a), __builtin_bit_cast(rdx_h2, b), c, false);
}
#else
__device__ __forceinline__ float h2f(hst x) { return __bfloat162float(x); }
__device__ __forceinline__ hst f2h(float x) { return __float2bfloat16(x); }
__device__ __forceinline__ uint32_t hbits_of(hst x) { return (uint32_t)__bfloat16_as_ushort(x); }
__device__ __forceinline__ float hlo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hhi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ rdx_f32x16 mfma32x32x16(hx8 a, hx8 b, rdx_f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ rdx_f32x4 mfma16x16x32(hx8 a, hx8 b, rdx_f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// c + a.lo * b.lo + a.hi * b.hi of two packed 16-bit pairs, fp32 accumulate (v_dot2c_f32_bf16)
__device__ __forceinline__ float hdot2(uint32_t a, uint32_t b, float c) {
  typedef __attribute__((ext_vector_type(2))) __bf16 rdx_b2;
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(rdx_b2, a), __builtin_bit_cast(rdx_b2, b), c, false);
}
#endif
__device__ __forceinline__ float hround(float x) { return h2f(f2h(x)); }
__device__ __forceinline__ uint32_t hbits(float x) { return hbits_of(f2h(x)); }
__device__ __forceinline__ uint32_t hpack2(float lo, float hi) { return hbits(lo) | (hbits(hi) << 16); }
// ds_read_b64_tr_b16 from an LDS address (4 16-bit elements of the lane's transposed column)
__device__ __forceinline__ hx4v ds_tr4(const void* lds) {
  return __builtin_bit_cast(hx4v, __builtin_amdgcn_ds_read_tr16_b64_v4i16((rdx_lds_s4v*)(lds)));
}

// GELU (erf form, HF "gelu" = torch.nn.functional.gelu) for the GEMM epilogues (csrc/hgemm.hip, csrc/lgemm.hip), with erf by Abramowitz & Stegun 7.1.26
// (|error| <= 1.5e-7, below the fp32 rounding the result then takes to bf16 / fp16): one reciprocal, one exp2 and
// five FMAs instead of erff's piecewise polynomial, which made the VALU tail of a 256 x 256 FFN1 tile longer than its
// stores. With z = x / sqrt(2) and q = P(t) exp(-z^2) = 1 - erf(|z|): 1 + erf(z) = 2 - q (z >= 0) or q (z < 0), and
// exp(-z^2) = exp(-x^2 / 2) also gives the normal density of the GELU derivative.
struct GeluParts {
  float one_p_erf;   // 1 + erf(x / sqrt(2))
  float e;           // exp(-x^2 / 2)
};
__device__ __forceinline__ GeluParts gelu_parts(float x) {
  const float ax = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float y = fmaf(t, 1.061405429f, -1.453152027f);
  y = fmaf(t, y, 1.421413741f);
  y = fmaf(t, y, -0.284496736f);
  y = fmaf(t, y, 0.254829592f);
  y *= t;
  const float e = __builtin_amdgcn_exp2f(-x * x * 0.72134752044448170f);   // exp(-x^2/2) = 2^(-x^2 log2(e) / 2)
  const float q = y * e;
  return GeluParts{x >= 0.f ? 2.0f - q : q, e};
}
__device__ __forceinline__ float gelu(float x) { return 0.5f * x * gelu_parts(x).one_p_erf; }
__device__ __forceinline__ float gelu_grad(float x) {
  const GeluParts g = gelu_parts(x);
  return fmaf(x * 0.39894228040143268f, g.e, 0.5f * g.one_p_erf);
}
// Storage-type adapters: all arithmetic is fp32.
template <typename T> __device__ __forceinline__ float ld(const T* p, int64_t i);
template <> __device__ __forceinline__ float ld<float>(const float* p, int64_t i) { return p[i]; }
template <> __device__ __forceinline__ float ld<hst>(const hst* p, int64_t i) { return h2f(p[i]); }
template <typename T> __device__ __forceinline__ void st(T* p, int64_t i, float v);
template <> __device__ __forceinline__ void st<float>(float* p, int64_t i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void st<hst>(hst* p, int64_t i, float v) { p[i] = f2h(v); }

__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }
// F.softplus(x) with the default threshold 20 (mamba_ssm: delta <= 20 ? log1p(exp(delta)) : delta)
__device__ __forceinline__ float softplusf_(float x) { return x <= 20.f ? log1pf(expf(x)) : x; }

// Sum over the 16 lanes of a DPP row (lanes 16r..16r+15); every lane of the row gets the sum.
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, false));  // row_ror:8
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xF, 0xF, false));  // row_ror:4
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x122, 0xF, 0xF, false));  // row_ror:2
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x121, 0xF, 0xF, false));  // row_ror:1
  return v;
}

// Sum over the 64 lanes, the same value in every lane, on the VALU's lane-crossing paths instead of LDS permutes
// (six dependent ds_bpermute round trips were the latency floor of every one-wave-per-row reduction): xor 1 and
// xor 2 by DPP quad_perm, the quads of each 8-lane half by row_half_mirror (quads 0 <-> 1), the halves of a row by
// row_mirror (quads 0 <-> 3, 1 <-> 2), then rows by permlane16_swap and halves of the wave by permlane32_swap.
// Every step adds a lane's value to its mirror's, whose value is the same sum in the other order, so all lanes hold
// the bit-identical total. Call with the whole wave active (DPP reads of switched-off lanes return 0).
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f32<0xB1>(v);    // quad_perm [1, 0, 3, 2]: xor 1
  v += dpp_f32<0x4E>(v);    // quad_perm [2, 3, 0, 1]: xor 2
  v += dpp_f32<0x141>(v);   // row_half_mirror
  v += dpp_f32<0x140>(v);   // row_mirror
  {
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(p[0]) + __uint_as_float(p[1]);    // rows 0 + 1, 2 + 3
  }
  {
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(p[0]) + __uint_as_float(p[1]);    // lanes 0-31 + 32-63
  }
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Counter-hash dropout shared by every fused kernel: element `idx` is kept iff hash(seed, idx) >= p * 2^32,
// so a backward pass regenerates the forward mask from (seed, salt, idx) alone.
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
// dropout keep decision for element index idx = ((b*H + h)*T + i)*T + j
__device__ __forceinline__ bool drop_keep(uint64_t seed, uint64_t idx, uint32_t thr) {
  // one murmur3 finaliser over the (bijectively) mixed 64-bit index and seed
  const uint32_t x = (((uint32_t)idx ^ (uint32_t)seed) * 0x9E3779B1u) ^ (uint32_t)(idx >> 32) ^
                     ((uint32_t)(seed >> 32) * 0x85ebca6bu);
  return fmix32(x) >= thr;
}
// The same decision for an index below 2^32 (then idx >> 32 contributes 0), with the seed words mixed once:
// drop_keep32(drop_key32(seed), idx, thr) == drop_keep(seed, idx, thr) for every idx < 2^32.
struct DropKey32 {
  uint32_t lo, hi;
};
__device__ __forceinline__ DropKey32 drop_key32(uint64_t seed) {
  return DropKey32{(uint32_t)seed, (uint32_t)(seed >> 32) * 0x85ebca6bu};
}
__device__ __forceinline__ bool drop_keep32(DropKey32 k, uint32_t idx, uint32_t thr) {
  return fmix32(((idx ^ k.lo) * 0x9E3779B1u) ^ k.hi) >= thr;
}
// Attention dropout (csrc/attention.hip): one hash per PAIR of keys (2j, 2j + 1) of a score row; key 2j
// is kept iff the low 16 bits of the hash are >= thr16 = p * 2^16, key 2j + 1 iff the high 16 bits are.
// Pair id = row * ceil(T / 2) + key / 2 with row = (b * H + h) * T + q. pair_hash32 == pair_hash for
// pair ids below 2^32.
__device__ __forceinline__ uint32_t pair_hash(uint64_t seed, uint64_t pid) {
  return fmix32((((uint32_t)pid ^ (uint32_t)seed) * 0x9E3779B1u) ^ (uint32_t)(pid >> 32) ^
                ((uint32_t)(seed >> 32) * 0x85ebca6bu));
}
__device__ __forceinline__ uint32_t pair_hash32(DropKey32 k, uint32_t pid) {
  return fmix32(((pid ^ k.lo) * 0x9E3779B1u) ^ k.hi);
}
__device__ __forceinline__ bool half_keep(uint32_t h, bool odd, uint32_t thr16) {
  return (odd ? (h >> 16) : (h & 0xffffu)) >= thr16;
}
__device__ __forceinline__ uint64_t attn_seed(const int64_t* seed_dev, int salt) {
  return (uint64_t)seed_dev[0] * 0x9E3779B97F4A7C15ull + (uint64_t)(uint32_t)salt * 0xD1B54A32D192ED03ull;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace rdx
