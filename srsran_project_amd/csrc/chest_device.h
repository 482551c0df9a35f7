// chest_device.h -- device helpers of the PUSCH DM-RS channel estimator shared by its expansion kernel
// (pusch_chest.hip chest_expand_kernel) and the PUSCH demodulator's fused equalizer (pusch_demod.hip),
// which rebuilds each RE's estimate from the estimator's per-subcarrier values with the SAME operations
// instead of reading an expanded estimate tensor from HBM; the virtual pilots of the FD filter are shared with
// the PUCCH Format 2 estimator (pucch.hip).
// Complex products follow the reference's AVX2+FMA srsran_simd_cf_prod
// (re = fma(a.re, b.re, -a.im b.im), im = fma(a.re, b.im, a.im b.re)).
#pragma once

#include <hip/hip_runtime.h>

#include "bf16_device.h"

#include <cstdint>

#include "pusch_chest_args.h"

namespace srs_amd {
namespace chdev {

constexpr float TWOPI_F = 6.28318530717958647692f;

__device__ __forceinline__ float2 cmul(float2 a, float2 b)
{
  return make_float2(__builtin_fmaf(a.x, b.x, -(a.y * b.y)), __builtin_fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 from_cbf16(uint32_t u)
{
  return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u));
}
__device__ __forceinline__ uint32_t bf16_bits(float f)
{
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}
__device__ __forceinline__ uint32_t to_cbf16(float2 v)
{
  return cbf16_pack(v.x, v.y); // == bf16_bits(v.x) | bf16_bits(v.y) << 16 (bf16_device.h)
}
__device__ __forceinline__ float2 polar1(float theta)
{
  float s, c;
  sincosf(theta, &s, &c);
  return make_float2(c, s);
}

// cmul as one packed multiply and one packed FMA (v_pk_mul_f32, v_pk_fma_f32): per component the same two roundings
// as cmul -- the product a.y b.y (or a.y b.x) rounded, then one fused multiply-add -- so the bits are cmul's.
__device__ __forceinline__ float2 cmul_pk(float2 a, float2 b)
{
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 av = {a.x, a.y}, bv = {b.x, b.y};
  f2       t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(t) : "v"(av), "v"(bv)); // (a.y b.y, a.y b.x)
  // (a.x b.x - t.x, a.x b.y + t.y)
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_lo:[0,0,1]" : "=v"(r) : "v"(av), "v"(bv), "v"(t));
  return make_float2(r.x, r.y);
}

// CFO phase of OFDM symbol l for a port whose estimator accumulators are acc[0..7]
// (port_channel_estimator_average_impl.cpp:184-193).
__device__ __forceinline__ float2 cfo_phase(const chest_args& a, const float* acc, uint32_t l)
{
  return polar1(TWOPI_F * a.epoch[l] * acc[4]);
}
__device__ __forceinline__ bool cfo_rotates(const chest_args& a, const float* acc)
{
  return a.compensate_cfo && acc[3] != 0.0f;
}

// The cbf16 estimate of symbol l of a subcarrier inside the allocation from the LSE slices it reads
// (x0 = slice i0 of the symbol -- td_i0[l], 0 when averaging -- and x1 = slice i0 + 1): the time-domain
// strategy (average or interpolation), bf16 rounding, then the CFO rotation and a second rounding
// (do_compute, port_channel_estimator_average_impl.cpp:184-193 / 390-440).
__device__ __forceinline__ uint32_t expand_pair(const chest_args& a, float2 x0, float2 x1, uint32_t l, bool rot,
                                                float2 ph)
{
  float2 e = x0;
  if (a.td != SRS_AMD_CHEST_TD_AVERAGE && a.td_interp[l]) {
    const float w = a.td_w[l];
    e             = make_float2(__builtin_fmaf(x1.x - x0.x, w, x0.x), __builtin_fmaf(x1.y - x0.y, w, x0.y));
  }
  uint32_t out = to_cbf16(e);
  if (rot) {
    out = to_cbf16(cmul_pk(from_cbf16(out), ph));
  }
  return out;
}

// Slice index i0 of symbol l (the first of the two expand_pair reads).
__device__ __forceinline__ int lse_index(const chest_args& a, uint32_t l)
{
  return a.td == SRS_AMD_CHEST_TD_AVERAGE ? 0 : a.td_i0[l];
}

// expand_pair with every LSE slice of the subcarrier in registers (x[0 .. nof_lse)).
template <int NLSE>
__device__ __forceinline__ uint32_t expand_value(const chest_args& a, const float2 (&x)[NLSE], uint32_t l, bool rot,
                                                 float2 ph)
{
  auto lse = [&](int i) { // x[i] without dynamic register indexing
    float2 r = x[0];
#pragma unroll
    for (int s = 1; s < NLSE; ++s) {
      r = i == s ? x[s] : r;
    }
    return r;
  };
  const int i0 = lse_index(a, l);
  return expand_pair(a, lse(i0), lse(i0 + 1), l, rot, ph);
}

// compute_v_pilots (port_channel_estimator_helpers.cpp:334-378) over one wave: lane i < n <= 12 computes the
// modulus / argument of value i and output value i; the short serial parts (phase unwrapping, the four
// sums) run redundantly in every lane on the shuffled values, in the reference's order.  One lane running
// the whole function was a chain of 3 n transcendental functions on the slice kernel's critical path.
__device__ inline void virtual_pilots_wave(float2* out, const float2* in, int n, bool is_start)
{
#pragma clang fp contract(off)
  const int lane = static_cast<int>(threadIdx.x & 63u);
  float     av = 0, gv = 0;
  if (lane < n) {
    av = sqrtf(in[lane].x * in[lane].x + in[lane].y * in[lane].y);
    gv = atan2f(in[lane].y, in[lane].x);
  }
  float absv[CH_MAXV], argv[CH_MAXV];
#pragma unroll
  for (int i = 0; i < CH_MAXV; ++i) {
    absv[i] = __shfl(av, i);
    argv[i] = __shfl(gv, i);
  }
  // unwrap_list (unwrap.cpp:42-62)
  const float width = 3.14159265358979323846f;
  float       k     = 0;
#pragma unroll
  for (int i = 0; i < CH_MAXV - 1; ++i) {
    if (i < n - 1) {
      const float old_a = argv[i], next_a = argv[i + 1];
      argv[i] += 2.0f * k * width;
      const float jump = next_a - old_a;
      if (fabsf(jump) > width) {
        k = k - copysignf(1.0f, jump);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < CH_MAXV; ++i) {
    if (i == n - 1) {
      argv[i] += 2.0f * k * width;
    }
  }
  const float mean_x    = static_cast<float>(n * (n - 1)) / 2.0f / n;
  const float norm_x_sq = static_cast<float>((n - 1) * n * (2 * n - 1)) / 6.0f;
  float       sa = 0, sg = 0, ma = 0, mg = 0;
#pragma unroll
  for (int i = 0; i < CH_MAXV; ++i) {
    if (i < n) {
      ma += absv[i];
      mg += argv[i];
      sa += absv[i] * static_cast<float>(i);
      sg += argv[i] * static_cast<float>(i);
    }
  }
  ma /= n;
  mg /= n;
  sa -= mean_x * ma * n;
  sa /= (norm_x_sq - n * mean_x * mean_x);
  sg -= mean_x * mg * n;
  sg /= (norm_x_sq - n * mean_x * mean_x);
  const float ia  = ma - sa * mean_x;
  const float ig  = mg - sg * mean_x;
  const int   off = is_start ? -n : n;
  if (lane < n) {
    const int   iv  = lane + off;
    const float rho = sa * iv + ia;
    const float ph  = sg * iv + ig + ((rho > 0) ? 0.0f : 3.14159265358979323846f);
    const float r   = fabsf(rho);
    out[lane]       = make_float2(r * cosf(ph), r * sinf(ph));
  }
}

} // namespace chdev
} // namespace srs_amd
