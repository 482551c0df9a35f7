// chest_device.h -- device helpers of the PUSCH DM-RS channel estimator shared by its expansion kernel
// (pusch_chest.hip chest_expand_kernel) and the PUSCH demodulator's fused equalizer (pusch_demod.hip),
// which rebuilds each RE's estimate from the estimator's per-subcarrier values with the SAME operations
// instead of reading an expanded estimate tensor from HBM.
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
    out = to_cbf16(cmul(from_cbf16(out), ph));
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

} // namespace chdev
} // namespace srs_amd
